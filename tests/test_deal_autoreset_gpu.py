"""The NPC-aware deal (traffic) decides how many NPC slots a car wave
loads: the env's class, its NPC count after the previous step.  A step with
MEV_AUTO_RESET files every env that ended into class 0 (its auto-reset empties the
fleet).  When the next step runs WITHOUT the auto-reset, those envs keep their NPCs
(the reference steps on: env.py only resets on request), so that class is no bound:
the step must deal afresh (mev_capi.cpp deal_ar).  Here every env truncates at step 10
under auto-reset, the next steps run without it, then with it again; every output
and the NPC state are compared with the oracle (reset() then step() where the device
auto-reset), on the fused traffic kernel and on the traffic early split."""
import numpy as np
import pytest

from conftest import use_step_kernel
import golden_replay as G
import oracle_replay as R

pytestmark = pytest.mark.gpu

ROUTES3 = [(1, 4), (2, 8), (3, 12), (4, 7), (5, 11), (6, 3), (7, 10), (8, 2), (9, 6), (10, 1), (11, 5), (12, 9)]


@pytest.mark.parametrize("split", [1, 3])
def test_deal_classes_survive_a_step_without_auto_reset(mev, split):
    E, RAYS, MAXS = 64, 32, 10
    meta = dict(rays=RAYS, num_lanes=3, n_agents=1, use_team=False, respawn=True, max_steps=MAXS, traffic=True,
                density=5.0, reward=[10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2])
    h = mev.Handle(num_envs=E, num_agents=1, lidar_rays=RAYS, obs_dim=127, traffic_flow=1, traffic_density=5.0,
                   max_steps=MAXS, max_npcs=32, seed=11)
    use_step_kernel(mev, h, 2)
    h.set_serve(0)  # launched steps: the deal runs (the step server deals by identity)
    h.set_env_deal(True)
    h.set_step_split(split)
    assert h.step_split() == (2 if split == 3 else 0), h.step_split()
    troutes = [h.route_id(s - 1, 12 + t - 1) for s, t in ROUTES3]
    h.set_traffic_routes(troutes)
    h.reset()
    st = h.get_state()
    oracles = []
    for e in range(E):
        o = R.make_oracle(meta)
        o.set_traffic_routes(troutes)
        o.reset([int(r) for r in st["route"][e]])
        oracles.append(o)
    rng = np.random.default_rng(5)
    ended = np.zeros(E, bool)
    # auto-reset steps 1-10 (every env truncates at 10), 11-16 without it, 17-30 with it again
    plan = [True] * MAXS + [False] * 6 + [True] * 14
    kept = 0
    for t, ar in enumerate(plan):
        a = rng.uniform(-1, 1, (E, 1, 2)).astype(np.float32)
        spawn = np.where(rng.uniform(size=E) < 0.5, rng.integers(0, len(troutes), E), -1).astype(np.int32)
        out = h.step(a, spawn_route=spawn, auto_reset=ar)
        gst = h.get_state()
        for e in range(E):
            o = oracles[e]
            if ended[e] and ar:  # the device reset this env before stepping it
                o.reset([int(r) for r in gst["route"][e]])
            elif ended[e]:
                kept += int(o.get_state()[1].shape[0] > 0)
            r = o.step(a[e], spawn_route=int(spawn[e]))
            tag = f"step {t + 1} (auto_reset {ar}) env {e}"
            assert G.bits_equal(out["obs"][e], r["obs"]), tag + ": obs"
            assert G.bits_equal(out["reward"][e], r["rew"]), tag + ": reward"
            assert [int(out["terminated"][e]), int(out["truncated"][e]), int(out["agents_alive"][e]),
                    int(out["step"][e])] == [r["terminated"], r["truncated"], r["agents_alive"], r["step"]], tag
            _, npcs, _ = o.get_state()
            k = len(npcs)
            assert int(gst["npc_count"][e]) == k, tag + ": npc count"
            for a_, b_ in (("npc_x", "x"), ("npc_y", "y"), ("npc_v", "v"), ("npc_heading", "h")):
                assert G.bits_equal(gst[a_][e, :k], npcs[b_]), tag + ": " + a_
            ended[e] = bool(r["terminated"] or r["truncated"])
    assert kept > E // 2, kept  # ended envs with NPCs stepped without the reset: the case at stake
    h.close()
