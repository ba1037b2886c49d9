"""MEV_AUTO_RESET against the oracle: a device step that auto-resets an env whose
previous step ended must equal the reference wrapper's reset() followed by
step() (reference env.py:147-161: IntersectionEnv::reset + add_car_with_route per
agent, cpp/IntersectionEnv.cpp:66-131, then IntersectionEnv::step), with the
routes the device drew for that reset (mev_set_reset_routes pool, read back with
mev_get_state) -- bit for bit on every output, on both kernel paths."""
import numpy as np
import pytest

from conftest import STEP_KERNELS, use_step_kernel
import oracle_replay as R

pytestmark = pytest.mark.gpu

ROUTES3 = [(1, 4), (2, 8), (3, 12), (4, 7), (5, 11), (6, 3), (7, 10), (8, 2), (9, 6), (10, 1), (11, 5), (12, 9)]


@pytest.mark.parametrize("kernel", STEP_KERNELS)
@pytest.mark.parametrize("pool", [False, True])
def test_auto_reset_equals_oracle_reset_then_step(mev, kernel, pool):
    E, N, RAYS, T, MAXS = 24, 3, 32, 70, 12
    meta = dict(rays=RAYS, num_lanes=3, n_agents=N, use_team=True, respawn=True, max_steps=MAXS, traffic=False,
                density=0.5, reward=[10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2])
    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=RAYS, obs_dim=127, use_team_reward=1, max_steps=MAXS,
                   seed=7, device=0)
    use_step_kernel(mev, h, kernel)
    all_routes = [h.route_id(s - 1, 12 + t - 1) for s, t in ROUTES3]
    if pool:
        h.set_reset_routes(all_routes)  # every reset draws each agent's route from the pool
    h.reset()
    st = h.get_state()
    oracles = []
    for e in range(E):
        o = R.make_oracle(meta)
        o.reset([int(r) for r in st["route"][e]])
        oracles.append(o)
    obs0 = h.observations()
    for e in range(E):
        assert np.array_equal(obs0[e].view(np.uint32), oracles[e].observe().view(np.uint32)), e
    rng = np.random.default_rng(3)
    ended = np.zeros(E, bool)
    resets = 0
    for t in range(T):
        a = rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)
        out = h.step(a, auto_reset=True)
        st = h.get_state()
        for e in range(E):
            o = oracles[e]
            if ended[e]:  # the device reset this env before stepping it: reset() then step()
                routes = [int(r) for r in st["route"][e]]
                if not pool:
                    assert routes == [all_routes[i % 12] for i in range(N)]
                o.reset(routes)
                resets += 1
            r = o.step(a[e])
            assert np.array_equal(out["obs"][e].view(np.uint32), r["obs"].view(np.uint32)), (t, e)
            assert np.array_equal(out["reward"][e].view(np.uint32), r["rew"].view(np.uint32)), (t, e)
            assert np.array_equal(out["status"][e], r["status"]) and np.array_equal(out["done"][e], r["done"])
            assert [int(out["terminated"][e]), int(out["truncated"][e]), int(out["agents_alive"][e]),
                    int(out["step"][e])] == [r["terminated"], r["truncated"], r["agents_alive"], r["step"]], (t, e)
            ended[e] = bool(r["terminated"] or r["truncated"])
    assert resets >= E  # max_steps 12 over 70 steps: every env was auto-reset several times
    h.close()
