"""Bit-exact parity of the gfx950 step against golden vectors from the REAL
reference simulator (tests/golden/*.npz, see tests/golden/gen_golden.py).
Every output is compared with exact bit equality — stricter than the 1e-5
float tolerance BASELINE.json asks for (obs, rewards, ego/NPC state) and the
bit-exact requirement on crash/success flags."""
import pytest

import golden_replay as G
from conftest import STEP_KERNELS

pytestmark = pytest.mark.gpu

# (per-car LiDAR objects, gen_golden.py gen_lidars: one handle per LiDAR configuration,
# replayed through the drop-in in test_dropin_gpu.py)
SINGLE = [n for n in G.scenario_names() if not n.startswith("inject_egos") and "car_lidars" not in G.load(n)["meta"]]


def _replay(mev, names, kernel):
    reps = G.replay(mev, names, kernel=kernel)
    if reps is None:
        pytest.skip(f"step kernel {kernel} does not apply to this configuration")
    return reps


@pytest.mark.parametrize("kernel", STEP_KERNELS)
@pytest.mark.parametrize("name", SINGLE)
def test_golden_scenario(mev, name, kernel):
    (rep,) = _replay(mev, name, kernel)
    assert rep.ok, f"{name}: {rep.mismatches[:5]} (steps checked {rep.steps})"


@pytest.mark.parametrize("kernel", STEP_KERNELS)
def test_injected_states_batched(mev, kernel):
    # six different injected scenarios as six envs of ONE handle
    reps = _replay(mev, G.scenario_names("inject_egos"), kernel)
    bad = [(r.name, r.mismatches[:3]) for r in reps if not r.ok]
    assert not bad, bad


@pytest.mark.parametrize("kernel", STEP_KERNELS)
@pytest.mark.parametrize("name", ["cfg3_team_policy", "traffic_d20"])
def test_same_scenario_replicated_envs(mev, name, kernel):
    # the same scenario in 37 envs of one handle: every env must match the reference
    reps = _replay(mev, [name] * 37, kernel)
    bad = [i for i, r in enumerate(reps) if not r.ok]
    assert not bad, reps[bad[0]].mismatches[:5]


@pytest.mark.parametrize("kernel", STEP_KERNELS)
def test_dense_traffic_goldens_cover_sequential_fallback(mev, kernel):
    """The traffic goldens at density 20 bit-exact on both kernel paths, and
    reporting how often the NPC controller left its parallel rounds for the
    sequential turns (round B changed a throttle)."""
    reps = _replay(mev, ["traffic_d20"] * 8, kernel)
    bad = [r.mismatches[:3] for r in reps if not r.ok]
    assert not bad, bad
    print(f"kernel {kernel}: sequential NPC turns over 8 x traffic_d20: {reps[0].seq_turns}")


PACKABLE = [n for n in SINGLE if G.load(n)["meta"]["n_agents"] <= 4 and not G.load(n)["meta"]["traffic"]]


@pytest.mark.parametrize("pack", [2, 4, 8])
@pytest.mark.parametrize("name", PACKABLE)
def test_golden_scenario_packed_waves(mev, name, pack):
    """Several envs per fused k_step wave (mev_set_step_pack): each golden
    scenario replicated into 7 envs (the last wave partly filled), every env
    bit-exact against the reference."""
    reps = G.replay(mev, [name] * 7, kernel=2, pack=pack)
    assert reps is not None
    bad = [(i, r.mismatches[:3]) for i, r in enumerate(reps) if not r.ok]
    assert not bad, bad


@pytest.mark.parametrize("split", [1, 2, 3])
@pytest.mark.parametrize("name", [n for n in SINGLE if not G.load(n)["meta"]["traffic"]])
def test_golden_scenario_split_waves(mev, name, split):
    """Each non-traffic golden on the fused kernel with one wave per workgroup
    (split 1), with the car part and the LiDAR in two waves (split 2) -- the
    small-batch default, forced off and on here -- and with the early split
    (3: the LiDAR wave marches the road from the poses after the kinematics; envs
    whose beams exceed one 512-beam pool take the automatic choice); all bit-exact."""
    (rep,) = G.replay(mev, name, kernel=2, split=split)
    assert rep.ok, f"{name}: {rep.mismatches[:5]} (steps checked {rep.steps})"


# (goldens with other car sizes run the runtime-layout kernel, which has no split)
TRAFFIC_ONE_EGO = [n for n in SINGLE if G.load(n)["meta"]["traffic"] and G.load(n)["meta"]["n_agents"] <= 1
                   and not G.has_dims(G.load(n)) and G.npc_slots([G.load(n)]) == 32]


@pytest.mark.parametrize("name", TRAFFIC_ONE_EGO)
def test_golden_scenario_traffic_early_split(mev, name):
    """The traffic early split (two car waves -- NPC phase and car part of one env
    each -- and one LiDAR wave for their egos per workgroup; E divisible by 16): each
    one-ego traffic golden replicated into 32 envs, every env bit-exact against the
    reference, with the split asserted to be the path that ran."""
    h = G.make_handle(mev, G.load(name)["meta"], 32)
    h.set_step_kernel(2)
    h.set_step_split(3)
    assert h.step_split() == 2, "traffic early split not selected"
    h.close()
    reps = G.replay(mev, [name] * 32, kernel=2, split=3)
    bad = [(i, r.mismatches[:3]) for i, r in enumerate(reps) if not r.ok]
    assert not bad, bad


@pytest.mark.parametrize("pack", [2, 4, 8])
def test_golden_routes_packed_in_one_handle(mev, pack):
    """The 12 config-2 route scenarios as 12 envs of ONE handle, 2 or 4 envs per
    fused wave: neighbours in a wave hold different states, each env bit-exact."""
    names = [n for n in SINGLE if n.startswith("cfg2_r64_route")]
    reps = G.replay(mev, names, kernel=2, pack=pack)
    bad = [(r.name, r.mismatches[:3]) for r in reps if not r.ok]
    assert not bad, bad
