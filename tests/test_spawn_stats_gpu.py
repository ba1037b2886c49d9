"""NPC spawn stream semantics.  The reference draws its spawn
coin and route from an unseeded thread_local std::mt19937 (TrafficFlow.cpp:
275-330), so parity is by distribution: per env-step a spawn is attempted with
p = 1 - exp(-density*dt) (computed with glibc expf on the host), the route is
uniform over the traffic routes, and a spawn within 2.5 car lengths (135 px) of
any car is dropped (is_spawn_blocked, :240-259).  Each env draws from its own
Philox4x32-10 counter stream (handle seed, step counter, env)."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

E = 8192


def _one_step_spawns(mev, density, seed):
    h = mev.Handle(num_envs=E, num_agents=1, lidar_rays=16, traffic_flow=1, traffic_density=density,
                   max_npcs=8, seed=seed)
    h.step(np.zeros((E, 1, 2), np.float32))
    st = h.get_state()
    troutes = h.default_traffic_routes()
    h.close()
    return st, troutes


def test_spawn_rate_and_route_distribution(mev):
    density = -math.log(0.7) * 60.0  # p = 0.3 per step at dt = 1/60
    st, troutes = _one_step_spawns(mev, density, seed=11)
    p = 1.0 - float(np.float32(math.exp(-np.float32(density) * np.float32(1 / 60))))
    # the ego starts at IN_1: routes starting in its own arm (within 135 px) are blocked
    h = mev.Handle(num_envs=1, num_agents=1, lidar_rays=16)
    ego_spawn = h.route_info(int(h.get_state()["route"][0, 0]))[2][:2]
    free = [r for r in troutes if np.hypot(*(h.route_info(int(r))[2][:2] - ego_spawn)) >= 135.0]
    h.close()
    assert 0 < len(free) < len(troutes)
    spawned = st["npc_count"][:, 0] if st["npc_count"].ndim == 2 else st["npc_count"]
    n = int((spawned > 0).sum())
    expect = E * p * len(free) / len(troutes)
    sd = math.sqrt(E * (expect / E) * (1 - expect / E))
    assert abs(n - expect) < 5 * sd, (n, expect, sd)
    # routes of the spawned NPCs: uniform over the unblocked routes (chi-square, 5 sigma-ish bound)
    r = st["npc_route"][spawned > 0, 0]
    assert set(np.unique(r).tolist()) <= set(int(x) for x in free)
    counts = np.array([(r == f).sum() for f in free], np.float64)
    chi2 = float(((counts - n / len(free)) ** 2 / (n / len(free))).sum())
    dof = len(free) - 1
    assert chi2 < dof + 5 * math.sqrt(2 * dof), chi2


def test_spawn_streams_depend_on_seed_and_env(mev):
    a, _ = _one_step_spawns(mev, 30.0, seed=1)
    b, _ = _one_step_spawns(mev, 30.0, seed=1)
    c, _ = _one_step_spawns(mev, 30.0, seed=2)
    assert np.array_equal(a["npc_count"], b["npc_count"]) and np.array_equal(a["npc_route"], b["npc_route"])
    assert not np.array_equal(a["npc_count"], c["npc_count"])
    # envs are not copies of each other
    assert 0 < int((a["npc_count"] > 0).sum()) < E
