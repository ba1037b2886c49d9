"""Route-table re-layout in the middle of an episode.

mev_add_route_n with a path longer than the table's rows (160 points, or the longest written
path so far) re-lays every row out at the new length and re-uploads the table
(mev_capi.cpp fill_row; RouteTab::plen / row).  Route ids, and so every car's state, stay.
Here one handle runs 20 steps, takes a 700-point route (re-layout), puts some egos and NPCs on
it and runs on; a second handle had the same long route from the start and runs the same
steps and writes.  Every output and the full state must be bit-equal after every step, on
both kernel paths, with traffic (NPCs on the written routes, Philox spawns) and without."""
import numpy as np
import pytest

from conftest import STEP_KERNELS, use_step_kernel

pytestmark = pytest.mark.gpu

E, T0, T1 = 16, 20, 40


def _long_path(h, n):
    """Lane route (0 -> 13) resampled at n points (linear interpolation in f64)."""
    path = h.route_info(h.route_id(0, 12))[0][: h.route_len(h.route_id(0, 12))].astype(np.float64)
    t = np.linspace(0.0, len(path) - 1.0, n)
    i0 = np.minimum(np.floor(t).astype(int), len(path) - 2)
    w = (t - i0)[:, None]
    return (path[i0] * (1.0 - w) + path[i0 + 1] * w).astype(np.float32)


def _make(mev, traffic, kernel):
    h = mev.Handle(num_envs=E, num_agents=3, lidar_rays=32, traffic_flow=int(traffic), traffic_density=3.0,
                   max_npcs=32, seed=5)
    use_step_kernel(mev, h, kernel)
    return h


@pytest.mark.parametrize("traffic", [False, True])
@pytest.mark.parametrize("kernel", STEP_KERNELS)
def test_relayout_mid_episode_matches_layout_from_start(mev, traffic, kernel):
    a = _make(mev, traffic, kernel)
    b = _make(mev, traffic, kernel)
    short = _long_path(a, 90)  # a shorter written path first: its row padding must survive the re-layout
    assert a.add_route(short, 1) == b.add_route(short, 1)
    long_ = _long_path(a, 700)
    rb = b.add_route(long_, 1)  # b: the long route (and 720-point rows) from the start
    rng = np.random.default_rng(3)
    acts = rng.uniform(-1, 1, (T0 + T1, E, 3, 2)).astype(np.float32)
    for h in (a, b):
        h.reset()
    for t in range(T0):
        oa, ob = a.step(acts[t]), b.step(acts[t])
        for k in oa:
            assert np.array_equal(np.asarray(oa[k]).view(np.uint8), np.asarray(ob[k]).view(np.uint8)), (t, k)
    ra = a.add_route(long_, 1)  # a: re-layout now
    assert ra == rb and a.route_len(ra) == 700
    assert np.array_equal(a.route_info(ra)[0], b.route_info(rb)[0])
    # some egos (and, with traffic, NPCs) onto the long route, mid-path, in both handles alike
    for h in (a, b):
        st = h.get_state()
        st["route"][::3, 1] = ra
        st["path_index"][::3, 1] = 300
        st["x"][::3, 1], st["y"][::3, 1] = long_[300]
        if traffic:
            h.set_traffic_routes([ra, h.route_id(1, 14), h.route_id(5, 18)])
            k = st["npc_count"]
            for e in range(0, E, 2):
                if k[e] < 32:
                    st["npc_route"][e, k[e]] = ra
                    st["npc_path_index"][e, k[e]] = 200 + e
                    st["npc_x"][e, k[e]], st["npc_y"][e, k[e]] = long_[200 + e]
                    st["npc_v"][e, k[e]] = 2.0
                    st["npc_alive"][e, k[e]] = 1
                    k[e] += 1
        h.set_state(st)
    for t in range(T0, T0 + T1):
        oa, ob = a.step(acts[t]), b.step(acts[t])
        for k in oa:
            assert np.array_equal(np.asarray(oa[k]).view(np.uint8), np.asarray(ob[k]).view(np.uint8)), (t, k)
        sa, sb = a.get_state(), b.get_state()
        for k in sa:
            assert np.array_equal(np.asarray(sa[k]).view(np.uint8), np.asarray(sb[k]).view(np.uint8)), (t, k)
    assert int(a.get_state()["path_index"][0, 1]) > 300  # the ego moved along the long route
    a.close()
    b.close()
