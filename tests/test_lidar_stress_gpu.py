"""LiDAR stress parity: dense random car clusters (overlapping, touching,
straddling the screen edge and the road edges), every heading, wide and narrow
fields of view, up to 1024 beams, exact (step 4) and accumulated-table (step
3.3) march distances.  Cars are placed with zero speed and stepped once with
zero actions and respawn off, so the survivors observe the cluster from where it
was placed; that step's observation is compared bit for bit with the C
restatement's (oracle/marl_oracle.c, pinned to the reference by
tests/test_oracle.py).  (The observation right after set_state carries a
max-range LiDAR block, as the reference's does, so it tests nothing here.)  This is where the k_lidar
shortcuts — the safe-stretch skipping, the angular beam ranges of each box and
the slab-bounded probe ranges — would show a dropped or spurious hit."""
import zlib

import numpy as np
import pytest

import golden_replay as G
from conftest import STEP_KERNELS, use_step_kernel
import oracle_replay as ORP

CAR_DTYPE, OracleEnv = ORP.O.CAR_DTYPE, ORP.O.OracleEnv

pytestmark = pytest.mark.gpu

CASES = [
    dict(name="n16_r64", n=16, rays=64, fov=360.0, maxd=250.0, step=4.0),
    dict(name="n32_r256", n=32, rays=256, fov=360.0, maxd=250.0, step=4.0),
    dict(name="n8_r1024", n=8, rays=1024, fov=360.0, maxd=250.0, step=4.0),
    dict(name="n12_r96_fov120_tab", n=12, rays=96, fov=120.0, maxd=180.0, step=3.3),
    dict(name="n6_r7_fov30", n=6, rays=7, fov=30.0, maxd=400.0, step=4.0),
    dict(name="n24_r64_lanes2_short", n=24, rays=64, fov=270.0, maxd=60.0, step=4.0, lanes=2),
]


def _cluster_state(rng, h, n):
    st = h.get_state()
    E = h.E
    for e in range(E):
        mode = e % 4
        if mode == 0:    # tight cluster anywhere on screen
            c = rng.uniform(0, 750, 2)
            xy = c + rng.normal(0, 35, (n, 2))
        elif mode == 1:  # along a road edge
            off = rng.choice([-1, 1]) * (42 * 3 + rng.normal(0, 6))
            t = rng.uniform(0, 750, n)
            xy = np.stack([375 + off + rng.normal(0, 3, n), t], 1)
            if rng.uniform() < 0.5:
                xy = xy[:, ::-1]
        elif mode == 2:  # straddling the screen border
            xy = rng.uniform(-30, 780, (n, 2))
            side = rng.integers(0, 4, n)
            xy[side == 0, 0] = rng.uniform(-25, 25, (side == 0).sum())
            xy[side == 1, 0] = rng.uniform(725, 775, (side == 1).sum())
            xy[side == 2, 1] = rng.uniform(-25, 25, (side == 2).sum())
            xy[side == 3, 1] = rng.uniform(725, 775, (side == 3).sum())
        else:            # a chain of touching boxes through the centre, pixel-aligned
            t = np.arange(n) * rng.choice([24.0, 27.0, 54.0]) + rng.uniform(0, 1)
            ang = rng.uniform(-np.pi, np.pi)
            xy = np.stack([375 + np.cos(ang) * (t - t.mean()), 375 - np.sin(ang) * (t - t.mean())], 1)
            m = rng.uniform(size=n) < 0.5
            xy[m] = np.round(xy[m])
        st["x"][e], st["y"][e] = xy[:, 0], xy[:, 1]
        hd = rng.uniform(-np.pi, np.pi, n)
        axis = rng.uniform(size=n) < 0.3  # axis-aligned headings (rays parallel to box edges)
        hd[axis] = rng.integers(-2, 3, axis.sum()) * (np.pi / 2)
        st["heading"][e] = hd
        st["alive"][e] = (rng.uniform(size=n) > 0.1).astype(st["alive"].dtype)
        st["v"][e] = 0.0
        st["acc"][e] = 0.0
        st["steering"][e] = 0.0
    h.set_state(st)
    return st


def _oracle_obs(case, st, e, D):
    n = case["n"]
    o = OracleEnv(num_lanes=case.get("lanes", 3), n_agents=n, rays=case["rays"], fov=case["fov"],
                  max_dist=case["maxd"], step=case["step"], obs_dim=D, respawn=False)
    cars = ORP.O.new_cars(n)
    for a, b in {"x": "x", "y": "y", "v": "v", "h": "heading", "acc": "acc", "steer": "steering",
                 "sx": "spawn_x", "sy": "spawn_y", "sv": "spawn_v", "sh": "spawn_heading", "prev_dist": "prev_dist",
                 "pa0": "prev_a0", "pa1": "prev_a1", "path_index": "path_index", "route": "route",
                 "intention": "intention", "alive": "alive"}.items():
        cars[a] = st[b][e]
    o.set_state(cars, ORP.O.new_cars(0), int(st["step_count"][e]))
    r = o.step(np.zeros((n, 2), np.float32))
    o.close()
    return r["obs"]


@pytest.mark.parametrize("kernel", STEP_KERNELS)
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_lidar_matches_oracle_on_dense_clusters(mev, case, kernel):
    rng = np.random.default_rng(zlib.crc32(case["name"].encode()))
    n, R_ = case["n"], case["rays"]
    D = 31 + R_
    E = 256 if R_ < 1024 else 64
    h = mev.Handle(num_envs=E, num_agents=n, num_lanes=case.get("lanes", 3), lidar_rays=R_, obs_dim=D,
                   lidar_fov_deg=case["fov"], lidar_max_dist=case["maxd"], lidar_step=case["step"], respawn_enabled=0)
    use_step_kernel(mev, h, kernel)
    stops = 0
    for rnd in range(5):
        st = _cluster_state(rng, h, n)
        out = h.step(np.zeros((E, n, 2), np.float32))
        got = out["obs"]
        for e in range(E):
            want = _oracle_obs(case, st, e, D)
            if not G.bits_equal(got[e], want):
                bad = np.argwhere(got[e].view(np.uint32) != want.view(np.uint32))
                i, c = bad[0]
                raise AssertionError(
                    f"{case['name']} round {rnd} env {e}: {len(bad)} words differ, first agent {i} col {c}: "
                    f"got {got[e][i, c]!r} want {want[i, c]!r}; agent poses "
                    f"{[(float(st['x'][e, j]), float(st['y'][e, j]), float(st['heading'][e, j]), int(st['alive'][e, j])) for j in range(n)]}; "
                    f"differing (agent, col): {bad[:12].tolist()}")
        # beams that stopped (road or car) — the comparison above is not vacuous
        stops += int(((got[:, :, 31:] > 0) & (got[:, :, 31:] < 1.0)).sum())
    assert stops > 0
    h.close()
