"""Diagnostic: per-wave road-march iteration counts (exp_iters build)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402

mev = pkgload.load()
mev._capi.VARIANT = "exp_iters"
h = mev.Handle(num_envs=4096, num_agents=8, lidar_rays=64, use_team_reward=1)
rng = np.random.default_rng(0)
for t in range(300):
    h.step(rng.uniform(-1, 1, (4096, 8, 2)).astype(np.float32), auto_reset=True)
it = h.debug_stamps().reshape(-1).astype(np.int64)
it = it[: 4096 * 8 // int(os.environ.get("MEV_LIDAR_G", "4"))]  # one entry per k_lidar wave
print("wave iterations: mean %.2f median %d p90 %d p99 %d max %d" % (it.mean(), np.median(it), np.percentile(it, 90),
                                                                   np.percentile(it, 99), it.max()))
print(np.bincount(it)[:80])
