"""Diagnostic: cars_post's parts (k_step, config 3 shape) from the stampspost build
(cars_post split by s_memtime stamps: bonuses + flags, ego write-back, observation head up
to the neighbour ranks, the head's features, the head's stores).  Shares only.
    MEV_LIB_VARIANT=stampspost python tools/post_profile.py"""
import os
import sys

os.environ.setdefault("MEV_LIB_VARIANT", "stampspost")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402

PARTS = ["bonuses+flags", "ego write-back", "head: reads+dist+rank", "head: features", "head: stores"]


def main():
    mev = pkgload.load()
    E, N, R = 4096, 8, 64
    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=R, use_team_reward=1)
    rng = np.random.default_rng(0)
    acc = []
    for t in range(200):
        a = rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)
        h.step(a, auto_reset=True)
        if t >= 100:
            s = h.debug_stamps().astype(np.int64).reshape(E, 8)
            acc.append(np.diff(s[:, :6], axis=1))
    d = np.concatenate(acc)
    tot = d.sum(1)
    print(f"cars_post per env: median {np.median(tot):.0f} cycles")
    for k, name in enumerate(PARTS):
        print(f"  {name:24s} median {np.median(d[:, k]):8.0f}  mean {d[:, k].mean():8.0f}  share {d[:, k].sum() / tot.sum():6.1%}")


if __name__ == "__main__":
    main()
