"""Time k_cars / k_lidar of a library variant with HIP events (experiments).
    python tools/kernel_time.py [variant ...]     e.g.  "" exp_noroad exp_nocars exp_none
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pkgload  # noqa: E402


def run(variant, E=4096, N=8, R=64, steps=200):
    mev = pkgload.load()
    cap = mev._capi
    old = cap.VARIANT
    cap.VARIANT = variant
    try:
        h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=R, use_team_reward=1)
    finally:
        cap.VARIANT = old
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    h.set_stream(st.cuda_stream)
    acts = torch.rand((steps, E, N, 2), device=dev) * 2 - 1
    obs = torch.zeros((E, N, 31 + R), device=dev)
    out = dict(obs=obs.data_ptr())
    for t in range(20):
        h.step(acts[t].data_ptr(), out=out, auto_reset=True, device=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for t in range(steps):
        h.step(acts[t].data_ptr(), out=out, auto_reset=True, device=True)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    h.close()
    return ms


if __name__ == "__main__":
    for v in (sys.argv[1:] or [""]):
        print(f"variant {v or 'product':12s}: {run(v) * 1e3:8.1f} us/step")
