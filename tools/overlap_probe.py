"""Experiment: does running two half-size env batches on two streams (so one
half's k_cars overlaps the other half's k_lidar) beat one full batch?
    python tools/overlap_probe.py [--envs 4096] [--splits 1 2 4]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    import torch
    import pkgload
    mev = pkgload.load()
    dev = torch.device("cuda", 0)
    for sp in a.splits:
        E = a.envs // sp
        hs, sts, acts = [], [], []
        for i in range(sp):
            h = mev.Handle(num_envs=E, num_agents=8, lidar_rays=64, use_team_reward=1, seed=i)
            st = torch.cuda.Stream(dev)
            h.set_stream(st.cuda_stream)
            hs.append(h)
            sts.append(st)
            acts.append(torch.rand((a.steps, E, 8, 2), device=dev) * 2 - 1)
        obs = [torch.zeros((E, 8, 95), device=dev) for _ in range(sp)]
        for t in range(50):
            for i in range(sp):
                hs[i].step(acts[i][t].data_ptr(), out=dict(obs=obs[i].data_ptr()), auto_reset=True, device=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(a.steps):
            for i in range(sp):
                hs[i].step(acts[i][t].data_ptr(), out=dict(obs=obs[i].data_ptr()), auto_reset=True, device=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(f"splits={sp}: {dt * 1e6:7.1f} us/step  {a.envs * 8 / dt / 1e6:7.1f} M agent-steps/s", flush=True)
        for h in hs:
            h.close()


if __name__ == "__main__":
    main()
