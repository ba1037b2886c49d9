"""Which kernel path is faster at which batch size (auto-selection rule of
mev_set_step_kernel(0)): config-3 shape (8 agents x 64 beams, team reward) at
growing env counts, both paths, per-step wall time on a device-resident loop.
    python tools/path_sweep.py [--envs 1,16,64,256,512,1024,2048]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_sweep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", default="1,16,64,256,512,1024,2048")
    ap.add_argument("--steps", type=int, default=1000)
    a = ap.parse_args()
    for E in (int(x) for x in a.envs.split(",")):
        cfg = dict(name=f"E{E}", desc=f"{E} envs x 8 agents x 64 beams, team reward", E=E, N=8, R=64, team=1)
        row = {"envs": E}
        for k in (1, 2):
            r = bench_sweep.run(cfg, a.steps, 100, k)
            row["two_kernel_us" if k == 1 else "fused_us"] = round(r["ms_per_step"] * 1e3, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
