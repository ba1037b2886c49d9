"""Throughput of the BASELINE configs on one GPU (documentation; bench.py is the
contract and measures config 3).  Same method as bench.py: actions resident
in HBM, outputs to HBM, auto-reset, warm-up then timed steps; per-kernel
device time from the library's events (every 4th step).
    python tools/bench_sweep.py [--steps 500] [--only cfg4] [--out profiles/r1_sweep.json]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [
    dict(name="cfg1", desc="1 env x 1 agent x 16 beams", E=1, N=1, R=16),
    dict(name="cfg2", desc="4096 envs x 1 agent x 64 beams", E=4096, N=1, R=64),
    dict(name="cfg3", desc="4096 envs x 8 agents x 64 beams, team reward", E=4096, N=8, R=64, team=1),
    dict(name="cfg4", desc="4096 envs x 1 agent x 64 beams, traffic density 0.5", E=4096, N=1, R=64, traffic=1),
    dict(name="cfg5/GPU", desc="4096 envs x 8 agents x 128 beams, team reward (per-GPU share of 32768)",
         E=4096, N=8, R=128, team=1),
    dict(name="96-beam", desc="4096 envs x 8 agents x 96 beams (reference default LiDAR), obs 127",
         E=4096, N=8, R=96, D=127),
    dict(name="cfg4-k64", desc="config 4 with 64 NPC slots per env (VecIntersectionEnv's default max_npcs)",
         E=4096, N=1, R=64, traffic=1, K=64),
    dict(name="1x96", desc="4096 envs x 1 agent x 96 beams (the reference's defaults: one agent, default LiDAR)",
         E=4096, N=1, R=96),
]


def run(cfg, steps, warmup, step_kernel=0, pack=0, split=0):
    import torch
    import pkgload
    mev = pkgload.load()
    dev = torch.device("cuda", 0)
    E, N, R = cfg["E"], cfg["N"], cfg["R"]
    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=R, obs_dim=cfg.get("D", 0),
                   use_team_reward=cfg.get("team", 0), traffic_flow=cfg.get("traffic", 0), traffic_density=0.5,
                   max_npcs=cfg.get("K", 32))
    if step_kernel:
        h.set_step_kernel(step_kernel)
    if pack:
        h.set_step_pack(pack)
    if split:
        h.set_step_split(split)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    h.set_stream(st.cuda_stream)
    acts = torch.rand((warmup + steps, E, N, 2), device=dev) * 2 - 1
    out = {k: torch.zeros_like(torch.as_tensor(v), device=dev) for k, v in h.alloc_outputs().items()}
    for t in range(warmup):
        h.step(acts[t], out=out, auto_reset=True, device=True)
    torch.cuda.synchronize()
    fused = h.step_kernel() == 2
    h.kernel_timing(25)  # sparse: the events add their own launch latency
    t0 = time.perf_counter()
    for t in range(steps):
        h.step(acts[warmup + t], out=out, auto_reset=True, device=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    c, l_, n = h.kernel_times()
    npc = float(h.get_state()["npc_count"].mean()) if cfg.get("traffic") else 0.0
    pk = h.step_pack()
    split = h.step_split()
    h.close()
    r = dict(name=cfg["name"], workload=cfg["desc"], agent_steps_per_s=round(E * N / dt, 1),
             ms_per_step=round(dt * 1e3, 5), step_kernel="k_step (fused)" if fused else "k_cars + k_lidar",
             # traffic early split: two car waves (one env each) + one LiDAR wave per workgroup
             # (kTsplitEnvs, mev_kernels.hip)
             envs_per_wave=pk, waves_per_workgroup=(3 if cfg.get("traffic") and split == 2 else
                                                    2 if split else 1),
             mean_npcs=round(npc, 3))
    if fused:
        r["k_step_ms_events"] = round(c / n, 5)
    else:
        r["k_cars_ms_events"], r["k_lidar_ms_events"] = round(c / n, 5), round(l_ / n, 5)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="comma-separated config names (e.g. cfg4)")
    ap.add_argument("--step-kernel", type=int, default=0, help="0 auto, 1 k_cars + k_lidar, 2 fused k_step")
    ap.add_argument("--pack", type=int, default=0, help="envs per fused wave: 0 auto, 1, 2, 4")
    ap.add_argument("--split", type=int, default=0, help="mev_set_step_split: 0 auto, 1 off, 2 on, 3 early split")
    ap.add_argument("--envs", type=int, default=0, help="override the configs' env count")
    a = ap.parse_args()
    res = []
    for cfg in CONFIGS:
        if a.only and cfg["name"] not in a.only.split(","):
            continue
        if a.envs:
            cfg = dict(cfg, E=a.envs, desc=cfg["desc"].replace(str(cfg["E"]), str(a.envs), 1))
        r = run(cfg, a.steps if cfg["E"] > 1 else 200, a.warmup, a.step_kernel, a.pack, a.split)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
