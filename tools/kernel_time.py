"""Per-kernel device time of k_cars / k_lidar (the library's own HIP events,
mev_kernel_timing) for library variants and LiDAR group sizes (experiments).
    python tools/kernel_time.py [variant[:G] ...]   e.g.  "" :4 exp_noroad exp_nocars:8
MEV_LIDAR_G=G selects the k_lidar group size (agents per wave pool)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(variant, E=4096, N=8, R=64, steps=300):
    import torch
    import pkgload
    mev = pkgload.load()
    cap = mev._capi
    cap.VARIANT = variant
    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=R, use_team_reward=1)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    h.set_stream(st.cuda_stream)
    acts = torch.rand((steps, E, N, 2), device=dev) * 2 - 1
    obs = torch.zeros((E, N, 31 + R), device=dev)
    out = dict(obs=obs.data_ptr())
    for t in range(30):
        h.step(acts[t].data_ptr(), out=out, auto_reset=True, device=True)
    torch.cuda.synchronize()
    h.kernel_timing(True)
    for t in range(steps):
        h.step(acts[t].data_ptr(), out=out, auto_reset=True, device=True)
    c, l_, n = h.kernel_times()
    h.close()
    return c / n * 1e3, l_ / n * 1e3


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        v, g = sys.argv[2], sys.argv[3]
        c, l_ = run(v)
        print(f"variant {v or 'product':12s} G={g or 'auto':4s}: k_cars {c:7.1f} us  k_lidar {l_:7.1f} us", flush=True)
        sys.exit(0)
    for spec in (sys.argv[1:] or [""]):
        v, _, g = spec.partition(":")
        env = dict(os.environ)
        if g:
            env["MEV_LIDAR_G"] = g
        # one process per spec: the group size is read once per process
        subprocess.run([sys.executable, __file__, "--one", v, g], env=env, check=True)
