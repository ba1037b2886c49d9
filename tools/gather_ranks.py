"""Multi-rank check of the C ABI gather (MEV_GATHER_TO_ROOT): `--ranks G`
processes, all on device 0 unless --devices says otherwise, each stepping its
shard of E envs; the root compares every rank's gathered rows with one handle
stepping all G*E envs with the same actions (bit for bit).  Prints GATHER OK,
or SKIP when RCCL refuses several ranks on one device.  Used by
tests/test_gather_gpu.py on the one-GPU box."""
import argparse
import datetime
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(args):
    import numpy as np
    import torch
    import torch.distributed as dist
    import torch.utils.dlpack as tdl

    import pkgload

    mev = pkgload.load()
    from marl_traffic_intersection_amd import sharding

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = (rank % args.devices)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
    E, N, R, T = args.envs, 4, 32, 12
    total = E * world
    cfg = dict(num_agents=N, lidar_rays=R, use_team_reward=1, max_steps=8, device=dev)
    h = mev.Handle(num_envs=E, **cfg)
    store = dist.distributed_c10d._get_default_store()
    try:
        sharding.comm_bootstrap(h, store, world, rank, root=0, slots=E)
    except mev.MevError as exc:
        ok = torch.tensor([0.0])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if rank == 0:
            print(f"SKIP: RCCL refused {world} ranks on {args.devices} device(s): {exc}"[:400], flush=True)
        dist.destroy_process_group()
        return 0
    ok = torch.tensor([1.0])
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if ok.item() == 0:
        dist.destroy_process_group()
        return 0
    ref = mev.Handle(num_envs=total, **cfg) if rank == 0 else None
    lay = sharding.PackedOutputs(E, N, h.D)
    rng = np.random.default_rng(11)
    bad = 0
    for t in range(T):
        acts = rng.uniform(-1, 1, (total, N, 2)).astype(np.float32)
        h.step(acts[rank * E:(rank + 1) * E], auto_reset=True, gather=True)
        h.gather_wait(60000)
        if rank == 0:
            want = ref.step(acts, auto_reset=True)
            h.gather_result()
            buf = tdl.from_dlpack(h.output_dlpack("gathered")).cpu().numpy()
            got = lay.unpack_gathered(buf, total, world)
            for k, v in got.items():
                a, b = np.ascontiguousarray(v), np.ascontiguousarray(want[k])
                if a.dtype == np.float32:
                    a, b = a.view(np.uint32), b.view(np.uint32)
                if not np.array_equal(a, b):
                    bad += 1
                    print(f"mismatch step {t} field {k}", flush=True)
        dist.barrier()
    h.comm_destroy()
    h.close()
    if rank == 0:
        ref.close()
        print("GATHER OK" if bad == 0 else f"GATHER FAILED ({bad} mismatches)", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if bad == 0 else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--devices", type=int, default=1)
    ap.add_argument("--envs", type=int, default=24)
    args = ap.parse_args()
    if "RANK" in os.environ:
        sys.exit(rank_main(args))
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, __file__] + sys.argv[1:],
                              env=dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.ranks),
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
             for r in range(args.ranks)]
    rc = 0
    for p in procs:
        try:
            c = p.wait(timeout=120)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            c = 124
        rc = rc or c
    sys.exit(rc)


if __name__ == "__main__":
    main()
