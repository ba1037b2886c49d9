"""bench.py — agent-steps/s of the batched intersection environment on MI355X.

Workload (BASELINE.json metric, config 3): per GPU 4096 envs x 8 ego agents,
64-beam LiDAR, team reward, respawn on, max_steps 2000, per-env auto-reset.
One "step" = IntersectionEnv::step + get_observations for all of the GPU's
4096 envs: one launch of the fused k_step kernel (one wave per env: physics,
status, collisions, rewards, respawn, observation head, then the 64-beam LiDAR
of the env's 8 agents as one pooled beam queue, all from the wave's LDS), with
the actions already resident in HBM (pre-generated uniform [-1, 1) f32) and
obs [E, 8, 95] / reward / done / status / terminated / truncated written to HBM.

--gpus N > 1: one process per GPU.  Run directly, bench.py starts the N rank
processes itself (children, before any GPU call); under torchrun it reads
RANK / LOCAL_RANK / WORLD_SIZE.  Every rank steps its own 4096 envs (weak
scaling: envs are independent, so the step has no data-path collective; a
barrier and a max-over-ranks reduction bracket the timed region): "value".
A second timed phase ("gather_to_root") repeats the steps with the
north star's per-step RCCL gather of every rank's packed outputs to rank 0,
issued from the C ABI (MEV_GATHER_TO_ROOT) on a communication stream that
overlaps the next step; --no-gather skips it.

Prints ONE JSON line on rank 0, including "roofline" for the dominant kernel
(k_step, the only kernel of a step; HBM fraction from HIP events on its stream,
VALU-issue fraction from the committed SQ counter pass) and "cpu_baseline" (the
pinned C restatement on every host core, with the reference's survey-container
numbers quoted beside it).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

E_PER_GPU = 4096
N_AGENTS = 8
RAYS = 64
OBS_DIM = 31 + RAYS
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def algorithmic_bytes_per_agent_step(rays: int) -> int:
    """actions 8 + ego hot state r/w 80 + obs 4*(31+R) + reward 4 + done/status 2."""
    return 8 + 80 + 4 * (31 + rays) + 4 + 2


def lidar_bytes_per_agent_step(rays: int) -> int:
    """k_lidar's share: reads the ego pose x, y, heading (12 B) and alive (1 B), writes obs[31:31+R] (4R B)."""
    return 13 + 4 * rays


def cars_bytes_per_agent_step(rays: int) -> int:
    """k_cars's share: actions 8 + hot state r/w 80 + obs head 4*31 + reward 4 + done/status 2."""
    return 8 + 80 + 4 * 31 + 4 + 2


# The reference's own C++ simulator timed in the survey container (8 vCPU Xeon, env.py
# driver, one env per process): it cannot run on the GPU box, which
# receives only this repository.  Quoted beside the live port timing.
REFERENCE_SURVEY_CPU = {
    "value_1_process": 6668, "value_8_processes": 37362, "unit": "agent-steps/s", "cores": 8,
    "host": "survey container, Intel Xeon (family 6, model 0xCF), 8 vCPUs",
    "config": "reference cpp/ (g++ -O2) through env.py, 8 agents, team reward, 64 beams",
    "source": "BASELINE.md (measured during the survey, not published by the reference)",
}


def host_cores() -> int:
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota if one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(seconds_budget: float = 20.0):
    """The pinned C restatement of the step (oracle/marl_oracle.c, bit-exact against the
    reference's golden vectors; test infrastructure used here only as the baseline), one
    thread per host core on every core this process may use, each thread its own env
    (the ctypes call releases the GIL, so the threads run in parallel)."""
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    oracle.lib()
    threads = host_cores()
    # ~1.2 ms per 8-agent env-step on one core: ~seconds_budget CPU-seconds in total
    steps = max(100, int(seconds_budget / threads / 1.2e-3))
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda t: oracle.bench(N_AGENTS, RAYS, True, steps, t), range(threads)))
    wall = time.perf_counter() - t0
    v = threads * steps * N_AGENTS / wall
    return {"value": round(v, 1), "unit": "agent-steps/s", "cores": threads, "kind": "port",
            "sample": f"C restatement of the step (oracle/marl_oracle.c, gcc -O2, bit-exact vs the reference "
                      f"goldens), {threads} threads (every host core available to this process) x 1 env x {steps} "
                      f"steps each, 8 agents, 64 beams, team reward, uniform random actions, auto-reset; "
                      f"wall {wall:.1f} s",
            "reference_survey": REFERENCE_SURVEY_CPU}


def dist_table_needed(max_dist: float = 250.0, step: float = 4.0) -> bool:
    """Whether the handle reads accumulated probe distances (k_step<_, true>): the float sum
    dist += step of Lidar.cpp:33 differs from k*step (mirrors mev_create)."""
    import numpy as np
    d, k = np.float32(0.0), 0
    while d < np.float32(max_dist):
        if d != np.float32(k) * np.float32(step):
            return True
        d = np.float32(d + np.float32(step))
        k += 1
    return False


VALU_PEAK_G = 1024 * 2.4e9 / 2 / 1e9  # wave64 VALU instructions/s: 1024 SIMD-32 x 2.4 GHz / 2 cycles


def valu_roofline(kernel_ms: float, envs: int):
    """VALU issue fraction of k_step: SQ_INSTS_VALU per launch (committed rocprofv3 pass,
    profiles/valu_counters.json) / the live kernel time, against 1024 SIMDs issuing one wave64
    VALU instruction per 2 cycles at 2.4 GHz (MI355X_MICROARCH.md, Wave scheduling)."""
    f = os.path.join(ROOT, "profiles", "valu_counters.json")
    if not os.path.exists(f):
        return None
    pm = json.load(open(f))
    k = pm.get("k_step")
    if not k or pm.get("envs") != envs or pm.get("agents") != N_AGENTS or pm.get("rays") != RAYS:
        return None
    inst = float(k["SQ_INSTS_VALU_per_launch"])
    achieved = inst / (kernel_ms * 1e-3) / 1e9
    return {"achieved": round(achieved, 2), "peak": VALU_PEAK_G, "unit": "G wave-instr/s",
            "frac": round(achieved / VALU_PEAK_G, 4), "SQ_INSTS_VALU_per_launch": inst,
            "source": "profiles/valu_counters.json (rocprofv3 --pmc pass of this bench) / live kernel_ms"}


class stdout_to_stderr:
    """RCCL prints its version banner on fd 1 at communicator init: keep the bench's stdout
    to the one JSON line by pointing fd 1 at stderr around the init."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n: int) -> int:
    """--gpus N without a launcher: start N rank processes of this script (one per GPU) and
    supervise them.  No GPU call happens in this process; the children are started, not
    exec'd.  If a rank fails, the others are stopped (by PID) and its exit code returned."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for pr in list(live):
            code = pr.poll()
            if code is None:
                continue
            live.remove(pr)
            if code != 0 and rc == 0:
                rc = code
                for other in live:
                    other.kill()
        time.sleep(0.05)
    return rc


def dry_run(args):
    """The rank-side control plane of main() without a GPU (tests/test_bench_launcher.py)."""
    import datetime
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("MEV_DRYRUN_FAIL_RANK") == str(rank):
        sys.exit(3)  # test hook: a rank that dies before the rendezvous (the launcher must stop the rest)
    if world > 1:
        with stdout_to_stderr():
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("mev_comm_id", bytes(range(128)))  # stands in for mev_comm_unique_id()
        uid = bytes(store.get("mev_comm_id"))
        assert uid == bytes(range(128))
        dist.barrier()
    t = torch.tensor([float(rank + 1), float(os.getpid())], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "max_over_ranks": t[0].item(),
                          "steps": args.steps, "warmup": args.warmup, "config": args.config, "rays": RAYS,
                          "value_includes_gather": args.config == 5}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def verify_gather(env, _capi, E, N, D, world, rank, gfmt, ls, dev, act, timeout_ms):
    """Every rank (the gathered step is collective): snapshot the state, take one more step
    with the gather, restore the snapshot and take the same step plainly (no gather, its own
    output buffers).  The root decodes every rank's gathered rows (sharding.PackedOutputs; the
    state format through mev_unpack_gathered on the device) and checks them: finite, valid
    status codes, and its own row equal, bit for bit, to the plain step's outputs."""
    import torch
    import torch.utils.dlpack as tdl
    from marl_traffic_intersection_amd import sharding

    snap = torch.empty(env.snapshot_size(), dtype=torch.uint8, device=dev)
    env.snapshot(snap, device=True)
    env.step(act.data_ptr(), 1.0 / 60.0, auto_reset=True, device=True, gather=True)
    env.gather_wait(timeout_ms)
    got = None
    if rank == 0:
        ptr, per_rank, w = env.gather_result()
        if not ptr or w != world:
            got = "missing"
        else:
            lay = sharding.PackedOutputs(E, N, D, fmt=gfmt, lidar_slots=ls,
                                         table=env.lidar_decode_table() if gfmt == 1 else None,
                                         handle=env if gfmt == 2 else None)
            stacked = tdl.from_dlpack(env.output_dlpack("gathered"))
            got = {k: v.clone() for k, v in lay.unpack_gathered(stacked, world * E, world).items()}
    torch.cuda.synchronize(dev)
    env.restore(snap, device=True)
    plain = {k: torch.zeros_like(torch.as_tensor(v), device=dev) for k, v in env.alloc_outputs().items()}
    env.step(act.data_ptr(), 1.0 / 60.0, out=plain, auto_reset=True, device=True)
    torch.cuda.synchronize(dev)
    if rank != 0:
        return None
    if isinstance(got, str):
        return got
    if not (torch.isfinite(got["obs"]).all().item() and torch.isfinite(got["reward"]).all().item()
            and int(got["status"].max().item()) <= 5):
        return "FAILED: non-finite or invalid rows"
    for k in sharding.PackedOutputs.FIELDS:
        a, b = got[k][:E].contiguous(), plain[k]
        if a.dtype == torch.float32:
            a, b = a.view(torch.int32), b.view(torch.int32)
        if not torch.equal(a, b):
            return f"FAILED: root row {k} differs from the plain step"
    what = {0: "f32 rows", 1: "31-float heads + u8 LiDAR codes", 2: "post-step state + u8 LiDAR codes, heads rebuilt "
            "on the root"}[gfmt]
    return (f"decoded {world} rank rows ({what}): finite, valid status codes; the root's row bit-equal to the same "
            f"step taken without the gather from the same snapshot")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs", type=int, default=E_PER_GPU, help="envs per GPU")
    ap.add_argument("--config", type=int, choices=(3, 5), default=3,
                    help="3: BASELINE config 3, the metric (4096 envs x 8 agents x 64 beams per GPU, value = the "
                         "steps without a collective); 5: BASELINE config 5 (32768 envs x 8 agents x 128 beams over "
                         "8 GPUs = 4096 per GPU, value = the steps WITH the per-step RCCL gather of every rank's "
                         "outputs to rank 0)")
    ap.add_argument("--rays", type=int, default=0, help="LiDAR beams (default: 64 for config 3, 128 for config 5)")
    ap.add_argument("--no-gather", action="store_true",
                    help="skip the second timed phase (every step's outputs gathered to rank 0 over RCCL)")
    ap.add_argument("--gather-timeout", type=float, default=120.0, help="seconds before a stuck gather is aborted")
    ap.add_argument("--gather-format", choices=("state", "u8", "f32"), default="state",
                    help="packed gather rows (all lossless): state = each agent's post-step state + one LiDAR code "
                         "per beam, the 31-float heads rebuilt on the root; u8 = 31-float heads + LiDAR codes; "
                         "f32 = plain rows")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed steps for this long before the warm-up (SIMD clock ramp from idle); 0 = none")
    ap.add_argument("--kernel-events", action="store_true",
                    help="record the library's per-kernel HIP events on every --event-every-th timed step (the "
                         "fused k_step's roofline uses the stream events around the timed region instead; the "
                         "sampled events add launch latency inside it: +0.9 us per step at 20 steps, "
                         "profiles/r6_events_ab.txt).  Always on for the two-kernel path, whose per-kernel "
                         "times need them")
    ap.add_argument("--no-kernel-events", action="store_true", help="never record per-kernel HIP events")
    ap.add_argument("--event-every", type=int, default=50, help="record the per-kernel events on every n-th step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--step-kernel", type=int, default=0,
                    help="0 automatic (fused k_step at this size), 1 k_cars + k_lidar, 2 fused")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank plumbing: launcher, gloo control plane, RCCL-id "
                         "exchange through the store, max over ranks; no GPU work, no metric")
    args = ap.parse_args()
    global RAYS, OBS_DIM
    RAYS = args.rays if args.rays > 0 else (128 if args.config == 5 else 64)
    OBS_DIM = 31 + RAYS
    if args.config == 5 and args.no_gather:
        ap.error("--config 5 measures the steps with the gather: --no-gather does not apply")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus))  # one child process per GPU; this process never touches the GPU
    if args.dry_run:
        return dry_run(args)

    import torch
    import pkgload

    mev = pkgload.load()
    from marl_traffic_intersection_amd import _capi

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MEV_BENCH_SHARE_DEVICE") == "1":
        # rehearsal of the N-rank path on fewer GPUs (ranks share devices round-robin); never the
        # default: on a node with N GPUs every rank owns its own device
        local_rank %= max(1, torch.cuda.device_count())
    dist = None
    torch.cuda.set_device(local_rank)
    if world > 1:
        # control plane only (barriers, max over ranks, the RCCL id): gloo on the host; the
        # data-path collective is the library's own RCCL gather (mev_comm_init)
        import datetime
        import torch.distributed as dist
        with stdout_to_stderr():  # gloo's C++ "connected to N peer ranks" banner: stdout carries only the line
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=max(60.0, args.gather_timeout + 60.0)))
            dist.barrier()
    dev = torch.device("cuda", local_rank)
    E, N, D = args.envs, N_AGENTS, OBS_DIM
    K, W = args.steps, args.warmup

    def max_over_ranks(vals):
        if dist is None:
            return vals
        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(x) for x in t.tolist()]

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    env = mev.Handle(num_envs=E, num_agents=N, lidar_rays=RAYS, use_team_reward=1, respawn_enabled=1,
                     max_steps=2000, seed=rank, device=local_rank)
    env.set_step_kernel(args.step_kernel)
    stream = torch.cuda.Stream(dev)  # the env kernels and the events are all ordered on it
    torch.cuda.set_stream(stream)
    env.set_stream(stream.cuda_stream)

    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    actions = torch.rand((W + K, E, N, 2), device=dev, generator=g, dtype=torch.float32) * 2.0 - 1.0

    # ---- phase 1 (the metric): every rank steps its own envs, outputs stay in its HBM
    outs = [{k: torch.zeros_like(torch.as_tensor(v), device=dev) for k, v in env.alloc_outputs().items()}
            for _ in range(2)]
    env.reset(device=True)

    def step(t):
        env.step(actions[t].data_ptr(), 1.0 / 60.0, out=outs[t & 1], auto_reset=True, device=True)

    # Clock settle (untimed, before the W warm-up steps): an idle MI355X needs ~0.1 s of load before
    # its SIMD clock reaches the level it then holds for the rest of a rollout; without it a short run
    # (the driver's 5 warm-up + 20 timed steps) times the ramp -- k_step averaged 36.9 us over such
    # 20 steps against 34.4 us over 1000.  The steps are the metric's own (same handle,
    # actions and outputs); the envs are reset afterwards, so the warm-up and timed steps start from
    # the same state as without it.
    settle_steps = 0
    if args.settle_ms > 0:
        t_end = time.perf_counter() + args.settle_ms * 1e-3
        while time.perf_counter() < t_end:
            for _ in range(64):
                step(settle_steps % (W + K))
                settle_steps += 1
            torch.cuda.synchronize(dev)
        env.reset(device=True)
    for t in range(W):
        step(t)
    torch.cuda.synchronize(dev)
    fused = env.step_kernel() == 2  # one k_step launch per step (else k_cars + k_lidar)
    kernel_events = (args.kernel_events or not fused) and not args.no_kernel_events
    if kernel_events:
        env.kernel_timing(args.event_every)
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(K):
        step(W + k)
    ev1.record(stream)
    barrier()
    elapsed = time.perf_counter() - t0
    stream_ms = ev0.elapsed_time(ev1) / K
    cars_ms = lidar_ms = None
    if kernel_events:
        c_sum, l_sum, n_steps = env.kernel_times()
        assert n_steps == (K + args.event_every - 1) // args.event_every, (n_steps, K)
        cars_ms, lidar_ms = c_sum / n_steps, l_sum / n_steps
        env.kernel_timing(0)
    elapsed, c_, l_, stream_ms = max_over_ranks([elapsed, cars_ms or 0.0, lidar_ms or 0.0, stream_ms])
    if cars_ms is not None:
        cars_ms, lidar_ms = c_, l_
    # sanity: outputs are finite and the sim advanced
    last = outs[(W + K - 1) & 1]
    assert torch.isfinite(last["obs"]).all().item(), "non-finite observations"

    # ---- phase 2: the same steps with every step's outputs gathered to rank 0 (RCCL, xGMI)
    gather = None
    comm_stuck = [False]  # a rank whose RCCL init never returned: exit without tearing the handle down
    if not args.no_gather:
        gather = {}
        try:
            if world > 1:
                store = dist.distributed_c10d._get_default_store()
                if rank == 0:
                    store.set("mev_comm_id", _capi.comm_unique_id())
                uid = bytes(store.get("mev_comm_id"))
            else:
                uid = _capi.comm_unique_id()
            # ncclCommInitRank blocks until every rank has joined: bounded here so that a
            # rank that never joins costs the gather phase, not the bench line
            import threading
            init_err = []

            gfmt = {"f32": _capi.MEV_GATHER_F32, "u8": _capi.MEV_GATHER_LIDAR_U8,
                    "state": _capi.MEV_GATHER_STATE}[args.gather_format]
            env.set_gather_format(gfmt)

            def _init():
                try:
                    with stdout_to_stderr():
                        env.comm_init(uid, world, rank, root=0, slots=E)
                except Exception as exc:  # reported below
                    init_err.append(exc)

            th = threading.Thread(target=_init, daemon=True)
            th.start()
            th.join(args.gather_timeout)
            if th.is_alive():
                comm_stuck[0] = True
                raise RuntimeError(f"RCCL communicator init did not finish within {args.gather_timeout:.0f} s")
            if init_err:
                raise init_err[0]
            env.reset(device=True)
            for t in range(W):
                env.step(actions[t].data_ptr(), 1.0 / 60.0, auto_reset=True, device=True, gather=True)
            env.gather_wait(int(args.gather_timeout * 1000))
            ok = 1.0
        except Exception as exc:  # reported in the line; never lose the phase-1 result
            gather["error"] = f"rank {rank}: {exc}"[:300]
            ok = 0.0
        if dist is not None:
            t = torch.tensor([ok], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = float(t.item())
        if ok > 0:
            barrier()
            t0 = time.perf_counter()
            try:
                for k in range(K):
                    env.step(actions[W + k].data_ptr(), 1.0 / 60.0, auto_reset=True, device=True, gather=True)
                env.gather_wait(int(args.gather_timeout * 1000))
                ok = 1.0
            except Exception as exc:
                gather["error"] = f"rank {rank}: {exc}"[:300]
                ok = 0.0
            torch.cuda.synchronize(dev)
            g_elapsed = time.perf_counter() - t0
            if dist is not None:
                dist.barrier()
            g_elapsed, bad = max_over_ranks([g_elapsed, 1.0 - ok])
            if bad == 0.0:
                ls = env.lidar_slots()
                per = _capi.packed_layout(E, N, D, gfmt, ls)[1]  # bytes per rank per step
                per_f32 = _capi.packed_layout(E, N, D)[1]
                gather.update({
                    "value": round(world * E * N * K / g_elapsed, 1), "unit": "agent-steps/s",
                    "ms_per_step": round(g_elapsed / K * 1e3, 5), "format": args.gather_format,
                    "bytes_per_rank_per_step": per, "bytes_per_rank_per_step_f32_rows": per_f32,
                    "root_ingress_GBs": round(per * (world - 1) / (g_elapsed / K) / 1e9, 2),
                    "what": "phase 1's steps with every step's packed outputs (reward|done|status|terminated|"
                            "truncated and the observations; state: each agent's post-step state (22 B) + one LiDAR "
                            "code per beam, the 31-float heads rebuilt bit-exactly on the root by mev_unpack_gathered; "
                            "u8: 31-float heads + LiDAR codes; f32: plain rows) gathered to rank 0: one grouped "
                            "ncclSend/ncclRecv per step from the C ABI (MEV_GATHER_TO_ROOT), on a communication "
                            "stream overlapping the next step",
                    "bound": "at N > 1 the root receives (N - 1) x bytes_per_rank_per_step every step over its xGMI "
                             "links, so this phase is bound by the root's ingress, not by the step kernel; at N = 1 "
                             "the root's row is written in place and nothing moves"})
                try:
                    v = verify_gather(env, _capi, E, N, D, world, rank, gfmt, ls, dev, actions[W + K - 1],
                                      int(args.gather_timeout * 1000))
                except Exception as exc:
                    v = f"FAILED: rank {rank}: {exc}"[:300]
                if rank == 0:
                    gather["verified"] = v
            elif "error" not in gather:
                gather["error"] = "another rank failed in the gather phase"
        elif "error" not in gather:
            gather["error"] = "another rank failed to set up the gather"

    if rank == 0:
        total_agent_steps = world * E * N * K
        value = total_agent_steps / elapsed
        roofline = None
        traffic_of = {}
        pmc_file = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_file):
            try:
                pm = json.load(open(pmc_file))
                if pm.get("envs") == E and pm.get("agents") == N and pm.get("rays") == RAYS:
                    traffic_of = {k: v.get("hbm_bytes_per_launch") for k, v in pm.items() if isinstance(v, dict)}
            except Exception:
                traffic_of = {}
        if fused:
            # one k_step launch per step, back to back on the stream: its average launch
            # duration is the stream time between the two HIP events bracketing the timed
            # region / K (the inter-launch gap included; rocprofv3's per-dispatch average
            # in profiles/ is the same quantity without the gap)
            pb = algorithmic_bytes_per_agent_step(RAYS) * E * N
            achieved = pb / (stream_ms * 1e-3) / 1e9
            tab = 'true' if dist_table_needed() else 'false'
            # the instantiation launch_fused picks at this shape (rocprofv3 prints the same arguments:
            # TRAFFIC, TAB, NM, KM, PK, SPLIT, ESPLIT, P1 -- one env per wave, no split at >= 2048
            # workgroups; in the 8-slot layout P1 = the beam count for 64 / 96 / 128 beams, else 1 for a multiple
            # of 64, 2 otherwise)
            fixed8 = N_AGENTS <= 8 and RAYS <= 128
            p1 = (RAYS if RAYS in (64, 96, 128) else (1 if RAYS % 64 == 0 else 2)) if fixed8 else 0
            nc = 8 if fixed8 and p1 >= 64 and N_AGENTS == 8 else 0  # (compile-time agents per env)
            kname = f"mev::k_step<false, {tab}, {8 if fixed8 else 0}, 64, 1, false, false, {p1}, {nc}>"
            roofline = {
                "bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic_of.get("k_step"),
                "kernel": kname, "kernel_ms": round(stream_ms, 5),
                "kernel_ms_source": "stream HIP events around the timed region / steps (one launch per step)",
                "algorithmic_bytes_per_agent_step": algorithmic_bytes_per_agent_step(RAYS), "bytes_per_launch": pb,
                "valu": valu_roofline(stream_ms, E),
                "binding_bound": "VALU issue (the working set is MALL/L2-resident; see valu.frac)",
            }
            if cars_ms is not None:
                roofline["kernel_ms_library_events"] = round(cars_ms, 5)
                roofline["kernel_events"] = (f"library HIP events around the k_step launch on every "
                                             f"{args.event_every}th timed step (they add their own launch latency)")
        elif lidar_ms is not None:
            lb = lidar_bytes_per_agent_step(RAYS) * E * N
            pb = algorithmic_bytes_per_agent_step(RAYS) * E * N
            achieved = lb / (lidar_ms * 1e-3) / 1e9
            roofline = {
                "bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic_of.get("k_lidar"),
                "kernel": "mev::k_lidar<false>", "kernel_ms": round(lidar_ms, 5),
                "algorithmic_bytes_per_agent_step": lidar_bytes_per_agent_step(RAYS), "bytes_per_launch": lb,
                "other_kernels": {"mev::k_cars<false>": {"kernel_ms": round(cars_ms, 5),
                                                    "algorithmic_bytes_per_agent_step": cars_bytes_per_agent_step(RAYS)}},
                "kernel_events": f"library HIP events around each kernel on every {args.event_every}th timed step",
                "step_pipeline": {"kernels_ms": round(cars_ms + lidar_ms, 5), "stream_ms_per_step": round(stream_ms, 5),
                                  "algorithmic_bytes_per_agent_step": algorithmic_bytes_per_agent_step(RAYS),
                                  "achieved_GBs": round(pb / ((cars_ms + lidar_ms) * 1e-3) / 1e9, 3)},
            }
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "clock_settle": {"steps": settle_steps, "ms": args.settle_ms,
                             "what": "untimed steps of the same workload before the warm-up (the SIMD clock's "
                                     "ramp from idle), then the envs reset; --settle-ms 0 turns it off"},
            "ms_per_step": round(elapsed / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: uniform [-1,1) f32 actions pre-generated on device, default 3-lane routes",
            "config": {"workload": f"config 3: {E} envs/GPU x {N} agents x {RAYS}-beam lidar, team reward, "
                                   f"respawn on, max_steps 2000, per-env auto-reset",
                       "envs_per_gpu": E, "agents": N, "rays": RAYS, "obs_dim": D,
                       "parallelism": f"env-sharded x{world} (one process per GPU, no data-path collective)"},
            "roofline": roofline,
            "gather_to_root": gather,
            "cpu_baseline": None,
        }
        if args.config == 5:
            # BASELINE config 5: the sharded step WITH the north star's per-step gather of the stacked
            # outputs to rank 0 is the workload; phase 1 (no collective) is reported beside it
            res["metric"] = ("agent-steps/sec (whole node) at 32768 envs x 8 agents x 128-beam lidar, env-sharded "
                             "over 8 GPUs with the per-step RCCL gather to rank 0 (BASELINE config 5)")
            res["no_gather"] = {"value": res["value"], "ms_per_step": res["ms_per_step"]}
            ok = bool(gather) and "value" in gather
            res["value"] = gather["value"] if ok else None
            res["ms_per_step"] = gather["ms_per_step"] if ok else None
            res["config"]["workload"] = (f"config 5: {world * E} envs ({E} per GPU) x {N} agents x {RAYS}-beam lidar, "
                                         f"team reward, respawn on, max_steps 2000, per-env auto-reset; every step's "
                                         f"outputs gathered to rank 0 ({args.gather_format} rows)")
            res["config"]["parallelism"] = (f"env-sharded x{world} (one process per GPU) + one RCCL gather of every "
                                            f"rank's packed outputs to rank 0 per step (value)")
        if world == 1 and not args.no_cpu_baseline:
            try:
                res["cpu_baseline"] = cpu_baseline()
            except Exception as exc:  # never let the baseline kill the bench line
                res["cpu_baseline"] = {"error": str(exc)[:200]}
        print(json.dumps(res), flush=True)
    if comm_stuck[0]:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)  # the init thread is stuck inside RCCL; nothing else to clean up safely
    env.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
