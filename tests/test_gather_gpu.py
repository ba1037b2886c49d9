"""The C ABI's multi-GPU gather (mev_comm_init + MEV_GATHER_TO_ROOT) and the
DLPack export, on one MI355X.

* world 1: a handle stepping with the gather writes its outputs into its row of
  the root's gather buffer; that row must equal, bit for bit, the outputs of a
  plain handle stepping the same envs with the same actions (and mev_get_outputs
  of the gathering handle must return the same);
* two ranks on the box's one GPU (tools/gather_ranks.py): rank 1's rows arrive
  in the root's buffer through ncclSend/ncclRecv, checked against one handle
  stepping all envs; skipped if RCCL refuses two ranks on one device;
* DLPack: the internal output buffers as torch tensors, zero copy."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.gpu

FIELDS = ("obs", "reward", "done", "status", "terminated", "truncated")


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


@pytest.mark.parametrize("fmt", [0, 1, 2], ids=["f32", "lidar_u8", "state"])
def test_gather_world1_row_equals_plain_step(mev, fmt):
    """fmt 1: the compact format (heads + one u8 code per beam), decoded through the
    library's table -- bit-identical to the plain rows, dead agents included.  fmt 2:
    the state format (post-step state + codes; the ranks write no heads), the rows
    rebuilt on the device by mev_unpack_gathered -- bit-identical too."""
    import torch
    import torch.utils.dlpack as tdl
    from marl_traffic_intersection_amd import _capi, sharding

    E, N, R, T = 48, 8, 64, 40
    cfg = dict(num_envs=E, num_agents=N, lidar_rays=R, use_team_reward=1, max_steps=25, device=0,
               respawn_enabled=0 if fmt else 1)  # no respawn: crashed agents stay dead (code 255 rows)
    plain = mev.Handle(**cfg)
    gat = mev.Handle(**cfg)
    try:
        if fmt:
            gat.set_gather_format(fmt)
        gat.comm_init(_capi.comm_unique_id(), world=1, rank=0, root=0, slots=E + 3)
        lay = sharding.PackedOutputs(E + 3, N, plain.D, fmt=fmt, lidar_slots=gat.lidar_slots(),
                                     table=gat.lidar_decode_table() if fmt == 1 else None,
                                     handle=gat if fmt == 2 else None)
        if fmt:
            assert lay.nbytes < (0.6 if fmt == 1 else 0.3) * sharding.PackedOutputs(E + 3, N, plain.D).nbytes
        rng = np.random.default_rng(5)
        for t in range(T):
            act = rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)
            ref = plain.step(act, auto_reset=True)
            extra = {"agents_alive": np.zeros(E, np.int32), "step": np.zeros(E, np.int32)}
            gat.step(act, auto_reset=True, gather=True, out=extra)
            gat.gather_wait(30000)
            ptr, nbytes, world = gat.gather_result()
            assert world == 1 and nbytes == lay.nbytes and ptr
            dbuf = tdl.from_dlpack(gat.output_dlpack("gathered"))
            assert tuple(dbuf.shape) == (1, lay.nbytes)
            if fmt == 2:  # decoded on the device by the library
                got = {k: v.cpu().numpy() for k, v in lay.unpack(dbuf[0]).items()}
            else:
                got = lay.unpack(dbuf.cpu().numpy()[0])
            for k in FIELDS:
                assert np.array_equal(_bits(got[k][:E]), _bits(ref[k])), (t, k)
                tail = got[k][E:, :, :31] if (fmt == 1 and k == "obs") else got[k][E:]
                assert not np.any(tail), (t, k)  # unused slots stay zero
            assert np.array_equal(extra["agents_alive"], ref["agents_alive"])
            assert np.array_equal(extra["step"], ref["step"])
            last = gat.get_outputs()  # mev_get_outputs reads where the step wrote: the packed row
            for k in FIELDS:
                assert np.array_equal(_bits(last[k]), _bits(ref[k])), (t, k)
        gat.comm_destroy()
    finally:
        plain.close()
        gat.close()


@pytest.mark.parametrize("fmt", [0, 1], ids=["f32", "lidar_u8"])
def test_gather_world1_traffic_early_split(mev, fmt):
    """Config-4 shape at 1024 envs (the traffic early split: four car waves and one
    LiDAR wave per workgroup, which writes the LiDAR codes and the dead egos' rows
    itself): the gathered row equals the plain step's bit for bit, with dead egos (code
    255 rows) and no auto-reset.  (The state format is refused with traffic.)"""
    from marl_traffic_intersection_amd import _capi, sharding
    import torch.utils.dlpack as tdl

    E, T = 1024, 80
    cfg = dict(num_envs=E, num_agents=1, lidar_rays=64, traffic_flow=1, traffic_density=2.0, max_npcs=32,
               respawn_enabled=0, device=0)
    plain = mev.Handle(**cfg)
    gat = mev.Handle(**cfg)
    try:
        assert plain.step_split() == 2 and gat.step_split() == 2
        if fmt:
            gat.set_gather_format(fmt)
        gat.comm_init(_capi.comm_unique_id(), world=1, rank=0, root=0)
        lay = sharding.PackedOutputs(E, 1, plain.D, fmt=fmt, lidar_slots=gat.lidar_slots(),
                                     table=gat.lidar_decode_table() if fmt == 1 else None)
        # every 7th env's ego dead (Car::alive written through set_state; the reference's step
        # never revives it): the LiDAR wave writes those rows itself (zeros / code 255)
        for h in (plain, gat):
            st = h.get_state()
            st["alive"][::7, 0] = 0
            h.set_state(st)
        rng = np.random.default_rng(6)
        dead = 0
        for t in range(T):
            act = rng.uniform(-1, 1, (E, 1, 2)).astype(np.float32)
            act[..., 0] = np.abs(act[..., 0])  # (throttle on: egos reach walls and cars)
            # (no auto-reset: the dead egos stay dead, the envs that ended stay over; the same
            # seed: the same Philox spawns)
            ref = plain.step(act)
            gat.step(act, gather=True,
                     out={"agents_alive": np.zeros(E, np.int32), "step": np.zeros(E, np.int32)})
            gat.gather_wait(30000)
            dbuf = tdl.from_dlpack(gat.output_dlpack("gathered"))
            got = lay.unpack(dbuf.cpu().numpy()[0])
            for k in FIELDS:
                assert np.array_equal(_bits(got[k]), _bits(ref[k])), (t, k)
            dead += int((ref["agents_alive"] == 0).sum())
        assert dead > 0  # dead egos' rows were exercised
        gat.comm_destroy()
    finally:
        plain.close()
        gat.close()


def test_gather_argument_errors(mev):
    from marl_traffic_intersection_amd import _capi

    h = mev.Handle(num_envs=4, num_agents=2, lidar_rays=16, device=0)
    try:
        act = np.zeros((4, 2, 2), np.float32)
        with pytest.raises(mev.MevError, match="communicator"):
            h.step(act, gather=True)
        with pytest.raises(mev.MevError):
            h.gather_result()
        h.comm_init(_capi.comm_unique_id(), 1, 0, 0)
        with pytest.raises(mev.MevError, match="NULL output pointers"):
            h.step(act, gather=True, out=h.alloc_outputs())
        with pytest.raises(mev.MevError, match="no step"):
            h.gather_result()
        with pytest.raises(mev.MevError, match="already"):
            h.comm_init(_capi.comm_unique_id(), 1, 0, 0)
        with pytest.raises(mev.MevError):
            h.comm_destroy()
            h.comm_init(_capi.comm_unique_id(), 1, 0, 0, slots=3)  # slots < num_envs
    finally:
        h.close()


def test_dlpack_outputs_alias_the_internal_buffers(mev):
    import torch

    E, N, R = 16, 3, 32
    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=R, use_team_reward=1, device=0)
    try:
        torch.cuda.set_device(0)
        acts = torch.rand((E, N, 2), device="cuda:0") * 2 - 1
        for _ in range(5):
            h.step(acts, device=True, auto_reset=True)  # no output pointers: the internal buffers
        h.sync()
        t = h.output_tensors()
        host = h.get_outputs()
        assert t["obs"].shape == (E, N, h.D) and t["obs"].dtype == torch.float32 and t["obs"].is_cuda
        assert t["agents_alive"].dtype == torch.int32 and t["done"].dtype == torch.uint8
        for k, v in host.items():
            assert np.array_equal(_bits(t[k].cpu().numpy()), _bits(v)), k
        ptrs = {}
        for k in ("obs", "reward", "done", "status", "terminated", "truncated"):
            ptrs[k] = t[k].data_ptr()
        h.step(acts, device=True)  # zero copy: the same tensors see the next step
        h.sync()
        assert t["obs"].data_ptr() == ptrs["obs"]
        assert np.array_equal(_bits(t["obs"].cpu().numpy()), _bits(h.observations()))
    finally:
        h.close()


def test_gather_two_ranks_on_one_device():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gather_ranks.py"), "--ranks", "2"],
                       capture_output=True, text=True, timeout=150, cwd=ROOT)
    out = r.stdout + r.stderr
    if "SKIP" in r.stdout:
        pytest.skip(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and "GATHER OK" in r.stdout, out[-3000:]


def test_output_views_follow_host_and_gather_steps(mev):
    """mev_device_outputs / DLPack views hold the LAST outputs whichever buffers the step
    wrote: a small handle's host-mode step (pinned zero-copy block), a device step into
    caller buffers, and a packed gather row are each copied into the internal buffers
    before the views are handed out."""
    import torch
    from marl_traffic_intersection_amd import _capi

    E, N, R = 16, 3, 32
    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=R, use_team_reward=1, device=0)
    try:
        torch.cuda.set_device(0)
        h.set_stream(torch.cuda.current_stream().cuda_stream)
        rng = np.random.default_rng(9)
        for _ in range(4):  # host mode: the pinned block (outputs <= 256 KB)
            host = h.step(rng.uniform(-1, 1, (E, N, 2)).astype(np.float32), auto_reset=True)
        t = h.output_tensors()
        torch.cuda.synchronize()
        for k, v in host.items():
            assert np.array_equal(_bits(t[k].cpu().numpy()), _bits(v)), k
        mine = {k: torch.zeros_like(torch.as_tensor(v), device="cuda:0") for k, v in h.alloc_outputs().items()}
        h.step(torch.rand((E, N, 2), device="cuda:0") * 2 - 1, out=mine, device=True)  # caller buffers
        t = h.output_tensors()
        torch.cuda.synchronize()
        for k in mine:
            assert torch.equal(t[k], mine[k]), k
        h.comm_init(_capi.comm_unique_id(), world=1, rank=0, root=0)
        h.step(torch.rand((E, N, 2), device="cuda:0") * 2 - 1, device=True, gather=True)  # packed row
        last = h.get_outputs()
        t = h.output_tensors(("obs", "reward", "done", "status", "terminated", "truncated"))
        torch.cuda.synchronize()
        for k, v in t.items():
            assert np.array_equal(_bits(v.cpu().numpy()), _bits(last[k])), k
        h.comm_destroy()
    finally:
        h.close()
