"""Env sharding over GPUs.

Envs never interact, so a batch of E envs is split into contiguous blocks,
env e -> rank floor(e * G / E), one process and one device handle per GPU,
with no communication inside a step.  The one collective is the gather of
every rank's step outputs to a root rank, and it lives in the C ABI
(mev_comm_init + the MEV_GATHER_TO_ROOT step flag: one grouped RCCL
ncclSend/ncclRecv per step over xGMI, on a communication stream that
overlaps the next step); the data path needs no torch.distributed.

The outputs of one step are packed into ONE flat byte buffer per rank so the
gather is a single message per peer (mev_packed_layout, include/marlenv.h):

    obs f32 [C, N, D] | reward f32 [C, N] | done u8 [C, N] | status u8 [C, N]
    | terminated u8 [C] | truncated u8 [C]     (fields 256-B aligned, total padded to 256 B)

with C = ceil(E / G) slots per rank (ranks with fewer envs leave the tail of
their slots unused).  This module holds the host-side pieces: the partition,
the layout's typed views, the RCCL-id bootstrap through a key-value store, and
a torch.distributed gather of packed buffers that the CPU tests use in place of
RCCL (gloo has no device path).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple


def shard_bounds(total_envs: int, world: int, rank: int) -> Tuple[int, int]:
    """(first env, env count) of `rank`: env e belongs to rank floor(e*world/total)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    start = -(-rank * total_envs // world)          # ceil(rank*E/G): smallest e with e*G/E >= rank
    stop = -(-(rank + 1) * total_envs // world)
    return start, stop - start


def env_owner(env: int, total_envs: int, world: int) -> int:
    return env * world // total_envs


class PackedOutputs:
    """Byte layout of one rank's step outputs: the library's mev_packed_layout2
    (host-only, no device), so these views match what MEV_GATHER_TO_ROOT writes.

    fmt = MEV_GATHER_LIDAR_U8 (the compact format): the message holds each row's
    31-float head and one u8 code per LiDAR beam; unpack() rebuilds the float
    rows through the library's decode table (`table`, Handle.lidar_decode_table()),
    bit-identical to the plain step's.

    fmt = MEV_GATHER_STATE: the message holds each agent's post-step state (22 B)
    and the LiDAR codes, no observation head; the rows are rebuilt on the device by
    the library (`handle`: a Handle with a communicator of this layout,
    mev_unpack_gathered), so unpack() takes torch device buffers only."""

    FIELDS = ("obs", "reward", "done", "status", "terminated", "truncated")

    def __init__(self, slots: int, agents: int, obs_dim: int, fmt: int = 0, lidar_slots: int = 0, table=None,
                 handle=None):
        from . import _capi

        self.C, self.N, self.D = int(slots), int(agents), int(obs_dim)
        self.fmt, self.L = int(fmt), int(lidar_slots)
        if self.fmt == _capi.MEV_GATHER_LIDAR_U8 and table is None:
            raise ValueError("the compact gather format needs the decode table (Handle.lidar_decode_table())")
        if self.fmt == _capi.MEV_GATHER_STATE and handle is None:
            raise ValueError("the state gather format is decoded by the library: pass the root's Handle")
        if handle is not None:
            # the library decodes with the handle's own layout (mev_unpack_gathered): a buffer
            # packed in another layout would be read out of bounds on the device
            comm = getattr(handle, "comm", None)
            got = (getattr(handle, "gather_format", 0), comm["slots"] if comm else None, handle.N, handle.D,
                   handle.lidar_slots())
            want = (self.fmt, self.C, self.N, self.D, self.L if self.fmt else handle.lidar_slots())
            if got != want:
                raise ValueError(f"the handle's gather layout (format, slots, agents, obs_dim, lidar_slots) {got} "
                                 f"differs from this layout's {want}")
        self.table = table
        self.handle = handle
        self.offsets, self.nbytes = _capi.packed_layout(self.C, self.N, self.D, self.fmt, self.L)
        self.offsets: Dict[str, int]
        self.used = (self.offsets["state"] + self.C * self.N * _capi.STATE_BYTES_PER_AGENT
                     if self.fmt == _capi.MEV_GATHER_STATE else
                     self.offsets["lidar"] + (self.C * self.N * self.L if self.fmt else 0))

    def pointers(self, base: int) -> Dict[str, int]:
        """Field pointers (for mev_step's output arguments) inside a buffer at `base`."""
        return {k: base + v for k, v in self.offsets.items()}

    def _shapes(self):
        C, N, D = self.C, self.N, self.D
        sh = {"obs": ((C, N, 31 if self.fmt else D), 4), "reward": ((C, N), 4), "done": ((C, N), 1),
              "status": ((C, N), 1), "terminated": ((C,), 1), "truncated": ((C,), 1)}
        if self.fmt == 2:  # MEV_GATHER_STATE: no observation field
            del sh["obs"]
        if self.fmt:
            sh["lidar"] = ((C, N, self.L), 1)
        return sh

    def unpack(self, buf) -> Dict[str, object]:
        """Outputs of one packed buffer (torch uint8 tensor or numpy uint8 array): views in the
        plain format; in the compact format "obs" is rebuilt [C, N, D] from heads + decoded codes."""
        out = {}
        is_torch = hasattr(buf, "view") and hasattr(buf, "data_ptr")
        for name, (shape, isz) in self._shapes().items():
            off = self.offsets[name]
            n = 1
            for s in shape:
                n *= s
            raw = buf[off: off + n * isz]
            if is_torch:
                import torch
                t = raw.view(torch.float32) if isz == 4 else raw
                out[name] = t.view(*shape)
            else:
                import numpy as np
                a = raw.view(np.float32) if isz == 4 else raw
                out[name] = a.reshape(shape)
        if self.fmt == 2:  # MEV_GATHER_STATE: the library rebuilds the rows on the device
            import torch
            if not is_torch or not buf.is_cuda:
                raise ValueError("the state gather format decodes device buffers (torch) only")
            out.pop("lidar")
            obs = torch.empty((self.C, self.N, self.D), dtype=torch.float32, device=buf.device)
            torch.cuda.current_stream(buf.device).synchronize()  # buf (and obs) ready for the handle's stream
            self.handle.unpack_gathered(buf.data_ptr(), 1, obs.data_ptr())
            self.handle.sync()
            out["obs"] = obs
        elif self.fmt:
            head, codes = out["obs"], out.pop("lidar")
            C, N, D, L = self.C, self.N, self.D, self.L
            if is_torch:
                import torch
                tab = torch.as_tensor(self.table, dtype=torch.float32, device=codes.device)
                obs = torch.zeros((C, N, D), dtype=torch.float32, device=codes.device)
                obs[..., :31] = head
                obs[..., 31:31 + L] = tab[codes.long()]
            else:
                import numpy as np
                obs = np.zeros((C, N, D), np.float32)
                obs[..., :31] = head
                obs[..., 31:31 + L] = np.asarray(self.table, np.float32)[codes]
            out["obs"] = obs
        return out

    def unpack_gathered(self, stacked, total_envs: int, world: int) -> Dict[str, object]:
        """[world, nbytes] gathered buffers -> outputs of all `total_envs` envs in env order."""
        parts: List[Dict[str, object]] = []
        for r in range(world):
            _, cnt = shard_bounds(total_envs, world, r)
            v = self.unpack(stacked[r])
            parts.append({k: x[:cnt] for k, x in v.items()})
        if hasattr(stacked, "data_ptr"):
            import torch
            return {k: torch.cat([p[k] for p in parts]) for k in self.FIELDS}
        import numpy as np
        return {k: np.concatenate([p[k] for p in parts]) for k in self.FIELDS}


def comm_bootstrap(handle, store, world: int, rank: int, root: int = 0, slots: int = 0,
                   key: str = "mev_comm_id") -> None:
    """Join the handle's RCCL communicator: the root draws the unique id
    (mev_comm_unique_id) and publishes it in `store` (any object with
    set/get, e.g. torch.distributed's TCPStore); every rank then calls
    mev_comm_init.  After this, handle.step(..., gather=True) gathers."""
    from . import _capi

    if rank == root:
        uid = _capi.comm_unique_id()
        store.set(key, uid)
    else:
        uid = bytes(store.get(key))
    handle.comm_init(uid, world, rank, root, slots)


def gather_to_root(buf, stacked: Optional[object], group=None, async_op: bool = True):
    """One gather of every rank's packed buffer into `stacked` ([world, nbytes]) on rank 0,
    through torch.distributed: the CPU tests' stand-in (gloo) for the library's RCCL gather."""
    import torch.distributed as dist
    gl = list(stacked.unbind(0)) if stacked is not None else None
    return dist.gather(buf, gather_list=gl, dst=0, group=group, async_op=async_op)
