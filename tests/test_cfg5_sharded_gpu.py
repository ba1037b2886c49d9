"""Config 5 -- 32768 envs x 8 agents x 128 beams, team reward, env-sharded over 8
ranks with the per-step gather of every rank's outputs to the root -- on one
MI355X.

One handle steps all 32768 envs.  Eight handles, one per rank's shard
(sharding.shard_bounds: contiguous blocks of 4096 envs), start from the same
state slices and step with the same actions, each with MEV_GATHER_TO_ROOT on a
world-of-one communicator, so the library itself writes every step's packed row
(obs | reward | done | status | terminated | truncated, mev_packed_layout).  The
eight rows are stacked as the root's [world][bytes] buffer would hold them and
reassembled with PackedOutputs.unpack_gathered: the result must equal the big
handle's outputs bit for bit at every step, with auto-resets in the window.
(At world > 1 the rows travel by ncclSend/ncclRecv; RCCL refuses two ranks on
one device, so that leg is the driver's multi-GPU run.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

E, N, RAYS, G, T, MAXS = 32768, 8, 128, 8, 50, 2000
FIELDS = ("obs", "reward", "done", "status", "terminated", "truncated")


@pytest.mark.parametrize("fmt", [0, 1, 2], ids=["f32", "lidar_u8", "state"])
def test_cfg5_shards_reassembled_from_packed_rows_equal_one_handle(mev, fmt):
    import torch
    import torch.utils.dlpack as tdl
    from marl_traffic_intersection_amd import _capi, sharding

    cfg = dict(num_agents=N, lidar_rays=RAYS, use_team_reward=1, respawn_enabled=1, max_steps=MAXS, device=0)
    big = mev.Handle(num_envs=E, **cfg)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(0)
    big.set_stream(stream.cuda_stream)
    D = big.D
    assert D == 31 + RAYS
    big.reset()
    warm = torch.Generator(device="cuda:0").manual_seed(3)
    for _ in range(30):  # move the envs apart
        big.step(torch.rand((E, N, 2), device="cuda:0", generator=warm) * 2 - 1, auto_reset=True, device=True)
    rng = np.random.default_rng(21)
    st = big.get_state()
    st["step_count"][:] = MAXS - rng.integers(1, 4 * T, E)  # truncations + auto-resets inside the window
    big.set_state(st)
    shards = []
    for r in range(G):
        s0, cnt = sharding.shard_bounds(E, G, r)
        assert cnt == E // G
        h = mev.Handle(num_envs=cnt, **cfg)
        h.set_stream(stream.cuda_stream)
        h.set_state({k: v[s0:s0 + cnt] for k, v in st.items()})
        if fmt:
            h.set_gather_format(fmt)
        h.comm_init(_capi.comm_unique_id(), world=1, rank=0, root=0, slots=cnt)
        shards.append((s0, cnt, h))
    lay = sharding.PackedOutputs(E // G, N, D, fmt=fmt, lidar_slots=big.lidar_slots(),
                                 table=shards[0][2].lidar_decode_table() if fmt == 1 else None,
                                 handle=shards[0][2] if fmt == 2 else None)
    out = {k: torch.zeros_like(torch.as_tensor(v), device="cuda:0") for k, v in big.alloc_outputs().items()}
    extra = [{"agents_alive": torch.zeros(cnt, dtype=torch.int32, device="cuda:0"),
              "step": torch.zeros(cnt, dtype=torch.int32, device="cuda:0")} for _, cnt, _ in shards]
    ended = 0
    for t in range(T):
        a = torch.rand((E, N, 2), device="cuda:0", generator=warm) * 2 - 1
        big.step(a, auto_reset=True, out=out, device=True)
        rows = []
        for (s0, cnt, h), ex in zip(shards, extra):
            h.step(a[s0:s0 + cnt].contiguous(), auto_reset=True, device=True, gather=True, out=ex)
            ptr, nbytes, world = h.gather_result()
            assert world == 1 and nbytes == lay.nbytes and ptr
            rows.append(tdl.from_dlpack(h.output_dlpack("gathered"))[0])
        stacked = torch.stack(rows)  # what the root's [world][bytes] buffer holds after the gather
        got = lay.unpack_gathered(stacked, E, G)
        for k in FIELDS:
            ref = out[k]
            g = got[k]
            assert g.shape == ref.shape, (t, k, g.shape, ref.shape)
            if ref.dtype == torch.float32:
                ref, g = ref.view(torch.int32), g.contiguous().view(torch.int32)
            assert torch.equal(g, ref), f"step {t + 1}: {k}"
        assert torch.equal(torch.cat([ex["step"] for ex in extra]), out["step"]), t
        assert torch.equal(torch.cat([ex["agents_alive"] for ex in extra]), out["agents_alive"]), t
        ended += int(out["truncated"].sum().item())
    assert ended > 100, f"only {ended} truncations in the window: auto-reset not exercised"
    # the shards' final state is the big handle's, slice by slice
    fin = big.get_state()
    for s0, cnt, h in shards:
        sst = h.get_state()
        for k, v in sst.items():
            assert np.array_equal(v, fin[k][s0:s0 + cnt]), k
        h.comm_destroy()
        h.close()
    big.close()
