"""Multi-rank HIP path on one GPU: two ranks share cuda:0 over gloo (RCCL
refuses two ranks on one device), so the real HipShardEngine pack /
all-gather / multi-segment join / count all-reduce run end to end."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, nR, nS, alpha, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import partitionedhashjoin_amd as phj
        from partitionedhashjoin_amd.distributed import HipShardEngine, distributed_join
        from partitionedhashjoin_amd.distributed import shard_range
        eng = HipShardEngine(0)
        # R holds keys [1 + off, |R| + off], S draws from [1, |R|]: S keys below
        # 1 + off miss, so the expected count is the S keys in [1 + off, |R|]
        off = nR // 3
        rlo, rhi = shard_range(nR, rank, world)
        slo, shi = shard_range(nS, rank, world)
        eng.ctx_r.generate_sequential(0, rhi - rlo, 1 + off, rlo)
        eng.ctx.generate_zipf(1, shi - slo, alpha, 1, nR, 77, slo)
        eng.share_build()
        expect_local = eng.ctx.count_in_range(1, 1 + off, nR)
        for _ in range(2):   # a second step reuses every buffer
            res = distributed_join(eng, phj.radix_params((8, 8)), nR, nS, rank, world, dist)
        out[rank] = (res.matches, expect_local, res.local_matches)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_hip_engine_multirank_on_one_gpu(world):
    nR, nS = 300_001, 4_000_003
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), nR, nS, 1.25, out), nprocs=world)
    expect = sum(out[r][1] for r in range(world))
    assert 0 < expect < nS
    assert {out[r][0] for r in range(world)} == {expect}
    # each rank's local count is exactly its own S shard's matches
    assert all(out[r][2] == out[r][1] for r in range(world))


def test_single_rank_generation_matches_sharded_generation():
    import partitionedhashjoin_amd as phj
    from partitionedhashjoin_amd.distributed import shard_range
    n = 4096 * 5 + 123
    with phj.Context(0) as full:
        full.generate_zipf(1, n, 1.05, 1, 10_000, 9)
        whole = full.download(1)
        parts = []
        for r in range(3):
            lo, hi = shard_range(n, r, 3)
            full.generate_zipf(1, hi - lo, 1.05, 1, 10_000, 9, lo)
            parts.append(full.download(1))
    import numpy as np
    assert np.array_equal(whole, np.concatenate(parts))


def _nccl_worker(rank, port, nR, nS, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import partitionedhashjoin_amd as phj
        from partitionedhashjoin_amd.distributed import HipShardEngine, distributed_join
        eng = HipShardEngine(0)
        off = nR // 4
        eng.ctx_r.generate_sequential(0, nR, 1 + off, 0)
        eng.ctx.generate_zipf(1, nS, 1.05, 1, nR, 5, 0)
        eng.share_build()
        expect = eng.ctx.count_in_range(1, 1 + off, nR)
        got = [distributed_join(eng, phj.radix_params((8, 8)), nR, nS, 0, 1, dist,
                                force_exchange=True).matches for _ in range(3)]
        out[0] = (got, expect)
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_branch_world_one():
    """The N>1 step (pack, asynchronous RCCL all-gather issued from the R
    stream, S issued from the second host thread, work.wait, multi-segment
    join, RCCL all-reduce) over the real nccl backend on a world of one: the
    8-GPU bench runs exactly this code with more ranks."""
    nR, nS = 1_000_003, 20_000_001
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_nccl_worker, args=(_free_port(), nR, nS, out), nprocs=1)
    got, expect = out[0]
    assert 0 < expect < nS
    assert got == [expect] * 3


def _np_worker(rank, world, port, backend, nR, nS, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import partitionedhashjoin_amd as phj
        from partitionedhashjoin_amd.distributed import HipShardEngine, distributed_join_nopart, shard_range
        eng = HipShardEngine(0)
        off = nR // 3
        rlo, rhi = shard_range(nR, rank, world)
        slo, shi = shard_range(nS, rank, world)
        eng.ctx_r.generate_sequential(0, rhi - rlo, 1 + off, rlo)
        eng.ctx.generate_zipf(1, shi - slo, 1.25, 1, nR, 31, slo)
        eng.share_build()
        expect_local = eng.ctx.count_in_range(1, 1 + off, nR)
        for _ in range(2):
            res = distributed_join_nopart(eng, phj.nopart_params(), nR, nS, rank, world, dist,
                                          force_exchange=True)
        out[rank] = (res.matches, expect_local, res.local_matches)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("backend,world", [("gloo", 2), ("gloo", 3), ("nccl", 1)])
def test_nopart_replicated_build_multirank(backend, world):
    """NoPartitioning over range shards: all-gather of the R shards, global
    table per rank, local S probe, count all-reduce."""
    nR, nS = 300_001, 4_000_003
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_np_worker, args=(world, _free_port(), backend, nR, nS, out), nprocs=world)
    expect = sum(out[r][1] for r in range(world))
    assert 0 < expect < nS
    assert {out[r][0] for r in range(world)} == {expect}
    assert all(out[r][2] == out[r][1] for r in range(world))
