"""Full-size multi-GPU configurations (BASELINE.json C3 and C5, plus the
NoPartitioning member step) through the multi-member step of csrc/phj_group.h.

Eight members share device 0 (PHJ_CTX_LOCAL: the exchange is done by device
copies, RCCL refuses two ranks per device), each running the step an 8-GPU
rank runs on its range shards: R shard pass 1 + pass 2 into the exchange block,
S shard pass 1, the gathered blocks' tables, the on-chip probe, the count sum.
The inputs are the full 10M⋈200M relations with misses (R from 1 + SHIFT,
every 7th S key negated, as in test_gpu_fullsize.py), so the count is far from
|S|; it is checked against the device range count, the oracle's independent
sort-and-search semi-join count and the closed form.
"""
import numpy as np
import pytest

import partitionedhashjoin_amd as phj
from oracle import oracle as O

pytestmark = pytest.mark.gpu

NR, NS = 10_000_000, 200_000_000
SHIFT, NEG_EVERY, GEN_SEED, THREADS = 3, 7, 20240601, 16
SEED = 0x1234_5678_9ABC_DEF1
WORLD = 8


@pytest.mark.parametrize("name,params,alpha", [
    ("C3-radix-8+8-murmur3-s1.05-x8", phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED), 1.05),
    ("C5-radix-8+8-murmur3-s1.25-x8", phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED), 1.25),
    ("nopart-xxh3-s1.05-x8", phj.nopart_params(hash=phj.HASH_XXH3, seed=SEED), 1.05),
])
def test_full_size_eight_members(name, params, alpha):
    with phj.Context(devices=[0] * WORLD, flags=phj.CTX_LOCAL) as g:
        assert g.info() == (WORLD, 0, WORLD)
        g.generate_sequential(phj.SIDE_BUILD, NR, 1 + SHIFT)
        g.generate_zipf(phj.SIDE_PROBE, NS, alpha, 1, NR, GEN_SEED)
        S = g.download(phj.SIDE_PROBE, NS)   # the members' shards, concatenated
        S[::NEG_EVERY, 0] = -S[::NEG_EVERY, 0]
        g.upload(phj.SIDE_PROBE, S)          # re-sharded
        keys = S[:, 0]
        expect = int(np.count_nonzero((keys > SHIFT) & (keys <= NR + SHIFT)))
        assert 0.4 * NS < expect < 0.85 * NS
        assert g.count_in_range(phj.SIDE_PROBE, 1 + SHIFT, NR + SHIFT) == expect
        R = g.download(phj.SIDE_BUILD, NR)
        assert O.semijoin_count(R, S, threads=THREADS) == expect
        del R, S, keys
        for _ in range(2):   # the second step reuses every buffer
            assert g.join(params).matches == expect, name
