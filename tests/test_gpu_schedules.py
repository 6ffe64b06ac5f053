"""GPU parity of every kernel schedule the context can be tuned to.

The tuning knobs (read from the environment when a context is created) pick
between kernel schedules that must produce the same bytes: tile size
(PHJ_TILE) and workgroup size (PHJ_BLOCK) of the histogram/scatter kernels,
nontemporal tuple loads (PHJ_NT_LOAD), the join's sub-partitioning of large
partitions (PHJ_SUBPART), the chunked pass 1 of unordered partitions
(PHJ_P1_CHUNK) and its persistent workgroups per shard (PHJ_P1_SLOTS,
PHJ_P1_WPC2), shard count (PHJ_P1_TPS, PHJ_P1_KO_TPS) and size threshold
(PHJ_P1_MIN_TILES), the on-chip probe (PHJ_P2PROBE), fused LDS join vs HBM
tables (PHJ_FUSED), the partitioned bucket tables vs CSR tables (PHJ_PTAB) and
the per-kernel timers (PHJ_TIMERS). Every knob the context reads appears here
(tests/test_tooling.py checks that). Each is checked against the oracle's
stable partition (or, for the unordered layout, the same tuples in every
partition) and semi-join count.
"""
import numpy as np
import pytest

import partitionedhashjoin_amd as phj
from test_gpu_parity import assert_same_partitions
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 0x0BAD_5EED_0BAD_5EED

SCHEDULES = [
    {},
    {"PHJ_BLOCK": "256", "PHJ_TILE": "4096"},
    {"PHJ_BLOCK": "256", "PHJ_TILE": "2048"},
    {"PHJ_BLOCK": "512", "PHJ_TILE": "2048"},
    {"PHJ_BLOCK": "512", "PHJ_TILE": "8192"},
    {"PHJ_BLOCK": "1024", "PHJ_TILE": "8192"},
    {"PHJ_BLOCK": "333"},                      # not compiled: falls back to 512 x 4096
    {"PHJ_BLOCK": "256", "PHJ_TILE": "2048", "PHJ_P1_MIN_TILES": "0"},    # chunked whole-tuple pass 1, non-PACK form
    {"PHJ_BLOCK": "1024", "PHJ_TILE": "8192", "PHJ_P1_MIN_TILES": "0"},   # ... 16 waves (scan words 0-15, reservations 16+)
    {"PHJ_FUSED": "0", "PHJ_PTAB": "0"},
    {"PHJ_FUSED": "0"},
    {"PHJ_FUSED": "0", "PHJ_PTAB": "2"},
    {"PHJ_SUBPART": "0"},
    {"PHJ_TIMERS": "0"},
    {"PHJ_P1_CHUNK": "0"},                                      # on-chip probe over a stable pass 1 (raw keys)
    {"PHJ_P1_MIN_TILES": "0"},                                  # chunked pass 1 at every size
    {"PHJ_P1_MIN_TILES": "0", "PHJ_P1_SLOTS": "-1"},            # one tile per workgroup
    {"PHJ_P1_MIN_TILES": "0", "PHJ_P1_SLOTS": "3"},             # long persistent walks
    {"PHJ_P1_MIN_TILES": "0", "PHJ_P1_TPS": "4"},               # 16 shards on small relations
    {"PHJ_P1_MIN_TILES": "0", "PHJ_P1_TPS": "8", "PHJ_P1_SLOTS": "1"},  # 8 shards, one workgroup each
    {"PHJ_NT_LOAD": "0"},                                       # no nontemporal tuple loads
    {"PHJ_NT_LOAD": "2", "PHJ_P1_MIN_TILES": "0"},              # nontemporal loads in both passes
    {"PHJ_P2PROBE": "0"},                                       # radix: probe side's pass 2 through HBM
    {"PHJ_P2PROBE": "0", "PHJ_P1_MIN_TILES": "0"},              # ... after the chunked pass 1
    {"PHJ_P1_WPC2": "0"},                                       # keys-only pass 1 on every LDS slot
    {"PHJ_P1_WPC2": "1"},                                       # ... on half a workgroup per CU
    {"PHJ_P1_KO_TPS": "4"},                                     # keys-only pass 1: 16 shards on small relations
    {"PHJ_CLUSTER": "0"},                                       # radix count: code tables in HBM (k_probe_ht), not the LDS join
    {"PHJ_CL_CAP": "8192"},                                     # LDS join: 64 KB tables, two workgroups per CU
    {"PHJ_CL_BITS": "11"},                                      # LDS join: 2048 clusters (two digits per pass-1 thread)
    {"PHJ_CL_BITS": "10", "PHJ_P1_KO_TPS": "4"},                # ... 1024 clusters over 16 shards
    {"PHJ_CL_CAP": "8192", "PHJ_CL_BITS": "11"},                # ... 64 KB tables over 2048 clusters
    {"PHJ_P1_PIPE": "0"},                                       # keys-only pass 1 resolving its claims in the same tile
    {"PHJ_P1_PIPE": "0", "PHJ_CL_BITS": "11"},                  # ... with four digits per thread
    {"PHJ_P1_BLOCK": "512"},                                    # pipelined pass 1 in 512 x 8 workgroups
    {"PHJ_P1_BLOCK": "512", "PHJ_CL_BITS": "11"},               # ... four digits per thread
    {"PHJ_R_CHUNK": "0"},                                       # LDS join: R by the stable pass (codes contiguous per cluster)
    {"PHJ_R_CHUNK": "0", "PHJ_CL_BITS": "11"},                  # ... 2048 clusters
    {"PHJ_R_ORDER": "0"},                                       # LDS join: R's pass 1 beside S's
    {"PHJ_R_ORDER": "2"},                                       # ... before it
    {"PHJ_COUNT_PIN": "0"},                                     # LDS join: the count read back by a copy
]

CASES = [((8, 8), 0, phj.HASH_MURMUR3), ((11, 0), 0, phj.HASH_XXH3), ((1, 0), 1000, phj.HASH_XXH3),
         ((3, 5), 0, phj.HASH_XXH3)]


def _sched_id(s):
    return ",".join(f"{k[4:]}={v}" for k, v in s.items()) or "default"


@pytest.fixture(params=SCHEDULES, ids=[_sched_id(s) for s in SCHEDULES])
def tuned_ctx(request, monkeypatch):
    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    c = phj.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("n", [1, 4095, 4097, 250_007])
def test_partition_layout(tuned_ctx, n):
    rng = np.random.default_rng(n)
    # a hot key (skew) plus uniform keys
    keys = rng.integers(-80_000, 80_000, n, dtype=np.int64)
    keys[rng.random(n) < 0.3] = 42
    rel = np.stack([keys, np.arange(n, dtype=np.int64)], axis=1)
    tuned_ctx.upload(phj.SIDE_PROBE, rel)
    for bits, nparts, hk in CASES:
        P, radix = (nparts, False) if nparts else (1 << (bits[0] + bits[1]), True)
        ok = O.HASH_MURMUR3 if hk == phj.HASH_MURMUR3 else O.HASH_XXH3
        out, ob = O.partition(rel, P, radix, ok, SEED, workers=2)
        for stable in (True, False):
            p = phj.radix_params(bits=bits, num_partitions=nparts, hash=hk, seed=SEED, stable=stable)
            v = tuned_ctx.partition(phj.SIDE_PROBE, p)
            k, pay, bounds = tuned_ctx.download_partitioned(v)
            assert np.array_equal(bounds[:P + 1].astype(np.uint64), ob), (bits, nparts, stable)
            if stable:
                assert np.array_equal(k, out[:, 0]), (bits, nparts)
                assert np.array_equal(pay, out[:, 1]), (bits, nparts)
            else:
                assert_same_partitions(k, pay, bounds, out, ob)


def test_join_counts(tuned_ctx):
    R, S = O.generate_tables(30_000, 400_003, 1.05, 21, threads=4)
    S[::7, 0] += 30_000   # misses
    expect = O.semijoin_count(R, S)
    tuned_ctx.upload(phj.SIDE_BUILD, R)
    tuned_ctx.upload(phj.SIDE_PROBE, S)
    for p in (phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED),
              phj.radix_params(num_partitions=1024, hash=phj.HASH_XXH3, seed=SEED),
              phj.radix_params(num_partitions=32, hash=phj.HASH_XXH3, seed=SEED),
              phj.radix_params(num_partitions=1, hash=phj.HASH_MURMUR3, seed=SEED),
              phj.radix_params(num_partitions=777, hash=phj.HASH_XXH3, seed=SEED),
              phj.radix_params((6, 0), hash=phj.HASH_XXH3, seed=SEED),
              phj.nopart_params(hash=phj.HASH_XXH3, seed=SEED),
              phj.nopart_params(hash=phj.HASH_MURMUR3, seed=SEED, table_ratio=1.0)):
        assert tuned_ctx.join(p).matches == expect
