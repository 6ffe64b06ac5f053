"""The CPU oracle against the golden vectors and the reference's own tests.

Pins: XXH3 against python xxhash; the generators
against the reference's own compiled Random/Zipf/Sequential code; the hash
tables against the reference's unit-test assertions
(tests/NoPartitioningHashJoin/HashTableTest.hpp, tests/DataGenerator/ZipfTest.hpp);
the joins against brute-force semi-join counts.
"""
import json
import os
import threading

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_xxh3_golden():
    for v in load("xxh3.json")["vectors"]:
        assert O.xxh3(v["key"], v["seed"]) == v["hash"], v


def test_murmur3_golden():
    for v in load("murmur3.json")["vectors"]:
        assert O.murmur3(v["key"], v["seed"]) == v["hash"], v


def test_xxhasher_mod_matches_reference_definition():
    # XXHasher::Hash = XXH3_64bits_withSeed(&key, 8, seed) % cardinality (XXHasher.hpp:19-22)
    for v in load("xxh3.json")["vectors"][:50]:
        for card in (1, 3, 32, 1000, 12_500_000):
            assert O.lib().or_hash_mod(O.HASH_XXH3, v["key"], v["seed"], card) == v["hash"] % card


def test_lcg_golden():
    for g in load("generators.json")["lcg"]:
        assert np.array_equal(O.lcg_sequence(g["seed"], len(g["values"])), np.array(g["values"]))


def test_zipf_generate_golden():
    for g in load("generators.json")["zipf"]:
        got = O.zipf_samples(g["alpha"], g["card"], g["seed"], len(g["samples"]))
        assert got.tolist() == g["samples"], (g["alpha"], g["card"])


def test_fill_zipf_golden():
    for g in load("generators.json")["fill_zipf"]:
        t = O.fill_zipf(g["batches"] * O.GEN_BATCH, g["alpha"], g["lo"], g["hi"], g["seed"], threads=3)
        assert t[:, 0].tolist() == g["ids"]
        assert t[:, 1].tolist() == g["payloads"]


def test_fill_sequential_golden():
    g = load("generators.json")["fill_sequential"][0]
    t = O.fill_sequential(g["n"], g["start"])
    assert t[:8, 0].tolist() == g["ids_head"]
    assert t[-8:, 0].tolist() == g["ids_tail"]
    assert t[-8:, 1].tolist() == g["payload_tail"]


def test_zipf_high_skew_reference_test():
    # ZipfTest.TestHighSkew (tests/DataGenerator/ZipfTest.hpp:15-51)
    s = O.zipf_samples(0.99, 10, 123456789, 10_000)
    assert s.min() >= 1 and s.max() <= 10
    freq = np.bincount(s.astype(np.int64), minlength=11)[1:]
    present = freq[freq > 0]
    assert np.all(present[:-1] >= present[1:])


def test_zipf_invalid_arguments():
    with pytest.raises(ValueError):
        O.fill_zipf(10, 1.05, 5, 5, 1)        # [x, x] rejected (Zipf.cpp:61-67)
    with pytest.raises(ValueError):
        O.fill_zipf(10, 0.001, 1, 10, 1)      # alpha < 0.01 (Zipf.cpp:19-21)


@pytest.mark.parametrize("cls,ratio", [(O.LinearProbingTable, 1.0 / 0.75), (O.SeparateChainingTable, 0.3)])
def test_insert_get_and_exists(cls, ratio):
    # testInsertGetAndExists (HashTableTest.hpp:10-26)
    t = cls(10, ratio=ratio, seed=99)
    t.insert(123456789, 0xABC0)
    assert t.exists(123456789)
    assert t.get(123456789) == 0xABC0
    assert not t.exists(987654321)
    assert t.get(987654321) is None


@pytest.mark.parametrize("cls,ratio", [(O.LinearProbingTable, 1.0 / 0.75), (O.SeparateChainingTable, 0.3)])
def test_iterator(cls, ratio):
    # testIterator (HashTableTest.hpp:28-44): the same key 10 times -> GetAll returns 10
    t = cls(10, ratio=ratio, seed=5)
    for i in range(10):
        t.insert(123456789, 0x1000 + 16 * i)
    assert sorted(t.get_all(123456789)) == [0x1000 + 16 * i for i in range(10)]


@pytest.mark.parametrize("cls,ratio", [(O.LinearProbingTable, 1.0 / 0.75), (O.SeparateChainingTable, 0.1)])
def test_multithreaded_insert(cls, ratio):
    # testMultiThreaded (HashTableTest.hpp:46-82); the reference's LinearProbing case
    # runs testIterator by mistake (:163) — here both tables get the real test.
    n = 1000
    t = cls(n, ratio=ratio, seed=3)
    ranges = [(i * n // 4, (i + 1) * n // 4) for i in range(4)]
    ths = [threading.Thread(target=lambda lo, hi: [t.insert(k, 16) for k in range(lo, hi)], args=r)
           for r in ranges]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert all(t.exists(k) for k in range(n))


def test_linear_probing_geometry():
    # getNumberOfBuckets = ceil(ratio * n) (LinearProbing.cpp:7-12)
    assert O.LinearProbingTable(10_000_000).num_buckets == 12_500_000
    with pytest.raises(ValueError):
        O.LinearProbingTable(0)


@pytest.mark.parametrize("case", load("semijoin.json")["cases"], ids=lambda c: c["name"])
def test_semijoin_golden(case):
    R, S = case["R"], case["S"]
    if len(S) == 0:
        S = np.zeros(0, dtype=np.int64)
    assert O.semijoin_count(R, S) == case["matches"]
    assert O.join_nopart(R, S, seed=11).matches == case["matches"]
    for P, radix in ((1, False), (7, False), (32, False), (16, True)):
        assert O.join_radix(R, S, P=P, radix=radix, part_hash=O.HASH_MURMUR3).matches == case["matches"]


def test_empty_build_nopartitioning_raises():
    with pytest.raises(ValueError, match="numberOfObjects"):
        O.join_nopart(np.zeros(0, dtype=np.int64), [1, 2])


@pytest.mark.parametrize("P,radix,hk", [(32, False, O.HASH_XXH3), (1000, False, O.HASH_XXH3),
                                        (256, True, O.HASH_MURMUR3), (1, False, O.HASH_XXH3)])
def test_partition_is_stable_and_complete(P, radix, hk):
    rng = np.random.default_rng(P)
    rel = np.stack([rng.integers(-1000, 1000, 50_000, dtype=np.int64),
                    np.arange(50_000, dtype=np.int64)], axis=1)
    out, bounds = O.partition(rel, P, radix, hk, 77, workers=5)
    assert bounds[0] == 0 and bounds[-1] == rel.shape[0] and np.all(np.diff(bounds.astype(np.int64)) >= 0)
    q = O.partition_ids(rel[:, 0], P, radix, hk, 77)
    expect = rel[np.argsort(q, kind="stable")]
    assert np.array_equal(out, expect)
    # worker count does not change the layout (partition-major, then input order)
    out1, _ = O.partition(rel, P, radix, hk, 77, workers=1)
    assert np.array_equal(out, out1)


@pytest.mark.parametrize("alpha", [1.05, 1.25])
def test_joins_agree_on_generated_tables(alpha):
    R, S = O.generate_tables(100_000, 1_000_000, alpha, seed=17)
    assert S[:, 0].min() >= 1 and S[:, 0].max() <= 100_000
    expect = S.shape[0]
    assert O.semijoin_count(R, S) == expect
    assert O.join_nopart(R, S, workers=3).matches == expect
    for P in (32, 1024):
        r = O.join_radix(R, S, P=P, workers=7)
        assert r.matches == expect
        assert r.partition_ms >= 0 and r.build_ms >= 0 and r.probe_ms >= 0
    S[::3, 0] *= -1
    assert O.join_radix(R, S, P=256, radix=True, part_hash=O.HASH_MURMUR3).matches == O.semijoin_count(R, S)


def test_c1_nopartitioning_single_thread_1m_16m():
    # BASELINE config C1: NoPartitioning, 1M ⋈ 16M, XXH3, the CPU reference path
    # single-threaded (src/main.cpp:81-108 with one worker). SURVEY.md §8(c)
    # observed count 16 000 000 on the reference's own compiled join.
    R, S = O.generate_tables(1_000_000, 16_000_000, 1.05, seed=20240601)
    r = O.join_nopart(R, S, hash_kind=O.HASH_XXH3, seed=0x9E3779B97F4A7C15, workers=1)
    assert r.workers == 1
    assert r.matches == 16_000_000 == O.semijoin_count(R, S)
    # with misses (keys 1..3 leave R, a seventh of S negated) the count follows
    R[:, 0] += 3
    S[::7, 0] = -S[::7, 0]
    expect = int(np.count_nonzero((S[:, 0] > 3) & (S[:, 0] <= 1_000_003)))
    assert O.join_nopart(R, S, workers=1).matches == expect == O.semijoin_count(R, S)
