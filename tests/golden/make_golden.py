#!/usr/bin/env python3
"""Regenerate the golden vectors in tests/golden/ (run in the build container).

Sources (no reference source is copied; only inputs/outputs are recorded):
  xxh3.json     XXH3_64bits_withSeed over the 8 little-endian key bytes, from
                the python `xxhash` package (3.8.1, libxxhash 0.8.2) — the
                third-party hash the reference calls (src/Common/XXHasher.hpp:20).
  murmur3.json  fmix64(key ^ seed) from the canonical MurmurHash3 constants,
                computed here in pure Python (no oracle code involved).
  generators.json
                outputs of the reference's OWN generator code
                (src/Common/Random.cpp, src/DataGenerator/{Zipf,Sequential}.cpp)
                compiled unmodified into oracle/_ref/libref_gen.so.
  semijoin.json small adversarial relations with their semi-join counts,
                computed by brute force in pure Python.
  reference_results/*.txt
                the reference's own published result files (data), used to pin
                the JSON output format of the phjoin CLI.
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

M64 = (1 << 64) - 1
I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


def fmix64(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & M64
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & M64
    return k ^ (k >> 33)


def keys_and_seeds(rng):
    specials = [0, 1, -1, 2, I64_MIN, I64_MAX, 123456789, 1 << 32, -(1 << 32), 10_000_000]
    seeds = [0, 1, 0x9E3779B97F4A7C15, M64, 0x1234_5678_9ABC_DEF1, 20240601]
    out = [(k, s) for k in specials for s in seeds]
    for _ in range(200):
        out.append((rng.randint(I64_MIN, I64_MAX), rng.randint(0, M64)))
    return out


def main():
    import xxhash
    rng = random.Random(20240601)
    pairs = keys_and_seeds(rng)
    xx = [{"key": k, "seed": s,
           "hash": xxhash.xxh3_64_intdigest(k.to_bytes(8, "little", signed=True), seed=s)}
          for k, s in pairs]
    with open(os.path.join(HERE, "xxh3.json"), "w") as f:
        json.dump({"source": f"python xxhash {xxhash.VERSION} (libxxhash {xxhash.XXHASH_VERSION})",
                   "vectors": xx}, f)
    mm = [{"key": k, "seed": s, "hash": fmix64((k & M64) ^ s)} for k, s in pairs]
    with open(os.path.join(HERE, "murmur3.json"), "w") as f:
        json.dump({"source": "fmix64(key ^ seed), canonical MurmurHash3 finalizer constants",
                   "vectors": mm}, f)

    from oracle import oracle as O
    if O.ref() is None:
        raise SystemExit("oracle/_ref/libref_gen.so missing: build it where /root/reference exists")
    gen = {"source": "reference src/Common/Random.cpp + src/DataGenerator/{Zipf,Sequential}.cpp "
                     "compiled unmodified (oracle/ref/Makefile)",
           "lcg": [], "zipf": [], "fill_zipf": [], "fill_sequential": []}
    for seed in (1, 123456789, 2147483646, 42):
        gen["lcg"].append({"seed": seed, "values": O.ref_lcg_sequence(seed, 64).tolist()})
    # ZipfTest.TestHighSkew parameters (tests/DataGenerator/ZipfTest.hpp:16-19) and the workloads' skews
    for alpha, card, seed in ((0.99, 10, 123456789), (1.05, 10_000_000, 7), (1.25, 10_000_000, 7),
                              (0.5, 1000, 3), (1.0, 1_000_000, 11), (2.0, 100, 5)):
        gen["zipf"].append({"alpha": alpha, "card": card, "seed": seed,
                            "samples": [int(x) for x in O.ref_zipf_samples(alpha, card, seed, 256)]})
    for alpha, lo, hi, seed, batches in ((1.05, 1, 1_000_000, 20240601, 2), (1.25, 1, 10_000_000, 5, 1)):
        t = O.ref_fill_zipf(alpha, lo, hi, seed, batches)
        gen["fill_zipf"].append({"alpha": alpha, "lo": lo, "hi": hi, "seed": seed, "batches": batches,
                                 "ids": t[:, 0].tolist(), "payloads": t[:, 1].tolist()})
    t = O.ref_fill_sequential(1, 20_000)
    gen["fill_sequential"].append({"start": 1, "n": 20_000, "ids_head": t[:8, 0].tolist(),
                                   "ids_tail": t[-8:, 0].tolist(), "payload_tail": t[-8:, 1].tolist()})
    with open(os.path.join(HERE, "generators.json"), "w") as f:
        json.dump(gen, f)

    cases = [
        {"name": "survey_0_1", "R": [1, 1, 2, 0, -1, I64_MIN, I64_MAX],
         "S": [1, 2, 3, 0, -1, -1, I64_MIN, I64_MAX, 5, 1]},
        {"name": "empty_probe", "R": [1, 2, 3], "S": []},
        {"name": "no_match", "R": [1, 2, 3], "S": [4, 5, 6, -1]},
        {"name": "all_duplicates", "R": [7] * 50, "S": [7] * 20 + [8] * 5},
    ]
    r = random.Random(9)
    cases.append({"name": "random_small", "R": [r.randint(-500, 500) for _ in range(700)],
                  "S": [r.randint(-1000, 1000) for _ in range(3000)]})
    for c in cases:
        keys = set(c["R"])
        c["matches"] = sum(1 for s in c["S"] if s in keys)
    with open(os.path.join(HERE, "semijoin.json"), "w") as f:
        json.dump({"source": "brute-force set membership in pure Python", "cases": cases}, f)
    print("golden vectors written")


if __name__ == "__main__":
    main()
