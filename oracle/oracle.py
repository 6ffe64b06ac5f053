"""TEST INFRASTRUCTURE ONLY — ctypes view of the CPU oracle (oracle/liboracle.so)
and of the reference's own generator code (oracle/_ref/libref_gen.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (partitionedhashjoin_amd/) never does. Relations are
numpy int64 arrays of shape (n, 2) = {id, payload}, the Common::Tuple layout
(src/Common/Table.hpp:20-25).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref_gen.so")

HASH_XXH3 = 0
HASH_MURMUR3 = 1
GEN_BATCH = 4096

_lib = None
_ref = None

_P = C.c_void_p
_u64 = C.c_uint64
_i64 = C.c_int64
_d = C.c_double
_i = C.c_int


class OrResult(C.Structure):
    _fields_ = [("matches", _u64), ("partition_ms", _d), ("build_ms", _d), ("probe_ms", _d),
                ("probe_only_ms", _d), ("wall_ms", _d), ("workers", _i)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def build():
    """Compile liboracle.so (and oracle/_ref when /root/reference is present)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    if os.path.isdir("/root/reference/src"):
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "ref")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        sig = {
            "or_xxh3_64": (_u64, [_i64, _u64]),
            "or_murmur3": (_u64, [_i64, _u64]),
            "or_hash": (_u64, [_i, _i64, _u64]),
            "or_hash_mod": (_u64, [_i, _i64, _u64, _u64]),
            "or_hash_many": (None, [_i, _P, _u64, _u64, _P]),
            "or_lcg_step": (_i64, [_i64]),
            "or_lcg_next": (_d, [C.POINTER(_i64)]),
            "or_zipf_generate": (_u64, [_d, _u64, C.POINTER(_i64)]),
            "or_batch_seed": (_i64, [_u64, _u64]),
            "or_fill_sequential": (None, [_P, _u64, _i64]),
            "or_fill_zipf": (_i, [_P, _u64, _d, _i64, _i64, _u64, _i]),
            "or_lp_new": (_P, [_d, _u64, _i, _u64]),
            "or_lp_free": (None, [_P]),
            "or_lp_num_buckets": (_u64, [_P]),
            "or_lp_insert": (None, [_P, _i64, _P]),
            "or_lp_get": (_P, [_P, _i64]),
            "or_lp_exists": (_i, [_P, _i64]),
            "or_lp_get_all": (_u64, [_P, _i64, _P, _u64]),
            "or_sc_new": (_P, [_d, _u64, _i, _u64]),
            "or_sc_free": (None, [_P]),
            "or_sc_num_buckets": (_u64, [_P]),
            "or_sc_insert": (_i, [_P, _i64, _P]),
            "or_sc_get": (_P, [_P, _i64]),
            "or_sc_exists": (_i, [_P, _i64]),
            "or_sc_get_all": (_u64, [_P, _i64, _P, _u64]),
            "or_partition": (_i, [_P, _u64, _u64, _i, _i, _u64, _i, _P, _P]),
            "or_partition_id": (_u64, [_i64, _u64, _i, _i, _u64]),
            "or_join_nopart": (_i, [_P, _u64, _P, _u64, _i, _u64, _d, _i, C.POINTER(OrResult)]),
            "or_join_radix": (_i, [_P, _u64, _P, _u64, _u64, _i, _i, _u64, _i, _u64, _d, _i,
                                   C.POINTER(OrResult)]),
            "or_semijoin_count_sorted": (_u64, [_P, _u64, _P, _u64, _i]),
            "or_semijoin_count_keys": (_u64, [_P, _u64, _P, _u64, _i]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def ref():
    """The reference's own generator code (None where it was never built)."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_PATH):
            return None
        L = C.CDLL(REF_PATH)
        L.ref_lcg_sequence.argtypes = [C.c_long, _u64, _P]
        L.ref_zipf_samples.argtypes = [_d, _u64, C.c_long, _u64, _P]
        L.ref_fill_zipf.argtypes = [_d, _i64, _i64, _u64, _u64, _u64, _P]
        L.ref_fill_sequential.argtypes = [_i64, _u64, _P]
        for f in (L.ref_lcg_sequence, L.ref_zipf_samples, L.ref_fill_zipf, L.ref_fill_sequential):
            f.restype = _i
        _ref = L
    return _ref


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_P)


def relation(n: int) -> np.ndarray:
    return np.zeros((n, 2), dtype=np.int64)


def as_relation(a) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.int64))
    if a.ndim == 1:
        a = np.stack([a, np.arange(a.shape[0], dtype=np.int64)], axis=1)
    assert a.ndim == 2 and a.shape[1] == 2
    return np.ascontiguousarray(a)


# ---- hashing ----
def xxh3(key: int, seed: int) -> int:
    return lib().or_xxh3_64(key, seed)


def murmur3(key: int, seed: int) -> int:
    return lib().or_murmur3(key, seed)


def hash_keys(kind: int, keys, seed: int) -> np.ndarray:
    keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
    out = np.zeros(keys.shape[0], dtype=np.uint64)
    lib().or_hash_many(kind, _ptr(keys), keys.shape[0], seed, _ptr(out))
    return out


# ---- generators ----
def fill_sequential(n: int, start: int = 1) -> np.ndarray:
    t = relation(n)
    lib().or_fill_sequential(_ptr(t), n, start)
    return t


def fill_zipf(n: int, alpha: float, lo: int, hi: int, seed: int, threads: int = 8) -> np.ndarray:
    t = relation(n)
    rc = lib().or_fill_zipf(_ptr(t), n, alpha, lo, hi, seed, threads)
    if rc != 0:
        raise ValueError("invalid Zipf range or skew")
    return t


def lcg_sequence(seed: int, n: int) -> np.ndarray:
    st = _i64(seed)
    L = lib()
    return np.array([L.or_lcg_next(C.byref(st)) for _ in range(n)], dtype=np.float64)


def zipf_samples(alpha: float, card: int, seed: int, n: int) -> np.ndarray:
    st = _i64(seed)
    L = lib()
    return np.array([L.or_zipf_generate(alpha, card, C.byref(st)) for _ in range(n)],
                    dtype=np.uint64)


def generate_tables(nR: int, nS: int, alpha: float, seed: int, threads: int = 8):
    """generateTables (src/main.cpp:35-79) with a seed: R Sequential from 1, S Zipf over [1, |R|]."""
    R = fill_sequential(nR, 1)
    S = fill_zipf(nS, alpha, 1, nR, seed, threads)
    return R, S


# ---- partition / joins ----
def partition_ids(keys, P: int, radix: bool, hash_kind: int, seed: int) -> np.ndarray:
    L = lib()
    return np.array([L.or_partition_id(int(k), P, int(radix), hash_kind, seed) for k in keys],
                    dtype=np.uint64)


def partition(rel: np.ndarray, P: int, radix: bool, hash_kind: int, seed: int, workers: int = 4):
    rel = as_relation(rel)
    n = rel.shape[0]
    out = relation(n)
    bounds = np.zeros(P + 1, dtype=np.uint64)
    rc = lib().or_partition(_ptr(rel), n, P, int(radix), hash_kind, seed, workers, _ptr(out),
                            _ptr(bounds))
    if rc != 0:
        raise ValueError("bad partition arguments")
    return out, bounds


def join_nopart(R, S, hash_kind=HASH_XXH3, seed=0, ratio=1.25, workers=4) -> OrResult:
    R, S = as_relation(R), as_relation(S)
    res = OrResult()
    rc = lib().or_join_nopart(_ptr(R), R.shape[0], _ptr(S), S.shape[0], hash_kind, seed, ratio,
                              workers, C.byref(res))
    if rc != 0:
        raise ValueError("LinearProbingHashTable: numberOfObjects must be greater than zero.")
    return res


def join_radix(R, S, P=32, radix=False, part_hash=HASH_XXH3, part_seed=1, table_hash=HASH_XXH3,
               table_seed=2, ratio=1.25, workers=4) -> OrResult:
    R, S = as_relation(R), as_relation(S)
    res = OrResult()
    rc = lib().or_join_radix(_ptr(R), R.shape[0], _ptr(S), S.shape[0], P, int(radix), part_hash,
                             part_seed, table_hash, table_seed, ratio, workers, C.byref(res))
    if rc != 0:
        raise ValueError("bad radix join arguments")
    return res


def semijoin_count(R, S, threads=4) -> int:
    R, S = as_relation(R), as_relation(S)
    return int(lib().or_semijoin_count_sorted(_ptr(R), R.shape[0], _ptr(S), S.shape[0], threads))


def semijoin_count_keys(rkeys: np.ndarray, skeys: np.ndarray, threads=4) -> int:
    rkeys = np.ascontiguousarray(rkeys, dtype=np.int64)
    skeys = np.ascontiguousarray(skeys, dtype=np.int64)
    return int(lib().or_semijoin_count_keys(_ptr(rkeys), rkeys.shape[0], _ptr(skeys),
                                            skeys.shape[0], threads))


class LinearProbingTable:
    """HashTables::LinearProbingHashTable<Tuple,3,XXHasher> (LinearProbing.hpp:90-210)."""

    def __init__(self, n, ratio=1.25, hash_kind=HASH_XXH3, seed=0):
        self._t = lib().or_lp_new(ratio, n, hash_kind, seed)
        if not self._t:
            raise ValueError("LinearProbingHashTable::LinearProbingHashTable: numberOfObjects "
                             "must be greater than zero.")

    def __del__(self):
        if getattr(self, "_t", None):
            lib().or_lp_free(self._t)

    @property
    def num_buckets(self):
        return lib().or_lp_num_buckets(self._t)

    def insert(self, key, value: int):
        lib().or_lp_insert(self._t, key, value)

    def get(self, key):
        return lib().or_lp_get(self._t, key)

    def exists(self, key):
        return bool(lib().or_lp_exists(self._t, key))

    def get_all(self, key):
        n = lib().or_lp_get_all(self._t, key, None, 0)
        out = (_P * max(n, 1))()
        lib().or_lp_get_all(self._t, key, C.cast(out, _P), n)
        return [out[i] for i in range(n)]


class SeparateChainingTable:
    """HashTables::SeparateChainingHashTable<Tuple,3,XXHasher> (SeparateChaining.hpp:143-277)."""

    def __init__(self, n, ratio=0.25, hash_kind=HASH_XXH3, seed=0):
        self._t = lib().or_sc_new(ratio, n, hash_kind, seed)
        if not self._t:
            raise ValueError("SeparateChainingHashTable: numberOfObjects must be greater than zero.")

    def __del__(self):
        if getattr(self, "_t", None):
            lib().or_sc_free(self._t)

    def insert(self, key, value: int):
        if lib().or_sc_insert(self._t, key, value) != 0:
            raise RuntimeError("BucketAllocator exceeded its limit.")

    def get(self, key):
        return lib().or_sc_get(self._t, key)

    def exists(self, key):
        return bool(lib().or_sc_exists(self._t, key))

    def get_all(self, key):
        n = lib().or_sc_get_all(self._t, key, None, 0)
        out = (_P * max(n, 1))()
        lib().or_sc_get_all(self._t, key, C.cast(out, _P), n)
        return [out[i] for i in range(n)]


# ---- reference generator code (oracle/_ref) ----
def ref_lcg_sequence(seed: int, n: int):
    R = ref()
    if R is None:
        return None
    out = np.zeros(n, dtype=np.float64)
    assert R.ref_lcg_sequence(seed, n, _ptr(out)) == 0
    return out


def ref_zipf_samples(alpha: float, card: int, seed: int, n: int):
    R = ref()
    if R is None:
        return None
    out = np.zeros(n, dtype=np.uint64)
    assert R.ref_zipf_samples(alpha, card, seed, n, _ptr(out)) == 0
    return out


def ref_fill_zipf(alpha: float, lo: int, hi: int, seed: int, batches: int):
    R = ref()
    if R is None:
        return None
    out = relation(batches * GEN_BATCH)
    assert R.ref_fill_zipf(alpha, lo, hi, seed, batches, GEN_BATCH, _ptr(out)) == 0
    return out


def ref_fill_sequential(start: int, n: int):
    R = ref()
    if R is None:
        return None
    out = relation(n)
    assert R.ref_fill_sequential(start, n, _ptr(out)) == 0
    return out
