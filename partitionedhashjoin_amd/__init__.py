"""partitionedhashjoin_amd — MI355X-native radix-partitioned / no-partitioning hash join.

The product is the HIP library libphj_hip.so (C ABI: include/phj.h) plus the
C++ host driver `phjoin` that keeps the reference's CLI, Configuration and
Table<Tuple> API (ragoragino/partitionedhashjoin, src/main.cpp). This Python
module is plumbing over the same C ABI for tests, bench.py and the
torch.distributed multi-GPU driver. It never falls back to a CPU path:
without the built HIP library every entry point raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi
from ._capi import (ALGO_NO_PARTITIONING, ALGO_RADIX, CTX_EXCHANGE, CTX_LOCAL, HASH_MURMUR3, HASH_XXH3,
                    PATH_CODE_TABLES, PATH_LDS_JOIN, PATH_NO_PARTITIONING, PATH_PARTITIONED, SIDE_BUILD,
                    SIDE_PROBE, JoinParams, JoinResult, Partitioned, PhjError)

__all__ = ["Context", "shard_range", "exchange_layout", "join_path", "PATH_LDS_JOIN", "PATH_CODE_TABLES",
           "PATH_PARTITIONED", "PATH_NO_PARTITIONING", "count_contribution", "count_verdict", "comm_unique_id", "CTX_EXCHANGE", "CTX_LOCAL", "radix_params", "nopart_params", "JoinParams", "JoinResult",
           "Partitioned", "PhjError", "ALGO_RADIX", "ALGO_NO_PARTITIONING", "HASH_XXH3",
           "HASH_MURMUR3", "SIDE_BUILD", "SIDE_PROBE", "DEFAULT_SEED"]

DEFAULT_SEED = 0x9E3779B97F4A7C15
PART_STABLE = 0x1   # include/phj.h PHJ_PART_STABLE
TABLE_CHAINED = 0x2   # include/phj.h PHJ_TABLE_CHAINED
DEFER_TIMERS = 0x4   # include/phj.h PHJ_DEFER_TIMERS: timers read later by Context.timers_report()
LEAN_TIMERS = 0x8    # include/phj.h PHJ_LEAN_TIMERS: only the critical path's large kernels timed


def radix_params(bits=(8, 8), num_partitions=0, hash=HASH_MURMUR3, seed=DEFAULT_SEED,
                 stable=False, chained=False) -> JoinParams:
    """RadixCluster parameters. num_partitions > 0 reproduces the reference's
    `hash % P` partitioning (`phjoin -p P`); otherwise q = hash & (2^(b0+b1)-1).
    stable=True asks `partition` for the reference's exact layout (input order
    inside each partition, RadixCluster/HashJoin.hpp:394-412); otherwise the
    order inside a partition is unspecified (PHJ_PART_STABLE, include/phj.h).
    chained=True builds bucket-chained tables, the reference's
    SeparateChainingHashTable (PHJ_TABLE_CHAINED)."""
    p = JoinParams()
    p.flags = (PART_STABLE if stable else 0) | (TABLE_CHAINED if chained else 0)
    p.algo = ALGO_RADIX
    p.hash = hash
    p.hash_seed = seed
    p.num_partitions = num_partitions
    p.radix_bits[0] = bits[0]
    p.radix_bits[1] = bits[1] if len(bits) > 1 else 0
    p.table_ratio = 0.0
    return p


def nopart_params(hash=HASH_XXH3, seed=DEFAULT_SEED, table_ratio=0.0) -> JoinParams:
    p = JoinParams()
    p.algo = ALGO_NO_PARTITIONING
    p.hash = hash
    p.hash_seed = seed
    p.table_ratio = table_ratio
    return p


def shard_range(n: int, rank: int, world: int):
    """Rows [lo, hi) of an n-row relation held by `rank` of `world` ranks: the
    range sharding of every multi-device context (phj_shard_range; host only)."""
    L = _capi.load()
    lo, hi = C.c_uint64(), C.c_uint64()
    L.phj_shard_range(n, rank, world, C.byref(lo), C.byref(hi))
    return lo.value, hi.value


def exchange_layout(max_shard: int, num_partitions: int):
    """(codes_elems, block_elems) of one rank's exchange block: codes, zero
    padded, then num_partitions + 1 uint32 bounds (phj_exchange_layout; host only)."""
    L = _capi.load()
    a, b = C.c_uint64(), C.c_uint64()
    L.phj_exchange_layout(max_shard, num_partitions, C.byref(a), C.byref(b))
    return a.value, b.value


def exchange_geometry(params: JoinParams, total_build: int):
    """(num_segments, shift, sub_bits, sub_shift, cluster) of the member step's
    exchange block for radix params and a global build side of total_build rows
    (phj_exchange_geometry; host only, default tuning)."""
    L = _capi.load()
    n, sh, sb, ss, cl = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_int()
    rc = L.phj_exchange_geometry(C.byref(params), total_build, C.byref(n), C.byref(sh), C.byref(sb), C.byref(ss),
                                 C.byref(cl))
    if rc != 0:
        raise PhjError(rc, "phj_exchange_geometry: radix params required")
    return n.value, sh.value, sb.value, ss.value, bool(cl.value)


def join_path(params: JoinParams, build_n: int, probe_n: int) -> int:
    """The counting path phj_join takes on one device (phj_join_path; host
    only, default tuning): PATH_LDS_JOIN, PATH_CODE_TABLES, PATH_PARTITIONED
    or PATH_NO_PARTITIONING."""
    rc = _capi.load().phj_join_path(C.byref(params), build_n, probe_n)
    if rc < 0:
        raise PhjError(rc, "phj_join_path: bad params")
    return rc


def count_contribution(count: int, failed: bool = False) -> np.ndarray:
    """The two uint64 words a rank adds to the count all-reduce (phj_count_contribution)."""
    L = _capi.load()
    w = (C.c_uint64 * 2)()
    L.phj_count_contribution(count, 1 if failed else 0, w)
    return np.array([w[0], w[1]], dtype=np.uint64)


def count_verdict(words) -> int:
    """The global count from the all-reduced words; PhjError(PHJ_ERR_STATE) when a
    rank failed (phj_count_verdict)."""
    L = _capi.load()
    w = (C.c_uint64 * 2)(int(words[0]), int(words[1]))
    m = C.c_uint64()
    rc = L.phj_count_verdict(w, C.byref(m))
    if rc != 0:
        raise PhjError(rc, f"{int(words[1])} rank(s) failed during the join")
    return m.value


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 makes it; every rank passes it to
    Context.rank)."""
    L = _capi.load()
    buf = C.create_string_buffer(_capi.UNIQUE_ID_BYTES)
    rc = L.phj_comm_unique_id(buf)
    if rc != 0:
        raise PhjError(rc, "phj_comm_unique_id failed (RCCL unavailable?)")
    return buf.raw


class Context:
    """A phj_ctx: one HIP device (Context(device)), several devices driven by
    this process (Context(devices=[...]), the multi-GPU join; flags
    CTX_EXCHANGE / CTX_LOCAL), or one rank of a multi-process job
    (Context.rank)."""

    def __init__(self, device: int = 0, devices=None, flags: int = 0, _handle=None):
        self._L = _capi.load()
        self._keep = {}
        if _handle is not None:
            self._h = _handle
            self.device = device
            return
        h = C.c_void_p()
        if devices is None:
            rc = self._L.phj_ctx_create_device(device, C.byref(h))
            what = f"phj_ctx_create_device({device})"
        else:
            arr = (C.c_int * len(devices))(*devices)
            rc = self._L.phj_ctx_create_ex(len(devices), arr, flags, C.byref(h))
            what = f"phj_ctx_create_ex({list(devices)}, flags={flags})"
            device = devices[0]
        if rc != 0:
            raise PhjError(rc, f"{what} failed")
        self._h = h
        self.device = device

    @classmethod
    def rank(cls, device: int, nranks: int, rank: int, unique_id: bytes) -> "Context":
        """One device of a multi-process job (phj_ctx_create_rank): every call
        on it is collective over the ranks."""
        L = _capi.load()
        h = C.c_void_p()
        rc = L.phj_ctx_create_rank(device, nranks, rank, unique_id, C.byref(h))
        if rc != 0:
            raise PhjError(rc, f"phj_ctx_create_rank(device={device}, {rank}/{nranks}) failed")
        return cls(device, _handle=h)

    def info(self):
        """(world, rank of the first local device, local devices)"""
        w, r, n = C.c_int(), C.c_int(), C.c_int()
        self._check(self._L.phj_ctx_info(self._h, C.byref(w), C.byref(r), C.byref(n)))
        return w.value, r.value, n.value

    # -- lifecycle --
    def close(self):
        if getattr(self, "_h", None):
            self._L.phj_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise PhjError(rc, self._L.phj_last_error(self._h).decode())

    def set_stream(self, stream_ptr: int | None):
        self._check(self._L.phj_ctx_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        self._check(self._L.phj_ctx_synchronize(self._h))

    # -- relations --
    def upload(self, side: int, rel: np.ndarray):
        rel = np.ascontiguousarray(rel, dtype=np.int64)
        assert rel.ndim == 2 and rel.shape[1] == 2
        self._check(self._L.phj_relation_upload(self._h, side, rel.ctypes.data_as(C.c_void_p),
                                                rel.shape[0]))

    def bind_device(self, side: int, ptr: int, n: int, keepalive=None):
        self._keep[side] = keepalive
        self._check(self._L.phj_relation_bind_device(self._h, side, C.c_void_p(ptr), n))

    def relation_ptr(self, side: int):
        n = C.c_uint64()
        p = self._L.phj_relation_device_ptr(self._h, side, C.byref(n))
        return p, n.value

    def download(self, side: int, n: int | None = None) -> np.ndarray:
        if n is None:
            n = self.relation_ptr(side)[1]
        out = np.zeros((n, 2), dtype=np.int64)
        self._check(self._L.phj_relation_download(self._h, side, out.ctypes.data_as(C.c_void_p), n))
        return out

    def generate_sequential(self, side: int, n: int, start: int = 1, first_index: int = 0):
        self._check(self._L.phj_relation_generate_sequential(self._h, side, n, start, first_index))

    def generate_zipf(self, side: int, n: int, alpha: float, lo: int, hi: int, seed: int,
                      first_index: int = 0):
        self._check(self._L.phj_relation_generate_zipf(self._h, side, n, alpha, lo, hi, seed,
                                                       first_index))

    def count_in_range(self, side: int, lo: int, hi: int) -> int:
        c = C.c_uint64()
        self._check(self._L.phj_relation_count_in_range(self._h, side, lo, hi, C.byref(c)))
        return c.value

    # -- join --
    def prepare(self, params: JoinParams) -> None:
        """Allocate join's workspace for the bound relations (nothing runs)."""
        self._check(self._L.phj_prepare(self._h, C.byref(params)))

    def join(self, params: JoinParams) -> JoinResult:
        r = JoinResult()
        self._check(self._L.phj_join(self._h, C.byref(params), C.byref(r)))
        return r

    def join_materialize(self, params: JoinParams) -> JoinResult:
        """phj_join_materialize: the join's rows (JoinedTuple) in a device buffer;
        r.matches rows. Read them with joined()."""
        r = JoinResult()
        self._check(self._L.phj_join_materialize(self._h, C.byref(params), C.byref(r)))
        return r

    def joined(self, n: int | None = None) -> np.ndarray:
        """Rows of the last materialised join as an (n, 3) int64 array
        {id, payloadA (build), payloadB (probe)}."""
        total = C.c_uint64(0)
        self._L.phj_joined_rows(self._h, C.byref(total))
        n = total.value if n is None else n
        out = np.zeros((n, 3), dtype=np.int64)
        self._check(self._L.phj_joined_download(self._h, out.ctypes.data_as(C.c_void_p), n))
        return out

    def partition(self, side: int, params: JoinParams) -> Partitioned:
        v = Partitioned()
        self._check(self._L.phj_partition(self._h, side, C.byref(params), C.byref(v)))
        return v

    def join_partitioned(self, params: JoinParams, segments) -> JoinResult:
        arr = (Partitioned * len(segments))(*segments)
        r = JoinResult()
        self._check(self._L.phj_join_partitioned(self._h, C.byref(params), len(segments), arr,
                                                 C.byref(r)))
        return r

    def join_partitioned_async(self, params: JoinParams, segments, dev_count: int) -> None:
        """Enqueue build + probe; the count lands at device address dev_count (uint64)."""
        arr = (Partitioned * len(segments))(*segments)
        self._check(self._L.phj_join_partitioned_async(self._h, C.byref(params), len(segments), arr,
                                                       C.c_void_p(dev_count)))

    def timers_report(self) -> JoinResult:
        r = JoinResult()
        self._check(self._L.phj_timers_report(self._h, C.byref(r)))
        return r

    def download_partitioned(self, v: Partitioned):
        keys = np.zeros(v.n, dtype=np.int64)
        pays = np.zeros(v.n, dtype=np.int64)
        bounds = np.zeros(v.num_partitions + 1, dtype=np.uint32)
        self._check(self._L.phj_partitioned_download(
            self._h, C.byref(v), keys.ctypes.data_as(C.c_void_p), pays.ctypes.data_as(C.c_void_p),
            bounds.ctypes.data_as(C.c_void_p)))
        return keys, pays, bounds

    def probe_pass1(self, params: JoinParams):
        """Test hook (phj_probe_pass1): the probe side's pass-1 output as the
        counting join's on-chip probe consumes it, pass-1 digit major.
        Returns (keys or hash codes, bounds1 (nb1 + 1), is_codes)."""
        n = self.relation_ptr(SIDE_PROBE)[1]
        out = np.zeros(n, dtype=np.int64)
        b1 = np.zeros(2049, dtype=np.uint32)
        nb1, codes = C.c_uint32(), C.c_int()
        self._check(self._L.phj_probe_pass1(self._h, C.byref(params), out.ctypes.data_as(C.c_void_p), n,
                                            b1.ctypes.data_as(C.c_void_p), C.byref(nb1), C.byref(codes)))
        return out, b1[:nb1.value + 1].copy(), bool(codes.value)

    def debug_poison_chunk_table(self, side: int, params: JoinParams, byte: int = 0xFF) -> None:
        """Test hook (phj_debug_poison_chunk_table): leave `side`'s chunk table
        as a stale one would be (every byte = `byte`, marked clean)."""
        self._check(self._L.phj_debug_poison_chunk_table(self._h, side, C.byref(params), byte))

    def debug_poison_alloc(self, byte: int = 0xFF) -> None:
        """Test hook (phj_debug_poison_alloc): every workspace buffer this
        context (and each of its members) allocates from now on is filled with
        `byte` (-1: off), so a read of a word nothing wrote shows."""
        self._check(self._L.phj_debug_poison_alloc(self._h, byte))

    def debug_fail_member(self, member: int) -> None:
        """Test hook (phj_debug_fail_member): local member `member` fails the
        next join before the exchange (-1: none)."""
        self._check(self._L.phj_debug_fail_member(self._h, member))

    def debug_exchange_block(self, member: int, elems: int) -> np.ndarray:
        """Test hook (phj_debug_exchange_block): local member `member`'s packed
        exchange block of the last radix join (`elems` int64)."""
        out = np.zeros(elems, dtype=np.int64)
        self._check(self._L.phj_debug_exchange_block(self._h, member, out.ctypes.data_as(C.c_void_p), elems))
        return out

    def hash_keys(self, kind: int, seed: int, keys) -> np.ndarray:
        keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
        out = np.zeros(keys.shape[0], dtype=np.uint64)
        self._check(self._L.phj_hash_keys(self._h, kind, seed, keys.ctypes.data_as(C.c_void_p),
                                          keys.shape[0], out.ctypes.data_as(C.c_void_p)))
        return out
