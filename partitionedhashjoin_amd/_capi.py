"""ctypes binding of include/phj.h (libphj_hip.so, built in-tree).

Plumbing for tests and bench.py: the product's host driver is C++
(partitionedhashjoin_amd/host, the `phjoin` CLI). This module fails loudly
when the HIP library is missing — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PHJ_LIB") or os.path.join(HERE, "libphj_hip.so")   # PHJ_LIB: an A/B build of the same sources

PHJ_OK = 0
PHJ_ERR_INVALID = -1
PHJ_ERR_NOMEM = -2
PHJ_ERR_HIP = -3
PHJ_ERR_STATE = -4
PHJ_ERR_RANGE = -5

ALGO_NO_PARTITIONING = 0
ALGO_RADIX = 1
HASH_XXH3 = 0
HASH_MURMUR3 = 1
SIDE_BUILD = 0
SIDE_PROBE = 1
MAX_TIMERS = 32
TIMER_NAME = 24

# Every symbol include/phj.h declares (tests check the .so exports them all).
EXPORTED = [
    "phj_abi_version", "phj_ctx_create", "phj_ctx_destroy", "phj_last_error",
    "phj_ctx_set_stream", "phj_ctx_synchronize", "phj_relation_upload",
    "phj_relation_bind_device", "phj_relation_device_ptr", "phj_relation_download",
    "phj_relation_generate_sequential", "phj_relation_generate_zipf",
    "phj_relation_count_in_range", "phj_join", "phj_partition", "phj_join_partitioned",
    "phj_partitioned_download", "phj_hash_keys", "phj_timers_report", "phj_join_partitioned_async",
    "phj_prepare", "phj_join_materialize", "phj_joined_rows", "phj_joined_download",
    "phj_ctx_create_ex", "phj_ctx_create_device", "phj_comm_unique_id", "phj_ctx_create_rank",
    "phj_ctx_info", "phj_shard_range", "phj_probe_pass1", "phj_debug_poison_chunk_table", "phj_debug_poison_alloc", "phj_debug_fail_member", "phj_debug_exchange_block", "phj_exchange_geometry",
    "phj_exchange_layout", "phj_count_contribution", "phj_count_verdict", "phj_join_path",
]
ABI_VERSION = 2
CTX_EXCHANGE = 0x1   # phj_ctx_create_ex: the multi-GPU path on one device (RCCL world of one)
CTX_LOCAL = 0x2      # ... exchange by device copies; devices may repeat (rehearsal on one GPU)
UNIQUE_ID_BYTES = 128
PATH_NO_PARTITIONING, PATH_LDS_JOIN, PATH_CODE_TABLES, PATH_PARTITIONED = 0, 1, 2, 3   # phj_join_path


class Tuple(C.Structure):
    """phj_tuple == Common::Tuple (src/Common/Table.hpp:20-25)."""
    _fields_ = [("id", C.c_int64), ("payload", C.c_int64)]


class JoinParams(C.Structure):
    _fields_ = [("algo", C.c_int32), ("hash", C.c_int32), ("hash_seed", C.c_uint64),
                ("num_partitions", C.c_uint32), ("radix_bits", C.c_uint8 * 2),
                ("flags", C.c_uint8), ("reserved", C.c_uint8),
                ("table_ratio", C.c_double)]


class JoinResult(C.Structure):
    _fields_ = [("matches", C.c_uint64), ("partition_ms", C.c_double), ("build_ms", C.c_double),
                ("probe_ms", C.c_double), ("total_ms", C.c_double), ("exchange_ms", C.c_double),
                ("algorithmic_bytes", C.c_uint64), ("num_partitions", C.c_uint32),
                ("num_timers", C.c_uint32), ("timer_ms", C.c_double * MAX_TIMERS),
                ("timer_bytes", C.c_uint64 * MAX_TIMERS),
                ("timer_name", (C.c_char * TIMER_NAME) * MAX_TIMERS)]

    def timers(self):
        return [(self.timer_name[i].value.decode(), self.timer_ms[i], self.timer_bytes[i])
                for i in range(self.num_timers)]

    def as_dict(self):
        return {"matches": self.matches, "partition_ms": self.partition_ms,
                "build_ms": self.build_ms, "probe_ms": self.probe_ms, "total_ms": self.total_ms,
                "exchange_ms": self.exchange_ms,
                "algorithmic_bytes": self.algorithmic_bytes,
                "num_partitions": self.num_partitions, "timers": self.timers()}


class Partitioned(C.Structure):
    _fields_ = [("keys", C.c_void_p), ("payloads", C.c_void_p), ("bounds", C.c_void_p),
                ("n", C.c_uint64), ("num_partitions", C.c_uint32), ("reserved", C.c_uint32)]


_lib = None


class PhjError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"phj error {code}: {msg}")
        self.code = code


def load():
    """Load libphj_hip.so; raise if it was not built (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `make` or __graft_entry__.build() first "
                          "(the HIP extension is required; there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    u64, i64, i, d = C.c_uint64, C.c_int64, C.c_int, C.c_double
    sig = {
        "phj_abi_version": (i, []),
        "phj_ctx_create": (i, [i, C.POINTER(i), C.POINTER(P)]),
        "phj_ctx_create_ex": (i, [i, C.POINTER(i), C.c_uint32, C.POINTER(P)]),
        "phj_ctx_create_device": (i, [i, C.POINTER(P)]),
        "phj_comm_unique_id": (i, [C.c_char_p]),
        "phj_ctx_create_rank": (i, [i, i, i, C.c_char_p, C.POINTER(P)]),
        "phj_ctx_info": (i, [P, C.POINTER(i), C.POINTER(i), C.POINTER(i)]),
        "phj_shard_range": (None, [u64, i, i, C.POINTER(u64), C.POINTER(u64)]),
        "phj_exchange_layout": (None, [u64, C.c_uint32, C.POINTER(u64), C.POINTER(u64)]),
        "phj_count_contribution": (None, [u64, i, C.POINTER(u64)]),
        "phj_count_verdict": (i, [C.POINTER(u64), C.POINTER(u64)]),
        "phj_join_path": (i, [C.POINTER(JoinParams), u64, u64]),
        "phj_ctx_destroy": (None, [P]),
        "phj_last_error": (C.c_char_p, [P]),
        "phj_ctx_set_stream": (i, [P, P]),
        "phj_ctx_synchronize": (i, [P]),
        "phj_relation_upload": (i, [P, i, P, u64]),
        "phj_relation_bind_device": (i, [P, i, P, u64]),
        "phj_relation_device_ptr": (P, [P, i, C.POINTER(u64)]),
        "phj_relation_download": (i, [P, i, P, u64]),
        "phj_relation_generate_sequential": (i, [P, i, u64, i64, u64]),
        "phj_relation_generate_zipf": (i, [P, i, u64, d, i64, i64, u64, u64]),
        "phj_relation_count_in_range": (i, [P, i, i64, i64, C.POINTER(u64)]),
        "phj_join": (i, [P, C.POINTER(JoinParams), C.POINTER(JoinResult)]),
        "phj_partition": (i, [P, i, C.POINTER(JoinParams), C.POINTER(Partitioned)]),
        "phj_join_partitioned": (i, [P, C.POINTER(JoinParams), i, C.POINTER(Partitioned),
                                     C.POINTER(JoinResult)]),
        "phj_partitioned_download": (i, [P, C.POINTER(Partitioned), P, P, P]),
        "phj_hash_keys": (i, [P, i, u64, P, u64, P]),
        "phj_probe_pass1": (i, [P, P, P, u64, P, P, P]),
        "phj_debug_poison_chunk_table": (i, [P, i, P, i]),
        "phj_debug_poison_alloc": (i, [P, i]),
        "phj_debug_fail_member": (i, [P, i]),
        "phj_debug_exchange_block": (i, [P, i, P, u64]),
        "phj_exchange_geometry": (i, [P, u64, P, P, P, P, P]),
        "phj_timers_report": (i, [P, C.POINTER(JoinResult)]),
        "phj_join_partitioned_async": (i, [P, C.POINTER(JoinParams), i, C.POINTER(Partitioned), P]),
        "phj_prepare": (i, [P, C.POINTER(JoinParams)]),
        "phj_join_materialize": (i, [P, C.POINTER(JoinParams), C.POINTER(JoinResult)]),
        "phj_joined_rows": (P, [P, C.POINTER(u64)]),
        "phj_joined_download": (i, [P, P, u64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L
