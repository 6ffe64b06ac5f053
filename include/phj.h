/*
 * phj.h — C ABI of the MI355X-native partitioned hash join (libphj_hip.so).
 *
 * This is the drop-in boundary under the reference's join API. The reference
 * (ragoragino/partitionedhashjoin, C++17, CPU only) exposes
 *
 *   RadixClustering::HashJoiner<HashTableFactory, HasherType>::Run(
 *       shared_ptr<Table<Tuple>> tableA /+build+/, shared_ptr<Table<Tuple>> tableB /+probe+/,
 *       shared_ptr<IHashJoinTimer> timer)                 src/RadixCluster/HashJoin.hpp:100-104
 *   NoPartitioning::HashJoiner<HashTableFactory>::Run(...) src/NoPartitioning/HashJoin.hpp:23-27
 *
 * and reads the relations through Table<Tuple>::operator[] / GetSize()
 * (src/Common/Table.hpp:42-46). Those entry points are kept in C++ by the
 * host driver (partitionedhashjoin_amd/host/Gpu/HashJoin.hpp); underneath, they call
 * only the functions below: plain pointers and sizes, no exceptions, no
 * torch types. Conventions: 0 = PHJ_OK, negative = error (message via
 * phj_last_error). A context owns every device buffer it allocates (grow
 * only, allocated outside the timed phases) and is not thread-safe. It spans
 * one device (one stream) or several (SURVEY.md §8(b),(e)): the relations
 * are range-sharded across the devices, phj_join runs the multi-GPU join
 * (partition the shards, RCCL all-gather of the partitioned build keys over
 * xGMI, local build + probe, all-reduce of the count) and one worker thread
 * per local device issues its work, as the reference's thread pool carries
 * its parallelism (src/main.cpp:235-241).
 */
#ifndef PHJ_H
#define PHJ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PHJ_ABI_VERSION 2

/* Common::Tuple (src/Common/Table.hpp:20-25): alignas(16) {int64 id; int64 payload}. */
typedef struct phj_tuple {
    int64_t id;
    int64_t payload;
} phj_tuple;

typedef struct phj_ctx phj_ctx;

/* status codes */
#define PHJ_OK 0
#define PHJ_ERR_INVALID -1 /* bad argument (reference: std::invalid_argument) */
#define PHJ_ERR_NOMEM -2   /* device allocation failed */
#define PHJ_ERR_HIP -3     /* HIP runtime / kernel launch error */
#define PHJ_ERR_STATE -4   /* call order (e.g. join before relations are bound) */
#define PHJ_ERR_RANGE -5   /* size beyond a documented limit */

/* Common::JoinAlgorithmType values (src/Common/Configuration.hpp:12-15). */
#define PHJ_ALGO_NO_PARTITIONING 0
#define PHJ_ALGO_RADIX 1

/* hash functions: XXH3_64bits_withSeed over the 8-byte key (XXHasher.hpp:19-22)
 * and the Murmur3 fmix64 finalizer over key ^ seed (BASELINE config C2). */
#define PHJ_HASH_XXH3 0
#define PHJ_HASH_MURMUR3 1

/* relation sides: tableA = build (R), tableB = probe (S) (HashJoin.hpp:99) */
#define PHJ_SIDE_BUILD 0
#define PHJ_SIDE_PROBE 1

typedef struct phj_join_params {
    int32_t algo;            /* PHJ_ALGO_* */
    int32_t hash;            /* PHJ_HASH_* */
    uint64_t hash_seed;      /* XXHasher seed (random in the reference, explicit here) */
    /* Radix partition id q(key):
     *   num_partitions > 0 : q = hash % num_partitions  (reference `-p P`, HashJoin.hpp:349-351)
     *   num_partitions == 0: q = hash & (2^(b0+b1) - 1) (power-of-two radix, radix_bits = {b0, b1})
     * Partitioning takes one pass when q has <= 11 bits and two otherwise
     * (pass digits: high bits first). Maximum 22 bits (4,194,304 partitions). */
    uint32_t num_partitions;
    uint8_t radix_bits[2];
    uint8_t flags;           /* PHJ_PART_* */
    uint8_t reserved;
    /* NoPartitioning: hash-table slots per build tuple (>= 1). 0 selects the default. */
    double table_ratio;
} phj_join_params;

/* flags: PHJ_PART_STABLE asks phj_partition for the reference's exact layout
 * (a STABLE partition: partition-major, then input order, as partitionTable
 * writes it, RadixCluster/HashJoin.hpp:394-412). Without it a 2-pass
 * partition may order the tuples inside each partition arbitrarily (the
 * first pass then needs no histogram pass over the relation); partition
 * contents, bounds and every join count are identical either way. */
#define PHJ_PART_STABLE 0x1
/* flags: PHJ_TABLE_CHAINED (radix join) builds every partition's table as the
 * reference's SeparateChainingHashTable does (SeparateChaining.hpp:143-277:
 * buckets of slots, overflow chained on), in compacted form: per partition a
 * bucket-chained table in HBM whose buckets are contiguous runs (CSR offsets,
 * phj_join.h k_build_small / k_build_big), probed by k_probe. Without it the
 * counting join uses the open-addressed code tables of LinearProbing
 * semantics (phj_table.h). Counts are identical either way; the host driver's
 * SeparateChainingFactory sets it. Ignored by NoPartitioning. */
#define PHJ_TABLE_CHAINED 0x2
/* flags: PHJ_DEFER_TIMERS (one device) leaves this join's timers in the
 * context instead of reading them into the result: no event queries and no
 * extra synchronisation after the count is read back. Timers accumulate over
 * such joins; phj_timers_report returns their sums (the LDS join's build /
 * probe split then uses the last join's clocks) and resets them. Result
 * fields partition_ms .. total_ms and the timer list stay zero. A benchmark
 * loop sets it to keep the readout off its timed steps (bench.py). */
#define PHJ_DEFER_TIMERS 0x4
/* flags: PHJ_LEAN_TIMERS records only the timers of the large kernels (the
 * probe side's pass 1, the LDS join's build and probe, the exchange): every
 * event recorded between two kernels delays the second by ~4 us. The build
 * side's pass-1 timers are not recorded, the big clusters' tables
 * (`build.big`) are listed at zero. */
#define PHJ_LEAN_TIMERS 0x8
#define PHJ_MAX_TIMERS 32
#define PHJ_TIMER_NAME 24

typedef struct phj_join_result {
    uint64_t matches;            /* #probe tuples with >= 1 equal build key (semi-join count:
                                    the "Joined N tuples" of RadixCluster/HashJoin.hpp:320-321) */
    double partition_ms;         /* reference phase keys (Results.hpp:274-276), device time */
    double build_ms;
    double probe_ms;             /* probe alone (the reference's NoPartitioning probe also
                                    counts its build, Results.hpp:202; see phj host driver) */
    double total_ms;             /* first kernel start .. count on host */
    double exchange_ms;          /* multi-device: the build-side exchange (RCCL all-gather), 0 on one device */
    uint64_t algorithmic_bytes;  /* HBM bytes the algorithm must move */
    uint32_t num_partitions;     /* final partition count (radix) */
    uint32_t num_timers;
    double timer_ms[PHJ_MAX_TIMERS];        /* per-kernel device time (hipEvents on the ctx stream),
                                               summed over the records of that name */
    uint64_t timer_bytes[PHJ_MAX_TIMERS];   /* algorithmic bytes of those launches (summed) */
    char timer_name[PHJ_MAX_TIMERS][PHJ_TIMER_NAME];
} phj_join_result;

/* A partitioned relation on the device: SoA key/payload columns in partition
 * order, bounds[num_partitions + 1] offsets (uint32). Views are owned by the
 * ctx that produced them (valid until the next partition call on that side)
 * or by the caller (gathered shards on multi-GPU). */
typedef struct phj_partitioned {
    const int64_t *keys;
    const int64_t *payloads;
    const uint32_t *bounds;
    uint64_t n;
    uint32_t num_partitions;
    uint32_t reserved;
} phj_partitioned;

/* ---- context ---- */
/* One context over `ngpus` HIP devices (devs[i] = device of rank i; NULL means
 * 0 .. ngpus-1), SURVEY.md §8(b). ngpus == 1 gives a single-device context.
 * With ngpus > 1 every relation call takes the whole relation and range-shards
 * it (rank r holds rows [r*n/ngpus, (r+1)*n/ngpus)), and phj_join / phj_prepare
 * run the multi-GPU join with RCCL collectives (at most 16 ranks). This is the
 * reference's Run() with its thread pool (src/main.cpp:235-241, dispatch
 * :260-276) replaced by devices. */
int phj_ctx_create(int ngpus, const int *devs, phj_ctx **out);
/* flags for phj_ctx_create_ex */
#define PHJ_CTX_EXCHANGE 0x1 /* take the multi-GPU path even on one device (an RCCL world of one) */
#define PHJ_CTX_LOCAL 0x2    /* exchange by device copies between this process's members instead of
                                RCCL; devices may repeat (rehearses N ranks on one GPU) */
int phj_ctx_create_ex(int ngpus, const int *devs, uint32_t flags, phj_ctx **out);
/* A single-device context (ABI v1's phj_ctx_create(device)). */
int phj_ctx_create_device(int device, phj_ctx **out);
/* One device of a multi-process job (one process per GPU, e.g. torchrun):
 * rank 0 makes an id with phj_comm_unique_id and hands it to every rank (any
 * channel); each rank creates its context with it. On such a context every
 * call is collective (all ranks make the same calls in the same order), the
 * relation calls take this rank's shard (generators: rows [first_index,
 * first_index + n) of the global relation), and phj_join returns the global
 * count. */
#define PHJ_UNIQUE_ID_BYTES 128
int phj_comm_unique_id(uint8_t *id /* [PHJ_UNIQUE_ID_BYTES] */);
int phj_ctx_create_rank(int device, int nranks, int rank, const uint8_t *id, phj_ctx **out);
/* ranks of the job, global rank of this context's first device, devices in this context */
int phj_ctx_info(const phj_ctx *ctx, int *world, int *rank0, int *nlocal);
/* Host-only: rows [lo, hi) of an n-row relation held by `rank` of `world` ranks
 * (the range sharding of every multi-device context). */
void phj_shard_range(uint64_t n, int rank, int world, uint64_t *lo, uint64_t *hi);
/* ---- the multi-GPU exchange protocol (host-only; csrc/phj_group.h) ----
 * Replaces nothing in the reference (its parallel split is a thread pool,
 * src/main.cpp:235-241). These ARE the rules phj_join's member step applies,
 * exported so that a caller driving its own transport, and the CPU tests over
 * gloo, follow the same layout and reduction:
 *  - the exchange block of one rank (the all-gathered unit, int64 elements):
 *    its build codes in final partition order, zero padded to *codes_elems
 *    (a multiple of 64, >= the largest rank's shard), then the partition bounds
 *    (num_partitions + 1 uint32, two per element), *block_elems in all; a rank
 *    that failed before the all-gather still takes part with an all-zero
 *    block (bounds all 0: an empty build segment);
 *  - the count all-reduce (sum, uint64): every rank contributes the two words
 *    of phj_count_contribution; phj_count_verdict turns the sum into the global
 *    count, or PHJ_ERR_STATE when any rank failed. */
void phj_exchange_layout(uint64_t max_shard, uint32_t num_partitions, uint64_t *codes_elems,
                         uint64_t *block_elems);
/* The counting path phj_join takes on one device for params p over a build
 * side of build_n and a probe side of probe_n rows (default tuning; host
 * only, no device touched): PHJ_PATH_LDS_JOIN (the clusters' tables built in
 * LDS, phj_cluster.h), PHJ_PATH_CODE_TABLES (code tables in HBM, the probe
 * side's pass 2 on chip), PHJ_PATH_PARTITIONED (both sides fully partitioned,
 * fused or HBM-table join), PHJ_PATH_NO_PARTITIONING; negative: an error code.
 * The LDS join needs the probe side's keys-only chunked pass 1, whose chunk
 * pools address slots with 32 bits: above that bound it is declined. Replaces
 * the choice main() makes between the reference's joins (src/main.cpp:260-276),
 * refined inside RadixCluster by size. */
#define PHJ_PATH_NO_PARTITIONING 0
#define PHJ_PATH_LDS_JOIN 1
#define PHJ_PATH_CODE_TABLES 2
#define PHJ_PATH_PARTITIONED 3
int phj_join_path(const phj_join_params *p, uint64_t build_n, uint64_t probe_n);

/* The segment geometry phj_join's member step uses for radix params p and a
 * global build side of total_build rows (default tuning): the block's codes
 * are grouped by d(c) = (q(c) >> *shift), q = the plan's (sub-)partition
 * number of code c (q = c & (P - 1) for radix bits; (c % P) << s | bits
 * 40.. for h % P, s = *sub_bits; radix bits below the cluster width take
 * *sub_bits hash bits just above them), with *num_segments + 1 bounds.
 * *cluster = 1: the LDS join's clusters (phj_cluster.h), else the final
 * partitions of the code tables. PHJ_ERR_INVALID for bad params. */
int phj_exchange_geometry(const phj_join_params *p, uint64_t total_build, uint32_t *num_segments,
                          uint32_t *shift, uint32_t *sub_bits, uint32_t *sub_shift, int *cluster);
void phj_count_contribution(uint64_t count, int failed, uint64_t words[2]);
int phj_count_verdict(const uint64_t words[2], uint64_t *matches);
void phj_ctx_destroy(phj_ctx *ctx);
const char *phj_last_error(const phj_ctx *ctx);
/* Run on an external stream (e.g. torch.cuda.current_stream()); NULL = ctx-owned stream.
 * Multi-device contexts: only with one local device. The building blocks below
 * (phj_partition ... phj_hash_keys) likewise act on the single local device of a
 * rank context and return PHJ_ERR_STATE on a context with several local devices;
 * phj_join_materialize is single-device only. */
int phj_ctx_set_stream(phj_ctx *ctx, void *hip_stream);
int phj_ctx_synchronize(phj_ctx *ctx);
int phj_abi_version(void);

/* ---- relations (Table<Tuple>: &(*table)[0], GetSize(), Table.hpp:42-46) ---- */
/* Copy a host relation to ctx-owned device memory (H2D, synchronous). */
int phj_relation_upload(phj_ctx *ctx, int side, const phj_tuple *host, uint64_t n);
/* Borrow a device relation (caller keeps it alive while the ctx uses it). */
int phj_relation_bind_device(phj_ctx *ctx, int side, const phj_tuple *dev, uint64_t n);
/* Device pointer of the bound relation (NULL if none; NULL with *n = the rows
 * of all local devices on a context with several). */
const phj_tuple *phj_relation_device_ptr(phj_ctx *ctx, int side, uint64_t *n);
/* Copy the bound relation back to host (n tuples). */
int phj_relation_download(phj_ctx *ctx, int side, phj_tuple *host, uint64_t n);
/* On-device generators: Sequential::FillTable (Sequential.cpp:6-40)
 * and Zipf::FillTable (Zipf.cpp:58-108) over [lo, hi] with LCG streams seeded
 * per 4096-tuple batch. Rows [first_index, first_index + n) of the full
 * relation are generated (a range shard on multi-GPU; 0 = the whole table),
 * so shards concatenate to exactly the single-device relation. The Zipf
 * kernel draws with phj_pow.h, a restatement of glibc's pow (the one the
 * reference's std::pow calls) evaluated in glibc's FMA-build operation order,
 * so its samples equal the host generator's and the reference's bit for bit
 * (tests/test_gpu_generators.py). */
int phj_relation_generate_sequential(phj_ctx *ctx, int side, uint64_t n, int64_t start,
                                     uint64_t first_index);
int phj_relation_generate_zipf(phj_ctx *ctx, int side, uint64_t n, double alpha, int64_t lo,
                               int64_t hi, uint64_t seed, uint64_t first_index);
/* Count tuples of the bound relation with lo <= id <= hi (device reduction). */
int phj_relation_count_in_range(phj_ctx *ctx, int side, int64_t lo, int64_t hi, uint64_t *count);

/* ---- the join (HashJoiner::Run) ---- */
/* Synchronous: partition (radix) / build / probe on the device, count back on the host. */
int phj_join(phj_ctx *ctx, const phj_join_params *p, phj_join_result *r);

/* Allocate (grow-only) every workspace buffer phj_join with these params needs
 * for the relations currently bound, launching nothing: the reference keeps
 * its allocations outside the timed phases (RadixCluster/HashJoin.hpp:195-198),
 * and a first phj_join after phj_prepare allocates nothing. Optional. */
int phj_prepare(phj_ctx *ctx, const phj_join_params *p);

/* ---- materialised join ---- */
/* Common::JoinedTuple (src/Common/Table.hpp:27-33): {id, payloadA, payloadB}, 24 B. */
typedef struct phj_joined {
    int64_t id;
    int64_t payload_a; /* build (tableA) payload of the first match: HashTable::Get (LinearProbing.hpp:160-180) */
    int64_t payload_b; /* probe (tableB) payload */
} phj_joined;
/* The join of phj_join (same params, same count), materialised: one row per
 * probe tuple with a match, into a ctx-owned device buffer. This is the
 * Table<JoinedTuple> the reference's Run() declares but returns empty
 * (NoPartitioning/HashJoin.hpp:186, RadixCluster/HashJoin.hpp:240). Rows are
 * in the probe side's storage order (input order for NoPartitioning,
 * partition order for the radix join). The radix form needs one build
 * segment. Synchronous; r->matches = number of rows. */
int phj_join_materialize(phj_ctx *ctx, const phj_join_params *p, phj_join_result *r);
/* The rows of the last phj_join_materialize: device pointer (ctx-owned, valid
 * until the next materialised join) and count. */
const phj_joined *phj_joined_rows(phj_ctx *ctx, uint64_t *n);
/* Copy the first n rows of the last phj_join_materialize to host memory. */
int phj_joined_download(phj_ctx *ctx, phj_joined *host, uint64_t n);

/* ---- building blocks (multi-GPU: range-sharded relations, RCCL exchange) ---- */
/* Radix-partition the bound relation of `side`; fills `out` with ctx-owned views.
 * Asynchronous on the ctx stream (order later work on the same stream). */
int phj_partition(phj_ctx *ctx, int side, const phj_join_params *p, phj_partitioned *out);
/* Build bucket-chained tables over the union of `nbuild` partitioned build
 * segments (e.g. every rank's shard after an all-gather) and probe the ctx's
 * partitioned probe relation. Build segments may omit payloads (NULL in every
 * segment): the join only tests key equality, as the reference's Join() only
 * tests Get() for null (RadixCluster/HashJoin.hpp:295-301). Probe the ctx's
 * partitioned probe relation (phj_partition(PHJ_SIDE_PROBE) with the same
 * params must precede). Synchronous; fills r (build_ms, probe_ms, matches). */
int phj_join_partitioned(phj_ctx *ctx, const phj_join_params *p, int nbuild,
                         const phj_partitioned *build, phj_join_result *r);
/* Asynchronous form of phj_join_partitioned for stream-ordered pipelines
 * (multi-GPU: the count feeds an RCCL all-reduce on the same stream): enqueues
 * build and probe on the ctx stream and stores the count (uint64) at
 * `dev_count`, a device address; no host synchronization. The phase timers
 * are read later with phj_timers_report. */
int phj_join_partitioned_async(phj_ctx *ctx, const phj_join_params *p, int nbuild,
                               const phj_partitioned *build, uint64_t *dev_count);
/* Per-kernel device timers recorded since the last report (e.g. after
 * phj_partition / phj_join_partitioned_async calls, possibly several joins),
 * summed by timer name; synchronizes the ctx stream, then resets. */
int phj_timers_report(phj_ctx *ctx, phj_join_result *r);
/* Copy a partitioned view (keys, payloads: n; bounds: P+1) to host or device
 * buffers (any may be NULL). Synchronous when any destination is host memory;
 * with device destinations only, the copies are enqueued on the ctx stream
 * and the call returns at once. */
int phj_partitioned_download(phj_ctx *ctx, const phj_partitioned *v, int64_t *keys,
                             int64_t *payloads, uint32_t *bounds);

/* ---- hashing on the device (tests / host parity) ---- */
/* out[i] = hash(keys[i]) for n host keys, evaluated by the device kernel. */
int phj_hash_keys(phj_ctx *ctx, int hash, uint64_t seed, const int64_t *keys, uint64_t n,
                  uint64_t *out);

/* ---- test hook: the probe side's pass 1 of the counting join ----
 * Replaces nothing in the reference: it exposes the intermediate that
 * phj_join's on-chip probe consumes instead of the reference's partitioned
 * probe table (src/RadixCluster/HashJoin.hpp:394-412, first of two passes),
 * so tests can compare it with the oracle at full size. Runs the probe side's
 * pass 1 for params (single-device ctx, radix join taking the on-chip path)
 * and copies its output, concatenated in pass-2 tile order (pass-1 digit
 * major, unordered inside a digit), to keys[0, n) (n = |S|), and the digit
 * bounds to bounds1[0, nb1 + 1). *nb1 = pass-1 digits; *codes = 1 when the
 * output holds hash codes h(key) (the keys-only pass), 0 for keys. bounds1
 * must hold at least 2049 entries. */
int phj_probe_pass1(phj_ctx *ctx, const phj_join_params *p, int64_t *keys, uint64_t n, uint32_t *bounds1,
                    uint32_t *nb1, int *codes);

/* ---- test hook: a stale chunk table ----
 * Replaces nothing in the reference. Fills the chunk table of `side`'s chunked
 * pass 1 (the one the last chunked pass on that side used; if there is none
 * yet, the one phj_join with params p would use) with `byte` and marks it
 * clean, as a table left stale by an earlier pass would be. The chunked passes bound-check every
 * chunk id and chain index they read back, so the next join returns
 * PHJ_ERR_STATE (nothing is written through a stale entry) and clears the
 * table; the join after it is exact again. Single-device ctx. */
int phj_debug_poison_chunk_table(phj_ctx *ctx, int side, const phj_join_params *p, int byte);

/* ---- test hook: poisoned workspace ----
 * Replaces nothing in the reference. From now on every device buffer the
 * context (each member of a multi-device or rank context) allocates for its
 * workspace is filled with `byte` (-1: off) before first use, as memory an
 * earlier context freed may come back. No join may read a word it did not
 * write first: the chunk tables, cursors, count pairs and exchange blocks are
 * cleared or written by the library itself, so every count stays exact. */
int phj_debug_poison_alloc(phj_ctx *ctx, int byte);

/* ---- test hook: a failing rank ----
 * Replaces nothing in the reference. On a multi-device or rank context, local
 * member `member` (-1: none) fails the next phj_join before the exchange. The
 * protocol must still end cleanly: with the local exchange every member returns
 * PHJ_ERR_STATE; over RCCL the failed rank sends a zeroed (valid, empty) block
 * into the all-gather and {0, 1} into the count all-reduce, so every rank
 * returns PHJ_ERR_STATE ("1 rank(s) failed") with no collective left waiting. */
int phj_debug_fail_member(phj_ctx *ctx, int member);

/* ---- test hook: the exchange block a member packed ----
 * Replaces nothing in the reference. Copies local member `member`'s exchange
 * block of the last radix phj_join (phj_exchange_layout's layout, `elems`
 * int64) to host memory, so tests can compare the library's own pack with the
 * protocol's definition. */
int phj_debug_exchange_block(phj_ctx *ctx, int member, int64_t *out, uint64_t elems);

#ifdef __cplusplus
}
#endif

#endif /* PHJ_H */
