/*
 * phj_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the hot path of ragoragino/partitionedhashjoin
 * (reference mounted read-only at /root/reference). It is the parity checker
 * for the MI355X product in partitionedhashjoin_amd/: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * Nothing in the product links, imports or calls this code.
 *
 * Parity pinning:
 *   - XXH3_64bits_withSeed (8-byte input): pinned against python `xxhash`
 *     3.8.1 (libxxhash 0.8.2) golden vectors in tests/golden/.
 *   - LCG + Zipf + Sequential generators: pinned against the reference's own
 *     src/Common/Random.cpp, src/DataGenerator/{Zipf,Sequential}.cpp compiled
 *     unmodified into oracle/_ref (oracle/ref/Makefile), golden vectors in
 *     tests/golden/.
 *   - Hash tables / joins: the reference's join path cannot be compiled here
 *     (needs Boost and an xxh3.h header the image lacks); the restatement is
 *     pinned by the reference's own unit-test assertions
 *     (tests/NoPartitioningHashJoin/HashTableTest.hpp) re-expressed in
 *     tests/test_oracle.py, and by an independent sort/binary-search count.
 */
#ifndef PHJ_ORACLE_H
#define PHJ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Common::Tuple (src/Common/Table.hpp:20-25): {int64 id; int64 payload}, 16 B. */
typedef struct or_tuple {
    int64_t id;
    int64_t payload;
} or_tuple;

enum { OR_HASH_XXH3 = 0, OR_HASH_MURMUR3 = 1 };

/* ---- hashing (src/Common/XXHasher.hpp:19-22) ---- */
uint64_t or_xxh3_64(int64_t key, uint64_t seed);
uint64_t or_murmur3(int64_t key, uint64_t seed);
uint64_t or_hash(int kind, int64_t key, uint64_t seed);
void or_hash_many(int kind, const int64_t* keys, uint64_t n, uint64_t seed, uint64_t* out);
/* hash(key) % cardinality, exactly XXHasher::Hash */
uint64_t or_hash_mod(int kind, int64_t key, uint64_t seed, uint64_t card);

/* ---- generators (src/Common/Random.cpp:9-30, src/DataGenerator/{Zipf,Sequential}.cpp) ---- */
int64_t or_lcg_step(int64_t state);
double or_lcg_next(int64_t *state);
uint64_t or_zipf_generate(double alpha, uint64_t cardinality, int64_t *state);
int64_t or_batch_seed(uint64_t base_seed, uint64_t batch);
void or_fill_sequential(or_tuple *t, uint64_t n, int64_t start);
/* returns 0 or -1 (invalid range / alpha: Zipf.cpp:19-21,61-67) */
int or_fill_zipf(or_tuple *t, uint64_t n, double alpha, int64_t lo, int64_t hi,
                 uint64_t seed, int threads);

/* ---- LinearProbing (src/HashTables/LinearProbing.hpp:22-210) ---- */
typedef struct or_lp_table or_lp_table;
or_lp_table *or_lp_new(double ratio, uint64_t n, int hash_kind, uint64_t seed);
void or_lp_free(or_lp_table *t);
uint64_t or_lp_num_buckets(const or_lp_table *t);
void or_lp_insert(or_lp_table *t, int64_t key, const void *value); /* thread-safe */
const void *or_lp_get(or_lp_table *t, int64_t key);
int or_lp_exists(or_lp_table *t, int64_t key);
uint64_t or_lp_get_all(or_lp_table *t, int64_t key, const void **out, uint64_t cap);

/* ---- SeparateChaining (src/HashTables/SeparateChaining.hpp:143-277) ---- */
typedef struct or_sc_table or_sc_table;
or_sc_table *or_sc_new(double ratio, uint64_t n, int hash_kind, uint64_t seed);
void or_sc_free(or_sc_table *t);
uint64_t or_sc_num_buckets(const or_sc_table *t);
int or_sc_insert(or_sc_table *t, int64_t key, const void *value); /* thread-safe; -1 on overflow */
const void *or_sc_get(or_sc_table *t, int64_t key);
int or_sc_exists(or_sc_table *t, int64_t key);
uint64_t or_sc_get_all(or_sc_table *t, int64_t key, const void **out, uint64_t cap);

/* ---- partitioning ----
 * Partition id q(key):  mode "mod":   q = hash(key) % P          (RadixCluster/HashJoin.hpp:349-351)
 *                       mode "radix": q = hash(key) & (2^bits-1) (extension: power-of-two radix)
 * Output: a STABLE partition (partition-major, then input order), which is
 * exactly the layout the reference's per-worker prefix-sum scatter produces
 * (HashJoin.hpp:394-412). bounds has P+1 entries. */
int or_partition(const or_tuple *in, uint64_t n, uint64_t P, int radix, int hash_kind,
                 uint64_t seed, int workers, or_tuple *out, uint64_t *bounds);
/* q for one key (radix: P must be a power of two) */
uint64_t or_partition_id(int64_t key, uint64_t P, int radix, int hash_kind, uint64_t seed);

/* ---- joins ---- */
typedef struct or_result {
    uint64_t matches;       /* semi-join count: #S tuples with >= 1 match in R */
    double partition_ms;    /* reference timer semantics (Results.hpp:167-247) */
    double build_ms;
    double probe_ms;        /* NoPartitioning: as reported (includes build, Results.hpp:202) */
    double probe_only_ms;   /* NoPartitioning: probe phase alone */
    double wall_ms;
    int workers;
} or_result;

/* NoPartitioning::HashJoiner::Run (src/NoPartitioning/HashJoin.hpp:54-187) with
 * LinearProbingFactory<Tuple,3,XXHasher> (src/main.cpp:216). Returns -1 when
 * |R| == 0 (LinearProbing.hpp: numberOfObjects must be > 0). */
int or_join_nopart(const or_tuple *R, uint64_t nR, const or_tuple *S, uint64_t nS,
                   int hash_kind, uint64_t table_seed, double ratio, int workers,
                   or_result *res);

/* RadixClustering::HashJoiner::Run (src/RadixCluster/HashJoin.hpp:190-331).
 * radix==0: q = hash%P (reference); radix==1: q = hash & (P-1). */
int or_join_radix(const or_tuple *R, uint64_t nR, const or_tuple *S, uint64_t nS,
                  uint64_t P, int radix, int part_hash_kind, uint64_t part_seed,
                  int table_hash_kind, uint64_t table_seed, double ratio, int workers,
                  or_result *res);

/* Independent check: sort R keys, binary-search every S key. */
uint64_t or_semijoin_count_sorted(const or_tuple *R, uint64_t nR, const or_tuple *S,
                                  uint64_t nS, int threads);
/* Same, over key columns (int64 arrays). */
uint64_t or_semijoin_count_keys(const int64_t *rkeys, uint64_t nR, const int64_t *skeys,
                                uint64_t nS, int threads);

#ifdef __cplusplus
}
#endif

#endif
