/*
 * phj_oracle.c — TEST INFRASTRUCTURE ONLY (see phj_oracle.h).
 *
 * CPU restatement of the reference hot path. Every function cites the
 * reference file:line it follows (paths relative to /root/reference/).
 * Multi-threaded with plain pthreads so it can also serve as bench.py's
 * cpu_baseline ("kind": "port").
 */
#define _GNU_SOURCE
#include "phj_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define OR_GEN_BATCH 4096u   /* tuples per seeded LCG stream */
#define OR_LCG_M 2147483647LL
#define OR_MIN_BATCH 10000u  /* RadixCluster/Configuration.hpp:7, NoPartitioning/Configuration.hpp:7 */

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

/* ------------------------------------------------------------------ */
/* tiny parallel-for on pthreads (stands in for Common::ThreadPool)     */
/* ------------------------------------------------------------------ */
typedef void (*or_task_fn)(void *arg, int id);
typedef struct {
    or_task_fn fn;
    void *arg;
    int id;
} or_task;

static void *or_task_main(void *p) {
    or_task *t = (or_task *)p;
    t->fn(t->arg, t->id);
    return NULL;
}

static void or_parallel(int n, or_task_fn fn, void *arg) {
    if (n <= 1) {
        if (n == 1) fn(arg, 0);
        return;
    }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n);
    or_task *tk = (or_task *)malloc(sizeof(or_task) * (size_t)n);
    for (int i = 0; i < n; i++) {
        tk[i].fn = fn;
        tk[i].arg = arg;
        tk[i].id = i;
        if (i > 0) pthread_create(&th[i], NULL, or_task_main, &tk[i]);
    }
    fn(arg, 0);
    for (int i = 1; i < n; i++) pthread_join(th[i], NULL);
    free(th);
    free(tk);
}

/* Worker/batch split used by every reference stage:
 * batch = size / W; if batch < MinBatchSize: W = ceil(size/MinBatch), batch = MinBatch;
 * the last worker takes the remainder (e.g. NoPartitioning/HashJoin.hpp:84-110). */
static void or_split(uint64_t size, int pool, uint64_t *workers, uint64_t *batch) {
    uint64_t w = pool < 1 ? 1 : (uint64_t)pool;
    uint64_t b = (uint64_t)((double)size / (double)w);
    if (b < OR_MIN_BATCH) {
        w = (uint64_t)ceil((double)size / (double)OR_MIN_BATCH);
        b = OR_MIN_BATCH;
    }
    *workers = w;
    *batch = b;
}

static void or_range(uint64_t i, uint64_t w, uint64_t batch, uint64_t size, uint64_t *lo,
                     uint64_t *hi) {
    *lo = batch * i;
    *hi = (i == w - 1) ? size : batch * (i + 1);
    if (*lo > size) *lo = size;
    if (*hi > size) *hi = size;
}

/* ------------------------------------------------------------------ */
/* hashing                                                             */
/* ------------------------------------------------------------------ */
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

/* XXH3_64bits_withSeed(&key, 8, seed) as called by XXHasher::Hash
 * (src/Common/XXHasher.hpp:20). Third-party algorithm (xxHash >= 0.8, the
 * "len 4..8" short-input path; reference pins only "xxHash 0.7" in
 * CMakeLists.txt:14): the 8 input bytes are the little-endian int64 key;
 * secret = XXH3 default kSecret, of which bytes [8,24) enter this path. */
uint64_t or_xxh3_64(int64_t key, uint64_t seed) {
    const uint64_t k = (uint64_t)key;
    const uint32_t in1 = (uint32_t)k;          /* readLE32(input)     */
    const uint32_t in2 = (uint32_t)(k >> 32);  /* readLE32(input + 4) */
    const uint32_t s32 = (uint32_t)seed;
    const uint32_t sw = (s32 >> 24) | ((s32 >> 8) & 0xff00u) | ((s32 << 8) & 0xff0000u) | (s32 << 24);
    seed ^= (uint64_t)sw << 32;
    const uint64_t secret8 = 0x1cad21f72c81017cULL;   /* kSecret[8..16)  LE */
    const uint64_t secret16 = 0xdb979083e96dd4deULL;  /* kSecret[16..24) LE */
    const uint64_t bitflip = (secret8 ^ secret16) - seed;
    const uint64_t input64 = (uint64_t)in2 + ((uint64_t)in1 << 32);
    uint64_t h = input64 ^ bitflip;
    /* XXH3_rrmxmx(h, len = 8) */
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= 0x9FB21C651E98DF25ULL;
    h ^= (h >> 35) + 8u;
    h *= 0x9FB21C651E98DF25ULL;
    h ^= h >> 28;
    return h;
}

/* Murmur3 64-bit finalizer (fmix64) over key ^ seed — the BASELINE.json C2
 * "Murmur3" option (an extension: the reference only has XXHasher). */
uint64_t or_murmur3(int64_t key, uint64_t seed) {
    uint64_t k = (uint64_t)key ^ seed;
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

uint64_t or_hash(int kind, int64_t key, uint64_t seed) {
    return kind == OR_HASH_MURMUR3 ? or_murmur3(key, seed) : or_xxh3_64(key, seed);
}

/* or_hash over an array (test infrastructure: full-size code checks). */
void or_hash_many(int kind, const int64_t* keys, uint64_t n, uint64_t seed, uint64_t* out) {
    for (uint64_t i = 0; i < n; i++) out[i] = or_hash(kind, keys[i], seed);
}

/* XXHasher::Hash(key, cardinality) = hash % cardinality (XXHasher.hpp:19-22). */
uint64_t or_hash_mod(int kind, int64_t key, uint64_t seed, uint64_t card) {
    return or_hash(kind, key, seed) % card;
}

/* ------------------------------------------------------------------ */
/* generators                                                          */
/* ------------------------------------------------------------------ */
/* MultiplicativeLCGRandomNumberGenerator::Next (src/Common/Random.cpp:9-30):
 * Park-Miller minimal standard, a=16807, m=2^31-1, Schrage's method. */
int64_t or_lcg_step(int64_t state) {
    const int64_t a = 16807, q = 127773, r = 2836;
    const int64_t x_div_q = state / q;
    const int64_t x_mod_q = state % q;
    const int64_t x_new = (a * x_mod_q) - (r * x_div_q);
    return x_new > 0 ? x_new : x_new + OR_LCG_M;
}

double or_lcg_next(int64_t *state) {
    *state = or_lcg_step(*state);
    return (double)(*state) / (double)OR_LCG_M;
}

/* Zipf::generate (src/DataGenerator/Zipf.cpp:14-56), rejection sampling. */
uint64_t or_zipf_generate(double alpha, uint64_t cardinality, int64_t *state) {
    const double errorDifferential = 0.01;
    double skewDifferential = 1.001 - alpha;
    const double diff = 1.0 - alpha;
    if (fabs(diff) < errorDifferential) {
        skewDifferential = errorDifferential * ((diff < 0) ? 1 : -1);
        alpha = 1.0 - skewDifferential;
    }
    const double normalizationConstant =
        (pow((double)cardinality, skewDifferential) - alpha) / skewDifferential;
    for (;;) {
        const double u1 = or_lcg_next(state);
        const double u2 = or_lcg_next(state);
        double inv;
        if (u1 * normalizationConstant <= 1.0) {
            inv = u1 * normalizationConstant;
        } else {
            inv = pow((u1 * normalizationConstant) * skewDifferential + alpha,
                      1.0 / skewDifferential);
        }
        const double sample = floor(inv + 1);
        const double densityOriginal = pow(sample, -alpha);
        const double densitySampling =
            sample <= 1.0 ? 1.0 / normalizationConstant
                          : pow(inv, -alpha) / normalizationConstant;
        const double ratio = densityOriginal / (densitySampling * normalizationConstant);
        if (u2 < ratio) return (uint64_t)sample;
    }
}

/* Seeded replacement for the reference's per-batch std::random_device seed
 * (Zipf.cpp:86 → Random.cpp:32-36): batch b of OR_GEN_BATCH tuples uses
 * GetNewGenerator(seed_b) (Random.cpp:38-41) with seed_b in [1, 2^31-2]. */
int64_t or_batch_seed(uint64_t base_seed, uint64_t batch) {
    const uint64_t M = 2147483646ULL;
    return (int64_t)(1 + (((base_seed % M) * 1000003ULL + batch) % M));
}

/* Sequential::FillTable (src/DataGenerator/Sequential.cpp:6-40): id = start+i, payload = i. */
void or_fill_sequential(or_tuple *t, uint64_t n, int64_t start) {
    for (uint64_t i = 0; i < n; i++) {
        t[i].id = start + (int64_t)i;
        t[i].payload = (int64_t)i;
    }
}

typedef struct {
    or_tuple *t;
    uint64_t n, nbatches;
    double alpha;
    uint64_t card;
    int64_t correction;
    uint64_t seed;
    int threads;
} zipf_job;

static void zipf_worker(void *p, int id) {
    zipf_job *j = (zipf_job *)p;
    for (uint64_t b = (uint64_t)id; b < j->nbatches; b += (uint64_t)j->threads) {
        int64_t st = or_batch_seed(j->seed, b);
        const uint64_t lo = b * OR_GEN_BATCH;
        const uint64_t hi = lo + OR_GEN_BATCH < j->n ? lo + OR_GEN_BATCH : j->n;
        for (uint64_t i = lo; i < hi; i++) {
            j->t[i].id = (int64_t)or_zipf_generate(j->alpha, j->card, &st) + j->correction;
            j->t[i].payload = (int64_t)i;
        }
    }
}

/* Zipf::FillTable (src/DataGenerator/Zipf.cpp:58-108) over closed range [lo, hi]. */
int or_fill_zipf(or_tuple *t, uint64_t n, double alpha, int64_t lo, int64_t hi, uint64_t seed,
                 int threads) {
    if (lo >= hi) return -1;        /* Zipf.cpp:61-67 */
    if (alpha < 0.01) return -1;    /* Zipf.cpp:19-21 */
    zipf_job j;
    j.t = t;
    j.n = n;
    j.nbatches = (n + OR_GEN_BATCH - 1) / OR_GEN_BATCH;
    j.alpha = alpha;
    j.card = (uint64_t)(hi - lo + 1);
    j.correction = lo - 1;
    j.seed = seed;
    j.threads = threads < 1 ? 1 : threads;
    or_parallel(j.threads, zipf_worker, &j);
    return 0;
}

/* ------------------------------------------------------------------ */
/* LinearProbing (src/HashTables/LinearProbing.hpp)                     */
/* ------------------------------------------------------------------ */
#define OR_LP_SLOTS 3 /* LinearProbingFactory<Tuple, 3, XXHasher> (src/main.cpp:216) */

typedef struct __attribute__((aligned(64))) or_lp_bucket {
    int8_t fill;                       /* m_freePosition  :269 */
    int64_t keys[OR_LP_SLOTS];         /* m_keys          :270 */
    const void *vals[OR_LP_SLOTS];     /* m_values        :271 */
} or_lp_bucket;

struct or_lp_table {
    uint64_t nb;
    or_lp_bucket *b;
    atomic_flag *latch;
    int hk;
    uint64_t seed;
};

/* getNumberOfBuckets (LinearProbing.cpp:7-12): ceil(ratio * n) */
or_lp_table *or_lp_new(double ratio, uint64_t n, int hash_kind, uint64_t seed) {
    if (n == 0) return NULL; /* LinearProbing.hpp:295-299 throws invalid_argument */
    or_lp_table *t = (or_lp_table *)calloc(1, sizeof(or_lp_table));
    t->nb = (uint64_t)ceil(ratio * (double)n);
    if (t->nb == 0) t->nb = 1;
    t->b = (or_lp_bucket *)aligned_alloc(64, sizeof(or_lp_bucket) * t->nb);
    memset(t->b, 0, sizeof(or_lp_bucket) * t->nb);
    t->latch = (atomic_flag *)malloc(sizeof(atomic_flag) * t->nb);
    for (uint64_t i = 0; i < t->nb; i++) atomic_flag_clear(&t->latch[i]);
    t->hk = hash_kind;
    t->seed = seed;
    return t;
}

void or_lp_free(or_lp_table *t) {
    if (!t) return;
    free(t->b);
    free((void *)t->latch);
    free(t);
}

uint64_t or_lp_num_buckets(const or_lp_table *t) { return t ? t->nb : 0; }

/* Insert (LinearProbing.hpp:114-134): latch the home bucket; if full, move on. */
void or_lp_insert(or_lp_table *t, int64_t key, const void *value) {
    uint64_t h = or_hash_mod(t->hk, key, t->seed, t->nb);
    for (uint64_t step = 0; step < t->nb; step++) {
        while (atomic_flag_test_and_set_explicit(&t->latch[h], memory_order_acquire)) {
        }
        or_lp_bucket *bk = &t->b[h];
        int ok = 0;
        if (bk->fill != OR_LP_SLOTS) {
            bk->keys[bk->fill] = key;
            bk->vals[bk->fill] = value;
            bk->fill++;
            ok = 1;
        }
        atomic_flag_clear_explicit(&t->latch[h], memory_order_release);
        if (ok) return;
        h = (h + 1 == t->nb) ? 0 : h + 1;
    }
}

/* Get (LinearProbing.hpp:160-180): first match; stop at the first non-full bucket. */
const void *or_lp_get(or_lp_table *t, int64_t key) {
    uint64_t h = or_hash_mod(t->hk, key, t->seed, t->nb);
    for (uint64_t step = 0; step < t->nb; step++) {
        const or_lp_bucket *bk = &t->b[h];
        for (int i = 0; i < bk->fill; i++)
            if (bk->keys[i] == key) return bk->vals[i];
        if (bk->fill != OR_LP_SLOTS) return NULL;
        h = (h + 1 == t->nb) ? 0 : h + 1;
    }
    return NULL;
}

/* Exists (LinearProbing.hpp:137-157) */
int or_lp_exists(or_lp_table *t, int64_t key) {
    uint64_t h = or_hash_mod(t->hk, key, t->seed, t->nb);
    for (uint64_t step = 0; step < t->nb; step++) {
        const or_lp_bucket *bk = &t->b[h];
        for (int i = 0; i < bk->fill; i++)
            if (bk->keys[i] == key) return 1;
        if (bk->fill != OR_LP_SLOTS) return 0;
        h = (h + 1 == t->nb) ? 0 : h + 1;
    }
    return 0;
}

/* GetAll (LinearProbing.hpp:183-200) */
uint64_t or_lp_get_all(or_lp_table *t, int64_t key, const void **out, uint64_t cap) {
    uint64_t h = or_hash_mod(t->hk, key, t->seed, t->nb), cnt = 0;
    for (uint64_t step = 0; step < t->nb; step++) {
        const or_lp_bucket *bk = &t->b[h];
        for (int i = 0; i < bk->fill; i++)
            if (bk->keys[i] == key) {
                if (out && cnt < cap) out[cnt] = bk->vals[i];
                cnt++;
            }
        if (bk->fill != OR_LP_SLOTS) return cnt;
        h = (h + 1 == t->nb) ? 0 : h + 1;
    }
    return cnt;
}

/* ------------------------------------------------------------------ */
/* SeparateChaining (src/HashTables/SeparateChaining.hpp)               */
/* ------------------------------------------------------------------ */
typedef struct __attribute__((aligned(64))) or_sc_bucket {
    struct or_sc_bucket *next;   /* m_nextBucket  :97 */
    int8_t fill;                 /* m_freePosition :98 */
    int64_t keys[OR_LP_SLOTS];
    const void *vals[OR_LP_SLOTS];
} or_sc_bucket;

struct or_sc_table {
    uint64_t nb;
    or_sc_bucket **ptrs;     /* m_bucketPtrs   */
    or_sc_bucket *first;     /* m_firstBuckets */
    atomic_flag *latch;
    or_sc_bucket *pool;      /* BucketAllocator (:103-135) */
    uint64_t pool_size;
    atomic_uint_fast64_t pool_next;
    int hk;
    uint64_t seed;
};

/* ctor (SeparateChaining.hpp:149-172): ceil(ratio*n) heads; ceil(n/3) overflow buckets */
or_sc_table *or_sc_new(double ratio, uint64_t n, int hash_kind, uint64_t seed) {
    if (n == 0) return NULL;
    or_sc_table *t = (or_sc_table *)calloc(1, sizeof(or_sc_table));
    t->nb = (uint64_t)ceil(ratio * (double)n);
    if (t->nb == 0) t->nb = 1;
    t->ptrs = (or_sc_bucket **)calloc(t->nb, sizeof(or_sc_bucket *));
    t->first = (or_sc_bucket *)aligned_alloc(64, sizeof(or_sc_bucket) * t->nb);
    memset(t->first, 0, sizeof(or_sc_bucket) * t->nb);
    t->latch = (atomic_flag *)malloc(sizeof(atomic_flag) * t->nb);
    for (uint64_t i = 0; i < t->nb; i++) atomic_flag_clear(&t->latch[i]);
    t->pool_size = (uint64_t)ceil((double)n / (double)OR_LP_SLOTS);
    t->pool = (or_sc_bucket *)aligned_alloc(64, sizeof(or_sc_bucket) * (t->pool_size ? t->pool_size : 1));
    memset(t->pool, 0, sizeof(or_sc_bucket) * (t->pool_size ? t->pool_size : 1));
    atomic_init(&t->pool_next, 0);
    t->hk = hash_kind;
    t->seed = seed;
    return t;
}

void or_sc_free(or_sc_table *t) {
    if (!t) return;
    free(t->ptrs);
    free(t->first);
    free((void *)t->latch);
    free(t->pool);
    free(t);
}

uint64_t or_sc_num_buckets(const or_sc_table *t) { return t ? t->nb : 0; }

static int sc_bucket_insert(or_sc_bucket *b, int64_t key, const void *v) {
    if (b->fill == OR_LP_SLOTS) return 0;
    b->keys[b->fill] = key;
    b->vals[b->fill] = v;
    b->fill++;
    return 1;
}

/* Insert (SeparateChaining.hpp:175-213): head insertion of a fresh bucket when full. */
int or_sc_insert(or_sc_table *t, int64_t key, const void *value) {
    const uint64_t h = or_hash_mod(t->hk, key, t->seed, t->nb);
    int rc = 0;
    while (atomic_flag_test_and_set_explicit(&t->latch[h], memory_order_acquire)) {
    }
    if (t->ptrs[h] == NULL) {
        t->ptrs[h] = &t->first[h];
        sc_bucket_insert(t->ptrs[h], key, value);
    } else if (!sc_bucket_insert(t->ptrs[h], key, value)) {
        const uint64_t idx = atomic_fetch_add(&t->pool_next, 1);
        if (idx >= t->pool_size) {
            rc = -1; /* "BucketAllocator exceeded its limit." (:116-118) */
        } else {
            or_sc_bucket *nb = &t->pool[idx];
            nb->next = t->ptrs[h];
            t->ptrs[h] = nb;
            sc_bucket_insert(nb, key, value);
        }
    }
    atomic_flag_clear_explicit(&t->latch[h], memory_order_release);
    return rc;
}

/* Get (SeparateChaining.hpp:236-254) */
const void *or_sc_get(or_sc_table *t, int64_t key) {
    const uint64_t h = or_hash_mod(t->hk, key, t->seed, t->nb);
    for (const or_sc_bucket *b = t->ptrs[h]; b; b = b->next)
        for (int i = 0; i < b->fill; i++)
            if (b->keys[i] == key) return b->vals[i];
    return NULL;
}

int or_sc_exists(or_sc_table *t, int64_t key) { return or_sc_get(t, key) != NULL; }

/* GetAll (SeparateChaining.hpp:74-94, 257-265) */
uint64_t or_sc_get_all(or_sc_table *t, int64_t key, const void **out, uint64_t cap) {
    const uint64_t h = or_hash_mod(t->hk, key, t->seed, t->nb);
    uint64_t cnt = 0;
    for (const or_sc_bucket *b = t->ptrs[h]; b; b = b->next)
        for (int i = 0; i < b->fill; i++)
            if (b->keys[i] == key) {
                if (out && cnt < cap) out[cnt] = b->vals[i];
                cnt++;
            }
    return cnt;
}

/* ------------------------------------------------------------------ */
/* partitioning (src/RadixCluster/HashJoin.hpp:333-440)                 */
/* ------------------------------------------------------------------ */
uint64_t or_partition_id(int64_t key, uint64_t P, int radix, int hash_kind, uint64_t seed) {
    const uint64_t h = or_hash(hash_kind, key, seed);
    return radix ? (h & (P - 1)) : (h % P);
}

typedef struct {
    const or_tuple *in;
    or_tuple *out;
    uint64_t n, P, W, batch;
    int radix, hk;
    uint64_t seed;
    uint64_t *pst;    /* PrefixSumTable [W x P], worker-major (:41-61) */
    uint64_t *bounds; /* PartitionsInfo borders (:16-33), P+1 entries */
} part_job;

/* scanTable (:343-357) */
static void part_scan(void *p, int id) {
    part_job *j = (part_job *)p;
    uint64_t lo, hi;
    or_range((uint64_t)id, j->W, j->batch, j->n, &lo, &hi);
    uint64_t *row = j->pst + (uint64_t)id * j->P;
    for (uint64_t i = lo; i < hi; i++)
        row[or_partition_id(j->in[i].id, j->P, j->radix, j->hk, j->seed)]++;
}

/* partitionTable (:394-412): stable scatter out[border[p] + pos[w][p]++] = t */
static void part_scatter(void *p, int id) {
    part_job *j = (part_job *)p;
    uint64_t lo, hi;
    or_range((uint64_t)id, j->W, j->batch, j->n, &lo, &hi);
    uint64_t *row = j->pst + (uint64_t)id * j->P;
    for (uint64_t i = lo; i < hi; i++) {
        const uint64_t q = or_partition_id(j->in[i].id, j->P, j->radix, j->hk, j->seed);
        j->out[j->bounds[q] + row[q]++] = j->in[i];
    }
}

static int or_partition_w(const or_tuple *in, uint64_t n, uint64_t P, int radix, int hk,
                          uint64_t seed, uint64_t W, uint64_t batch, or_tuple *out,
                          uint64_t *bounds) {
    if (P == 0) return -1;
    if (radix && (P & (P - 1))) return -1;
    part_job j;
    j.in = in;
    j.out = out;
    j.n = n;
    j.P = P;
    j.W = W == 0 ? 1 : W;
    j.batch = batch;
    j.radix = radix;
    j.hk = hk;
    j.seed = seed;
    j.pst = (uint64_t *)calloc(j.W * P, sizeof(uint64_t));
    j.bounds = bounds;
    or_parallel((int)j.W, part_scan, &j);
    /* createPrefixSumTable (:360-390): per partition exclusive scan over workers */
    uint64_t run = 0;
    for (uint64_t q = 0; q < P; q++) {
        uint64_t acc = 0;
        for (uint64_t w = 0; w < j.W; w++) {
            const uint64_t c = j.pst[w * P + q];
            j.pst[w * P + q] = acc;
            acc += c;
        }
        /* ComputePartitionsBoundaries (:18-25) */
        bounds[q] = run;
        run += acc;
    }
    bounds[P] = run;
    or_parallel((int)j.W, part_scatter, &j);
    free(j.pst);
    return 0;
}

int or_partition(const or_tuple *in, uint64_t n, uint64_t P, int radix, int hash_kind,
                 uint64_t seed, int workers, or_tuple *out, uint64_t *bounds) {
    uint64_t W, batch;
    or_split(n, workers, &W, &batch);
    if (n == 0) {
        for (uint64_t q = 0; q <= P; q++) bounds[q] = 0;
        return P == 0 ? -1 : 0;
    }
    return or_partition_w(in, n, P, radix, hash_kind, seed, W, batch, out, bounds);
}

/* ------------------------------------------------------------------ */
/* joins                                                               */
/* ------------------------------------------------------------------ */
typedef struct {
    const or_tuple *R, *S;
    uint64_t nR, nS, W, batch;
    or_lp_table *table;
    _Atomic uint64_t count;
} np_job;

static void np_build(void *p, int id) {   /* buildHashTable (NoPartitioning/HashJoin.hpp:93-98) */
    np_job *j = (np_job *)p;
    uint64_t lo, hi;
    or_range((uint64_t)id, j->W, j->batch, j->nR, &lo, &hi);
    for (uint64_t i = lo; i < hi; i++) or_lp_insert(j->table, j->R[i].id, &j->R[i]);
}

static void np_probe(void *p, int id) {   /* probeHashTable (:144-157) */
    np_job *j = (np_job *)p;
    uint64_t lo, hi, c = 0;
    or_range((uint64_t)id, j->W, j->batch, j->nS, &lo, &hi);
    for (uint64_t i = lo; i < hi; i++)
        if (or_lp_get(j->table, j->S[i].id) != NULL) c++;
    atomic_fetch_add(&j->count, c);
}

/* NoPartitioning::HashJoiner::Run (src/NoPartitioning/HashJoin.hpp:54-74). */
int or_join_nopart(const or_tuple *R, uint64_t nR, const or_tuple *S, uint64_t nS, int hash_kind,
                   uint64_t table_seed, double ratio, int workers, or_result *res) {
    memset(res, 0, sizeof(*res));
    const double t0 = now_ms();
    /* Build (:76-126): table allocation is inside the build phase (:82) */
    or_lp_table *t = or_lp_new(ratio, nR, hash_kind, table_seed);
    if (!t) return -1;
    np_job j;
    j.R = R;
    j.S = S;
    j.nR = nR;
    j.nS = nS;
    j.table = t;
    atomic_init(&j.count, 0);
    or_split(nR, workers, &j.W, &j.batch);
    or_parallel((int)j.W, np_build, &j);
    const double t1 = now_ms();
    /* Probe (:128-187) */
    or_split(nS, workers, &j.W, &j.batch);
    if (nS > 0) or_parallel((int)j.W, np_probe, &j);
    const double t2 = now_ms();
    res->matches = atomic_load(&j.count);
    res->build_ms = t1 - t0;
    res->probe_ms = t2 - t0; /* HashJoinTimer::SetProbePhaseEnd measures from m_buildStart (Results.hpp:202) */
    res->probe_only_ms = t2 - t1;
    res->partition_ms = 0;
    res->wall_ms = t2 - t0;
    res->workers = workers;
    or_lp_free(t);
    return 0;
}

typedef struct {
    const or_tuple *pR, *pS;
    const uint64_t *bR, *bS;
    uint64_t P, W;
    int hk;
    uint64_t seed;
    double ratio;
    _Atomic uint64_t count;
    pthread_mutex_t mu;
    double max_build, max_probe; /* BuildAndProbeRepresentativeDurationMeasurer (:63-87) */
} rj_job;

/* join lambda (RadixCluster/HashJoin.hpp:258-323) */
static void rj_worker(void *p, int id) {
    rj_job *j = (rj_job *)p;
    double build = 0, probe = 0;
    uint64_t joined = 0;
    for (uint64_t q = (uint64_t)id; q < j->P; q += j->W) {
        const uint64_t ra = j->bR[q], rb = j->bR[q + 1];
        if (rb == ra) continue; /* :273-276 */
        or_lp_table *t = or_lp_new(j->ratio, rb - ra, j->hk, j->seed); /* :278 (outside build time) */
        double t0 = now_ms();
        for (uint64_t i = ra; i < rb; i++) or_lp_insert(t, j->pR[i].id, &j->pR[i]);
        double t1 = now_ms();
        for (uint64_t i = j->bS[q]; i < j->bS[q + 1]; i++)
            if (or_lp_get(t, j->pS[i].id) != NULL) joined++;
        double t2 = now_ms();
        build += t1 - t0;
        probe += t2 - t1;
        or_lp_free(t);
    }
    pthread_mutex_lock(&j->mu);
    if (build + probe > j->max_build + j->max_probe) {
        j->max_build = build;
        j->max_probe = probe;
    }
    pthread_mutex_unlock(&j->mu);
    atomic_fetch_add(&j->count, joined);
}

/* RadixClustering::HashJoiner::Run (src/RadixCluster/HashJoin.hpp:190-241). */
int or_join_radix(const or_tuple *R, uint64_t nR, const or_tuple *S, uint64_t nS, uint64_t P,
                  int radix, int part_hash_kind, uint64_t part_seed, int table_hash_kind,
                  uint64_t table_seed, double ratio, int workers, or_result *res) {
    memset(res, 0, sizeof(*res));
    if (P == 0 || (radix && (P & (P - 1)))) return -1;
    /* partitioned copies allocated outside the timer (:195-198) */
    or_tuple *pR = (or_tuple *)malloc(sizeof(or_tuple) * (nR ? nR : 1));
    or_tuple *pS = (or_tuple *)malloc(sizeof(or_tuple) * (nS ? nS : 1));
    uint64_t *bR = (uint64_t *)calloc(P + 1, sizeof(uint64_t));
    uint64_t *bS = (uint64_t *)calloc(P + 1, sizeof(uint64_t));
    /* GetPartitioningConfiguration (:149-188): W shared by both relations */
    uint64_t W = workers < 1 ? 1 : (uint64_t)workers;
    uint64_t batchA = (uint64_t)((double)nR / (double)W);
    uint64_t batchB = (uint64_t)((double)nS / (double)W);
    if (batchA < OR_MIN_BATCH) {
        W = (uint64_t)ceil((double)nR / (double)OR_MIN_BATCH);
        batchA = OR_MIN_BATCH;
    }
    if (batchB < OR_MIN_BATCH) {
        W = (uint64_t)ceil((double)nS / (double)OR_MIN_BATCH);
        batchB = OR_MIN_BATCH;
    }
    if (W == 0) W = 1;
    const double t0 = now_ms();
    if (nR) or_partition_w(R, nR, P, radix, part_hash_kind, part_seed, W, batchA, pR, bR);
    if (nS) or_partition_w(S, nS, P, radix, part_hash_kind, part_seed, W, batchB, pS, bS);
    const double t1 = now_ms();
    rj_job j;
    j.pR = pR;
    j.pS = pS;
    j.bR = bR;
    j.bS = bS;
    j.P = P;
    j.W = W;
    j.hk = table_hash_kind;
    j.seed = table_seed;
    j.ratio = ratio;
    atomic_init(&j.count, 0);
    pthread_mutex_init(&j.mu, NULL);
    j.max_build = j.max_probe = 0;
    if (nR && nS) or_parallel((int)W, rj_worker, &j);
    const double t2 = now_ms();
    res->matches = atomic_load(&j.count);
    res->partition_ms = t1 - t0;
    res->build_ms = j.max_build;
    res->probe_ms = j.max_probe;
    res->probe_only_ms = j.max_probe;
    res->wall_ms = t2 - t0;
    res->workers = (int)W;
    pthread_mutex_destroy(&j.mu);
    free(pR);
    free(pS);
    free(bR);
    free(bS);
    return 0;
}

/* ------------------------------------------------------------------ */
/* independent semi-join count                                         */
/* ------------------------------------------------------------------ */
static int cmp_i64(const void *a, const void *b) {
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

typedef struct {
    const int64_t *sorted;
    uint64_t nR;
    const int64_t *skeys;
    const or_tuple *S;
    uint64_t nS;
    int threads;
    _Atomic uint64_t count;
} sj_job;

static void sj_worker(void *p, int id) {
    sj_job *j = (sj_job *)p;
    const uint64_t per = (j->nS + (uint64_t)j->threads - 1) / (uint64_t)j->threads;
    const uint64_t lo = per * (uint64_t)id;
    const uint64_t hi = lo + per < j->nS ? lo + per : j->nS;
    uint64_t c = 0;
    for (uint64_t i = lo; i < hi; i++) {
        const int64_t k = j->skeys ? j->skeys[i] : j->S[i].id;
        uint64_t a = 0, b = j->nR;
        while (a < b) {
            const uint64_t m = a + (b - a) / 2;
            if (j->sorted[m] < k) a = m + 1;
            else b = m;
        }
        if (a < j->nR && j->sorted[a] == k) c++;
    }
    atomic_fetch_add(&j->count, c);
}

static uint64_t sj_run(int64_t *sorted, uint64_t nR, const int64_t *skeys, const or_tuple *S,
                       uint64_t nS, int threads) {
    qsort(sorted, nR, sizeof(int64_t), cmp_i64);
    sj_job j;
    j.sorted = sorted;
    j.nR = nR;
    j.skeys = skeys;
    j.S = S;
    j.nS = nS;
    j.threads = threads < 1 ? 1 : threads;
    atomic_init(&j.count, 0);
    if (nS && nR) or_parallel(j.threads, sj_worker, &j);
    return atomic_load(&j.count);
}

uint64_t or_semijoin_count_sorted(const or_tuple *R, uint64_t nR, const or_tuple *S, uint64_t nS,
                                  int threads) {
    int64_t *k = (int64_t *)malloc(sizeof(int64_t) * (nR ? nR : 1));
    for (uint64_t i = 0; i < nR; i++) k[i] = R[i].id;
    const uint64_t c = sj_run(k, nR, NULL, S, nS, threads);
    free(k);
    return c;
}

uint64_t or_semijoin_count_keys(const int64_t *rkeys, uint64_t nR, const int64_t *skeys,
                                uint64_t nS, int threads) {
    int64_t *k = (int64_t *)malloc(sizeof(int64_t) * (nR ? nR : 1));
    memcpy(k, rkeys, sizeof(int64_t) * nR);
    const uint64_t c = sj_run(k, nR, skeys, NULL, nS, threads);
    free(k);
    return c;
}
