// phj_capi.hip — the C ABI (include/phj.h) over the gfx950 kernels.
//
// Orchestration of the reference's HashJoiner::Run on one MI355X:
//   radix:          Partition(R), Partition(S)            RadixCluster/HashJoin.hpp:208-224
//                   -> build + probe per partition        :243-331
//   no-partitioning: Build(R) -> Probe(S)                 NoPartitioning/HashJoin.hpp:54-187
// Every kernel is launched on the ctx stream; device buffers are allocated
// once (grow-only) before the timed region; phases are timed with hipEvents
// on the same stream. Errors never cross the ABI as exceptions: they become
// negative status codes plus a message (phj_last_error).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

// Measurement builds only (scripts/ab_lib.sh, `make prof-lib`): the phase-clock
// forms of S's pass 1 and of the LDS join's builds, printed to stderr per join.
#ifndef PHJ_P1_PROF
#define PHJ_P1_PROF 0
#endif
#ifndef PHJ_CL_PROF
#define PHJ_CL_PROF 0
#endif

#include "../../include/phj.h"
#include "phj_cluster.h"
#include "phj_join.h"
#include "phj_mat.h"
#include "phj_partition.h"
#include "phj_table.h"

using namespace phj;

namespace {

constexpr double kNPDefaultRatio = 2.0;             // slots per build tuple
constexpr uint32_t kNPRegionBuckets = 1024;           // NoPartitioning region build: buckets per region (LDS 60 B each)
constexpr int kOnePassMax = 256;                      // hash % P: largest P partitioned in one pass

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// Launch-shape knobs (results never depend on them). Defaults are the tuned
// values; ctx_create_device reads their PHJ_* overrides (every one is run by
// tests/test_gpu_schedules.py).
struct Tuning {
    int tile = 4096;      // tile kernels: tuples per tile (2048, 4096 or 8192)
    int block = 512;      // threads per workgroup of the tile kernels (256, 512 or 1024; tile_shape)
    int nt_load = 1;      // nontemporal tuple loads in the partition passes: 1 pass 1, 2 both
    bool fused = true;    // radix join: fused per-partition LDS build + probe when partitions are small
    int ptab = 1;         // partitioned bucket tables: 0 never, 1 very large partitions, 2 always
    bool subpart = true;  // phj_join: sub-partition large partitions for the fused join
    bool timers = true;   // per-kernel timer events (phase events are always recorded)
    bool p1_chunk = true; // 2-pass, unordered partitions: chunked pass 1 without a histogram pass
    int p1_slots = 0;     // chunked pass 1: workgroups per shard (0 = fill the chip once, -1 = one per tile)
    int p1_wpc2 = 2;      // ... keys-only: workgroups per CU x 2 (0 = fill the chip once)
    int p1_tps = static_cast<int>(kTilesPerShard);   // chunked pass 1: tiles per shard (sets the shard count)
    int p1_min_tiles = 32768;  // chunked pass 1: smallest relation (in 4096-tuple tiles, ~134M tuples)
    int p1_ko_tps = 1024;      // ... the keys-only form for the on-chip probe: tiles per shard (at every size)
    int p2probe = 1;      // radix join, 2 passes: the probe side's pass 2 on-chip (k_probe_ht)
    int p1_pipe = 1;      // keys-only pass 1: claims resolved a tile later over pre-allocated chunks (k_chunk_codes_pipe)
    int r_chunk = 1;      // LDS join on one device: R through the chunked code pass, read by tiles ("tile mode")
    int count_pin = 1;    // LDS join: the last workgroup writes the count to pinned host memory (0: a copy back)
    int r_order = 1;      // LDS join: R's pass 1 beside S's (0), after it (1: measured C2 1.69 vs 1.72 ms, S.p1 1.05 vs 1.19), before it (2)
    int p1_block = 1024;  // ... its workgroup: 1024 x 4 codes (16 waves per CU; measured 1.20 -> 1.07 ms at C2) or 512 x 8, the same tile
    int cluster = 1;      // radix join: LDS cluster tables (phj_cluster.h) when the build side's clusters fit
    int cl_cap = static_cast<int>(kClCapMax);   // ... LDS table slots (8192: two workgroups per CU, 16384: one)
    int cl_bits = 0;      // ... clusters = 2^cl_bits (0: the fewest >= 256 whose average fits the table)
};

int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}

struct Plan {
    int hk = 0;
    uint64_t seed = 0;
    uint32_t mode = 0;    // 0: q = h & (P-1), 1: q = h % P
    uint64_t P = 0;       // logical partitions
    uint32_t npass = 1;
    uint32_t nb1 = 1, nb2 = 1;
    uint32_t bits1 = 0, bits2 = 0;
    uint32_t shift1 = 0, dmask1 = 0, dmask2 = 0;
    uint32_t Ppad = 1;    // nb1 * nb2 = final bounds length - 1
    uint32_t sub_bits = 0, sub_shift = 0;   // phj_join: sub-partitions per partition (refine_plan)
    bool stable = false;  // PHJ_PART_STABLE: the reference's order inside each partition (not compared by ==)
    bool chained = false; // PHJ_TABLE_CHAINED: bucket-chained (CSR) tables in HBM (not compared by ==: tables only)
    bool cluster = false; // phj_join: pass 1 = the LDS join's clusters (cluster_plan), the count path of phj_cluster.h
    bool operator==(const Plan& o) const {
        return hk == o.hk && seed == o.seed && mode == o.mode && P == o.P && npass == o.npass &&
               nb1 == o.nb1 && nb2 == o.nb2 && sub_bits == o.sub_bits && sub_shift == o.sub_shift;
    }
};

struct TimerRec {
    std::string name;
    uint64_t bytes;
    hipEvent_t a, b;
    int split = 0;   // 1 / 2: the build / probe share of a fused join launch (ctx->split clocks)
};

struct SideState {
    const phj_tuple* rel = nullptr;
    uint64_t n = 0;
    DevBuf owned;
    DevBuf kA, pA, kB, pB;
    DevBuf hist1, hist2, bounds1, tbase2, tseg2, bounds, partials;
    DevBuf dig;           // pass-2 digit column written by pass 1
    DevBuf ccur, ctab, tstart;   // chunked pass 1: digit cursors + pool counter, chunk table, pass-2 tile starts
    DevBuf csink;                // ... code form: sink words of the stores past the tile (never read)
    bool ctab_dirty = true;      // chunked pass 1: the chunk table may hold entries (clear before the next pass)
    bool hcoded = false;         // the last pass 1 wrote hash codes (keys only, k_chunk_codes)
    bool chunk_check = false;    // a chunked pass ran whose error word (chunk_err_word) nobody has read yet
    phj_partitioned view{};
    PassArgs p2{};               // p1_only: the pass-2 tile mapping over the pass-1 output
    uint32_t nt2 = 0;            // ... and its tile bound
    bool partitioned = false;
    Plan plan;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

uint32_t ceil_log2(uint64_t x) {
    uint32_t b = 0;
    while ((1ull << b) < x) b++;
    return b;
}

uint32_t next_pow2_u32(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

struct Group;   // phj_group.h: the members of a multi-device context

}  // namespace

struct phj_ctx {
    Group* group = nullptr;        // multi-device context (phj_group.h); null for one device
    int device = 0;
    hipStream_t stream = nullptr;  // the ctx stream (own or borrowed)
    hipStream_t aux = nullptr;     // ctx-owned: R-side partitioning runs here beside S
    hipStream_t ks = nullptr;      // stream the current launches go to (stream or aux)
    DevBuf* scan_scratch = nullptr; // scan partials of the side being partitioned
    int num_cus = 256;
    bool own_stream = false;
    SideState side[2];
    DevBuf scan_partials, prep, tkeys, tpays, toffs, gcursor, items, count, biglist;
    DevBuf ht_tab, ht_desc;   // on-chip join: code tables, descriptors (build_ht)
    DevBuf r_codes, r_bounds;         // ... the build side's codes in partition order and bounds (single device)
    DevBuf np_tab, np_pays;
    DevBuf np_ovf, np_ovfb, np_ovfn;   // region build: overflow tuples, their start buckets, count
    DevBuf np_uni;                     // code-table NoPartitioning: {uniform?, cap} (k_np_ct_plan)
    DevBuf fitems, split, cl_prof;
    DevBuf mat_mark, mat_cnt, mat_rows;   // materialised join: per-probe match, block offsets, rows
    uint64_t mat_n = 0;   // fused join: item slots; wave clocks {build, probe} since the last timer reset
    std::vector<hipEvent_t> evpool;
    size_t evnext = 0;
    std::vector<TimerRec> timers;
    std::string err;
    Tuning tune;
    bool last_fused = false;   // the last build_and_probe ran the fused kernel
    bool dry = false;          // phj_prepare: size and allocate the workspace, launch nothing
    hipEvent_t last_ev = nullptr;      // the last event recorded (mark) ...
    hipStream_t last_ev_stream = nullptr;  // ... on this stream ...
    uint32_t since_ev = 0;             // ... and the kernels launched since
    unsigned long long* count_host = nullptr;   // pinned: the count read back
    // fine-grained pinned {count, failed} written by the LDS join's last
    // workgroup (k_cluster_probe_big), its device address, and the launch's
    // finished-workgroup counter; count_pinned: this join's count is there
    unsigned long long* count_pin = nullptr;
    unsigned long long* count_pin_dev = nullptr;
    DevBuf cl_done;
    bool count_pin_failed = false, count_pinned = false;
    unsigned long long* split_words = nullptr;  // the LDS probe's {build, probe} clocks (count buffer words 2-3), this join
    bool defer_timers = false;  // the running join has PHJ_DEFER_TIMERS: its timers stay for phj_timers_report
    bool lean_timers = false;   // PHJ_LEAN_TIMERS: the build side's timers are not recorded
    bool timer_skipped = false; // the open timer was not recorded (timer_end records nothing)
    // the next chunked pass-1 bookkeeping kernel also clears this chunk state
    // (the LDS join: R's, cleared by S's k_pass1_finish_sizes on the same
    // stream), and the pass whose state p1_cleared names skips its memset
    void* p1_clear = nullptr;
    size_t p1_clear_bytes = 0;
    void* p1_cleared = nullptr;
    // the probe side's chunk state left all zero by the last join's final
    // workgroup (k_cluster_probe_big, s_clear) and its size; pending: asked
    // of the running join, confirmed when its count shows no failure
    void* s_zeroed = nullptr;
    size_t s_zeroed_bytes = 0;
    void* s_zero_pending = nullptr;
    size_t s_zero_pending_bytes = 0;
    int poison = -1;   // phj_debug_poison_alloc: every new workspace buffer is filled with this byte
};

namespace {

int set_err(phj_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define PHJ_HIP(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err(ctx, PHJ_ERR_HIP,                                                 \
                           std::string(#expr) + ": " + hipGetErrorString(e_));               \
    } while (0)

#define PHJ_LAUNCHED(ctx, what)                                                              \
    do {                                                                                     \
        (ctx)->since_ev++;                                                                   \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ != hipSuccess)                                                                \
            return set_err(ctx, PHJ_ERR_HIP, std::string("launch ") + what + ": " +         \
                                                 hipGetErrorString(e_));                     \
    } while (0)

#define PHJ_TRY(expr)           \
    do {                        \
        int rc_ = (expr);       \
        if (rc_ != PHJ_OK) return rc_; \
    } while (0)

int ensure(phj_ctx* c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return PHJ_OK;
    if (b.p) {
        PHJ_HIP(c, hipStreamSynchronize(c->stream));
        PHJ_HIP(c, hipStreamSynchronize(c->aux));
        PHJ_HIP(c, hipFree(b.p));
        b.p = nullptr;
        b.bytes = 0;
    }
    const size_t rounded = (bytes + 4095) & ~size_t(4095);
    hipError_t e = hipMalloc(&b.p, rounded);
    if (e != hipSuccess) {
        b.p = nullptr;
        return set_err(c, PHJ_ERR_NOMEM, "hipMalloc(" + std::to_string(rounded) + "): " + hipGetErrorString(e));
    }
    b.bytes = rounded;
    if (c->poison >= 0) {   // (test hook) no buffer may be read before it is written
        PHJ_HIP(c, hipMemsetAsync(b.p, c->poison, rounded, c->stream));
        PHJ_HIP(c, hipStreamSynchronize(c->stream));
    }
    return PHJ_OK;
}

void free_buf(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

hipEvent_t new_event() {
    hipEvent_t e = nullptr;
    // timing / same-device ordering only: no system-scope fence (a default
    // event's system-scope writeback costs ~10 us per record); the first
    // flag set the runtime accepts is used
    const unsigned tries[3] = {hipEventDisableSystemFence, hipEventReleaseToDevice, hipEventDefault};
    for (unsigned f : tries) {
        if (hipEventCreateWithFlags(&e, f) == hipSuccess) break;
        (void)hipGetLastError();
        e = nullptr;
    }
    return e;
}

hipEvent_t next_event(phj_ctx* c) {
    if (c->evnext == c->evpool.size()) {
        hipEvent_t e = new_event();
        if (!e) return nullptr;
        c->evpool.push_back(e);
    }
    return c->evpool[c->evnext++];
}

// phj_prepare: events for this many timer marks created up front (deferred
// timers keep every join's marks until phj_timers_report, ~4 per join under
// PHJ_LEAN_TIMERS: 64 joins' worth), so no hipEventCreate runs inside a timed loop
constexpr size_t kPrepEvents = 256;
int reserve_events(phj_ctx* c, size_t n) {
    while (c->evpool.size() < n) {
        hipEvent_t e = new_event();
        if (!e) return set_err(c, PHJ_ERR_HIP, "hipEventCreate failed");
        c->evpool.push_back(e);
    }
    if (c->timers.capacity() < n) c->timers.reserve(n);
    return PHJ_OK;
}

int mark(phj_ctx* c, hipEvent_t* out) {
    *out = next_event(c);
    if (!*out) return set_err(c, PHJ_ERR_HIP, "hipEventCreate failed");
    PHJ_HIP(c, hipEventRecord(*out, c->ks));
    c->last_ev = *out;
    c->last_ev_stream = c->ks;
    c->since_ev = 0;
    return PHJ_OK;
}

// mark, or the last event when it was recorded on this stream with nothing
// launched after it (the same point of the stream: one marker packet fewer)
int mark_shared(phj_ctx* c, hipEvent_t* out) {
    if (c->last_ev && c->last_ev_stream == c->ks && c->since_ev == 0) {
        *out = c->last_ev;
        return PHJ_OK;
    }
    return mark(c, out);
}

int timer_begin(phj_ctx* c, const char* name, uint64_t bytes) {
    if (!c->tune.timers) return PHJ_OK;
    c->timer_skipped = c->lean_timers && (std::strncmp(name, "R.", 2) == 0 || std::strcmp(name, "build.big") == 0);
    if (c->timer_skipped) return PHJ_OK;   // PHJ_LEAN_TIMERS
    TimerRec t{name, bytes, nullptr, nullptr};
    // back-to-back timers on one stream share the boundary event (the previous
    // timer's end is this one's start when nothing was launched in between)
    if (c->last_ev && c->last_ev_stream == c->ks && c->since_ev == 0) t.a = c->last_ev;
    else PHJ_TRY(mark(c, &t.a));
    c->timers.push_back(t);
    return PHJ_OK;
}

// Launch kfn on the current launch stream.
int launch_kernel(phj_ctx* c, const void* kfn, dim3 grid, dim3 block, void** args, size_t lds, const char* what) {
    PHJ_HIP(c, hipLaunchKernel(kfn, grid, block, args, lds, c->ks));
    PHJ_LAUNCHED(c, what);
    return PHJ_OK;
}

int timer_end(phj_ctx* c) {
    if (c->timer_skipped) {
        c->timer_skipped = false;
        return PHJ_OK;
    }
    return c->tune.timers ? mark(c, &c->timers.back().b) : PHJ_OK;
}

// One launch reported as two timers (build, probe) split by the kernel's own clocks.
int timer_begin_split(phj_ctx* c, uint64_t build_bytes, uint64_t probe_bytes) {
    if (!c->tune.timers) return PHJ_OK;
    PHJ_TRY(timer_begin(c, "build", build_bytes));
    c->timers.back().split = 1;
    c->timers.push_back(TimerRec{"probe", probe_bytes, c->timers.back().a, nullptr, 2});
    return PHJ_OK;
}

int timer_end_split(phj_ctx* c) {
    if (!c->tune.timers) return PHJ_OK;
    PHJ_TRY(mark(c, &c->timers.back().b));
    c->timers[c->timers.size() - 2].b = c->timers.back().b;
    return PHJ_OK;
}

constexpr size_t kMaxTimerRecs = 1u << 14;

void reset_timers(phj_ctx* c) {
    c->timers.clear();
    c->evnext = 0;
    c->last_ev = nullptr;
    c->split_words = nullptr;
    if (c->split.p) (void)hipMemsetAsync(c->split.p, 0, 16, c->ks);
}

// Build share of the fused join launches since the last reset (wave clocks).
double fused_build_fraction(phj_ctx* c) {
    unsigned long long cyc[2] = {0, 0};
    const void* src = c->split_words ? static_cast<const void*>(c->split_words) : c->split.p;
    if (!src || hipMemcpyAsync(cyc, src, 16, hipMemcpyDeviceToHost, c->ks) != hipSuccess ||
        hipStreamSynchronize(c->ks) != hipSuccess)
        return 0.5;
    const double t = static_cast<double>(cyc[0]) + static_cast<double>(cyc[1]);
    return t > 0 ? static_cast<double>(cyc[0]) / t : 0.5;
}

// Timers aggregated by name (sums over every record since the last reset:
// one join, or many when a caller reports once after several joins).
int fill_timers(phj_ctx* c, phj_join_result* r) {
    r->num_timers = 0;
    if (c->defer_timers) return PHJ_OK;   // PHJ_DEFER_TIMERS: read later by phj_timers_report
    double fb = -1.0;
    for (const TimerRec& t : c->timers) {
        float ms = 0;
        PHJ_HIP(c, hipEventElapsedTime(&ms, t.a, t.b));
        if (t.split) {
            if (fb < 0) fb = fused_build_fraction(c);
            ms = static_cast<float>(ms * (t.split == 1 ? fb : 1.0 - fb));
        }
        uint32_t i = 0;
        while (i < r->num_timers && std::strncmp(r->timer_name[i], t.name.c_str(), PHJ_TIMER_NAME - 1) != 0) i++;
        if (i == r->num_timers) {
            if (r->num_timers >= PHJ_MAX_TIMERS) continue;
            r->num_timers++;
            r->timer_ms[i] = 0;
            r->timer_bytes[i] = 0;
            std::snprintf(r->timer_name[i], PHJ_TIMER_NAME, "%s", t.name.c_str());
        }
        r->timer_ms[i] += ms;
        r->timer_bytes[i] += t.bytes;
    }
    return PHJ_OK;
}

double elapsed(phj_ctx* c, hipEvent_t a, hipEvent_t b) {
    if (c->defer_timers) return 0.0;   // PHJ_DEFER_TIMERS: no event queries in the join
    float ms = 0;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return -1.0;
    return ms;
}

int make_plan(phj_ctx* c, const phj_join_params* p, Plan& pl) {
    if (!p) return set_err(c, PHJ_ERR_INVALID, "null params");
    if (p->hash != PHJ_HASH_XXH3 && p->hash != PHJ_HASH_MURMUR3)
        return set_err(c, PHJ_ERR_INVALID, "unknown hash function");
    pl = Plan{};
    pl.stable = (p->flags & PHJ_PART_STABLE) != 0;
    pl.chained = (p->flags & PHJ_TABLE_CHAINED) != 0;
    pl.hk = p->hash;
    pl.seed = p->hash_seed;
    if (p->num_partitions > 0) {
        pl.mode = 1;
        pl.P = p->num_partitions;
        // one pass while the scatter's runs stay long (a 4096-tuple tile over
        // <= 256 digits); beyond, two passes with balanced digits: pass 1 on
        // q >> b2, pass 2 on q & (2^b2 - 1), 2^b2 ~ sqrt(P)
        if (pl.P <= static_cast<uint64_t>(kOnePassMax)) {
            pl.npass = 1;
            pl.nb1 = static_cast<uint32_t>(pl.P);
            pl.bits1 = ceil_log2(pl.P);
            pl.shift1 = 0;
            pl.dmask1 = 0xffffffffu;
        } else {
            if (pl.P > (1ull << (2 * kMaxDigitBits)))
                return set_err(c, PHJ_ERR_RANGE, "num_partitions above 2^22");
            const uint32_t b2 = std::min<uint32_t>(kMaxDigitBits, (ceil_log2(pl.P) + 1) / 2);
            pl.npass = 2;
            pl.nb2 = 1u << b2;
            pl.bits2 = b2;
            pl.nb1 = static_cast<uint32_t>((pl.P + pl.nb2 - 1) / pl.nb2);
            pl.bits1 = ceil_log2(pl.nb1);
            pl.shift1 = b2;
            pl.dmask1 = 0xffffffffu;
            pl.dmask2 = pl.nb2 - 1;
        }
    } else {
        const uint32_t b0 = p->radix_bits[0], b1 = p->radix_bits[1];
        if (b0 < 1 || b0 > static_cast<uint32_t>(kMaxDigitBits) || b1 > static_cast<uint32_t>(kMaxDigitBits))
            return set_err(c, PHJ_ERR_INVALID, "radix_bits must be in [1,11] x [0,11]");
        pl.mode = 0;
        pl.P = 1ull << (b0 + b1);
        pl.nb1 = 1u << b0;
        pl.bits1 = b0;
        pl.dmask1 = pl.nb1 - 1;
        pl.shift1 = b1;
        if (b1 == 0) {
            pl.npass = 1;
        } else {
            pl.npass = 2;
            pl.nb2 = 1u << b1;
            pl.bits2 = b1;
            pl.dmask2 = pl.nb2 - 1;
        }
    }
    pl.Ppad = pl.nb1 * pl.nb2;
    return PHJ_OK;
}

// phj_join only: when the requested partitions are too large for the fused LDS
// join (the reference's -p 32 .. 8192 at 10M build tuples), split every
// partition into 2^s sub-partitions of ~<= 170 build tuples (DigitFn sub_bits)
// and partition on the refined q in two balanced passes. The count is the
// same (a partition's hash table is simply organised by further hash bits);
// phj_partition keeps the exact layout of the requested partitions.
void refine_plan_sub(const phj_ctx* c, Plan& pl, uint64_t nR) {
    if (!c->tune.subpart || !c->tune.fused || pl.P == 0) return;
    const double expect = static_cast<double>(nR) / static_cast<double>(pl.P);
    if (expect * 3 <= static_cast<double>(kFusedTcap) * 2) return;
    const uint32_t logP = ceil_log2(pl.P);
    uint32_t s = 0;
    while (expect / static_cast<double>(1ull << s) > 170.0 && logP + s < 2u * kMaxDigitBits) s++;
    if (s == 0) return;
    pl.sub_bits = s;
    // radix: the hash bits just above the partition bits; hash % P: bits 40+
    // (the LDS table buckets use bits 32..39)
    pl.sub_shift = pl.mode == 0 ? logP : 40;
    const uint64_t range = (pl.mode == 0 ? (1ull << logP) : pl.P) << s;
    const uint32_t b2 = std::min<uint32_t>(kMaxDigitBits, (ceil_log2(range) + 1) / 2);
    pl.npass = 2;
    pl.nb2 = 1u << b2;
    pl.bits2 = b2;
    pl.dmask2 = pl.nb2 - 1;
    pl.nb1 = static_cast<uint32_t>((range + pl.nb2 - 1) / pl.nb2);
    pl.bits1 = ceil_log2(pl.nb1);
    pl.shift1 = b2;
    pl.dmask1 = 0xffffffffu;
    pl.Ppad = pl.nb1 * pl.nb2;
}

void refine_plan(const phj_ctx* c, Plan& pl, uint64_t nR) { refine_plan_sub(c, pl, nR); }

// The LDS join's plan (phj_cluster.h) from the requested one (make_plan):
// pass 1 partitions into K = 2^k clusters, the top k bits of the partition
// number q (refined by sub-partition bits when q has fewer than k bits: hash
// bits just above the radix bits, or bits 40+ under h % P, as refine_plan_sub),
// so every cluster is a union of whole requested partitions. K is the smallest
// power of two >= 256 (chains enough for S's pass-1 cursors) whose average
// cluster fills at most 0.8 of the LDS limit (the binomial spread of the
// cluster sizes, ~3 % at 10M / 1024); larger build sides than 2048 clusters
// hold take the code-table path. Returns false when the plan does not apply.
bool cluster_plan_k(const Plan& base, uint32_t k, Plan& pl) {
    pl = base;
    pl.cluster = true;
    pl.sub_bits = 0;
    pl.sub_shift = 0;
    uint32_t bits;   // bits of the (refined) partition number
    if (base.mode == 0) {
        const uint32_t logP = ceil_log2(base.P);
        if (logP < k) {
            pl.sub_bits = k - logP;
            pl.sub_shift = logP;
        }
        bits = std::max(logP, k);
    } else {
        uint32_t s = 0;
        while ((base.P << s) < (1ull << k)) s++;
        if (s) {
            pl.sub_bits = s;
            pl.sub_shift = 40;
        }
        bits = ceil_log2(base.P << s);
    }
    const uint64_t range = (base.mode == 0 ? (1ull << ceil_log2(base.P)) : base.P) << pl.sub_bits;
    const uint32_t shift = bits - k;
    pl.npass = 2;
    pl.shift1 = shift;
    pl.dmask1 = 0xffffffffu;
    pl.nb1 = static_cast<uint32_t>((range + (1ull << shift) - 1) >> shift);
    pl.bits1 = ceil_log2(pl.nb1);
    pl.nb2 = 1u << shift;
    pl.bits2 = shift;
    pl.dmask2 = pl.nb2 - 1;
    pl.Ppad = pl.nb1 * pl.nb2;
    return pl.nb1 >= 2 && pl.nb1 <= static_cast<uint32_t>(kMaxBins);
}

bool cluster_plan(const phj_ctx* c, const Plan& base, uint64_t nR, Plan& pl) {
    if (!c->tune.cluster || base.chained || nR == 0 || base.P == 0) return false;
    const double fit = 0.8 * cl_lim(static_cast<uint32_t>(c->tune.cl_cap));
    // h % P: the clusters are 2^shift consecutive refined partitions each, so
    // there may be fewer than 2^k of them; every k is tried until they fit
    const uint32_t k0 = c->tune.cl_bits > 0 ? static_cast<uint32_t>(c->tune.cl_bits) : 8;
    const uint32_t k1 = c->tune.cl_bits > 0 ? k0 : static_cast<uint32_t>(kMaxDigitBits);
    for (uint32_t k = k0; k <= k1; k++)
        if (cluster_plan_k(base, k, pl) && static_cast<double>(nR) / static_cast<double>(pl.nb1) <= fit) return true;
    return false;
}

DigitFn digit_fn(const Plan& pl, int pass) {
    DigitFn f{};
    f.seed = pl.seed;
    f.P = pl.P;
    f.mode = pl.mode;
    f.magic = pl.mode == 1 ? (~0ull) / pl.P : 0;
    f.sub_bits = pl.sub_bits;
    f.sub_shift = pl.sub_shift;
    if (pass == 1) {
        f.shift = pl.shift1;
        f.dmask = pl.dmask1;
    } else {
        f.shift = 0;
        f.dmask = pl.dmask2;
    }
    return f;
}


// E_0 of the plan's code tables (phj_table.h ht_empty): the lowest power of
// two whose final partition is not 0. Code 0 is in partition 0 under every
// partition function, so E_p = 0 serves every other partition. 1 for radix bits
// and h % P with P >= 2; 2^40 for h % 1 split into sub-partitions at bit 40
// (code 1 is in partition 0 there); 0 when the plan has one final partition
// (no code lies elsewhere: use_p2probe then declines the code tables).
uint64_t plan_empty0(const Plan& pl) {
    const DigitFn f = digit_fn(pl, 1);
    for (int b = 0; b < 64; b++)
        if (q_from_hash(1ull << b, f) != 0) return 1ull << b;
    return 0;
}

// E of cluster 0 (phj_cluster.h): the lowest power of two outside cluster 0
// (pass-1 digit 0); 0 when every code is in cluster 0.
uint64_t cluster_empty0(const Plan& pl) {
    const DigitFn f = digit_fn(pl, 1);
    for (int b = 0; b < 64; b++)
        if (((q_from_hash(1ull << b, f) >> f.shift) & f.dmask) != 0) return 1ull << b;
    return 0;
}

int scan_u32(phj_ctx* c, uint32_t* data, uint32_t len, uint32_t narrays, uint32_t stride,
             DevBuf* scratch = nullptr) {
    if (len == 0) return PHJ_OK;
    ScanArgs s{};
    s.data = data;
    s.len = len;
    s.stride = stride;
    s.nblk = (len + kScanBlockElems - 1) / kScanBlockElems;
    DevBuf& part = scratch ? *scratch : c->scan_partials;
    PHJ_TRY(ensure(c, part, static_cast<size_t>(s.nblk) * narrays * 4));
    if (c->dry) return PHJ_OK;
    s.partials = static_cast<uint32_t*>(part.p);
    hipLaunchKernelGGL(k_scan_reduce, dim3(s.nblk, narrays), dim3(kBlock), 0, c->ks, s);
    PHJ_LAUNCHED(c, "k_scan_reduce");
    hipLaunchKernelGGL(k_scan_apply, dim3(s.nblk, narrays), dim3(kBlock), 0, c->ks, s);
    PHJ_LAUNCHED(c, "k_scan_apply");
    return PHJ_OK;
}


// The pipelined code pass in 1024 x 4 workgroups: KPF tiles of keys in
// flight (S: 2, measured 1.08 -> 1.05 ms at C2; R: 1); a measurement build
// (-DPHJ_P1_PROF=1, scripts/ab_lib.sh) runs S's pass in the phase-clock form.
template <int HK, int DPT>
const void* pipe1024(int kpf) {
    if (kpf == 1) return reinterpret_cast<const void*>(&k_chunk_codes_pipe<1024, 4, HK, DPT, 0, false, 1>);
    return reinterpret_cast<const void*>(&k_chunk_codes_pipe<1024, 4, HK, DPT, 0, PHJ_P1_PROF != 0, 2>);
}

// Workgroups per CU of kernel kfn at `block` threads and `lds` bytes of dynamic
// LDS, as the runtime reports it (0 if it cannot), cached per host thread: the
// query reads the kernel's attributes through the runtime, host time before
// every launch of a join otherwise.
int occupancy(const void* kfn, int block, size_t lds) {
    struct Key {
        const void* f;
        int b;
        size_t l;
        bool operator==(const Key& o) const { return f == o.f && b == o.b && l == o.l; }
    };
    struct Hash {
        size_t operator()(const Key& k) const {
            return std::hash<const void*>()(k.f) ^ (static_cast<size_t>(k.b) << 20) ^ (k.l * 0x9E3779B97F4A7C15ull);
        }
    };
    thread_local std::unordered_map<Key, int, Hash> cache;
    const Key k{kfn, block, lds};
    auto it = cache.find(k);
    if (it != cache.end()) return it->second;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kfn, block, lds) != hipSuccess) {
        (void)hipGetLastError();
        occ = 0;
    }
    cache.emplace(k, occ);
    return occ;
}

template <int BLOCK, int ITEMS, bool IN_AOS, bool OUT_AOS>
int launch_pass_t(phj_ctx* c, int hk, const PassArgs& a, uint32_t grid, const std::string& prefix,
                  uint64_t n, uint32_t hist_len) {
    constexpr int T = BLOCK * ITEMS;
    constexpr int NW = BLOCK / 64;
    const size_t hist_lds = static_cast<size_t>(NW) * a.nbins * 4;
    const size_t sc_lds = scatter_lds_bytes(T, a.nbins, NW, a.chunk_cursor != nullptr);
    const std::string hname = prefix + ".hist", cname = prefix + ".scan", sname = prefix + ".scatter";
    if (a.chunk_cursor) {
        // chunked pass 1: no histogram / scan; the digit cursors and the pool
        // counter start at zero
        const bool zeroed = a.chunk_cursor == c->s_zeroed && chunk_state_bytes(a.nbins) <= c->s_zeroed_bytes;
        if (a.chunk_cursor == c->s_zeroed) c->s_zeroed = nullptr;   // (this pass writes it)
        if (a.chunk_cursor == c->p1_cleared) c->p1_cleared = nullptr;   // cleared by the kernel before it
        else if (!zeroed) PHJ_HIP(c, hipMemsetAsync(a.chunk_cursor, 0, chunk_state_bytes(a.nbins), c->ks));
        c->since_ev++;
        const uint64_t sbytes = n * (a.keys_only ? 24 : 32) + (a.out_dig ? n * (a.dig_wide ? 2 : 1) : 0);
        PHJ_TRY(timer_begin(c, sname.c_str(), sbytes));
        if constexpr (IN_AOS && OUT_AOS && ITEMS <= 8) {
            // persistent: as many workgroups per shard as fit the chip at once
            // (two per CU at 81 KB of LDS), never more than the shard's tiles
            const uint32_t ntiles = static_cast<uint32_t>((n + T - 1) / T);
            const uint32_t per = (ntiles + a.nshards - 1) / a.nshards;
            const bool pipe = a.keys_only && c->tune.p1_pipe && BLOCK == 512 && ITEMS == 8;
            const size_t lds = pipe ? chunk_pipe_lds_bytes(T, a.nbins) : a.keys_only ? chunk_codes_lds_bytes(T, a.nbins) : sc_lds;
            const void* kfn = nullptr;
            int kblock = BLOCK;
            // keys only, written as hash codes (the on-chip probe): k_chunk_codes;
            // whole tuples: VAR 3, LDS-atomic ranking, 16-B LDS entries (phj_partition.h)
            // (more digits than threads: the cluster plans, 512 x 4096 only)
            if (a.keys_only && pipe) {
                if constexpr (BLOCK == 512 && ITEMS == 8) {
                    const int dpt = a.nbins > 2 * BLOCK ? 4 : a.nbins > BLOCK ? 2 : 1;
                    if (c->tune.p1_block == 1024) {   // 16 waves per CU, 4 codes per thread
                        kblock = 1024;
                        // R's pass (LDS join, tile mode: ~10 tiles per workgroup at C2)
                        // keeps one tile in flight, which also gives it a kernel name of
                        // its own in rocprof summaries (S's is the roofline kernel)
                        const int kpf = prefix.rfind("R.", 0) == 0 ? 1 : 2;
                        kfn = hk == kMurmur3 ? (dpt == 4 ? pipe1024<kMurmur3, 2>(kpf) : pipe1024<kMurmur3, 1>(kpf))
                                             : (dpt == 4 ? pipe1024<kXXH3, 2>(kpf) : pipe1024<kXXH3, 1>(kpf));
                    } else if (hk == kMurmur3)
                        kfn = dpt == 4 ? reinterpret_cast<const void*>(&k_chunk_codes_pipe<BLOCK, ITEMS, kMurmur3, 4>)
                            : dpt == 2 ? reinterpret_cast<const void*>(&k_chunk_codes_pipe<BLOCK, ITEMS, kMurmur3, 2>)
                                       : reinterpret_cast<const void*>(&k_chunk_codes_pipe<BLOCK, ITEMS, kMurmur3, 1>);
                    else
                        kfn = dpt == 4 ? reinterpret_cast<const void*>(&k_chunk_codes_pipe<BLOCK, ITEMS, kXXH3, 4>)
                            : dpt == 2 ? reinterpret_cast<const void*>(&k_chunk_codes_pipe<BLOCK, ITEMS, kXXH3, 2>)
                                       : reinterpret_cast<const void*>(&k_chunk_codes_pipe<BLOCK, ITEMS, kXXH3, 1>);
                }
            } else if (a.keys_only) {
                if constexpr (BLOCK == 512 && ITEMS == 8) {
                    if (a.nbins > 2 * BLOCK)
                        kfn = hk == kMurmur3 ? reinterpret_cast<const void*>(&k_chunk_codes<BLOCK, ITEMS, kMurmur3, 4>)
                                             : reinterpret_cast<const void*>(&k_chunk_codes<BLOCK, ITEMS, kXXH3, 4>);
                    else if (a.nbins > BLOCK)
                        kfn = hk == kMurmur3 ? reinterpret_cast<const void*>(&k_chunk_codes<BLOCK, ITEMS, kMurmur3, 2>)
                                             : reinterpret_cast<const void*>(&k_chunk_codes<BLOCK, ITEMS, kXXH3, 2>);
                }
                if (!kfn && a.nbins > BLOCK) return set_err(c, PHJ_ERR_INVALID, "keys-only pass 1: more digits than threads");
                if (!kfn)
                    kfn = hk == kMurmur3 ? reinterpret_cast<const void*>(&k_chunk_codes<BLOCK, ITEMS, kMurmur3>)
                                         : reinterpret_cast<const void*>(&k_chunk_codes<BLOCK, ITEMS, kXXH3>);
            } else
                kfn = hk == kMurmur3 ? reinterpret_cast<const void*>(&k_scatter_chunked<BLOCK, ITEMS, kMurmur3, 3>)
                                     : reinterpret_cast<const void*>(&k_scatter_chunked<BLOCK, ITEMS, kXXH3, 3>);
            // workgroups per CU: what the LDS and the kernel's registers allow
            // (cached per kernel and LDS size; one cache per worker thread)
            const int occ = std::max(1, occupancy(kfn, kblock, lds));
            const uint32_t fit = std::max<uint32_t>(1, std::min<uint32_t>(static_cast<uint32_t>(occ), static_cast<uint32_t>(160 * 1024 / lds)));
            uint32_t slots = std::max<uint32_t>(1, std::min<uint32_t>(per, fit * c->num_cus / a.nshards));
            // keys-only (the on-chip join): PHJ_P1_WPC2 half-workgroups per CU, not
            // every slot the LDS allows, so R's partition and tables on the aux
            // stream get CUs beside S's persistent pass 1 instead of queueing behind it
            if (a.keys_only && c->tune.p1_wpc2 > 0)
                slots = std::max<uint32_t>(
                    1, std::min<uint32_t>(per, std::min<uint32_t>(fit * 2, static_cast<uint32_t>(c->tune.p1_wpc2)) *
                                                   c->num_cus / (2 * a.nshards)));
            if (c->tune.p1_slots > 0) slots = std::min<uint32_t>(per, c->tune.p1_slots);
            if (c->tune.p1_slots < 0) slots = per;   // one tile per workgroup
            PassArgs ak = a;
            const bool prof = PHJ_P1_PROF && pipe && kblock == 1024 && prefix.rfind("R.", 0) != 0;
            if (prof) {   // diagnostics (measurement build, PHJ_P1_PROF): synchronous, to stderr
                PHJ_TRY(ensure(c, c->cl_prof, 64 * 8));   // words 32.. (the LDS join's are 0..)
                ak.prof = static_cast<unsigned long long*>(c->cl_prof.p) + 32;
                PHJ_HIP(c, hipMemsetAsync(ak.prof, 0, kP1ProfWords * 8, c->ks));
            }
            void* kargs[] = {&ak, const_cast<uint32_t*>(&ntiles), const_cast<uint32_t*>(&per)};
            PHJ_TRY(launch_kernel(c, kfn, dim3(slots * a.nshards), dim3(kblock), kargs, lds, sname.c_str()));
            if (prof) {
                unsigned long long h[kP1ProfWords] = {};
                PHJ_HIP(c, hipMemcpyAsync(h, ak.prof, sizeof(h), hipMemcpyDeviceToHost, c->ks));
                PHJ_HIP(c, hipStreamSynchronize(c->ks));
                const double n = h[7] ? static_cast<double>(h[7]) : 1.0;
                std::fprintf(stderr, "p1_prof %s grid %u: cycles per tile: hash+rank %.0f B1 %.0f scan %.0f claims+B2 %.0f scatter+protocol %.0f B3 %.0f write %.0f; tiles %llu; "
                             "waves' max/mean B3->B1 %.0f/%.0f B1->B2 %.0f/%.0f B2->B3 %.0f/%.0f\n",
                             sname.c_str(), slots * a.nshards, h[0] / n, h[1] / n, h[2] / n, h[3] / n, h[4] / n, h[5] / n, h[6] / n, h[7],
                             h[8] / n, h[11] / n, h[9] / n, h[12] / n, h[10] / n, h[13] / n);
            }
        } else {
            (void)grid;
            return set_err(c, PHJ_ERR_INVALID, "chunked pass 1 needs AoS input and output, <= 8 tuples per thread");
        }
        return timer_end(c);
    }
    // algorithmic bytes: the histogram reads the key (a whole 16-B tuple when AoS)
    // or 1-2 B of a digit column; the scatter reads and writes every tuple once
    // (16 + 16 B) plus the digit column it leaves for pass 2
    const uint64_t hbytes = a.in_dig ? n * (a.dig_wide ? 2 : 1) : n * (IN_AOS ? 16 : 8);
    PHJ_TRY(timer_begin(c, hname.c_str(), hbytes));
    if (a.in_dig) {
        // wave per tile: 4 tiles per workgroup
        PassArgs ac = a;
        uint32_t cgrid = (grid + 3) / 4;
        cgrid = (cgrid + 7) & ~7u;
        const size_t clds = 4ull * a.nbins * 4;
        if (a.dig_wide)
            hipLaunchKernelGGL((k_hist_col<T, uint16_t>), dim3(cgrid), dim3(256), clds, c->ks, ac);
        else
            hipLaunchKernelGGL((k_hist_col<T, uint8_t>), dim3(cgrid), dim3(256), clds, c->ks, ac);
    } else if (hk == kMurmur3)
        hipLaunchKernelGGL((k_hist<BLOCK, ITEMS, IN_AOS, kMurmur3>), dim3(grid), dim3(BLOCK), hist_lds, c->ks, a);
    else
        hipLaunchKernelGGL((k_hist<BLOCK, ITEMS, IN_AOS, kXXH3>), dim3(grid), dim3(BLOCK), hist_lds, c->ks, a);
    PHJ_LAUNCHED(c, hname);
    PHJ_TRY(timer_end(c));
    PHJ_TRY(timer_begin(c, cname.c_str(), static_cast<uint64_t>(hist_len) * 12));
    PHJ_TRY(scan_u32(c, a.hist, hist_len, 1, hist_len, c->scan_scratch));
    PHJ_TRY(timer_end(c));
    PHJ_TRY(timer_begin(c, sname.c_str(), n * 32 + (a.out_dig ? n * (a.dig_wide ? 2 : 1) : 0)));
    if (hk == kMurmur3) {
        hipLaunchKernelGGL((k_scatter<BLOCK, ITEMS, IN_AOS, OUT_AOS, kMurmur3>), dim3(grid), dim3(BLOCK), sc_lds, c->ks, a);
    } else {
        hipLaunchKernelGGL((k_scatter<BLOCK, ITEMS, IN_AOS, OUT_AOS, kXXH3>), dim3(grid), dim3(BLOCK), sc_lds, c->ks, a);
    }
    PHJ_LAUNCHED(c, sname);
    PHJ_TRY(timer_end(c));
    return PHJ_OK;
}

// Workgroup size and tile of the tile kernels: the tuned shape when it is one
// of the compiled ones and its scatter fits the LDS, else 512 x 4096.
struct TileShape {
    int block, tile;
};

TileShape tile_shape(const phj_ctx* c, uint32_t nb) {
    const int b = c->tune.block, t = c->tune.tile;
    const bool compiled = (b == 256 && (t == 2048 || t == 4096)) || (b == 512 && (t == 2048 || t == 4096 || t == 8192)) ||
                          (b == 1024 && t == 8192);
    if (compiled && scatter_lds_bytes(t, nb, b / 64) <= 160 * 1024) return TileShape{b, t};
    return TileShape{512, 4096};
}

// One partition pass over `ntiles` tiles (an upper bound for segmented passes).
int launch_pass(phj_ctx* c, int hk, bool in_aos, bool out_aos, PassArgs a, uint32_t ntiles,
                const std::string& prefix, uint64_t n, uint32_t hist_len) {
    if (ntiles == 0) return PHJ_OK;
    uint32_t grid = ntiles;
    grid = (ntiles + 7) & ~7u;
    a.xcd_remap = 1;
    const TileShape sh = tile_shape(c, a.nbins);
    const int io = (in_aos ? 2 : 0) + (out_aos ? 1 : 0);
#define PHJ_PASS_CASES(B, I)                                                        \
    switch (io) {                                                                   \
        case 0: return launch_pass_t<B, I, false, false>(c, hk, a, grid, prefix, n, hist_len); \
        case 2: return launch_pass_t<B, I, true, false>(c, hk, a, grid, prefix, n, hist_len);  \
        case 3: return launch_pass_t<B, I, true, true>(c, hk, a, grid, prefix, n, hist_len);   \
        default: return set_err(c, PHJ_ERR_INVALID, "unsupported pass layout");     \
    }
    a.nt_store = 0;
    // nontemporal tuple loads: 1 = the chunked pass 1 only (the relation is read
    // once there; the stable pass 1 re-reads it after its histogram, and at
    // 25-100M tuples that re-read is measured 0.01-0.02 ms slower with them),
    // 2 = every pass
    a.nt_load = (c->tune.nt_load == 2 || (c->tune.nt_load == 1 && a.chunk_cursor != nullptr && prefix.size() >= 3 &&
                                         prefix.compare(prefix.size() - 3, 3, ".p1") == 0)) ? 1u : 0u;
    if (sh.block == 256 && sh.tile == 2048) PHJ_PASS_CASES(256, 8)
    if (sh.block == 256 && sh.tile == 4096) PHJ_PASS_CASES(256, 16)
    if (sh.block == 512 && sh.tile == 2048) PHJ_PASS_CASES(512, 4)
    if (sh.block == 512 && sh.tile == 8192) PHJ_PASS_CASES(512, 16)
    if (sh.block == 1024 && sh.tile == 8192) PHJ_PASS_CASES(1024, 8)
    PHJ_PASS_CASES(512, 8)
#undef PHJ_PASS_CASES
}

// Whether partition_state takes the chunked pass 1 for n tuples under plan pl
// (ko: the keys-only code form of the counting joins). Chunked pass 1
// (unordered partitions, tile kernels): pass-1 chunks are the pass-2 tiles,
// every digit's run of a tile fits one workgroup thread (nb1 <= block) and
// spans at most two chunks (tile1 == tile2), and every pool slot of the
// shards' pools is a uint32 (the pool bound below).
// Measured: it pays at 200M tuples (16 chains per digit) and
// loses to the stable pass below ~100M, where fewer shards (more
// workgroups per cursor line) or more partial chunks cost more than the
// histogram read saves; so it starts at p1_min_tiles tiles. The keys-only
// form for the on-chip probe (half the bytes, three workgroups per CU)
// wins at every size measured (25M-200M), with shards of p1_ko_tps tiles.
// use_cluster asks the same of the probe side (the LDS join needs S's codes).
bool chunked_pass1(const phj_ctx* c, const Plan& pl, uint64_t n64, bool ko) {
    if (pl.npass != 2 || pl.stable || !c->tune.p1_chunk || n64 == 0 || n64 >= (1ull << 32) - 2 * 4096) return false;
    const uint64_t n = n64;
    const TileShape sh = tile_shape(c, pl.nb1);
    const uint32_t tile = sh.tile;
    if (tile != tile_shape(c, pl.nb2).tile) return false;
    if (!ko && (n + tile - 1) / tile < static_cast<uint64_t>(c->tune.p1_min_tiles)) return false;
    if (pl.nb1 > static_cast<uint32_t>(sh.block) * (ko && sh.block == 512 && tile == 4096 ? 4u : 1u)) return false;
    if (tile / sh.block > 8) return false;   // registers: the next tile is prefetched
    if ((3 * (n / tile + kShards) + kShards * pl.nb1) * tile >= (1ull << 32)) return false;
    const bool pipe = ko && c->tune.p1_pipe && sh.block == 512 && tile == 4096;
    // the pipelined code pass's pool (pipe_pool_stride per shard)
    if (pipe && ((kPipeRes + 1) * (n / tile + kShards) + kShards * (3ull * pl.nb1 + 1)) * tile >= (1ull << 32)) return false;
    return true;
}

int partition_state(phj_ctx* c, SideState& S, const char* tag, const Plan& pl, bool p1_only,
                    unsigned long long* zero = nullptr, uint32_t max_shards = kShards) {
    c->scan_scratch = &S.partials;
    if (!S.rel && S.n > 0) return set_err(c, PHJ_ERR_STATE, "relation not bound");
    const uint64_t n64 = S.n;
    if (n64 >= (1ull << 32) - 2 * 4096) return set_err(c, PHJ_ERR_RANGE, "relation above 2^32 tuples per device");
    const uint32_t n = static_cast<uint32_t>(n64);
    const uint32_t tile = tile_shape(c, pl.nb1).tile;
    const uint32_t tile2 = pl.npass == 2 ? tile_shape(c, pl.nb2).tile : 0;
    const uint32_t nt1 = (n + tile - 1) / tile;
    const bool p1_aos = pl.npass == 2;
    // pass 1 leaves the pass-2 digit in a column (tile kernels only)
    // (p1_only: the probe re-hashes the keys itself, nothing reads the column)
    const bool dcol = pl.npass == 2 && !p1_only;
    const uint32_t dbytes = pl.bits2 > 8 ? 2 : 1;
    // Chunked pass 1 (unordered partitions, tile kernels): pass-1 chunks are
    // the pass-2 tiles, every digit's run of a tile fits one workgroup thread
    // (nb1 <= block) and spans at most two chunks (tile1 == tile2).
    // Measured: it pays at 200M tuples (16 chains per digit) and
    // loses to the stable pass below ~100M, where fewer shards (more
    // workgroups per cursor line) or more partial chunks cost more than the
    // histogram read saves; so it starts at p1_min_tiles tiles. The keys-only
    // form for the on-chip probe (half the bytes, three workgroups per CU)
    // wins at every size measured (25M-200M), with shards of p1_ko_tps tiles.
    const bool ko = p1_only;
    const bool chunked = chunked_pass1(c, pl, n64, ko);
    S.hcoded = chunked && ko;   // k_chunk_codes
    // chains per digit: ~kTilesPerShard tiles each, a power of two <= kShards
    // (max_shards < kShards: R in tile mode takes exactly that many, so a
    // cluster below the LDS limit has at most max_shards + lim / tile runs)
    uint32_t nshards = 1;
    const uint32_t tps = max_shards < kShards ? std::max<uint32_t>(1, (nt1 + max_shards - 1) / max_shards)
                                              : static_cast<uint32_t>(ko ? c->tune.p1_ko_tps : c->tune.p1_tps);
    while (nshards < max_shards && static_cast<uint64_t>(nshards) * tps < nt1) nshards <<= 1;
    // pool of pass-1 chunks, one region per shard: a shard takes at most
    // `per` tiles, each with two chunks reserved up front (k_scatter_chunked, k_chunk_codes;
    // unused ones are never touched), then at most per + nb1 chunks for its
    // chains' other starts (each chain wastes at most one partial chunk)
    const uint32_t per = (nt1 + nshards - 1) / nshards;
    // (the pipelined code pass: 2 static chunks per chain, kPipeRes per tile, then its counter)
    const bool pipe = ko && c->tune.p1_pipe && tile_shape(c, pl.nb1).block == 512 && tile == 4096;
    const uint32_t pool_stride = pipe ? pipe_pool_stride(per, pl.nb1) : 3 * per + pl.nb1;
    const uint32_t maxch = per + 1;   // chunks of one chain (every tuple of a shard in one digit)
    const size_t slots1 = chunked ? static_cast<size_t>(nshards) * pool_stride * tile : n;
    // pass-2 tiles (bound): one partial tile per segment, or per chain when chunked
    const uint32_t nt2 = pl.npass != 2 ? 0 : (n + tile2 - 1) / tile2 + pl.nb1 * (chunked ? nshards : 1);
    const uint32_t nt2max = nt2 + 8;
    // workspace (grow-only; allocation is outside the timed phases on reuse)
    PHJ_TRY(ensure(c, S.kA, slots1 * (p1_aos ? 16 : 8)));
    if (!p1_aos) PHJ_TRY(ensure(c, S.pA, static_cast<size_t>(n) * 8));
    if (!chunked) PHJ_TRY(ensure(c, S.hist1, static_cast<size_t>(nt1) * pl.nb1 * 4));
    PHJ_TRY(ensure(c, S.bounds1, (static_cast<size_t>(pl.nb1) + 1) * 4));
    if (pl.npass == 2) {
        PHJ_TRY(ensure(c, S.kB, static_cast<size_t>(n) * 8));
        PHJ_TRY(ensure(c, S.pB, static_cast<size_t>(n) * 8));
        PHJ_TRY(ensure(c, S.tbase2, (static_cast<size_t>(pl.nb1) + 1) * 4));
        PHJ_TRY(ensure(c, S.hist2, (static_cast<size_t>(nt2) + 8) * pl.nb2 * 4));
        PHJ_TRY(ensure(c, S.tseg2, (static_cast<size_t>(nt2) + 8) * 4));
        PHJ_TRY(ensure(c, S.bounds, (static_cast<size_t>(pl.Ppad) + 1) * 4));
        if (dcol) PHJ_TRY(ensure(c, S.dig, slots1 * dbytes + 64));
    }
    if (chunked) {
        PHJ_TRY(ensure(c, S.ccur, chunk_state_bytes(pl.nb1)));
        if (ko) PHJ_TRY(ensure(c, S.csink, static_cast<size_t>(kSinkGroups) * std::max(1024, tile_shape(c, pl.nb1).block) * 8));
        PHJ_TRY(ensure(c, S.tstart, static_cast<size_t>(nt2max) * 8));   // tile_start, tile_cnt
        // all zero between passes (kPublished): cleared when new, and when a
        // pass that published entries never reached k_tile_chunks (an error)
        // (a reallocation can return the same address: compare the size)
        const size_t before = S.ctab.bytes;
        PHJ_TRY(ensure(c, S.ctab, static_cast<size_t>(nshards) * pl.nb1 * maxch * 8));
        if (S.ctab.bytes != before) S.ctab_dirty = true;
        if (S.ctab_dirty && !c->dry) {
            PHJ_HIP(c, hipMemsetAsync(S.ctab.p, 0, S.ctab.bytes, c->ks));
            S.ctab_dirty = false;
        }
    }
    if (c->dry) {   // scan scratch of both passes, then nothing is launched
        if (!chunked) PHJ_TRY(scan_u32(c, nullptr, nt1 * pl.nb1, 1, nt1 * pl.nb1, c->scan_scratch));
        if (pl.npass == 2 && n) PHJ_TRY(scan_u32(c, nullptr, nt2 * pl.nb2, 1, nt2 * pl.nb2, c->scan_scratch));
        return PHJ_OK;
    }
    // pass 1: AoS relation -> SoA columns A
    PassArgs a{};
    a.in_keys = reinterpret_cast<const int64_t*>(S.rel);
    a.out_keys = static_cast<int64_t*>(S.kA.p);
    a.out_pays = static_cast<int64_t*>(S.pA.p);
    a.hist = static_cast<uint32_t*>(S.hist1.p);
    a.seg_bounds = nullptr;
    a.tile_base = nullptr;
    a.nseg = 1;
    a.n = n;
    a.ntiles1 = nt1;
    a.nbins = pl.nb1;
    a.nbits = pl.bits1;
    a.f = digit_fn(pl, 1);
    if (dcol) {
        a.out_dig = S.dig.p;
        a.dig_wide = dbytes == 2 ? 1u : 0u;
        a.dig2_mask = pl.dmask2;
    }
    if (chunked) {
        // the counting probe consumes pass 1 on chip and reads only keys
        a.keys_only = ko ? 1u : 0u;
        a.chunk_cursor = static_cast<uint32_t*>(S.ccur.p);
        a.sink = static_cast<unsigned long long*>(S.csink.p);
        a.chunk_tab = static_cast<unsigned long long*>(S.ctab.p);
        a.maxch = maxch;
        a.pool_stride = pool_stride;
        a.nshards = nshards;
        S.ctab_dirty = n > 0;   // until k_tile_chunks has cleared what pass 1 publishes
        S.chunk_check = n > 0;
    }
    uint32_t* tb2 = pl.npass == 2 ? static_cast<uint32_t*>(S.tbase2.p) : nullptr;
    PHJ_TRY(launch_pass(c, pl.hk, true, p1_aos, a, nt1, std::string(tag) + ".p1", n, nt1 * pl.nb1));
    if (chunked) {
        uint4* clr = nullptr;   // another pass's chunk state, cleared here (c->p1_clear)
        if (c->p1_clear) {
            clr = static_cast<uint4*>(c->p1_clear);
            c->p1_cleared = c->p1_clear;
            c->p1_clear = nullptr;
        }
        {
            hipLaunchKernelGGL(k_pass1_finish_sizes, dim3(1), dim3(kFinSizesBlock), 0, c->ks, a.chunk_cursor, pl.nb1, nshards, n, tile2,
                               static_cast<uint32_t*>(S.bounds1.p), tb2, zero, clr, static_cast<uint32_t>(c->p1_clear_bytes / 16));
            PHJ_LAUNCHED(c, "k_pass1_finish_sizes");
        }
    } else {
        hipLaunchKernelGGL(k_pass1_finish, dim3(1), dim3(kFinBlock), 0, c->ks, a.hist, nt1, pl.nb1, n,
                           pl.npass == 2 ? tile2 : tile, static_cast<uint32_t*>(S.bounds1.p), tb2);
        PHJ_LAUNCHED(c, "k_pass1_finish");
    }
    if (pl.npass == 1) {
        S.view.keys = static_cast<const int64_t*>(S.kA.p);
        S.view.payloads = static_cast<const int64_t*>(S.pA.p);
        S.view.bounds = static_cast<const uint32_t*>(S.bounds1.p);
    } else {
        PassArgs b{};
        b.in_keys = static_cast<const int64_t*>(S.kA.p);
        b.in_pays = p1_aos ? nullptr : static_cast<const int64_t*>(S.pA.p);
        b.out_keys = static_cast<int64_t*>(S.kB.p);
        b.out_pays = static_cast<int64_t*>(S.pB.p);
        b.hist = static_cast<uint32_t*>(S.hist2.p);
        b.seg_bounds = static_cast<const uint32_t*>(S.bounds1.p);
        b.tile_base = tb2;
        b.tile_seg = static_cast<const uint32_t*>(S.tseg2.p);
        b.nseg = pl.nb1;
        b.keys_only = a.keys_only;
        if (n) {
            if (chunked) {
                uint32_t* ts = static_cast<uint32_t*>(S.tstart.p);
                uint32_t* tc = ts + nt2max;
                {
                    hipLaunchKernelGGL(k_tile_chunks, dim3((pl.nb1 * nshards + kWaves - 1) / kWaves), dim3(kBlock), 0, c->ks, tb2,
                                       static_cast<uint32_t*>(S.ccur.p), pl.nb1, nshards,
                                       static_cast<unsigned long long*>(S.ctab.p), maxch, pool_stride, tile2,
                                       static_cast<uint32_t*>(S.tseg2.p), ts, tc);
                    PHJ_LAUNCHED(c, "k_tile_chunks");
                }
                S.ctab_dirty = false;
                b.tile_start = ts;
                b.tile_cnt = tc;
            } else {   // stable layout: tile -> digit
                hipLaunchKernelGGL(k_tile_seg, dim3((pl.nb1 + kWaves - 1) / kWaves), dim3(kBlock), 0, c->ks, tb2,
                                   pl.nb1, static_cast<uint32_t*>(S.tseg2.p));
                PHJ_LAUNCHED(c, "k_tile_seg");
            }
        }
        b.n = n;
        b.ntiles1 = 0;
        b.nbins = pl.nb2;
        b.nbits = pl.bits2;
        b.f = digit_fn(pl, 2);
        if (dcol) {
            b.in_dig = S.dig.p;
            b.dig_wide = dbytes == 2 ? 1u : 0u;
        }
        const uint32_t grid2 = n ? nt2 : 0;
        if (p1_only) {   // the caller consumes the pass-2 tiles itself (k_probe_ht)
            S.p2 = b;
            S.nt2 = grid2;
            S.view = phj_partitioned{};
            S.partitioned = false;
            S.plan = pl;
            return PHJ_OK;
        }
        PHJ_TRY(launch_pass(c, pl.hk, p1_aos, false, b, grid2, std::string(tag) + ".p2", n, grid2 * pl.nb2));
        const uint32_t nbnd = pl.Ppad + 1;
        hipLaunchKernelGGL(k_pass2_bounds, dim3((nbnd + kBlock - 1) / kBlock), dim3(kBlock), 0, c->ks,
                           b.hist, tb2, b.seg_bounds, pl.nb1, pl.nb2, n, static_cast<uint32_t*>(S.bounds.p));
        PHJ_LAUNCHED(c, "k_pass2_bounds");
        S.view.keys = static_cast<const int64_t*>(S.kB.p);
        S.view.payloads = static_cast<const int64_t*>(S.pB.p);
        S.view.bounds = static_cast<const uint32_t*>(S.bounds.p);
    }
    S.view.n = n;
    S.view.num_partitions = pl.Ppad;
    S.partitioned = true;
    S.plan = pl;
    return PHJ_OK;
}

// zero: a word the pass-1 bookkeeping clears (the on-chip probe's count),
// or null
int partition_side(phj_ctx* c, int s, const Plan& pl, bool p1_only = false, unsigned long long* zero = nullptr) {
    return partition_state(c, c->side[s], s == PHJ_SIDE_BUILD ? "R" : "S", pl, p1_only, zero);
}

// Build over `nseg` partitioned build segments and probe the ctx's partitioned
// probe side. Records "build" and "probe" timers; returns events bracketing them.
int build_and_probe(phj_ctx* c, const Plan& pl, int nseg, const phj_partitioned* segs,
                    hipEvent_t* e_build0, hipEvent_t* e_build1, hipEvent_t* e_probe1) {
    SideState& PS = c->side[PHJ_SIDE_PROBE];
    if (!c->dry && (!PS.partitioned || !(PS.plan == pl)))
        return set_err(c, PHJ_ERR_STATE, "probe relation not partitioned with these params");
    if (nseg < 1 || nseg > kMaxSegs) return set_err(c, PHJ_ERR_INVALID, "nbuild must be in [1,16]");
    const uint32_t P = pl.Ppad;
    SegList L{};
    L.nseg = static_cast<uint32_t>(nseg);
    L.P = P;
    uint64_t nR = 0;
    for (int g = 0; g < nseg; g++) {
        if (segs[g].num_partitions != P)
            return set_err(c, PHJ_ERR_INVALID, "build segment partition count mismatch");
        L.seg[g].keys = segs[g].keys;
        L.seg[g].pays = segs[g].payloads;
        if ((segs[g].payloads == nullptr) != (segs[0].payloads == nullptr))
            return set_err(c, PHJ_ERR_INVALID, "build segments must all carry payloads or none");
        L.seg[g].bounds = segs[g].bounds;
        nR += segs[g].n;
    }
    if (nR >= (1ull << 32) - 1) return set_err(c, PHJ_ERR_RANGE, "build side above 2^32 tuples");
    const uint64_t nS = c->dry ? PS.n : PS.view.n;
    // fused when the average partition fits one LDS round with margin (larger
    // ones take extra rounds, each re-probing the item's S keys)
    if (!pl.chained && c->tune.fused && (nR + P - 1) / P * 3 <= static_cast<uint64_t>(kFusedTcap) * 2) {
        // fused per-partition join with LDS tables: HashJoin.hpp:267-303
        const size_t nslots = nS / kFusedChunk + P + 1;
        PHJ_TRY(ensure(c, c->fitems, nslots * sizeof(FusedItem)));
        PHJ_TRY(ensure(c, c->count, 32));
        if (!c->split.p) {
            PHJ_TRY(ensure(c, c->split, 16));
            PHJ_HIP(c, hipMemsetAsync(c->split.p, 0, 16, c->ks));
        }
        if (c->dry) return PHJ_OK;
        PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 8, c->ks));
        PHJ_TRY(mark(c, e_build0));
        // algorithmic bytes: R keys once (build), S keys once (probe)
        PHJ_TRY(timer_begin_split(c, nR * 8, nS * 8));
        hipLaunchKernelGGL(k_fused_items, dim3((P + kWaves - 1) / kWaves), dim3(kBlock), 0, c->ks,
                           PS.view.bounds, P, static_cast<FusedItem*>(c->fitems.p));
        PHJ_LAUNCHED(c, "k_fused_items");
        FusedArgs fa{};
        fa.L = L;
        fa.skeys = PS.view.keys;
        fa.sbounds = PS.view.bounds;
        fa.items = static_cast<const FusedItem*>(c->fitems.p);
        fa.nitems = static_cast<uint32_t>(nslots - 1);
        fa.count = static_cast<unsigned long long*>(c->count.p);
        fa.cycles = static_cast<unsigned long long*>(c->split.p);
        fa.seed = pl.seed;
        const void* kfn = pl.hk == kMurmur3 ? reinterpret_cast<const void*>(&k_join_fused<kMurmur3, kFusedKPL, kFusedTcap>)
                                            : reinterpret_cast<const void*>(&k_join_fused<kXXH3, kFusedKPL, kFusedTcap>);
        int per_cu = 0;
        if ((per_cu = occupancy(kfn, kBlock, 0)) < 1) per_cu = 2;
        const size_t wblocks = (nslots + kWaves - 1) / kWaves;
        const uint32_t grid = static_cast<uint32_t>(
            std::max<size_t>(1, std::min<size_t>(wblocks, static_cast<size_t>(per_cu) * c->num_cus)));
        void* kargs[] = {&fa};
        PHJ_HIP(c, hipLaunchKernel(kfn, dim3(grid), dim3(kBlock), kargs, 0, c->ks));
        PHJ_LAUNCHED(c, "k_join_fused");
        PHJ_TRY(timer_end_split(c));
        PHJ_TRY(mark(c, e_probe1));
        *e_build1 = *e_probe1;
        c->last_fused = true;
        return PHJ_OK;
    }
    c->last_fused = false;
    // very large partitions (the reference's -p 32 .. 128 at 10M build tuples):
    // partitioned bucket tables, whose build is one pass of atomics over all
    // tuples; the CSR build below gives each partition one workgroup (3.9 ms at
    // -p 32 against 0.76), while its probe is faster from -p 1024 up
    if (!pl.chained && (c->tune.ptab > 1 || (c->tune.ptab == 1 && (nR + P - 1) / P >= 65536))) {
        // partitioned bucket tables in HBM (large partitions)
        const uint32_t ratio_x256 = static_cast<uint32_t>(kNPDefaultRatio * 256);
        const size_t nbk_bound = static_cast<size_t>(nR) * ratio_x256 / 256 / kNPSlots + 2 * static_cast<size_t>(P) + 1;
        PHJ_TRY(ensure(c, c->np_tab, nbk_bound * sizeof(NPBucket)));
        PHJ_TRY(ensure(c, c->np_pays, nbk_bound * kNPSlots * 8));
        PHJ_TRY(ensure(c, c->prep, (static_cast<size_t>(P) + 1) * 4));
        PHJ_TRY(ensure(c, c->count, 32));
        PtabArgs ta{};
        ta.L = L;
        uint64_t off = 0;
        for (int g = 0; g < nseg; g++) {
            ta.segoff[g] = static_cast<uint32_t>(off);
            off += segs[g].n;
        }
        ta.segoff[nseg] = static_cast<uint32_t>(off);
        ta.tab = static_cast<NPBucket*>(c->np_tab.p);
        ta.pays = static_cast<int64_t*>(c->np_pays.p);
        ta.tob = static_cast<const uint32_t*>(c->prep.p);
        ta.f = DigitFn{pl.seed, pl.P, pl.mode == 1 ? (~0ull) / pl.P : 0, pl.mode, 0, 0xffffffffu,
                       pl.sub_bits, pl.sub_shift, 0};
        ta.seed = pl.seed;
        if (c->dry) return scan_u32(c, nullptr, P + 1, 1, P + 1);
        PHJ_TRY(mark(c, e_build0));
        PHJ_TRY(timer_begin(c, "build", nR * 32 + nbk_bound * 64));
        PHJ_HIP(c, hipMemsetAsync(c->np_tab.p, 0, nbk_bound * sizeof(NPBucket), c->ks));
        hipLaunchKernelGGL(k_pt_prep, dim3((P + 1 + kBlock - 1) / kBlock), dim3(kBlock), 0, c->ks, L, ratio_x256,
                           static_cast<uint32_t*>(c->prep.p));
        PHJ_LAUNCHED(c, "k_pt_prep");
        PHJ_TRY(scan_u32(c, static_cast<uint32_t*>(c->prep.p), P + 1, 1, P + 1));
        if (nR) {
            const dim3 bg(static_cast<uint32_t>((nR + kBlock - 1) / kBlock));
            if (pl.hk == kMurmur3) hipLaunchKernelGGL((k_pt_build<kMurmur3>), bg, dim3(kBlock), 0, c->ks, ta);
            else hipLaunchKernelGGL((k_pt_build<kXXH3>), bg, dim3(kBlock), 0, c->ks, ta);
            PHJ_LAUNCHED(c, "k_pt_build");
        }
        PHJ_TRY(timer_end(c));
        PHJ_TRY(mark(c, e_build1));
        PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 8, c->ks));
        PHJ_TRY(timer_begin(c, "probe", nS * 8 + nS * 64));
        if (nS) {
            constexpr int IT = 4;
            const dim3 pg(static_cast<uint32_t>((nS + kBlock * IT - 1) / (kBlock * IT)));
            auto* cnt = static_cast<unsigned long long*>(c->count.p);
            const auto* tab = static_cast<const NPBucket*>(c->np_tab.p);
            const auto* tob = static_cast<const uint32_t*>(c->prep.p);
            if (pl.hk == kMurmur3)
                hipLaunchKernelGGL((k_pt_probe<kMurmur3, IT>), pg, dim3(kBlock), 0, c->ks, PS.view.keys,
                                   static_cast<uint32_t>(nS), tab, tob, ta.f, pl.seed, cnt);
            else
                hipLaunchKernelGGL((k_pt_probe<kXXH3, IT>), pg, dim3(kBlock), 0, c->ks, PS.view.keys,
                                   static_cast<uint32_t>(nS), tab, tob, ta.f, pl.seed, cnt);
            PHJ_LAUNCHED(c, "k_pt_probe");
        }
        PHJ_TRY(timer_end(c));
        PHJ_TRY(mark(c, e_probe1));
        return PHJ_OK;
    }
    const size_t stride = static_cast<size_t>(P) + 1;
    PHJ_TRY(ensure(c, c->prep, stride * 3 * 4));
    PHJ_TRY(ensure(c, c->tkeys, nR * 8));
    PHJ_TRY(ensure(c, c->tpays, nR * 8));
    const size_t noffs = nR + 2 * static_cast<size_t>(P) + 1;
    PHJ_TRY(ensure(c, c->toffs, noffs * 4));
    PHJ_TRY(ensure(c, c->gcursor, noffs * 4));
    // probe schedule: small per-partition tables (the radix case) -> one wave
    // per item of <= 512 S keys; larger tables -> one workgroup per item
    const uint64_t expect_m = (nR + P - 1) / P;
    // (measured on C2: the wave schedule wins at <= ~800 S keys per partition,
    // i.e. the multi-GPU shards; the workgroup schedule at 3000)
    const uint64_t expect_s = (nS + P - 1) / P;
    const bool wave_probe = expect_m * 2 <= kProbeWaveTcap && expect_s <= 1024;
    const uint32_t kChunk = wave_probe ? 64u * kProbeWaveKPL : kBlock * 8u;
    const size_t item_bound = P + (nS + kChunk - 1) / kChunk;
    PHJ_TRY(ensure(c, c->items, item_bound * sizeof(ProbeItem)));
    PHJ_TRY(ensure(c, c->count, 32));
    PHJ_TRY(ensure(c, c->biglist, static_cast<size_t>(P) * 4));
    uint32_t* prep = static_cast<uint32_t*>(c->prep.p);
    // LDS capacities from the expected partition size (larger partitions take
    // the global-memory path; results are identical).
    const uint64_t expect = (nR + P - 1) / P;
    const uint32_t kcap = expect * 2 > 8192 ? 256u : std::max<uint32_t>(256, next_pow2_u32(static_cast<uint32_t>(expect * 2)));
    const uint32_t ocap_build = 16384;
    const uint32_t ocap_wave = std::min<uint32_t>(2048, std::max<uint32_t>(64, kcap));
    if (c->dry) return scan_u32(c, nullptr, P + 1, 3, static_cast<uint32_t>(stride));

    PHJ_TRY(mark(c, e_build0));
    PHJ_TRY(timer_begin(c, "build", nR * 32));
    hipLaunchKernelGGL(k_join_prep, dim3((P + 1 + kBlock - 1) / kBlock), dim3(kBlock), 0, c->ks, L,
                       PS.view.bounds, kChunk, prep);
    PHJ_LAUNCHED(c, "k_join_prep");
    PHJ_TRY(scan_u32(c, prep, P + 1, 3, static_cast<uint32_t>(stride)));
    const uint32_t* tkb = prep;
    const uint32_t* tob = prep + stride;
    const uint32_t* itb = prep + 2 * stride;
    hipLaunchKernelGGL(k_items_expand, dim3((P + kWaves - 1) / kWaves), dim3(kBlock), 0, c->ks, itb, tkb, tob,
                       PS.view.bounds, P, kChunk, static_cast<ProbeItem*>(c->items.p));
    PHJ_LAUNCHED(c, "k_items_expand");
    BuildArgs ba{};
    ba.L = L;
    ba.tkb = tkb;
    ba.tob = tob;
    ba.tkeys = static_cast<int64_t*>(c->tkeys.p);
    ba.tpays = static_cast<int64_t*>(c->tpays.p);
    ba.toffs = static_cast<uint32_t*>(c->toffs.p);
    ba.gcursor = static_cast<uint32_t*>(c->gcursor.p);
    ba.ocap = ocap_build;
    ba.seed = pl.seed;
    // wave-per-partition build; partitions past a wave's LDS slice go to k_build_big
    ba.biglist = static_cast<uint32_t*>(c->biglist.p);
    ba.bigcount = static_cast<uint32_t*>(c->count.p) + 2;
    PHJ_HIP(c, hipMemsetAsync(ba.bigcount, 0, 4, c->ks));
    ba.ocap = ocap_wave;
    const uint32_t sgrid = (P + kWaves - 1) / kWaves;   // one wave per partition
    const size_t slds = static_cast<size_t>(ocap_wave) * 4 * kWaves;
    if (pl.hk == kMurmur3)
        hipLaunchKernelGGL((k_build_small<kMurmur3, kBuildKPL>), dim3(sgrid), dim3(kBlock), slds, c->ks, ba);
    else
        hipLaunchKernelGGL((k_build_small<kXXH3, kBuildKPL>), dim3(sgrid), dim3(kBlock), slds, c->ks, ba);
    PHJ_LAUNCHED(c, "k_build_small");
    ba.ocap = ocap_build;
    const size_t blds = 64 + static_cast<size_t>(ocap_build) * 4;
    if (pl.hk == kMurmur3)
        hipLaunchKernelGGL((k_build_big<kMurmur3>), dim3(256), dim3(kBlock), blds, c->ks, ba);
    else
        hipLaunchKernelGGL((k_build_big<kXXH3>), dim3(256), dim3(kBlock), blds, c->ks, ba);
    PHJ_LAUNCHED(c, "k_build_big");
    PHJ_TRY(timer_end(c));
    PHJ_TRY(mark(c, e_build1));

    PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 8, c->ks));
    ProbeArgs pa{};
    pa.skeys = PS.view.keys;
    pa.tkeys = static_cast<const int64_t*>(c->tkeys.p);
    pa.toffs = static_cast<const uint32_t*>(c->toffs.p);
    pa.items = static_cast<const ProbeItem*>(c->items.p);
    pa.nitems = itb + P;
    pa.count = static_cast<unsigned long long*>(c->count.p);
    pa.seed = pl.seed;
    PHJ_TRY(timer_begin(c, "probe", nS * 8 + nR * 8));
    // staged table slice per item: 512 keys (2 per lane) covers |R|/P up to ~300
    // (P = 65536 at 10M); larger per-partition tables stage 2048 keys or probe in place
    const bool small = expect * 2 <= 512;
    const void* kfn = nullptr;
#define PHJ_PROBE_PICK(HK_, IT_, KPT_) kfn = reinterpret_cast<const void*>(&k_probe<HK_, IT_, KPT_>)
    if (pl.hk == kMurmur3) { if (small) PHJ_PROBE_PICK(kMurmur3, 8, 2); else PHJ_PROBE_PICK(kMurmur3, 8, 8); }
    else { if (small) PHJ_PROBE_PICK(kXXH3, 8, 2); else PHJ_PROBE_PICK(kXXH3, 8, 8); }
#undef PHJ_PROBE_PICK
    if (wave_probe) {
        if (pl.hk == kMurmur3) kfn = reinterpret_cast<const void*>(&k_probe_wave<kMurmur3, kProbeWaveKPL, kProbeWaveTcap>);
        else kfn = reinterpret_cast<const void*>(&k_probe_wave<kXXH3, kProbeWaveKPL, kProbeWaveTcap>);
    }
    int per_cu = 0;
    if ((per_cu = occupancy(kfn, kBlock, 0)) < 1) per_cu = 2;
    const size_t item_blocks = wave_probe ? (item_bound + kWaves - 1) / kWaves : item_bound;
    const uint32_t pgrid = static_cast<uint32_t>(
        std::max<size_t>(1, std::min<size_t>(item_blocks, static_cast<size_t>(per_cu) * c->num_cus)));
    void* kargs[] = {&pa};
    PHJ_HIP(c, hipLaunchKernel(kfn, dim3(pgrid), dim3(kBlock), kargs, 0, c->ks));
    PHJ_LAUNCHED(c, "k_probe");
    PHJ_TRY(timer_end(c));
    PHJ_TRY(mark(c, e_probe1));
    return PHJ_OK;
}

// ---- the counting join's on-chip path (phj_table.h) ----

// The build side of the on-chip join on this device's relation: pass 1 as
// hash codes, contiguous per pass-1 digit (k_hist + scan + k_scatter_codes,
// 512 x 4096 tiles), then pass 2 into final partition order (k_ht_p2, one
// workgroup per pass-1 digit). `out` receives |R| codes, `bounds` the P + 1 partition
// bounds: one build segment of build_ht (they may point into an exchange block).
// A cluster plan (pl.cluster, phj_cluster.h) stops after pass 1: `out` = the
// codes contiguous per cluster, `bounds` = the nb1 + 1 cluster bounds.
int partition_build(phj_ctx* c, const Plan& pl, int64_t* out, uint32_t* bounds) {
    SideState& S = c->side[PHJ_SIDE_BUILD];
    c->scan_scratch = &S.partials;
    if (!S.rel && S.n > 0) return set_err(c, PHJ_ERR_STATE, "relation not bound");
    if (S.n >= (1ull << 32) - 2 * 4096) return set_err(c, PHJ_ERR_RANGE, "relation above 2^32 tuples per device");
    constexpr int BLOCK = 512, ITEMS = 8, T = BLOCK * ITEMS;
    const uint32_t n = static_cast<uint32_t>(S.n), nb = pl.nb1, P = pl.Ppad;
    const uint32_t nt = (n + T - 1) / T, hlen = nt * nb;
    PHJ_TRY(ensure(c, S.hist1, std::max<size_t>(1, hlen) * 4));
    if (!pl.cluster) PHJ_TRY(ensure(c, S.kA, std::max<size_t>(1, n) * 8));
    if (c->dry) return hlen ? scan_u32(c, nullptr, hlen, 1, hlen, c->scan_scratch) : PHJ_OK;
    if (n == 0) {
        PHJ_HIP(c, hipMemsetAsync(bounds, 0, (static_cast<size_t>(pl.cluster ? nb : P) + 1) * 4, c->ks));
        c->since_ev++;
        return PHJ_OK;
    }
    PassArgs a{};
    a.in_keys = reinterpret_cast<const int64_t*>(S.rel);
    a.out_keys = pl.cluster ? out : static_cast<int64_t*>(S.kA.p);
    a.hist = static_cast<uint32_t*>(S.hist1.p);
    a.nseg = 1;
    a.n = n;
    a.ntiles1 = nt;
    a.nbins = nb;
    a.nbits = pl.bits1;
    a.f = digit_fn(pl, 1);
    a.xcd_remap = 1;
    const uint32_t grid = (nt + 7) & ~7u;
    const size_t hlds = static_cast<size_t>(BLOCK / 64) * nb * 4;
    PHJ_TRY(timer_begin(c, "R.p1.hist", static_cast<uint64_t>(n) * 16));
    if (pl.hk == kMurmur3) hipLaunchKernelGGL((k_hist<BLOCK, ITEMS, true, kMurmur3>), dim3(grid), dim3(BLOCK), hlds, c->ks, a);
    else hipLaunchKernelGGL((k_hist<BLOCK, ITEMS, true, kXXH3>), dim3(grid), dim3(BLOCK), hlds, c->ks, a);
    PHJ_LAUNCHED(c, "k_hist");
    PHJ_TRY(timer_end(c));
    PHJ_TRY(timer_begin(c, "R.p1.scan", static_cast<uint64_t>(hlen) * 12));
    PHJ_TRY(scan_u32(c, a.hist, hlen, 1, hlen, c->scan_scratch));   // k_ht_p2 reads d1's run from it
    PHJ_TRY(timer_end(c));
    // algorithmic bytes: the 16-B tuple read, the 8-B code written
    PHJ_TRY(timer_begin(c, "R.p1.scatter", static_cast<uint64_t>(n) * 24));
    const size_t slds = scatter_codes_lds_bytes(T, nb);
    if (pl.hk == kMurmur3)
        hipLaunchKernelGGL((k_scatter_codes<BLOCK, ITEMS, kMurmur3>), dim3(grid), dim3(BLOCK), slds, c->ks, a);
    else
        hipLaunchKernelGGL((k_scatter_codes<BLOCK, ITEMS, kXXH3>), dim3(grid), dim3(BLOCK), slds, c->ks, a);
    PHJ_LAUNCHED(c, "k_scatter_codes");
    PHJ_TRY(timer_end(c));
    if (pl.cluster) {   // the cluster bounds from the scanned histogram
        hipLaunchKernelGGL(k_pass1_finish, dim3(1), dim3(kFinBlock), 0, c->ks, a.hist, nt, nb, n, static_cast<uint32_t>(T),
                           bounds, static_cast<uint32_t*>(nullptr));
        PHJ_LAUNCHED(c, "k_pass1_finish");
        return PHJ_OK;
    }
    HtPass2Args b{};
    b.codes = static_cast<const int64_t*>(S.kA.p);
    b.hist1 = a.hist;
    b.out = out;
    b.bounds = bounds;
    b.nt1 = nt;
    b.n = n;
    b.nb1 = nb;
    b.nb2 = pl.nb2;
    b.f2 = digit_fn(pl, 2);
    // algorithmic bytes: the codes read, written in partition order
    PHJ_TRY(timer_begin(c, "R.p2.scatter", static_cast<uint64_t>(n) * 16));
    // runs kept in registers when d1's runs average well inside kHtP2Keep
    const bool keep = static_cast<uint64_t>(n) / nb * 5 / 4 <= kHtP2Keep;
    if (keep) hipLaunchKernelGGL(k_ht_p2<true>, dim3(nb), dim3(kHtP2Block), ht_p2_lds_bytes(pl.nb2, true), c->ks, b);
    else hipLaunchKernelGGL(k_ht_p2<false>, dim3(nb), dim3(kHtP2Block), ht_p2_lds_bytes(pl.nb2, false), c->ks, b);
    PHJ_LAUNCHED(c, "k_ht_p2");
    return timer_end(c);
}

// Code tables of every final partition over `nseg` build segments (codes in
// partition order + P + 1 bounds each, e.g. the all-gathered shards), plus
// the descriptors k_probe_ht stages. nR = the codes of all segments.
int build_ht(phj_ctx* c, const Plan& pl, int nseg, const int64_t* const* codes, const uint32_t* const* bounds,
             uint64_t nR, const uint32_t* uni = nullptr) {
    if (nseg < 1 || nseg > kHtSegs) return set_err(c, PHJ_ERR_INVALID, "build segments must be in [1,16]");
    const uint32_t P = pl.Ppad;
    const uint64_t slots = 4 * nR + 2ull * P;
    if (slots >= (1ull << 32)) return set_err(c, PHJ_ERR_RANGE, "build side too large for 32-bit table slots");
    PHJ_TRY(ensure(c, c->ht_tab, slots * 8));
    PHJ_TRY(ensure(c, c->ht_desc, static_cast<size_t>(P) * 8));
    PHJ_TRY(ensure(c, c->count, 32));
    if (c->dry) return PHJ_OK;
    HtArgs a{};
    for (int g = 0; g < nseg; g++) {
        a.codes[g] = codes[g];
        a.bounds[g] = bounds[g];
    }
    a.nseg = static_cast<uint32_t>(nseg);
    a.nb1 = pl.nb1;
    a.nb2 = pl.nb2;
    a.e1 = plan_empty0(pl);
    a.table = static_cast<uint64_t*>(c->ht_tab.p);
    a.desc = static_cast<uint2*>(c->ht_desc.p);
    a.uni = uni;
    if (nseg == 1) hipLaunchKernelGGL(k_ht_fill<true>, dim3((P + kHtPpw - 1) / kHtPpw), dim3(256), 0, c->ks, a);
    else hipLaunchKernelGGL(k_ht_fill<false>, dim3((P + kHtPpw - 1) / kHtPpw), dim3(256), 0, c->ks, a);
    PHJ_LAUNCHED(c, "k_ht_fill");
    return PHJ_OK;
}

// phj_join takes the on-chip path for a 2-pass plan unless PHJ_P2PROBE=0 or a
// tuning knob changed the tile shape (the probe walks 512 x 4096 tiles).
bool use_p2probe(const phj_ctx* c, const Plan& pl, uint64_t nS, uint64_t nR) {
    (void)nS;
    return c->tune.p2probe && !pl.chained && pl.npass == 2 && tile_shape(c, pl.nb2).tile == 4096 && tile_shape(c, pl.nb2).block == 512 &&
           tile_shape(c, pl.nb1).tile == 4096 &&
           probe_ht_lds_bytes(kProbeBlock * kProbeItems, pl.nb2) <= 160 * 1024 &&
           4 * nR + 2ull * pl.Ppad < (1ull << 32) && plan_empty0(pl) != 0;
}

// phj_join takes the LDS join (phj_cluster.h) when the plan's clusters fit:
// out = the cluster plan. Needs the keys-only chunked pass 1 (512 x 4096 tiles).
// nS: the probe side (0: not known yet, e.g. the exchange geometry); it must
// take the keys-only chunked pass 1 under the cluster plan, else (a probe side
// above the pool's uint32 slot bound, ~2^32 / (kPipeRes + 1) codes per device)
// the join takes the stable pass 1 and the code tables (use_p2probe).
bool use_cluster(const phj_ctx* c, const Plan& pl, uint64_t nS, uint64_t nR, Plan& out) {
    if (!c->tune.p1_chunk || pl.stable) return false;
    if (!cluster_plan(c, pl, nR, out)) return false;
    // the chunked pass 1 runs on 512 x 4096 tiles for both of the plan's digit counts
    for (uint32_t nb : {out.nb1, out.nb2}) {
        const TileShape sh = tile_shape(c, nb);
        if (sh.tile != 4096 || sh.block != 512) return false;
    }
    if (nS > 0 && !chunked_pass1(c, out, nS, true)) return false;
    return cluster_empty0(out) != 0 && 4 * nR + 2ull * out.nb1 < (1ull << 32);
}

// Probe a probe-side pass-1 output (partition_state p1_only) against the
// tables of build_ht; the count lands in (clear) or is added to c->count.
int probe_ht(phj_ctx* c, const Plan& pl, SideState& PS, bool clear = true) {
    if (clear) PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 16, c->ks));
    if (PS.nt2 == 0) return PHJ_OK;
    HtProbeArgs pa{};
    pa.a = PS.p2;
    pa.desc = static_cast<const uint2*>(c->ht_desc.p);
    pa.table = static_cast<const uint64_t*>(c->ht_tab.p);
    pa.count = static_cast<unsigned long long*>(c->count.p);
    if (PS.chunk_check) {   // its error word is folded into the count pair
        pa.err = static_cast<const uint32_t*>(PS.ccur.p) + chunk_err_word(PS.plan.nb1);
        PS.chunk_check = false;
    }
    pa.seed = pl.seed;
    pa.e1 = plan_empty0(pl);
    pa.nb2 = pl.nb2;
    constexpr int B = kProbeBlock, I = kProbeItems;
    const size_t lds = probe_ht_lds_bytes(B * I, pl.nb2);
    // a keys-only pass 1 wrote codes (k_chunk_codes); a stable pass 1 left whole tuples
    // (the chunked pass-1 output is always codes; a radix plan's d2 is a bit field)
    const bool radix = pl.mode == 0 && pl.sub_bits == 0;
    const void* kfn = PS.hcoded ? (radix ? reinterpret_cast<const void*>(&k_probe_ht<B, I, kHashed, kProbeRadix | kProbeChunked>)
                                         : reinterpret_cast<const void*>(&k_probe_ht<B, I, kHashed, kProbeChunked>))
                      : pl.hk == kMurmur3 ? reinterpret_cast<const void*>(&k_probe_ht<B, I, kMurmur3>)
                                          : reinterpret_cast<const void*>(&k_probe_ht<B, I, kXXH3>);
    // persistent: as many workgroups as fit the chip at once (a multiple of 8:
    // XCD x owns tiles [x, x + 1) * ntiles / 8), never many more than tiles
    int per_cu = 0;
    if ((per_cu = occupancy(kfn, B, lds)) < 1) per_cu = 2;
    per_cu = std::min<int>(per_cu, static_cast<int>(160 * 1024 / lds));
    const uint32_t want = (PS.nt2 + 7) & ~7u;
    const uint32_t grid = std::max<uint32_t>(8, std::min<uint32_t>(want, static_cast<uint32_t>(per_cu) * c->num_cus) & ~7u);
    void* kargs[] = {&pa};
    PHJ_HIP(c, hipLaunchKernel(kfn, dim3(grid), dim3(B), kargs, lds, c->ks));
    PHJ_LAUNCHED(c, "k_probe_ht");
    return PHJ_OK;
}

// A stale chunk table met by a chunked pass (phj_partition.h chunk_err_word):
// the pass wrote nothing through it, and the join reports PHJ_ERR_STATE. Both
// sides' tables are cleared before their next pass.
int chunk_table_error(phj_ctx* c, uint32_t bits) {
    for (SideState& S : c->side) {
        S.ctab_dirty = true;
        S.chunk_check = false;
    }
    return set_err(c, PHJ_ERR_STATE, "chunked pass 1 read a chunk-table entry out of range (stale table, error bits " +
                                         std::to_string(bits) + "); nothing was written through it");
}

// The error words of chunked passes not folded into a count (a 4-B read back
// per side; the default on-chip join folds S's into the count instead).
int check_chunk_errors(phj_ctx* c) {
    for (SideState& S : c->side) {
        if (!S.chunk_check) continue;
        S.chunk_check = false;
        uint32_t e = 0;
        PHJ_HIP(c, hipMemcpyAsync(&e, static_cast<const uint32_t*>(S.ccur.p) + chunk_err_word(S.plan.nb1), 4,
                                  hipMemcpyDeviceToHost, c->ks));
        PHJ_HIP(c, hipStreamSynchronize(c->ks));
        if (e) return chunk_table_error(c, e);
    }
    return PHJ_OK;
}

// The LDS join over a cluster plan: the HBM tables of the clusters beyond the
// LDS limit (k_cluster_big_fill, on the current launch stream: R's chain),
// then (probe_cluster, on the main stream) k_cluster_probe over the probe
// side's pass-1 tiles. `nseg` build segments of codes contiguous per cluster
// and nb1 + 1 bounds each; nR = their codes. The count pair is added to.
// RT (tile mode, one device): R's chunked code pass; its tiles are the runs,
// its cluster offsets (bounds1) give each cluster's size and first code.
ClusterArgs cluster_args(phj_ctx* c, const Plan& pl, int nseg, const int64_t* const* codes,
                         const uint32_t* const* bounds, SideState* RT = nullptr) {
    ClusterArgs a{};
    if (RT) {
        nseg = 1;
        a.r_codes[0] = RT->p2.in_keys;
        a.r_bounds[0] = static_cast<const uint32_t*>(RT->bounds1.p);
        a.rt_base = RT->p2.tile_base;
        a.rt_start = RT->p2.tile_start;
        a.rt_cnt = RT->p2.tile_cnt;
        a.r_pool = RT->p2.in_keys;
    } else {
        for (int g = 0; g < nseg; g++) {
            a.r_codes[g] = codes[g];
            a.r_bounds[g] = bounds[g];
        }
    }
    a.nseg = static_cast<uint32_t>(nseg);
    a.nb1 = pl.nb1;
    a.cap = static_cast<uint32_t>(c->tune.cl_cap);
    a.lim = cl_lim(a.cap);
    a.e1 = cluster_empty0(pl);
    a.gtab = static_cast<uint64_t*>(c->ht_tab.p);
    a.count = static_cast<unsigned long long*>(c->count.p);
    return a;
}

int cluster_big_fill(phj_ctx* c, const Plan& pl, int nseg, const int64_t* const* codes, const uint32_t* const* bounds,
                     uint64_t nR, SideState* RT = nullptr) {
    if (nseg < 1 || nseg > kHtSegs) return set_err(c, PHJ_ERR_INVALID, "build segments must be in [1,16]");
    const uint64_t slots = 4 * nR + 2ull * pl.nb1;
    if (slots >= (1ull << 32)) return set_err(c, PHJ_ERR_RANGE, "build side too large for 32-bit table slots");
    PHJ_TRY(ensure(c, c->ht_tab, slots * 8));
    PHJ_TRY(ensure(c, c->count, 32));
    if (c->dry) return PHJ_OK;
    ClusterArgs a = cluster_args(c, pl, nseg, codes, bounds, RT);
    hipLaunchKernelGGL(k_cluster_big_fill, dim3(pl.nb1), dim3(256), 0, c->ks, a);
    PHJ_LAUNCHED(c, "k_cluster_big_fill");
    return PHJ_OK;
}

// The pinned count word pair (count_pin) and its device side; false: the
// count comes back by a copy (get_count).
bool count_pin_ready(phj_ctx* c) {
    if (c->count_pin) return true;
    if (c->count_pin_failed) return false;
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(&d, h, 0) != hipSuccess || ensure(c, c->cl_done, 4) != PHJ_OK ||
        hipMemset(c->cl_done.p, 0, 4) != hipSuccess) {
        (void)hipGetLastError();
        if (h) (void)hipHostFree(h);
        c->count_pin_failed = true;
        return false;
    }
    c->count_pin = static_cast<unsigned long long*>(h);
    c->count_pin_dev = static_cast<unsigned long long*>(d);
    return true;
}

// pin: the last kernel also writes the count pair to count_pin (get_count
// then only synchronises; one device-to-host copy fewer per join)
int probe_cluster(phj_ctx* c, const Plan& pl, SideState& PS, int nseg, const int64_t* const* codes,
                  const uint32_t* const* bounds, SideState* RT = nullptr, bool pin = false) {
    if (c->dry || PS.nt2 == 0) return PHJ_OK;
    if (!PS.hcoded) return set_err(c, PHJ_ERR_STATE, "the LDS join needs the keys-only pass 1 (codes)");
    ClusterArgs a = cluster_args(c, pl, nseg, codes, bounds, RT);
    SideState& RS = c->side[PHJ_SIDE_BUILD];
    if (RS.chunk_check) {   // R's chunked pass-1 error word, folded into the count pair as S's
        a.err_r = static_cast<const uint32_t*>(RS.ccur.p) + chunk_err_word(RS.plan.nb1);
        RS.chunk_check = false;
    }
    a.s_codes = PS.p2.in_keys;
    a.tile_base = PS.p2.tile_base;
    a.tile_seg = PS.p2.tile_seg;
    a.tile_start = PS.p2.tile_start;
    a.tile_cnt = PS.p2.tile_cnt;
    if (PS.chunk_check) {   // its error word is folded into the count pair
        a.err = static_cast<const uint32_t*>(PS.ccur.p) + chunk_err_word(PS.plan.nb1);
        PS.chunk_check = false;
    }
    // the clock split: words 2-3 of the count buffer, cleared with the count
    // pair by the pass-1 bookkeeping kernel (no memset per join)
    if (c->tune.timers) {
        a.split = static_cast<unsigned long long*>(c->count.p) + 2;
        c->split_words = a.split;
    }
    constexpr int B = kClBlock, I = kClItems;
    const size_t lds = cluster_lds_bytes(a.cap);   // the table + its 16-bit bucket fill counters
    constexpr bool PR = PHJ_CL_PROF != 0;   // measurement build: the builds' section clocks
    if (PR) {
        PHJ_TRY(ensure(c, c->cl_prof, 64 * 8));
        a.prof = static_cast<unsigned long long*>(c->cl_prof.p);
        PHJ_HIP(c, hipMemsetAsync(a.prof, 0, kClProfWords * 8, c->ks));
    }
    // three tiles of codes in flight, the next cluster's R codes prefetched
    // (measured: one / two tiles 0.406 / 0.360 ms against 0.355 at C2; tables by
    // 64-bit compare-and-swap 0.082 ms of builds against 0.055 by fill counters)
    const void* kfn = RT ? reinterpret_cast<const void*>(&k_cluster_probe<B, I, 3, true, PR, true>)
                         : reinterpret_cast<const void*>(&k_cluster_probe<B, I, 3, true, PR, false>);
    int per_cu = 0;
    if ((per_cu = occupancy(kfn, B, lds)) < 1) per_cu = 1;
    per_cu = std::max(1, std::min<int>(per_cu, static_cast<int>(160 * 1024 / (lds + 256))));
    // persistent, a multiple of 8 (XCD-grouped ranges), never many more than tiles
    const uint32_t want = (PS.nt2 + 7) & ~7u;
    const uint32_t grid = std::max<uint32_t>(8, std::min<uint32_t>(want, static_cast<uint32_t>(per_cu) * c->num_cus) & ~7u);
    void* kargs[] = {&a};
    PHJ_TRY(launch_kernel(c, kfn, dim3(grid), dim3(B), kargs, lds, "k_cluster_probe"));
    if (PR) {   // diagnostics (measurement build): synchronous, to stderr, in microseconds summed over workgroups
        unsigned long long h[kClProfWords] = {};
        PHJ_HIP(c, hipMemcpyAsync(h, a.prof, sizeof(h), hipMemcpyDeviceToHost, c->ks));
        PHJ_HIP(c, hipStreamSynchronize(c->ks));
        std::fprintf(stderr, "cl_prof grid %u: cold %.1f us, clear+runs %.1f us, inserts %.1f us, prefetch %.1f us; builds %llu, cold %llu\n",
                     grid, h[0] / 100.0, h[1] / 100.0, h[2] / 100.0, h[3] / 100.0, h[4], h[5]);
    }
    // the big clusters' tiles against their HBM tables (workgroups of the
    // other clusters return at once)
    a.split = nullptr;
    a.err = nullptr;
    a.err_r = nullptr;
    if (pin && c->tune.count_pin && count_pin_ready(c)) {
        // a value no launch writes (failed holds error bits): get_count falls
        // back to the copy if the kernel left it
        reinterpret_cast<volatile unsigned long long*>(c->count_pin)[1] = ~0ull;
        a.host_out = c->count_pin_dev;
        a.done = static_cast<uint32_t*>(c->cl_done.p);
        c->count_pinned = true;
        // S's chunk state is read no more after this launch: cleared for the next join
        a.s_clear = static_cast<uint4*>(PS.ccur.p);
        a.s_clear16 = static_cast<uint32_t>(chunk_state_bytes(PS.plan.nb1) / 16);
        c->s_zero_pending = PS.ccur.p;
        c->s_zero_pending_bytes = chunk_state_bytes(PS.plan.nb1);
    }
    hipLaunchKernelGGL(k_cluster_probe_big, dim3(std::max<uint32_t>(kProbeBigGrid, (pl.nb1 + 255) / 256)), dim3(256), 0, c->ks, a);
    PHJ_LAUNCHED(c, "k_cluster_probe_big");
    return PHJ_OK;
}

// The count comes back through a pinned host word (a pageable destination is
// staged by the runtime: a slower copy on the step's critical path). pair:
// the on-chip probes' {count, failed}, failed set when S's pass 1 met a stale
// chunk table (fold_pass1_error).
int get_count(phj_ctx* c, uint64_t* out, bool pair = false) {
    if (c->count_pinned) {   // written by the join's last workgroup (probe_cluster)
        c->count_pinned = false;
        const volatile unsigned long long* v = c->count_pin;
        if (c->defer_timers) {
            // no event is read in this join: poll the pinned word (the
            // driver's stream synchronisation wakes later), asking every
            // 4096 polls whether the stream has finished without it
            for (uint32_t i = 1; v[1] == ~0ull; i++) {
                if ((i & 4095u) == 0) {
                    const hipError_t q = hipStreamQuery(c->ks);
                    if (q == hipSuccess) break;
                    if (q != hipErrorNotReady) PHJ_HIP(c, q);
                }
                __builtin_ia32_pause();
            }
            std::atomic_thread_fence(std::memory_order_acquire);
        } else {
            PHJ_HIP(c, hipStreamSynchronize(c->ks));
        }
        const unsigned long long failed = v[1];
        if (failed == 0) {   // the last workgroup cleared S's chunk state
            c->s_zeroed = c->s_zero_pending;
            c->s_zeroed_bytes = c->s_zero_pending_bytes;
        }
        c->s_zero_pending = nullptr;
        if (failed != ~0ull) {
            *out = v[0];
            if (pair && failed) {
                c->side[PHJ_SIDE_PROBE].chunk_check = true;   // read its word for the message
                const int rc = check_chunk_errors(c);
                return rc != PHJ_OK ? rc : chunk_table_error(c, 0);
            }
            return check_chunk_errors(c);
        }
    }
    if (!c->count_host && hipHostMalloc(reinterpret_cast<void**>(&c->count_host), 16, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        c->count_host = nullptr;
    }
    unsigned long long h[2] = {0, 0};
    unsigned long long* dst = c->count_host ? c->count_host : h;
    PHJ_HIP(c, hipMemcpyAsync(dst, c->count.p, pair ? 16 : 8, hipMemcpyDeviceToHost, c->ks));
    PHJ_HIP(c, hipStreamSynchronize(c->ks));
    *out = dst[0];
    if (pair && dst[1]) {
        c->side[PHJ_SIDE_PROBE].chunk_check = true;   // read its word for the message
        const int rc = check_chunk_errors(c);
        return rc != PHJ_OK ? rc : chunk_table_error(c, 0);
    }
    return check_chunk_errors(c);
}

// The NoPartitioning count over region code tables (phj_table.h, k_np_probe_ct):
// R partitioned into 2^k regions of ~300 codes by two radix passes of its hash
// codes (the build), one code table per region; S probed unpartitioned.
int join_nopart_ct(phj_ctx* c, const phj_join_params* p, phj_join_result* r) {
    SideState& R = c->side[PHJ_SIDE_BUILD];
    SideState& S = c->side[PHJ_SIDE_PROBE];
    uint32_t k = 2;
    while (k < 22 && (R.n >> k) > 300) k++;
    phj_join_params pp = *p;
    pp.algo = PHJ_ALGO_RADIX;
    pp.num_partitions = 0;
    pp.flags = 0;
    pp.radix_bits[1] = static_cast<uint8_t>(k / 2);
    pp.radix_bits[0] = static_cast<uint8_t>(k - k / 2);
    Plan pl;
    PHJ_TRY(make_plan(c, &pp, pl));
    const uint32_t P = pl.Ppad;
    const uint64_t slot_bound = 4 * R.n + 2ull * P;
    PHJ_TRY(ensure(c, c->r_codes, std::max<uint64_t>(1, R.n) * 8));
    PHJ_TRY(ensure(c, c->r_bounds, (static_cast<size_t>(P) + 1) * 4));
    PHJ_TRY(ensure(c, c->np_uni, 16));
    PHJ_TRY(ensure(c, c->count, 32));
    const int64_t* rcodes = static_cast<const int64_t*>(c->r_codes.p);
    const uint32_t* rbnd = static_cast<const uint32_t*>(c->r_bounds.p);
    auto* uni = static_cast<uint32_t*>(c->np_uni.p);
    if (c->dry) {
        PHJ_TRY(partition_build(c, pl, static_cast<int64_t*>(c->r_codes.p), static_cast<uint32_t*>(c->r_bounds.p)));
        return build_ht(c, pl, 1, &rcodes, &rbnd, R.n, uni);
    }
    hipEvent_t e0, e1, e2;
    PHJ_TRY(mark(c, &e0));
    // the partition is part of the build (its R.* timers show it)
    PHJ_TRY(partition_build(c, pl, static_cast<int64_t*>(c->r_codes.p), static_cast<uint32_t*>(c->r_bounds.p)));
    // algorithmic bytes: the codes read, the tables written (~1.7 slots per code)
    PHJ_TRY(timer_begin(c, "np.build", R.n * 8 * 3));
    hipLaunchKernelGGL(k_np_ct_plan, dim3(1), dim3(256), 0, c->ks, rbnd, P, slot_bound, uni);
    PHJ_LAUNCHED(c, "k_np_ct_plan");
    PHJ_TRY(build_ht(c, pl, 1, &rcodes, &rbnd, R.n, uni));
    PHJ_TRY(timer_end(c));
    PHJ_TRY(mark(c, &e1));
    PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 8, c->ks));
    if (S.n > 0) {
        // algorithmic bytes: S's tuples read once (16 B), R's tables (~2 slots per code) once
        PHJ_TRY(timer_begin(c, "np.probe", S.n * 16 + R.n * 16));
        constexpr int IT = 4;
        const void* kfn = p->hash == PHJ_HASH_MURMUR3 ? reinterpret_cast<const void*>(&k_np_probe_ct<kMurmur3, IT>)
                                                      : reinterpret_cast<const void*>(&k_np_probe_ct<kXXH3, IT>);
        int per_cu = 0;
        if ((per_cu = occupancy(kfn, 256, 0)) < 1) per_cu = 8;
        const uint64_t want = (S.n + 256ull * IT - 1) / (256ull * IT);
        const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(want, static_cast<uint64_t>(per_cu) * c->num_cus)));
        const auto* S_rel = reinterpret_cast<const longlong2*>(S.rel);
        const auto* tab = static_cast<const uint64_t*>(c->ht_tab.p);
        const auto* dsc = static_cast<const uint2*>(c->ht_desc.p);
        const uint32_t* un = uni;
        auto* cnt = static_cast<unsigned long long*>(c->count.p);
        uint64_t nS64 = S.n, seed = p->hash_seed, e1 = plan_empty0(pl);
        uint32_t Pv = P;
        void* kargs[] = {const_cast<longlong2**>(&S_rel), &nS64, const_cast<uint64_t**>(&tab), const_cast<uint2**>(&dsc),
                         const_cast<uint32_t**>(&un), &Pv, &seed, &e1, &cnt};
        PHJ_HIP(c, hipLaunchKernel(kfn, dim3(grid), dim3(256), kargs, 0, c->ks));
        PHJ_LAUNCHED(c, "k_np_probe_ct");
        PHJ_TRY(timer_end(c));
    }
    PHJ_TRY(mark(c, &e2));
    uint64_t m = 0;
    PHJ_TRY(get_count(c, &m));
    r->matches = m;
    r->partition_ms = 0;
    r->build_ms = elapsed(c, e0, e1);
    r->probe_ms = elapsed(c, e1, e2);
    r->total_ms = elapsed(c, e0, e2);
    r->num_partitions = 0;
    r->algorithmic_bytes = R.n * (16 + 8 + 8 + 8) + R.n * 24 + S.n * 16 + R.n * 16;
    return fill_timers(c, r);
}

// marks != nullptr: the probe also writes, per probe tuple, its match's payload
// slot (phj_join_materialize)
int join_nopart(phj_ctx* c, const phj_join_params* p, phj_join_result* r, uint32_t* marks = nullptr) {
    SideState& R = c->side[PHJ_SIDE_BUILD];
    SideState& S = c->side[PHJ_SIDE_PROBE];
    if (p->hash != PHJ_HASH_XXH3 && p->hash != PHJ_HASH_MURMUR3)
        return set_err(c, PHJ_ERR_INVALID, "unknown hash function");
    if (R.n == 0)  // LinearProbing.hpp:295-299
        return set_err(c, PHJ_ERR_INVALID,
                       "LinearProbingHashTable::LinearProbingHashTable: numberOfObjects must be greater than zero.");
    if (R.n >= (1ull << 32)) return set_err(c, PHJ_ERR_RANGE, "build side above 2^32 tuples");
    if (!marks && R.n < (1ull << 30)) return join_nopart_ct(c, p, r);
    const double ratio = p->table_ratio > 0 ? p->table_ratio : kNPDefaultRatio;
    if (ratio < 1.0) return set_err(c, PHJ_ERR_INVALID, "table_ratio must be >= 1");
    const double nbd = std::ceil(static_cast<double>(R.n) * ratio / kNPSlots);
    if (nbd >= 4294967295.0) return set_err(c, PHJ_ERR_RANGE, "table too large");
    const uint32_t nb0 = std::max<uint32_t>(1, static_cast<uint32_t>(nbd));
    // region build: 2^rbits regions of <= kNPRegionBuckets buckets (LDS-sized)
    NPHome g{nb0, nb0, 0, 0};
    g.rbits = std::min<uint32_t>(22, std::max<uint32_t>(1, ceil_log2((nb0 + kNPRegionBuckets - 1) / kNPRegionBuckets)));
    g.nbr = (nb0 + (1u << g.rbits) - 1) >> g.rbits;
    const uint64_t nbw = static_cast<uint64_t>(g.nbr) << g.rbits;
    if (nbw >= 4294967295ull || g.nbr > 2 * kNPRegionBuckets) return set_err(c, PHJ_ERR_RANGE, "table too large");
    g.nb = static_cast<uint32_t>(nbw);
    const uint32_t nb = g.nb;
    // the materialising probe stores a match as the uint32 slot b * 7 + s, and
    // kNoMatch (0xffffffff) must stay out of that range
    if (marks && static_cast<uint64_t>(nb) * kNPSlots >= kNoMatch)
        return set_err(c, PHJ_ERR_RANGE, "materialised NoPartitioning join: table above 2^32 - 1 slots");
    PHJ_TRY(ensure(c, c->np_tab, static_cast<size_t>(nb) * sizeof(NPBucket)));
    PHJ_TRY(ensure(c, c->np_pays, static_cast<size_t>(nb) * kNPSlots * 8));
    PHJ_TRY(ensure(c, c->count, 8));
    PHJ_TRY(ensure(c, c->np_ovf, R.n * 16));
    PHJ_TRY(ensure(c, c->np_ovfb, R.n * 4));
    PHJ_TRY(ensure(c, c->np_ovfn, 4));
    Plan rp;
    {
        phj_join_params pp = *p;
        pp.algo = PHJ_ALGO_RADIX;
        pp.num_partitions = 0;
        pp.flags = 0;
        pp.radix_bits[1] = static_cast<uint8_t>(g.rbits <= 8 ? 0 : g.rbits / 2);
        pp.radix_bits[0] = static_cast<uint8_t>(g.rbits - pp.radix_bits[1]);
        PHJ_TRY(make_plan(c, &pp, rp));
        if (c->dry) return partition_side(c, PHJ_SIDE_BUILD, rp);
    }
    hipEvent_t e0, e1, e2;
    const uint32_t nR = static_cast<uint32_t>(R.n);
    PHJ_TRY(mark(c, &e0));
    {
        // the partition is part of the build (its R.* timers show it)
        PHJ_TRY(partition_side(c, PHJ_SIDE_BUILD, rp));
        const phj_partitioned& v = R.view;
        PHJ_TRY(timer_begin(c, "np.build", static_cast<uint64_t>(nR) * 32 + static_cast<uint64_t>(nb) * 64));
        PHJ_HIP(c, hipMemsetAsync(c->np_ovfn.p, 0, 4, c->ks));
        const size_t lds = static_cast<size_t>(g.nbr) * (kNPSlots * 8 + 4);
        auto* ovn = static_cast<uint32_t*>(c->np_ovfn.p);
        auto* ov = static_cast<longlong2*>(c->np_ovf.p);
        auto* ovb = static_cast<uint32_t*>(c->np_ovfb.p);
        auto* tab = static_cast<NPBucket*>(c->np_tab.p);
        auto* pays = static_cast<int64_t*>(c->np_pays.p);
        const dim3 grid(1u << g.rbits);
        if (p->hash == PHJ_HASH_MURMUR3)
            hipLaunchKernelGGL((k_np_build_region<kMurmur3>), grid, dim3(kBlock), lds, c->ks, v.keys, v.payloads,
                               v.bounds, g, tab, pays, p->hash_seed, ovn, ov, ovb);
        else
            hipLaunchKernelGGL((k_np_build_region<kXXH3>), grid, dim3(kBlock), lds, c->ks, v.keys, v.payloads,
                               v.bounds, g, tab, pays, p->hash_seed, ovn, ov, ovb);
        PHJ_LAUNCHED(c, "k_np_build_region");
        hipLaunchKernelGGL(k_np_build_overflow, dim3(64), dim3(kBlock), 0, c->ks, ovn, ov, ovb, tab, pays, nb);
        PHJ_LAUNCHED(c, "k_np_build_overflow");
        PHJ_TRY(timer_end(c));
    }
    PHJ_TRY(mark(c, &e1));
    PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 8, c->ks));
    if (S.n > 0) {
        const uint64_t per = static_cast<uint64_t>(kBlock) * 4;
        const uint32_t pg = static_cast<uint32_t>(std::min<uint64_t>((S.n + per - 1) / per, 8192));
        PHJ_TRY(timer_begin(c, "np.probe", S.n * 16 + static_cast<uint64_t>(nb) * 64));
        const auto* S_rel = reinterpret_cast<const longlong2*>(S.rel);
        const auto* tab = static_cast<const NPBucket*>(c->np_tab.p);
        auto* cnt = static_cast<unsigned long long*>(c->count.p);
        // (the count takes join_nopart_ct below 2^30 build tuples; this bucket
        // probe serves larger build sides and, with marks, the materialised join)
        if (marks) {
            const uint32_t mg = static_cast<uint32_t>(std::min<uint64_t>((S.n + 4 * kBlock - 1) / (4 * kBlock), 8192));
            if (p->hash == PHJ_HASH_MURMUR3)
                hipLaunchKernelGGL((k_np_probe_mark<kMurmur3>), dim3(mg), dim3(kBlock), 0, c->ks, S_rel, S.n, tab, g,
                                   p->hash_seed, marks, cnt);
            else
                hipLaunchKernelGGL((k_np_probe_mark<kXXH3>), dim3(mg), dim3(kBlock), 0, c->ks, S_rel, S.n, tab, g,
                                   p->hash_seed, marks, cnt);
        } else if (p->hash == PHJ_HASH_MURMUR3) {
            hipLaunchKernelGGL((k_np_probe<kMurmur3, 4, 1>), dim3(pg), dim3(kBlock), 0, c->ks, S_rel, S.n, tab, g, p->hash_seed, cnt);
        } else {
            hipLaunchKernelGGL((k_np_probe<kXXH3, 4, 1>), dim3(pg), dim3(kBlock), 0, c->ks, S_rel, S.n, tab, g, p->hash_seed, cnt);
        }
        PHJ_LAUNCHED(c, "k_np_probe");
        PHJ_TRY(timer_end(c));
    }
    PHJ_TRY(mark(c, &e2));
    uint64_t m = 0;
    PHJ_TRY(get_count(c, &m));
    r->matches = m;
    r->partition_ms = 0;
    r->build_ms = elapsed(c, e0, e1);
    r->probe_ms = elapsed(c, e1, e2);
    r->total_ms = elapsed(c, e0, e2);
    r->num_partitions = 0;
    r->algorithmic_bytes = R.n * 32 + S.n * 16 + static_cast<uint64_t>(nb) * 64;
    return fill_timers(c, r);
}

int check_side(phj_ctx* c, int side) {
    if (!c) return PHJ_ERR_INVALID;
    (void)hipGetLastError();  // drop a stale error left by code outside this library
    if (side != PHJ_SIDE_BUILD && side != PHJ_SIDE_PROBE)
        return set_err(c, PHJ_ERR_INVALID, "side must be PHJ_SIDE_BUILD or PHJ_SIDE_PROBE");
    return PHJ_OK;
}

void drop_relation(phj_ctx* c, int side) {
    SideState& S = c->side[side];
    S.rel = nullptr;
    S.n = 0;
    S.partitioned = false;
}

uint64_t partition_bytes(const Plan& pl, uint64_t n) {
    // hist (16 B AoS read) + scatter (16 read + 16 write); pass 2: hist 8 + scatter 32
    return n * (16 + 32) + (pl.npass == 2 ? n * (8 + 32) : 0);
}

// Rows of a marked probe (phj_mat.h): block counts, exclusive scan, write.
int mat_compact(phj_ctx* c, uint64_t nS, const longlong2* s_aos, const int64_t* sk, const int64_t* sp,
                const int64_t* rpay) {
    const uint32_t nblk = static_cast<uint32_t>((nS + kMatBlock - 1) / kMatBlock);
    PHJ_TRY(ensure(c, c->mat_cnt, (static_cast<size_t>(nblk) + 1) * 4));
    PHJ_TRY(ensure(c, c->mat_rows, std::max<uint64_t>(1, nS) * sizeof(JoinedRow)));
    auto* cnt = static_cast<uint32_t*>(c->mat_cnt.p);
    const auto* mark = static_cast<const uint32_t*>(c->mat_mark.p);
    PHJ_TRY(timer_begin(c, "mat.write", nS * 20 + static_cast<uint64_t>(nS) * 4));
    PHJ_HIP(c, hipMemsetAsync(cnt, 0, (static_cast<size_t>(nblk) + 1) * 4, c->ks));
    if (nblk) {
        hipLaunchKernelGGL(k_mat_count, dim3(nblk), dim3(kBlock), 0, c->ks, mark, nS, cnt);
        PHJ_LAUNCHED(c, "k_mat_count");
    }
    PHJ_TRY(scan_u32(c, cnt, nblk + 1, 1, nblk + 1));
    if (nblk) {
        hipLaunchKernelGGL(k_mat_write, dim3(nblk), dim3(kBlock), 0, c->ks, mark, nS, s_aos, sk, sp, rpay, cnt,
                           static_cast<JoinedRow*>(c->mat_rows.p));
        PHJ_LAUNCHED(c, "k_mat_write");
    }
    return timer_end(c);
}

int join_radix_mark(phj_ctx* c, const phj_join_params* p, phj_join_result* r) {
    Plan pl;
    PHJ_TRY(make_plan(c, p, pl));
    SideState& R = c->side[PHJ_SIDE_BUILD];
    SideState& S = c->side[PHJ_SIDE_PROBE];
    const uint32_t requested = pl.Ppad;
    refine_plan(c, pl, R.n);
    const uint32_t P = pl.Ppad;
    if (!c->tune.fused || (R.n + P - 1) / P * 3 > static_cast<uint64_t>(kFusedTcap) * 2)
        return set_err(c, PHJ_ERR_INVALID, "materialised radix join needs the fused LDS join (PHJ_FUSED, PHJ_SUBPART)");
    hipEvent_t t0, t1, p1;
    PHJ_TRY(mark(c, &t0));
    PHJ_TRY(partition_side(c, PHJ_SIDE_PROBE, pl));
    PHJ_TRY(partition_side(c, PHJ_SIDE_BUILD, pl));
    PHJ_TRY(mark(c, &t1));
    const uint64_t nS = S.view.n;
    const size_t nslots = nS / kFusedChunk + P + 1;
    PHJ_TRY(ensure(c, c->fitems, nslots * sizeof(FusedItem)));
    PHJ_TRY(ensure(c, c->count, 32));
    PHJ_TRY(ensure(c, c->mat_mark, std::max<uint64_t>(1, nS) * 4));
    PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 8, c->ks));
    PHJ_HIP(c, hipMemsetAsync(c->mat_mark.p, 0xff, std::max<uint64_t>(1, nS) * 4, c->ks));
    PHJ_TRY(timer_begin(c, "mat.join", R.n * 8 + nS * 12));
    hipLaunchKernelGGL(k_fused_items, dim3((P + kWaves - 1) / kWaves), dim3(kBlock), 0, c->ks, S.view.bounds, P,
                       static_cast<FusedItem*>(c->fitems.p));
    PHJ_LAUNCHED(c, "k_fused_items");
    FusedArgs fa{};
    fa.L.nseg = 1;
    fa.L.P = P;
    fa.L.seg[0].keys = R.view.keys;
    fa.L.seg[0].pays = R.view.payloads;
    fa.L.seg[0].bounds = R.view.bounds;
    fa.skeys = S.view.keys;
    fa.sbounds = S.view.bounds;
    fa.items = static_cast<const FusedItem*>(c->fitems.p);
    fa.nitems = static_cast<uint32_t>(nslots - 1);
    fa.count = static_cast<unsigned long long*>(c->count.p);
    fa.seed = pl.seed;
    const uint32_t grid = static_cast<uint32_t>(
        std::max<size_t>(1, std::min<size_t>((nslots + kWaves - 1) / kWaves, static_cast<size_t>(4) * c->num_cus)));
    auto* mk = static_cast<uint32_t*>(c->mat_mark.p);
    if (pl.hk == kMurmur3)
        hipLaunchKernelGGL(k_join_fused_mark<kMurmur3>, dim3(grid), dim3(kBlock), 0, c->ks, fa, mk);
    else
        hipLaunchKernelGGL(k_join_fused_mark<kXXH3>, dim3(grid), dim3(kBlock), 0, c->ks, fa, mk);
    PHJ_LAUNCHED(c, "k_join_fused_mark");
    PHJ_TRY(timer_end(c));
    PHJ_TRY(mat_compact(c, nS, nullptr, S.view.keys, S.view.payloads, R.view.payloads));
    PHJ_TRY(mark(c, &p1));
    uint64_t m = 0;
    PHJ_TRY(get_count(c, &m));
    r->matches = m;
    r->partition_ms = elapsed(c, t0, t1);
    r->probe_ms = elapsed(c, t1, p1);
    r->total_ms = elapsed(c, t0, p1);
    r->num_partitions = requested;
    r->algorithmic_bytes = partition_bytes(pl, R.n) + partition_bytes(pl, S.n) + R.n * 8 + nS * 12 + m * 24;
    return fill_timers(c, r);
}

int ctx_create_device(int device, phj_ctx** out) {
    if (!out) return PHJ_ERR_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PHJ_ERR_HIP;
    if (device < 0 || device >= ndev) return PHJ_ERR_INVALID;
    if (hipSetDevice(device) != hipSuccess) return PHJ_ERR_HIP;
    phj_ctx* c = new phj_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return PHJ_ERR_HIP;
    }
    if (hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return PHJ_ERR_HIP;
    }
    c->ks = c->stream;
    c->own_stream = true;
    {
        const int t = env_int("PHJ_TILE", 4096);
        c->tune.tile = (t == 2048 || t == 8192) ? t : 4096;
    }
    c->tune.block = env_int("PHJ_BLOCK", 512);
    c->tune.nt_load = std::min(2, std::max(0, env_int("PHJ_NT_LOAD", 1)));
    c->tune.fused = env_int("PHJ_FUSED", 1) != 0;
    c->tune.ptab = env_int("PHJ_PTAB", 1);
    c->tune.subpart = env_int("PHJ_SUBPART", 1) != 0;
    c->tune.timers = env_int("PHJ_TIMERS", 1) != 0;
    c->tune.p1_chunk = env_int("PHJ_P1_CHUNK", 1) != 0;
    c->tune.cluster = env_int("PHJ_CLUSTER", 1) != 0;
    c->tune.p1_pipe = env_int("PHJ_P1_PIPE", 1) != 0;
    c->tune.cl_cap = env_int("PHJ_CL_CAP", static_cast<int>(kClCapMax)) == 8192 ? 8192 : static_cast<int>(kClCapMax);
    c->tune.cl_bits = std::max(0, std::min(kMaxDigitBits, env_int("PHJ_CL_BITS", 0)));
    c->tune.p2probe = env_int("PHJ_P2PROBE", 1);
    c->tune.p1_slots = env_int("PHJ_P1_SLOTS", 0);
    c->tune.p1_wpc2 = std::max(0, env_int("PHJ_P1_WPC2", 2));
    c->tune.r_order = std::min(2, std::max(0, env_int("PHJ_R_ORDER", 1)));
    c->tune.count_pin = env_int("PHJ_COUNT_PIN", 1);
    c->tune.r_chunk = env_int("PHJ_R_CHUNK", 1) != 0;
    c->tune.p1_block = env_int("PHJ_P1_BLOCK", 1024) == 512 ? 512 : 1024;
    c->tune.p1_tps = std::max(1, env_int("PHJ_P1_TPS", static_cast<int>(kTilesPerShard)));
    c->tune.p1_min_tiles = std::max(0, env_int("PHJ_P1_MIN_TILES", 32768));
    c->tune.p1_ko_tps = std::max(1, env_int("PHJ_P1_KO_TPS", 1024));
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
    }
    // gfx950 launches accept dynamic LDS up to the 160 KiB per workgroup without an
    // opt-in attribute; clear any error a probe of the runtime left behind
    (void)hipGetLastError();
    *out = c;
    return PHJ_OK;
}

}  // namespace

#include "phj_group.h"

namespace {

// A multi-device context with one local member forwards the single-device
// calls (building blocks) to it; with several members they are not defined.
template <class F>
int on_solo(phj_ctx* c, const char* what, F f) {
    phj_ctx* m = c->group->nlocal() == 1 ? c->group->mem[0] : nullptr;
    if (!m) return set_err(c, PHJ_ERR_STATE, std::string(what) + ": not available on a multi-device context");
    const int rc = f(m);
    if (rc != PHJ_OK) c->err = m->err;
    return rc;
}

}  // namespace

extern "C" {

int phj_abi_version(void) { return PHJ_ABI_VERSION; }

int phj_ctx_create_device(int device, phj_ctx** out) { return ctx_create_device(device, out); }

int phj_ctx_create_ex(int ngpus, const int* devs, uint32_t flags, phj_ctx** out) {
    if (!out) return PHJ_ERR_INVALID;
    *out = nullptr;
    if (ngpus < 1 || ngpus > kMaxSegs) return PHJ_ERR_INVALID;
    std::vector<int> d(ngpus);
    for (int i = 0; i < ngpus; i++) d[i] = devs ? devs[i] : i;
    if (ngpus == 1 && !(flags & (PHJ_CTX_EXCHANGE | PHJ_CTX_LOCAL))) return ctx_create_device(d[0], out);
    return group_create(ngpus, d.data(), flags, ngpus, 0, nullptr, out);
}

int phj_ctx_create(int ngpus, const int* devs, phj_ctx** out) { return phj_ctx_create_ex(ngpus, devs, 0, out); }

int phj_comm_unique_id(uint8_t* id) {
    if (!id) return PHJ_ERR_INVALID;
    RcclApi& api = rccl();
    if (!api.loaded) {
        std::fprintf(stderr, "phj_comm_unique_id: %s\n", api.err.c_str());
        return PHJ_ERR_HIP;
    }
    static_assert(sizeof(ncclUniqueId) == PHJ_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId u;
    if (api.GetUniqueId(&u) != ncclSuccess) return PHJ_ERR_HIP;
    std::memcpy(id, &u, sizeof(u));
    return PHJ_OK;
}

int phj_ctx_create_rank(int device, int nranks, int rank, const uint8_t* id, phj_ctx** out) {
    if (!out) return PHJ_ERR_INVALID;
    *out = nullptr;
    if (!id || nranks < 1 || nranks > kMaxSegs || rank < 0 || rank >= nranks) return PHJ_ERR_INVALID;
    return group_create(1, &device, 0, nranks, rank, id, out);
}

int phj_ctx_info(const phj_ctx* c, int* world, int* rank0, int* nlocal) {
    if (!c) return PHJ_ERR_INVALID;
    if (world) *world = c->group ? c->group->world : 1;
    if (rank0) *rank0 = c->group ? c->group->rank0 : 0;
    if (nlocal) *nlocal = c->group ? c->group->nlocal() : 1;
    return PHJ_OK;
}

void phj_shard_range(uint64_t n, int rank, int world, uint64_t* lo, uint64_t* hi) {
    uint64_t a = 0, b = 0;
    if (world >= 1 && rank >= 0 && rank < world) shard_range(n, rank, world, &a, &b);
    if (lo) *lo = a;
    if (hi) *hi = b;
}

void phj_exchange_layout(uint64_t max_shard, uint32_t num_partitions, uint64_t* codes_elems, uint64_t* block_elems) {
    const uint64_t cap = (max_shard + 63) / 64 * 64;   // both columns stay 16-B aligned in the gathered buffer
    if (codes_elems) *codes_elems = cap;
    if (block_elems) *block_elems = cap + (static_cast<uint64_t>(num_partitions) + 2) / 2;
}

int phj_join_path(const phj_join_params* p, uint64_t build_n, uint64_t probe_n) {
    if (!p) return PHJ_ERR_INVALID;
    if (p->algo == PHJ_ALGO_NO_PARTITIONING) return PHJ_PATH_NO_PARTITIONING;
    if (p->algo != PHJ_ALGO_RADIX) return PHJ_ERR_INVALID;
    phj_ctx tmp;   // default tuning (no device is touched)
    Plan pl, cpl;
    if (make_plan(&tmp, p, pl) != PHJ_OK) return PHJ_ERR_INVALID;
    if (use_cluster(&tmp, pl, probe_n, build_n, cpl)) return PHJ_PATH_LDS_JOIN;
    refine_plan(&tmp, pl, build_n);
    return use_p2probe(&tmp, pl, probe_n, build_n) ? PHJ_PATH_CODE_TABLES : PHJ_PATH_PARTITIONED;
}

int phj_exchange_geometry(const phj_join_params* p, uint64_t total_build, uint32_t* num_segments, uint32_t* shift,
                          uint32_t* sub_bits, uint32_t* sub_shift, int* cluster) {
    if (!p || p->algo != PHJ_ALGO_RADIX) return PHJ_ERR_INVALID;
    phj_ctx tmp;   // default tuning (no device is touched)
    Plan pl, cpl;
    if (make_plan(&tmp, p, pl) != PHJ_OK) return PHJ_ERR_INVALID;
    const bool cl = use_cluster(&tmp, pl, 0, total_build, cpl);
    if (cl) pl = cpl;
    else refine_plan(&tmp, pl, total_build);
    if (num_segments) *num_segments = cl ? pl.nb1 : pl.Ppad;
    if (shift) *shift = cl ? pl.shift1 : 0;
    if (sub_bits) *sub_bits = pl.sub_bits;
    if (sub_shift) *sub_shift = pl.sub_shift;
    if (cluster) *cluster = cl ? 1 : 0;
    return PHJ_OK;
}

void phj_count_contribution(uint64_t count, int failed, uint64_t* words) {
    words[0] = failed ? 0 : count;
    words[1] = failed ? 1 : 0;
}

int phj_count_verdict(const uint64_t* words, uint64_t* matches) {
    if (words[1] != 0) return PHJ_ERR_STATE;
    if (matches) *matches = words[0];
    return PHJ_OK;
}

void phj_ctx_destroy(phj_ctx* c) {
    if (!c) return;
    if (c->group) {
        group_destroy(c->group);
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->aux);
    if (c->count_host) (void)hipHostFree(c->count_host);
    if (c->count_pin) (void)hipHostFree(c->count_pin);
    for (SideState& S : c->side) {
        for (DevBuf* b : {&S.owned, &S.kA, &S.pA, &S.kB, &S.pB, &S.hist1, &S.hist2, &S.bounds1, &S.tbase2,
                          &S.bounds, &S.partials, &S.tseg2, &S.dig, &S.ccur, &S.ctab, &S.tstart, &S.csink})
            free_buf(*b);
    }
    for (DevBuf* b : {&c->ht_tab, &c->ht_desc, &c->r_codes, &c->r_bounds, &c->scan_partials, &c->prep, &c->tkeys, &c->tpays, &c->toffs, &c->gcursor, &c->items, &c->biglist,
                      &c->count, &c->np_tab, &c->np_pays, &c->np_ovf, &c->np_ovfb, &c->np_ovfn, &c->fitems, &c->split, &c->cl_prof, &c->mat_mark, &c->mat_cnt, &c->mat_rows, &c->cl_done})
        free_buf(*b);
    for (hipEvent_t e : c->evpool) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    (void)hipStreamDestroy(c->aux);
    delete c;
}

const char* phj_last_error(const phj_ctx* c) { return c ? c->err.c_str() : "null context"; }

int phj_ctx_set_stream(phj_ctx* c, void* stream) {
    if (!c) return PHJ_ERR_INVALID;
    if (c->group) return on_solo(c, "phj_ctx_set_stream", [&](phj_ctx* m) { return phj_ctx_set_stream(m, stream); });
    PHJ_HIP(c, hipSetDevice(c->device));
    PHJ_HIP(c, hipStreamSynchronize(c->stream));
    PHJ_HIP(c, hipStreamSynchronize(c->aux));
    if (c->own_stream) {
        PHJ_HIP(c, hipStreamDestroy(c->stream));
        c->own_stream = false;
    }
    if (stream) {
        c->stream = static_cast<hipStream_t>(stream);
    } else {
        PHJ_HIP(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
    }
    c->ks = c->stream;
    return PHJ_OK;
}

int phj_ctx_synchronize(phj_ctx* c) {
    if (!c) return PHJ_ERR_INVALID;
    if (c->group) {
        for (phj_ctx* m : c->group->mem) {
            const int rc = phj_ctx_synchronize(m);
            if (rc != PHJ_OK) return set_err(c, rc, m->err);
        }
        return PHJ_OK;
    }
    PHJ_HIP(c, hipStreamSynchronize(c->aux));
    PHJ_HIP(c, hipStreamSynchronize(c->stream));
    return PHJ_OK;
}

int phj_relation_upload(phj_ctx* c, int side, const phj_tuple* host, uint64_t n) {
    PHJ_TRY(check_side(c, side));
    if (n && !host) return set_err(c, PHJ_ERR_INVALID, "null host relation");
    if (c->group) return group_upload(c, side, host, n);
    PHJ_HIP(c, hipSetDevice(c->device));
    SideState& S = c->side[side];
    drop_relation(c, side);
    PHJ_TRY(ensure(c, S.owned, n * sizeof(phj_tuple)));
    if (n) {
        PHJ_HIP(c, hipMemcpyAsync(S.owned.p, host, n * sizeof(phj_tuple), hipMemcpyHostToDevice, c->ks));
        PHJ_HIP(c, hipStreamSynchronize(c->ks));
    }
    S.rel = static_cast<const phj_tuple*>(S.owned.p);
    S.n = n;
    return PHJ_OK;
}

int phj_relation_bind_device(phj_ctx* c, int side, const phj_tuple* dev, uint64_t n) {
    PHJ_TRY(check_side(c, side));
    if (n && !dev) return set_err(c, PHJ_ERR_INVALID, "null device relation");
    if (reinterpret_cast<uintptr_t>(dev) % 16) return set_err(c, PHJ_ERR_INVALID, "relation must be 16-byte aligned");
    if (c->group) {
        PHJ_TRY(on_solo(c, "phj_relation_bind_device", [&](phj_ctx* m) { return phj_relation_bind_device(m, side, dev, n); }));
        return exchange_sizes(c, *c->group, side);
    }
    drop_relation(c, side);
    c->side[side].rel = dev;
    c->side[side].n = n;
    return PHJ_OK;
}

const phj_tuple* phj_relation_device_ptr(phj_ctx* c, int side, uint64_t* n) {
    if (!c || (side != 0 && side != 1)) return nullptr;
    if (c->group) {   // several local devices: rows of all of them, no single pointer
        if (c->group->nlocal() == 1) return phj_relation_device_ptr(c->group->mem[0], side, n);
        if (n) {
            *n = 0;
            for (phj_ctx* m : c->group->mem) *n += m->side[side].n;
        }
        return nullptr;
    }
    if (n) *n = c->side[side].n;
    return c->side[side].rel;
}

int phj_relation_download(phj_ctx* c, int side, phj_tuple* host, uint64_t n) {
    PHJ_TRY(check_side(c, side));
    if (c->group) return group_download(c, side, host, n);
    SideState& S = c->side[side];
    if (n > S.n) return set_err(c, PHJ_ERR_INVALID, "download larger than the relation");
    PHJ_HIP(c, hipSetDevice(c->device));
    if (n) {
        PHJ_HIP(c, hipMemcpyAsync(host, S.rel, n * sizeof(phj_tuple), hipMemcpyDeviceToHost, c->ks));
        PHJ_HIP(c, hipStreamSynchronize(c->ks));
    }
    return PHJ_OK;
}

int phj_relation_generate_sequential(phj_ctx* c, int side, uint64_t n, int64_t start, uint64_t first_index) {
    PHJ_TRY(check_side(c, side));
    if (c->group)
        return group_generate(c, side, n, first_index, [&](phj_ctx* m, uint64_t k, uint64_t first) {
            return phj_relation_generate_sequential(m, side, k, start, first);
        });
    PHJ_HIP(c, hipSetDevice(c->device));
    SideState& S = c->side[side];
    drop_relation(c, side);
    PHJ_TRY(ensure(c, S.owned, n * sizeof(phj_tuple)));
    if (n) {
        const uint32_t g = static_cast<uint32_t>(std::min<uint64_t>((n + kBlock - 1) / kBlock, 65536));
        hipLaunchKernelGGL(k_gen_sequential, dim3(g), dim3(kBlock), 0, c->ks, static_cast<longlong2*>(S.owned.p), n, start,
                           first_index);
        PHJ_LAUNCHED(c, "k_gen_sequential");
        PHJ_HIP(c, hipStreamSynchronize(c->ks));
    }
    S.rel = static_cast<const phj_tuple*>(S.owned.p);
    S.n = n;
    return PHJ_OK;
}

int phj_relation_generate_zipf(phj_ctx* c, int side, uint64_t n, double alpha, int64_t lo, int64_t hi,
                               uint64_t seed, uint64_t first_index) {
    PHJ_TRY(check_side(c, side));
    if (lo >= hi) return set_err(c, PHJ_ERR_INVALID, "Range for Zipf generation is incorrectly specified");
    if (alpha < 0.01) return set_err(c, PHJ_ERR_INVALID, "Skew parameter must be greater than 0.01.");
    if (c->group)
        return group_generate(c, side, n, first_index, [&](phj_ctx* m, uint64_t k, uint64_t first) {
            return phj_relation_generate_zipf(m, side, k, alpha, lo, hi, seed, first);
        });
    PHJ_HIP(c, hipSetDevice(c->device));
    SideState& S = c->side[side];
    drop_relation(c, side);
    PHJ_TRY(ensure(c, S.owned, n * sizeof(phj_tuple)));
    if (n) {
        const uint64_t b0 = first_index / kGenBatch, b1 = (first_index + n + kGenBatch - 1) / kGenBatch;
        const uint32_t g = static_cast<uint32_t>((b1 - b0 + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(k_gen_zipf, dim3(g), dim3(kBlock), 0, c->ks, static_cast<longlong2*>(S.owned.p), n,
                           alpha, static_cast<uint64_t>(hi - lo + 1), lo - 1, seed, first_index);
        PHJ_LAUNCHED(c, "k_gen_zipf");
        PHJ_HIP(c, hipStreamSynchronize(c->ks));
    }
    S.rel = static_cast<const phj_tuple*>(S.owned.p);
    S.n = n;
    return PHJ_OK;
}

int phj_relation_count_in_range(phj_ctx* c, int side, int64_t lo, int64_t hi, uint64_t* count) {
    PHJ_TRY(check_side(c, side));
    if (!count) return set_err(c, PHJ_ERR_INVALID, "null count");
    if (c->group) {   // over this process's shards
        uint64_t t = 0;
        for (phj_ctx* m : c->group->mem) {
            uint64_t k = 0;
            const int rc = phj_relation_count_in_range(m, side, lo, hi, &k);
            if (rc != PHJ_OK) return set_err(c, rc, m->err);
            t += k;
        }
        *count = t;
        return PHJ_OK;
    }
    PHJ_HIP(c, hipSetDevice(c->device));
    SideState& S = c->side[side];
    PHJ_TRY(ensure(c, c->count, 8));
    PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 8, c->ks));
    if (S.n) {
        const uint32_t g = static_cast<uint32_t>(std::min<uint64_t>((S.n + kBlock - 1) / kBlock, 8192));
        hipLaunchKernelGGL(k_count_range, dim3(g), dim3(kBlock), 0, c->ks, reinterpret_cast<const longlong2*>(S.rel),
                           S.n, lo, hi, static_cast<unsigned long long*>(c->count.p));
        PHJ_LAUNCHED(c, "k_count_range");
    }
    return get_count(c, count);
}

int phj_partition(phj_ctx* c, int side, const phj_join_params* p, phj_partitioned* out) {
    PHJ_TRY(check_side(c, side));
    if (c->group) return on_solo(c, "phj_partition", [&](phj_ctx* m) { return phj_partition(m, side, p, out); });
    (void)hipGetLastError();
    if (p && p->algo != PHJ_ALGO_RADIX) return set_err(c, PHJ_ERR_INVALID, "phj_partition needs PHJ_ALGO_RADIX");
    Plan pl;
    PHJ_TRY(make_plan(c, p, pl));
    PHJ_HIP(c, hipSetDevice(c->device));
    // timers accumulate until phj_join / phj_join_partitioned / phj_timers_report
    // reports them; a caller that never reports loses the oldest records
    c->defer_timers = false;
    c->lean_timers = false;
    if (c->timers.size() > kMaxTimerRecs) reset_timers(c);
    PHJ_TRY(partition_side(c, side, pl));
    if (out) *out = c->side[side].view;
    return PHJ_OK;
}

int phj_join_partitioned(phj_ctx* c, const phj_join_params* p, int nbuild, const phj_partitioned* build,
                         phj_join_result* r) {
    if (!c || !r) return PHJ_ERR_INVALID;
    if (c->group)
        return on_solo(c, "phj_join_partitioned", [&](phj_ctx* m) { return phj_join_partitioned(m, p, nbuild, build, r); });
    if (!build) return set_err(c, PHJ_ERR_INVALID, "null build segments");
    if (p && p->algo != PHJ_ALGO_RADIX) return set_err(c, PHJ_ERR_INVALID, "phj_join_partitioned needs PHJ_ALGO_RADIX");
    (void)hipGetLastError();
    Plan pl;
    PHJ_TRY(make_plan(c, p, pl));
    PHJ_HIP(c, hipSetDevice(c->device));
    std::memset(r, 0, sizeof(*r));
    hipEvent_t b0, b1, p1;
    PHJ_TRY(build_and_probe(c, pl, nbuild, build, &b0, &b1, &p1));
    uint64_t m = 0;
    PHJ_TRY(get_count(c, &m));
    r->matches = m;
    r->build_ms = elapsed(c, b0, b1);
    r->probe_ms = elapsed(c, b1, p1);
    if (c->last_fused) {   // one fused launch: split by the kernel's own build / probe clocks
        const double t = elapsed(c, b0, p1), fb = fused_build_fraction(c);
        r->build_ms = t * fb;
        r->probe_ms = t * (1.0 - fb);
    }
    r->total_ms = elapsed(c, b0, p1);
    r->num_partitions = pl.Ppad;
    uint64_t nR = 0;
    for (int g = 0; g < nbuild; g++) nR += build[g].n;
    r->algorithmic_bytes = nR * 32 + c->side[PHJ_SIDE_PROBE].view.n * 8 + nR * 8;
    c->defer_timers = false;
    c->lean_timers = false;
    const int rc = fill_timers(c, r);  // includes the phj_partition launches since the last report
    reset_timers(c);
    return rc;
}

int phj_join_partitioned_async(phj_ctx* c, const phj_join_params* p, int nbuild, const phj_partitioned* build,
                               uint64_t* dev_count) {
    if (!c) return PHJ_ERR_INVALID;
    if (c->group)
        return on_solo(c, "phj_join_partitioned_async",
                       [&](phj_ctx* m) { return phj_join_partitioned_async(m, p, nbuild, build, dev_count); });
    if (!build || !dev_count) return set_err(c, PHJ_ERR_INVALID, "null build segments or count address");
    if (p && p->algo != PHJ_ALGO_RADIX)
        return set_err(c, PHJ_ERR_INVALID, "phj_join_partitioned_async needs PHJ_ALGO_RADIX");
    (void)hipGetLastError();
    Plan pl;
    PHJ_TRY(make_plan(c, p, pl));
    PHJ_HIP(c, hipSetDevice(c->device));
    hipEvent_t b0, b1, p1;
    PHJ_TRY(build_and_probe(c, pl, nbuild, build, &b0, &b1, &p1));
    PHJ_HIP(c, hipMemcpyAsync(dev_count, c->count.p, 8, hipMemcpyDeviceToDevice, c->ks));
    return PHJ_OK;
}

int phj_join(phj_ctx* c, const phj_join_params* p, phj_join_result* r) {
    if (!c || !r) return PHJ_ERR_INVALID;
    (void)hipGetLastError();
    if (!p) return set_err(c, PHJ_ERR_INVALID, "null params");
    if (c->group) {
        std::memset(r, 0, sizeof(*r));
        return group_join(c, p, r, false);
    }
    PHJ_HIP(c, hipSetDevice(c->device));
    std::memset(r, 0, sizeof(*r));
    c->defer_timers = (p->flags & PHJ_DEFER_TIMERS) != 0;
    c->lean_timers = (p->flags & PHJ_LEAN_TIMERS) != 0;
    c->timer_skipped = false;
    c->count_pinned = false;
    if (!c->defer_timers || c->timers.size() > kMaxTimerRecs) reset_timers(c);
    if (p->algo == PHJ_ALGO_NO_PARTITIONING) return join_nopart(c, p, r);
    if (p->algo != PHJ_ALGO_RADIX) return set_err(c, PHJ_ERR_INVALID, "Unrecognized join algorithm");
    Plan pl;
    PHJ_TRY(make_plan(c, p, pl));
    SideState& R = c->side[PHJ_SIDE_BUILD];
    SideState& S = c->side[PHJ_SIDE_PROBE];
    const uint32_t requested = pl.Ppad;   // reported; the join may sub-partition
    hipEvent_t t0, t1, tr, b0, b1, p1;
    Plan cpl;
    if (use_cluster(c, pl, S.n, R.n, cpl)) {
        // the LDS join (phj_cluster.h): S's pass 1 into clusters (codes) on
        // the main stream; R's pass 1 and the big clusters' HBM tables on the
        // aux stream beside it; then the probe builds each cluster's table in
        // LDS and probes S's codes against it
        PHJ_TRY(ensure(c, c->count, 32));
        // the result's phase marks: with deferred timers nothing reads them
        // (the result's phase times stay zero) and, R's chain on the main
        // stream, no stream waits on them: not recorded (each event between
        // two kernels delays the second by ~4 us)
        const int order = c->tune.r_order;
        const bool r_main = order == 1;
        const bool no_marks = c->defer_timers && r_main;
        t0 = tr = b0 = t1 = p1 = nullptr;
        auto phase_mark = [&](hipEvent_t* e) -> int { return no_marks ? PHJ_OK : mark_shared(c, e); };
        if (!no_marks) PHJ_TRY(mark(c, &t0));
        const int64_t* rcodes = nullptr;
        const uint32_t* rbnd = nullptr;
        // R's chain on the aux stream, after event `after`
        // R in tile mode (PHJ_R_CHUNK, default): R through the chunked code
        // pass as S (one launch; 8 shards, so a cluster below the LDS limit
        // has at most 8 + 3 runs), its tiles read by the builds; else the
        // stable pass (k_hist + scan + k_scatter_codes: codes contiguous per cluster)
        SideState* RT = nullptr;
        // after S's pass (PHJ_R_ORDER=1, default) R's chain runs on the main
        // stream itself: nothing runs beside it, and a cross-stream event wait
        // before the probe costs ~15 us (measured gap, r05z timeline)
        auto r_chain = [&](hipEvent_t after) -> int {
            if (!r_main) {
                PHJ_HIP(c, hipStreamWaitEvent(c->aux, after, 0));
                c->ks = c->aux;
            }
            int rc = PHJ_OK;
            if (c->tune.r_chunk && R.n > 0) {
                rc = partition_state(c, R, "R", cpl, true, nullptr, 8);
                if (rc == PHJ_OK && R.hcoded) RT = &R;
            }
            if (!RT) {
                if (rc == PHJ_OK) rc = ensure(c, c->r_codes, std::max<uint64_t>(1, R.n) * 8);
                if (rc == PHJ_OK) rc = ensure(c, c->r_bounds, (static_cast<size_t>(cpl.nb1) + 1) * 4);
                rcodes = static_cast<const int64_t*>(c->r_codes.p);
                rbnd = static_cast<const uint32_t*>(c->r_bounds.p);
                if (rc == PHJ_OK) rc = partition_build(c, cpl, static_cast<int64_t*>(c->r_codes.p), static_cast<uint32_t*>(c->r_bounds.p));
            }
            if (rc == PHJ_OK) rc = phase_mark(&b0);
            // the HBM tables of clusters beyond the LDS limit (none at the
            // balanced configurations; the LDS tables are built inside the probe)
            if (rc == PHJ_OK) rc = timer_begin(c, "build.big", 0);
            if (rc == PHJ_OK) rc = cluster_big_fill(c, cpl, 1, &rcodes, &rbnd, R.n, RT);
            if (rc == PHJ_OK) rc = timer_end(c);
            if (rc == PHJ_OK) rc = phase_mark(&tr);
            c->ks = c->stream;
            return rc;
        };
        // PHJ_R_ORDER: 0 = R's chain beside S's pass 1 (it waits for t0: the
        // previous step's probe read R's codes), 1 = after S's pass 1, 2 = before it
        if (order == 2) {
            PHJ_TRY(r_chain(t0));
            PHJ_HIP(c, hipStreamWaitEvent(c->stream, tr, 0));
        }
        // the code pass's bookkeeping kernel clears the count pair (an empty
        // S takes no chunked pass: a memset). R's chain after S's pass on the
        // same stream: S's bookkeeping kernel also clears R's chunk state (one
        // memset launch and its gap fewer before R's pass)
        const bool pre_clear = r_main && c->tune.r_chunk && R.n > 0 && !c->dry;
        if (pre_clear) {
            PHJ_TRY(ensure(c, R.ccur, chunk_state_bytes(cpl.nb1)));
            c->p1_clear = R.ccur.p;
            c->p1_clear_bytes = chunk_state_bytes(cpl.nb1);
        }
        const int prc = partition_side(c, PHJ_SIDE_PROBE, cpl, true, static_cast<unsigned long long*>(c->count.p));
        c->p1_clear = nullptr;
        if (prc != PHJ_OK) {
            c->p1_cleared = nullptr;
            return prc;
        }
        if (!S.hcoded) PHJ_HIP(c, hipMemsetAsync(c->count.p, 0, 32, c->stream));
        if (order != 2) {
            const int rc = r_chain(t0);
            c->p1_cleared = nullptr;   // (R's pass may not have taken the chunked form)
            PHJ_TRY(rc);
        }
        if (!r_main) PHJ_HIP(c, hipStreamWaitEvent(c->stream, tr, 0));
        PHJ_TRY(phase_mark(&t1));
        // one launch, reported as "build" (the workgroups' table builds in LDS:
        // R's codes read) and "probe" (S's codes read), split by the kernel's own clocks
        PHJ_TRY(timer_begin_split(c, R.n * 8, S.n * 8));
        if (c->lean_timers && c->tune.timers) {   // build.big not timed: a zero-length record keeps the phase listed
            const hipEvent_t e = c->timers.back().a;
            c->timers.insert(c->timers.end() - 2, TimerRec{"build.big", 0, e, e});
        }
        c->count_pinned = false;
        PHJ_TRY(probe_cluster(c, cpl, S, 1, &rcodes, &rbnd, RT, true));
        PHJ_TRY(timer_end_split(c));
        PHJ_TRY(phase_mark(&p1));
        uint64_t m = 0;
        PHJ_TRY(get_count(c, &m, true));
        r->matches = m;
        r->partition_ms = elapsed(c, t0, t1);
        {   // the probe launch split by its clocks (build = the LDS table builds + the big clusters' HBM tables)
            const double t = elapsed(c, t1, p1), fb = c->tune.timers && !c->defer_timers ? fused_build_fraction(c) : 0.0;
            r->build_ms = elapsed(c, b0, tr) + t * fb;
            r->probe_ms = t * (1.0 - fb);
        }
        r->total_ms = elapsed(c, t0, p1);
        r->num_partitions = requested;
        // R: 16 read + 8 written (pass 1), 8 read (probe); S: 16 read + 8 written, 8 read
        r->algorithmic_bytes = R.n * (24 + 8) + S.n * (24 + 8);
        return fill_timers(c, r);
    }
    refine_plan(c, pl, R.n);
    if (use_p2probe(c, pl, S.n, R.n)) {
        // S: pass 1 only (its pass 2 runs inside the probe); R: pass 1 as codes
        // and its tables on the aux stream, beside S (measured: R's chain
        // issued first, or run before S with S's pass 1 on every LDS slot, is
        // 0.05-0.1 ms slower; probing S in row ranges, each beside the next
        // range's pass 1, is 0.3 ms slower: DESIGN.md section 3)
        PHJ_TRY(ensure(c, c->count, 32));
        PHJ_TRY(mark(c, &t0));
        // the code pass's bookkeeping kernel clears the count (hcoded)
        PHJ_TRY(partition_side(c, PHJ_SIDE_PROBE, pl, true, static_cast<unsigned long long*>(c->count.p)));
        // R's chain waits for t0 (the previous step's probe read its tables);
        // the wait is issued after S's pass 1 so that launch goes out first
        PHJ_HIP(c, hipStreamWaitEvent(c->aux, t0, 0));
        c->ks = c->aux;
        int rc = ensure(c, c->r_codes, std::max<uint64_t>(1, R.n) * 8);
        if (rc == PHJ_OK) rc = ensure(c, c->r_bounds, (static_cast<size_t>(pl.Ppad) + 1) * 4);
        const int64_t* rcodes = static_cast<const int64_t*>(c->r_codes.p);
        const uint32_t* rbnd = static_cast<const uint32_t*>(c->r_bounds.p);
        if (rc == PHJ_OK) rc = partition_build(c, pl, static_cast<int64_t*>(c->r_codes.p), static_cast<uint32_t*>(c->r_bounds.p));
        if (rc == PHJ_OK) rc = mark(c, &b0);
        // algorithmic bytes: the codes read, the tables written (~1.7 slots per code)
        if (rc == PHJ_OK) rc = timer_begin(c, "build", R.n * 8 * 3);
        if (rc == PHJ_OK) rc = build_ht(c, pl, 1, &rcodes, &rbnd, R.n);
        if (rc == PHJ_OK) rc = timer_end(c);
        if (rc == PHJ_OK) rc = mark(c, &tr);
        c->ks = c->stream;
        PHJ_TRY(rc);
        PHJ_HIP(c, hipStreamWaitEvent(c->stream, tr, 0));
        PHJ_TRY(mark(c, &t1));
        // algorithmic bytes: the pass-1 output read once (16-B tuples, or 8-B
        // codes after a keys-only pass 1); the tables are re-read from L2
        PHJ_TRY(timer_begin(c, "probe", S.n * (S.p2.keys_only ? 8 : 16)));
        PHJ_TRY(probe_ht(c, pl, S, !S.hcoded));
        PHJ_TRY(timer_end(c));
        PHJ_TRY(mark(c, &p1));
        uint64_t m = 0;
        PHJ_TRY(get_count(c, &m, true));
        r->matches = m;
        r->partition_ms = elapsed(c, t0, t1);
        r->build_ms = elapsed(c, b0, tr);
        r->probe_ms = elapsed(c, t1, p1);
        r->total_ms = elapsed(c, t0, p1);
        r->num_partitions = requested;
        r->algorithmic_bytes = R.n * (24 + 16) + S.n * (16 + 8) + R.n * 24 + S.n * 8;
        return fill_timers(c, r);
    }
    // Partition(R) || Partition(S) (HashJoin.hpp:210-216): S (the long one) is
    // issued first on the ctx stream, R beside it on the aux stream
    PHJ_TRY(mark(c, &t0));
    PHJ_HIP(c, hipStreamWaitEvent(c->aux, t0, 0));
    PHJ_TRY(partition_side(c, PHJ_SIDE_PROBE, pl));
    c->ks = c->aux;
    int rc = partition_side(c, PHJ_SIDE_BUILD, pl);
    if (rc == PHJ_OK) rc = mark(c, &tr);
    c->ks = c->stream;
    PHJ_TRY(rc);
    PHJ_HIP(c, hipStreamWaitEvent(c->stream, tr, 0));
    PHJ_TRY(mark(c, &t1));
    PHJ_TRY(build_and_probe(c, pl, 1, &R.view, &b0, &b1, &p1));
    uint64_t m = 0;
    PHJ_TRY(get_count(c, &m));
    r->matches = m;
    r->partition_ms = elapsed(c, t0, t1);
    r->build_ms = elapsed(c, b0, b1);
    r->probe_ms = elapsed(c, b1, p1);
    if (c->last_fused) {   // one fused launch: split by the kernel's own build / probe clocks
        const double t = elapsed(c, b0, p1), fb = fused_build_fraction(c);
        r->build_ms = t * fb;
        r->probe_ms = t * (1.0 - fb);
    }
    r->total_ms = elapsed(c, t0, p1);
    r->num_partitions = requested;
    r->algorithmic_bytes = partition_bytes(pl, R.n) + partition_bytes(pl, S.n) + R.n * 32 + S.n * 8 + R.n * 8;
    return fill_timers(c, r);
}

int phj_prepare(phj_ctx* c, const phj_join_params* p) {
    if (!c) return PHJ_ERR_INVALID;
    if (!p) return set_err(c, PHJ_ERR_INVALID, "null params");
    if (c->group) {
        phj_join_result r{};
        return group_join(c, p, &r, true);
    }
    (void)hipGetLastError();
    PHJ_HIP(c, hipSetDevice(c->device));
    PHJ_TRY(reserve_events(c, kPrepEvents));
    struct DryScope {
        phj_ctx* c;
        ~DryScope() { c->dry = false; }
    } scope{c};
    c->dry = true;
    if (p->algo == PHJ_ALGO_NO_PARTITIONING) {
        phj_join_result r{};
        return join_nopart(c, p, &r);
    }
    if (p->algo != PHJ_ALGO_RADIX) return set_err(c, PHJ_ERR_INVALID, "Unrecognized join algorithm");
    Plan pl, cpl;
    PHJ_TRY(make_plan(c, p, pl));
    if (use_cluster(c, pl, c->side[PHJ_SIDE_PROBE].n, c->side[PHJ_SIDE_BUILD].n, cpl)) {
        const uint64_t nR = c->side[PHJ_SIDE_BUILD].n;
        PHJ_TRY(partition_side(c, PHJ_SIDE_PROBE, cpl, true));
        PHJ_TRY(ensure(c, c->r_codes, std::max<uint64_t>(1, nR) * 8));
        PHJ_TRY(ensure(c, c->r_bounds, (static_cast<size_t>(cpl.nb1) + 1) * 4));
        PHJ_TRY(partition_build(c, cpl, nullptr, nullptr));
        PHJ_TRY(cluster_big_fill(c, cpl, 1, nullptr, nullptr, nR));
        PHJ_HIP(c, hipStreamSynchronize(c->stream));
        return PHJ_OK;
    }
    refine_plan(c, pl, c->side[PHJ_SIDE_BUILD].n);
    if (use_p2probe(c, pl, c->side[PHJ_SIDE_PROBE].n, c->side[PHJ_SIDE_BUILD].n)) {
        const uint64_t nR = c->side[PHJ_SIDE_BUILD].n;
        PHJ_TRY(partition_side(c, PHJ_SIDE_PROBE, pl, true));
        PHJ_TRY(ensure(c, c->r_codes, std::max<uint64_t>(1, nR) * 8));
        PHJ_TRY(ensure(c, c->r_bounds, (static_cast<size_t>(pl.Ppad) + 1) * 4));
        PHJ_TRY(partition_build(c, pl, nullptr, nullptr));
        PHJ_TRY(build_ht(c, pl, 1, nullptr, nullptr, nR));
        PHJ_TRY(ensure(c, c->count, 32));
        PHJ_HIP(c, hipStreamSynchronize(c->stream));
        return PHJ_OK;
    }
    PHJ_TRY(partition_side(c, PHJ_SIDE_PROBE, pl));
    PHJ_TRY(partition_side(c, PHJ_SIDE_BUILD, pl));
    phj_partitioned seg{};
    seg.n = c->side[PHJ_SIDE_BUILD].n;
    seg.num_partitions = pl.Ppad;
    hipEvent_t b0, b1, p1;
    PHJ_TRY(build_and_probe(c, pl, 1, &seg, &b0, &b1, &p1));
    PHJ_HIP(c, hipStreamSynchronize(c->stream));
    return PHJ_OK;
}

int phj_timers_report(phj_ctx* c, phj_join_result* r) {
    if (!c || !r) return PHJ_ERR_INVALID;
    if (c->group) return on_solo(c, "phj_timers_report", [&](phj_ctx* m) { return phj_timers_report(m, r); });
    PHJ_HIP(c, hipSetDevice(c->device));
    PHJ_HIP(c, hipStreamSynchronize(c->ks));
    std::memset(r, 0, sizeof(*r));
    c->defer_timers = false;
    c->lean_timers = false;
    const int rc = fill_timers(c, r);
    reset_timers(c);
    return rc;
}

int phj_partitioned_download(phj_ctx* c, const phj_partitioned* v, int64_t* keys, int64_t* payloads,
                             uint32_t* bounds) {
    if (!c || !v) return PHJ_ERR_INVALID;
    if (c->group)
        return on_solo(c, "phj_partitioned_download",
                       [&](phj_ctx* m) { return phj_partitioned_download(m, v, keys, payloads, bounds); });
    PHJ_HIP(c, hipSetDevice(c->device));
    if (v->n && keys) PHJ_HIP(c, hipMemcpyAsync(keys, v->keys, v->n * 8, hipMemcpyDefault, c->ks));
    if (v->n && payloads) PHJ_HIP(c, hipMemcpyAsync(payloads, v->payloads, v->n * 8, hipMemcpyDefault, c->ks));
    if (bounds)
        PHJ_HIP(c, hipMemcpyAsync(bounds, v->bounds, (static_cast<size_t>(v->num_partitions) + 1) * 4,
                                  hipMemcpyDefault, c->ks));
    // device-only destinations stay stream-ordered; host destinations need the wait
    auto on_device = [](const void* ptr) {
        if (!ptr) return true;
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, ptr) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return at.type == hipMemoryTypeDevice;
    };
    if (!(on_device(keys) && on_device(payloads) && on_device(bounds))) {
        PHJ_HIP(c, hipStreamSynchronize(c->ks));
        PHJ_TRY(check_chunk_errors(c));   // a chunked pass that met a stale table wrote nothing through it
    }
    return PHJ_OK;
}

static_assert(sizeof(phj_joined) == 24 && sizeof(JoinedRow) == sizeof(phj_joined), "JoinedTuple layout");

int phj_join_materialize(phj_ctx* c, const phj_join_params* p, phj_join_result* r) {
    if (!c || !r) return PHJ_ERR_INVALID;
    if (c->group) return set_err(c, PHJ_ERR_STATE, "phj_join_materialize: single-device contexts only");
    (void)hipGetLastError();
    if (!p) return set_err(c, PHJ_ERR_INVALID, "null params");
    PHJ_HIP(c, hipSetDevice(c->device));
    std::memset(r, 0, sizeof(*r));
    c->defer_timers = false;
    c->lean_timers = false;
    reset_timers(c);
    c->mat_n = 0;
    if (p->algo == PHJ_ALGO_NO_PARTITIONING) {
        SideState& S = c->side[PHJ_SIDE_PROBE];
        if (S.n >= (1ull << 32)) return set_err(c, PHJ_ERR_RANGE, "probe side above 2^32 tuples");
        PHJ_TRY(ensure(c, c->mat_mark, std::max<uint64_t>(1, S.n) * 4));
        PHJ_TRY(join_nopart(c, p, r, static_cast<uint32_t*>(c->mat_mark.p)));
        hipEvent_t e0, e1;
        PHJ_TRY(mark(c, &e0));
        PHJ_TRY(mat_compact(c, S.n, reinterpret_cast<const longlong2*>(S.rel), nullptr, nullptr,
                            static_cast<const int64_t*>(c->np_pays.p)));
        PHJ_TRY(mark(c, &e1));
        PHJ_HIP(c, hipStreamSynchronize(c->ks));
        r->probe_ms += elapsed(c, e0, e1);
        r->total_ms += elapsed(c, e0, e1);
        r->algorithmic_bytes += r->matches * 24;
        PHJ_TRY(fill_timers(c, r));
    } else if (p->algo == PHJ_ALGO_RADIX) {
        PHJ_TRY(join_radix_mark(c, p, r));
    } else {
        return set_err(c, PHJ_ERR_INVALID, "Unrecognized join algorithm");
    }
    c->mat_n = r->matches;
    return PHJ_OK;
}

const phj_joined* phj_joined_rows(phj_ctx* c, uint64_t* n) {
    if (!c || c->group) return nullptr;
    if (n) *n = c->mat_n;
    return static_cast<const phj_joined*>(c->mat_rows.p);
}

int phj_joined_download(phj_ctx* c, phj_joined* host, uint64_t n) {
    if (!c) return PHJ_ERR_INVALID;
    if (c->group) return set_err(c, PHJ_ERR_STATE, "phj_joined_download: single-device contexts only");
    if (n > c->mat_n) return set_err(c, PHJ_ERR_RANGE, "more rows requested than the last materialised join made");
    if (n == 0) return PHJ_OK;
    if (!host) return set_err(c, PHJ_ERR_INVALID, "null destination");
    PHJ_HIP(c, hipSetDevice(c->device));
    PHJ_HIP(c, hipMemcpyAsync(host, c->mat_rows.p, n * sizeof(phj_joined), hipMemcpyDeviceToHost, c->stream));
    PHJ_HIP(c, hipStreamSynchronize(c->stream));
    return PHJ_OK;
}

int phj_probe_pass1(phj_ctx* c, const phj_join_params* p, int64_t* keys, uint64_t n, uint32_t* bounds1,
                    uint32_t* nb1, int* codes) {
    if (!c) return PHJ_ERR_INVALID;
    if (c->group) return set_err(c, PHJ_ERR_STATE, "phj_probe_pass1 takes a single-device context");
    if (!p || !bounds1 || !nb1 || !codes || (n && !keys)) return set_err(c, PHJ_ERR_INVALID, "null argument");
    (void)hipGetLastError();
    PHJ_HIP(c, hipSetDevice(c->device));
    if (p->algo != PHJ_ALGO_RADIX) return set_err(c, PHJ_ERR_INVALID, "radix join parameters required");
    SideState& S = c->side[PHJ_SIDE_PROBE];
    if (n != S.n) return set_err(c, PHJ_ERR_INVALID, "n must be the probe relation's size");
    Plan pl, cpl;
    PHJ_TRY(make_plan(c, p, pl));
    if (use_cluster(c, pl, S.n, c->side[PHJ_SIDE_BUILD].n, cpl)) {
        pl = cpl;   // phj_join's LDS join: pass 1 into its clusters
    } else {
        refine_plan(c, pl, c->side[PHJ_SIDE_BUILD].n);
        if (!use_p2probe(c, pl, S.n, c->side[PHJ_SIDE_BUILD].n))
            return set_err(c, PHJ_ERR_STATE, "these params do not take the on-chip probe");
    }
    c->defer_timers = false;
    c->lean_timers = false;
    reset_timers(c);
    c->ks = c->stream;
    PHJ_TRY(partition_side(c, PHJ_SIDE_PROBE, pl, true));
    const uint32_t nt = S.nt2;
    PHJ_TRY(ensure(c, c->prep, (static_cast<size_t>(nt) + 1) * 4));
    PHJ_TRY(ensure(c, S.kB, std::max<uint64_t>(1, n) * 8));
    auto* off = static_cast<uint32_t*>(c->prep.p);
    hipLaunchKernelGGL(k_tile_counts<4096>, dim3(nt / 256 + 1), dim3(256), 0, c->ks, S.p2, nt, off);
    PHJ_LAUNCHED(c, "k_tile_counts");
    PHJ_TRY(scan_u32(c, off, nt + 1, 1, nt + 1));
    if (nt) {
        hipLaunchKernelGGL(k_gather_pass1<4096>, dim3(nt), dim3(256), 0, c->ks, S.p2, off, static_cast<int64_t*>(S.kB.p));
        PHJ_LAUNCHED(c, "k_gather_pass1");
    }
    uint32_t total = 0;
    PHJ_HIP(c, hipMemcpyAsync(&total, off + nt, 4, hipMemcpyDeviceToHost, c->ks));
    PHJ_HIP(c, hipMemcpyAsync(bounds1, S.bounds1.p, (static_cast<size_t>(pl.nb1) + 1) * 4, hipMemcpyDeviceToHost, c->ks));
    if (n) PHJ_HIP(c, hipMemcpyAsync(keys, S.kB.p, n * 8, hipMemcpyDeviceToHost, c->ks));
    PHJ_HIP(c, hipStreamSynchronize(c->ks));
    PHJ_TRY(check_chunk_errors(c));
    if (total != n) return set_err(c, PHJ_ERR_STATE, "pass-1 tiles hold " + std::to_string(total) + " keys, not " + std::to_string(n));
    *nb1 = pl.nb1;
    *codes = S.hcoded ? 1 : 0;
    return PHJ_OK;
}

int phj_debug_poison_chunk_table(phj_ctx* c, int side, const phj_join_params* p, int byte) {
    if (!c) return PHJ_ERR_INVALID;
    PHJ_TRY(check_side(c, side));
    if (c->group) return set_err(c, PHJ_ERR_STATE, "phj_debug_poison_chunk_table takes a single-device context");
    if (!p || p->algo != PHJ_ALGO_RADIX) return set_err(c, PHJ_ERR_INVALID, "radix join parameters required");
    (void)hipGetLastError();
    PHJ_HIP(c, hipSetDevice(c->device));
    Plan pl, cpl;
    PHJ_TRY(make_plan(c, p, pl));
    bool p1_only;
    if (use_cluster(c, pl, c->side[PHJ_SIDE_PROBE].n, c->side[PHJ_SIDE_BUILD].n, cpl)) {
        pl = cpl;
        p1_only = side == PHJ_SIDE_PROBE;
    } else {
        refine_plan(c, pl, c->side[PHJ_SIDE_BUILD].n);
        // the pass phj_join runs on this side: keys-only codes for the on-chip probe
        p1_only = side == PHJ_SIDE_PROBE && use_p2probe(c, pl, c->side[PHJ_SIDE_PROBE].n, c->side[PHJ_SIDE_BUILD].n);
    }
    SideState& S = c->side[side];
    if (!S.ctab.p) {   // no pass has allocated it yet: size it for phj_join's pass
        struct DryScope {
            phj_ctx* c;
            ~DryScope() { c->dry = false; }
        } scope{c};
        c->dry = true;
        PHJ_TRY(partition_state(c, S, side == PHJ_SIDE_BUILD ? "R" : "S", pl, p1_only));
    }
    if (!S.ctab.p) return set_err(c, PHJ_ERR_STATE, "these params take no chunked pass on this side");
    PHJ_HIP(c, hipMemsetAsync(S.ctab.p, byte & 0xff, S.ctab.bytes, c->stream));
    PHJ_HIP(c, hipStreamSynchronize(c->stream));
    S.ctab_dirty = false;
    return PHJ_OK;
}

int phj_debug_poison_alloc(phj_ctx* c, int byte) {
    if (!c) return PHJ_ERR_INVALID;
    const int v = byte < 0 ? -1 : (byte & 0xff);
    c->poison = v;
    if (c->group)
        for (int i = 0; i < c->group->nlocal(); i++) c->group->mem[i]->poison = v;
    return PHJ_OK;
}

int phj_debug_fail_member(phj_ctx* c, int member) {
    if (!c) return PHJ_ERR_INVALID;
    if (!c->group) return set_err(c, PHJ_ERR_STATE, "phj_debug_fail_member takes a multi-device or rank context");
    if (member < -1 || member >= c->group->nlocal()) return set_err(c, PHJ_ERR_INVALID, "no such local member");
    c->group->fail_member = member;
    return PHJ_OK;
}

int phj_debug_exchange_block(phj_ctx* c, int member, int64_t* out, uint64_t elems) {
    if (!c || !out) return PHJ_ERR_INVALID;
    if (!c->group) return set_err(c, PHJ_ERR_STATE, "phj_debug_exchange_block takes a multi-device or rank context");
    Group& G = *c->group;
    if (member < 0 || member >= G.nlocal()) return set_err(c, PHJ_ERR_INVALID, "no such local member");
    const DevBuf& b = G.buf[member].recv;
    if (!b.p || b.bytes < static_cast<size_t>(G.world) * elems * 8) return set_err(c, PHJ_ERR_STATE, "no exchange block of that size");
    PHJ_HIP(c, hipSetDevice(G.mem[member]->device));
    PHJ_HIP(c, hipStreamSynchronize(G.mem[member]->aux));
    PHJ_HIP(c, hipMemcpy(out, own_block(G, member, elems), elems * 8, hipMemcpyDeviceToHost));
    return PHJ_OK;
}

int phj_hash_keys(phj_ctx* c, int hash, uint64_t seed, const int64_t* keys, uint64_t n, uint64_t* out) {
    if (!c) return PHJ_ERR_INVALID;
    if (c->group)
        return on_solo(c, "phj_hash_keys", [&](phj_ctx* m) { return phj_hash_keys(m, hash, seed, keys, n, out); });
    if (hash != PHJ_HASH_XXH3 && hash != PHJ_HASH_MURMUR3) return set_err(c, PHJ_ERR_INVALID, "unknown hash function");
    if (n == 0) return PHJ_OK;
    (void)hipGetLastError();
    PHJ_HIP(c, hipSetDevice(c->device));
    void *dk = nullptr, *dout = nullptr;
    PHJ_HIP(c, hipMalloc(&dk, n * 8));
    hipError_t e = hipMalloc(&dout, n * 8);
    if (e != hipSuccess) {
        (void)hipFree(dk);
        return set_err(c, PHJ_ERR_NOMEM, "hipMalloc failed");
    }
    int rc = PHJ_OK;
    do {
        if (hipMemcpy(dk, keys, n * 8, hipMemcpyHostToDevice) != hipSuccess) { rc = set_err(c, PHJ_ERR_HIP, "H2D"); break; }
        const uint32_t g = static_cast<uint32_t>((n + kBlock - 1) / kBlock);
        if (hash == PHJ_HASH_MURMUR3)
            hipLaunchKernelGGL((k_hash_keys<kMurmur3>), dim3(g), dim3(kBlock), 0, c->ks, static_cast<int64_t*>(dk), n, seed, static_cast<uint64_t*>(dout));
        else
            hipLaunchKernelGGL((k_hash_keys<kXXH3>), dim3(g), dim3(kBlock), 0, c->ks, static_cast<int64_t*>(dk), n, seed, static_cast<uint64_t*>(dout));
        if (hipGetLastError() != hipSuccess) { rc = set_err(c, PHJ_ERR_HIP, "k_hash_keys launch"); break; }
        if (hipStreamSynchronize(c->ks) != hipSuccess) { rc = set_err(c, PHJ_ERR_HIP, "sync"); break; }
        if (hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost) != hipSuccess) { rc = set_err(c, PHJ_ERR_HIP, "D2H"); break; }
    } while (0);
    (void)hipFree(dk);
    (void)hipFree(dout);
    return rc;
}

}  // extern "C"
