// phj_group.h — several devices behind one phj_ctx: the multi-GPU join
// (SURVEY.md §8(b) "phj_ctx_create(ngpus, devs)", §8(e)).
//
// The reference injects its parallelism into the joiner as a thread pool of
// hardware_concurrency() - 1 workers (src/main.cpp:235-241) and dispatches
// Run() from main (:260-276). Here the joiner's context spans G devices (one
// process, `phj_ctx_create(ngpus, devs)`), or is one device of a G-process
// job (one process per GPU, `phj_ctx_create_rank`). Either way every device
// ("member", global rank r) runs the same step on its range shards
// R_r = rows [r|R|/G, (r+1)|R|/G) and S_r:
//
//   aux stream:   partition R_r (2-pass radix) -> pack keys | bounds -> all-gather
//   main stream:  partition S_r (beside it) -> wait -> fused build + probe of
//                 S_r against the G gathered build segments -> all-reduce(count)
//
// S (95% of the bytes) never leaves its device and stays balanced under any
// key skew; only the build keys travel (the join tests key equality and never
// reads a build payload: RadixCluster/HashJoin.hpp:295-301). NoPartitioning
// replicates R instead (grouped broadcasts = an all-gather-v into one
// contiguous relation), builds the global table on every device and probes
// the local S shard (§8(e) "NoPartitioning multi-GPU").
//
// The exchange is RCCL over xGMI (librccl, resolved at run time so the
// library loads where RCCL is absent). PHJ_CTX_LOCAL replaces the
// collectives by device copies between the members of one process, so the
// multi-member orchestration runs with repeated devices (rehearsal on one GPU,
// where RCCL refuses two ranks per device). A process drives its local members
// from one worker thread each: issuing one member's ~30 launches costs
// ~0.15 ms of host time, which one thread would serialise across 8 devices.
#pragma once

#include <dlfcn.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <type_traits>

#include <rccl/rccl.h>

namespace {

// ---- RCCL, resolved with dlopen on first use ----
struct RcclApi {
    bool loaded = false;
    std::string err;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    decltype(&ncclBroadcast) Broadcast = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

RcclApi& rccl() {
    static RcclApi api = [] {
        RcclApi a;
        // an RCCL already in the process (e.g. torch's) is reused by its soname
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            a.err = std::string("dlopen(librccl.so.1): ") + (e ? e : "not found");
            return a;
        }
        bool ok = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            if (!fp) {
                ok = false;
                a.err = std::string("librccl: missing ") + name;
            }
        };
        sym(a.GetUniqueId, "ncclGetUniqueId");
        sym(a.CommInitRank, "ncclCommInitRank");
        sym(a.CommInitAll, "ncclCommInitAll");
        sym(a.CommDestroy, "ncclCommDestroy");
        sym(a.CommAbort, "ncclCommAbort");
        sym(a.AllGather, "ncclAllGather");
        sym(a.AllReduce, "ncclAllReduce");
        sym(a.Broadcast, "ncclBroadcast");
        sym(a.GroupStart, "ncclGroupStart");
        sym(a.GroupEnd, "ncclGroupEnd");
        sym(a.GetErrorString, "ncclGetErrorString");
        a.loaded = ok;
        return a;
    }();
    return api;
}

#define PHJ_NCCL(ctx, expr)                                                                   \
    do {                                                                                      \
        ncclResult_t r_ = (expr);                                                             \
        if (r_ != ncclSuccess)                                                                \
            return set_err(ctx, PHJ_ERR_HIP, std::string(#expr) + ": " + rccl().GetErrorString(r_)); \
    } while (0)

// ---- member threads: f(i) on thread i, the caller waits for all ----
class MemberThreads {
   public:
    explicit MemberThreads(int n) : n_(n), rc_(n, PHJ_OK) {
        for (int i = 0; i < n; i++) th_.emplace_back([this, i] { loop(i); });
    }
    ~MemberThreads() {
        {
            std::lock_guard<std::mutex> l(m_);
            stop_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    int run(const std::function<int(int)>& f) {
        {
            std::lock_guard<std::mutex> l(m_);
            f_ = &f;
            pending_ = n_;
            gen_++;
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return pending_ == 0; });
        f_ = nullptr;
        for (int rc : rc_)
            if (rc != PHJ_OK) return rc;
        return PHJ_OK;
    }

   private:
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<int(int)>* f = nullptr;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                f = f_;
            }
            const int rc = (*f)(i);
            {
                std::lock_guard<std::mutex> l(m_);
                rc_[i] = rc;
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_;
    std::vector<int> rc_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<int(int)>* f_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

// Reusable barrier of the member threads (PHJ_CTX_LOCAL exchange).
class Barrier {
   public:
    explicit Barrier(int n) : n_(n) {}
    void wait() {
        std::unique_lock<std::mutex> l(m_);
        const uint64_t g = gen_;
        if (++count_ == n_) {
            count_ = 0;
            gen_++;
            cv_.notify_all();
            return;
        }
        cv_.wait(l, [&] { return gen_ != g; });
    }

   private:
    int n_, count_ = 0;
    uint64_t gen_ = 0;
    std::mutex m_;
    std::condition_variable cv_;
};

void shard_range(uint64_t n, int rank, int world, uint64_t* lo, uint64_t* hi) {
    // rows [n*r/G, n*(r+1)/G): 128-bit products keep any n exact
    *lo = static_cast<uint64_t>((static_cast<unsigned __int128>(n) * rank) / world);
    *hi = static_cast<uint64_t>((static_cast<unsigned __int128>(n) * (rank + 1)) / world);
}

// Radix exchange block of one rank: build codes[maxn] | bounds[P + 1] (uint32,
// two per int64 element), the layout of phj_exchange_layout (include/phj.h).
struct PackLayout {
    uint64_t maxn, elems;
};

PackLayout pack_layout(uint64_t maxn, uint32_t P) {
    PackLayout l;
    phj_exchange_layout(maxn, P, &l.maxn, &l.elems);
    return l;
}

enum class Xchg { kRccl, kLocal };

struct MemberBufs {
    // recv: the gathered blocks of every rank; a member packs its own block in
    // place, at its global rank's offset (an in-place all-gather: no send
    // buffer, no copy of its own block)
    DevBuf recv, cnt, full;
    hipEvent_t packed = nullptr;
    bool rehearsal_packed = false;   // PHJ_REHEARSE: this member's block is packed (members > 0 pack once)
    // local NoPartitioning exchange: this member's R shard, published before the
    // barrier (peers never read a member's SideState, which it rebinds to its
    // replicated relation while they copy)
    const phj_tuple* shard = nullptr;
};

struct Group {
    int world = 1;     // global ranks
    int rank0 = 0;     // global rank of local member 0
    Xchg kind = Xchg::kRccl;
    std::vector<phj_ctx*> mem;
    std::vector<ncclComm_t> comm;
    std::vector<MemberBufs> buf;
    std::vector<uint64_t> n[2];   // shard sizes per global rank, per side
    std::unique_ptr<MemberThreads> threads;
    std::unique_ptr<Barrier> barrier;
    std::vector<phj_join_result> res;   // per member, the last join
    std::atomic<int> failed{0};          // local exchange: a member failed before the barrier
    bool rehearse = false;               // PHJ_REHEARSE (local exchange): members > 0 only feed the exchange
    int fail_member = -1;                // phj_debug_fail_member: this local member fails the next join before the exchange
    int nlocal() const { return static_cast<int>(mem.size()); }
};

// Count buffer: {sum, failed} received, {count, failed} sent, then one word
// per rank (exchange_sizes).
size_t cnt_bytes(const Group& G) { return 32 + static_cast<size_t>(G.world) * 8; }

// f(i) for every local member: on the member threads, or inline for one.
int for_members(phj_ctx* shell, Group& G, const std::function<int(int)>& f) {
    int rc;
    if (G.nlocal() == 1) {
        rc = f(0);
    } else {
        rc = G.threads->run(f);
    }
    if (rc != PHJ_OK) {
        for (int i = 0; i < G.nlocal(); i++)
            if (!G.mem[i]->err.empty()) {
                shell->err = "device " + std::to_string(G.rank0 + i) + ": " + G.mem[i]->err;
                break;
            }
    }
    return rc;
}

void group_destroy(Group* G) {
    if (!G) return;
    G->threads.reset();
    for (size_t i = 0; i < G->mem.size(); i++) {
        phj_ctx* c = G->mem[i];
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamSynchronize(c->aux);
        if (i < G->comm.size() && G->comm[i]) (void)rccl().CommDestroy(G->comm[i]);
        MemberBufs& B = G->buf[i];
        for (DevBuf* b : {&B.recv, &B.cnt, &B.full}) free_buf(*b);
        if (B.packed) (void)hipEventDestroy(B.packed);
    }
    for (phj_ctx* c : G->mem) phj_ctx_destroy(c);
    delete G;
}

// Sizes of every rank's shard after a local relation change: known on the
// host when the whole world is local, else one all-gather (the relation calls
// of a multi-process context are collective).
int exchange_sizes(phj_ctx* shell, Group& G, int side) {
    std::vector<uint64_t>& v = G.n[side];
    v.assign(G.world, 0);
    if (G.nlocal() == G.world) {
        for (int i = 0; i < G.nlocal(); i++) v[i] = G.mem[i]->side[side].n;
        return PHJ_OK;
    }
    phj_ctx* c = G.mem[0];
    MemberBufs& B = G.buf[0];
    PHJ_HIP(shell, hipSetDevice(c->device));
    PHJ_TRY(ensure(c, B.cnt, cnt_bytes(G)));
    auto* d = static_cast<uint64_t*>(B.cnt.p);
    const uint64_t mine = c->side[side].n;
    PHJ_HIP(shell, hipMemcpyAsync(d, &mine, 8, hipMemcpyHostToDevice, c->stream));
    PHJ_NCCL(shell, rccl().AllGather(d, d + 2, 1, ncclUint64, G.comm[0], c->stream));
    PHJ_HIP(shell, hipMemcpyAsync(v.data(), d + 2, static_cast<size_t>(G.world) * 8, hipMemcpyDeviceToHost, c->stream));
    PHJ_HIP(shell, hipStreamSynchronize(c->stream));
    return PHJ_OK;
}

// Member i's own exchange block: its global rank's slot of the gathered buffer.
int64_t* own_block(Group& G, int i, uint64_t elems) {
    return static_cast<int64_t*>(G.buf[i].recv.p) + static_cast<size_t>(G.rank0 + i) * elems;
}

uint64_t total(const std::vector<uint64_t>& v) {
    uint64_t t = 0;
    for (uint64_t x : v) t += x;
    return t;
}

// ---- the radix join step of one member ----

// All-gather of `elems` int64 per rank into B.recv (in place: each rank's block
// is already at its slot, own_block), on the member's current launch stream (aux). `ok` = this member packed its block; with the
// local exchange every member reaches the barrier even after an error, and
// nobody copies when any member failed (its block may not exist).
// With RCCL a member that failed before the collective still takes part in it
// (its peers have enqueued theirs and would otherwise wait forever): it sends
// an all-zero block, a valid empty build segment (every bound 0), so the peers
// build and probe sound tables, and it reports the failure through the count
// all-reduce (allreduce_count), which makes every rank return PHJ_ERR_STATE.
// Only when it has no buffers to take part with does it abort its
// communicator: the last resort, since ncclCommAbort tears down the local
// communicator only, and peers blocked in the collective over P2P/SHM may not
// see an error and keep waiting.
int abort_comm(Group& G, int i, int rc) {
    if (G.kind == Xchg::kRccl && G.comm[i]) {
        (void)rccl().CommAbort(G.comm[i]);
        G.comm[i] = nullptr;
    }
    return rc;
}

int allgather_blocks(Group& G, int i, uint64_t elems, bool ok, bool receive = true) {
    phj_ctx* c = G.mem[i];
    MemberBufs& B = G.buf[i];
    if (G.kind == Xchg::kRccl) {
        if (!G.comm[i]) return set_err(c, PHJ_ERR_STATE, "RCCL communicator aborted by an earlier failure");
        if (!B.recv.p || B.recv.bytes < static_cast<size_t>(G.world) * elems * 8)
            return abort_comm(G, i, ok ? set_err(c, PHJ_ERR_STATE, "exchange buffers missing") : PHJ_ERR_STATE);
        int64_t* mine = own_block(G, i, elems);
        if (!ok && hipMemsetAsync(mine, 0, elems * 8, c->ks) != hipSuccess)
            return abort_comm(G, i, PHJ_ERR_STATE);   // cannot send a valid empty segment
        PHJ_NCCL(c, rccl().AllGather(mine, B.recv.p, elems, ncclInt64, G.comm[i], c->ks));
        c->since_ev++;
        return ok ? PHJ_OK : PHJ_ERR_STATE;
    }
    if (ok && hipEventRecord(B.packed, c->ks) != hipSuccess) ok = false;
    if (!ok) G.failed.store(1);
    G.barrier->wait();
    if (G.failed.load()) return ok ? set_err(c, PHJ_ERR_STATE, "another member failed") : PHJ_ERR_STATE;
    if (!receive) return PHJ_OK;
    for (int h = 0; h < G.nlocal(); h++) {
        if (h == i) continue;   // (its own block is packed in place)
        phj_ctx* ch = G.mem[h];
        char* dst = static_cast<char*>(B.recv.p) + static_cast<size_t>(h) * elems * 8;
        const void* src = own_block(G, h, elems);   // (a peer writes only its other slots)
        PHJ_HIP(c, hipStreamWaitEvent(c->ks, G.buf[h].packed, 0));
        if (ch->device == c->device)
            PHJ_HIP(c, hipMemcpyAsync(dst, src, elems * 8, hipMemcpyDeviceToDevice, c->ks));
        else
            PHJ_HIP(c, hipMemcpyPeerAsync(dst, c->device, src, ch->device, elems * 8, c->ks));
    }
    c->since_ev++;
    return PHJ_OK;
}

// Sum of the members' device counts: RCCL all-reduce of {count, failed} on the
// main stream (B.cnt words 2-3 -> 0-1), so a member that failed after the
// exchange makes every rank return an error; or (local) the host adds the
// members' counts afterwards and the member threads carry the errors.
// `failed`: this member has no valid count but still takes part. pair: the
// local count is the on-chip probe's {count, failed} (fold_pass1_error), sent
// as this rank's two words.
int allreduce_count(Group& G, int i, const void* local_count, bool failed = false, bool pair = false) {
    phj_ctx* c = G.mem[i];
    MemberBufs& B = G.buf[i];
    if (G.kind == Xchg::kRccl) {
        if (!G.comm[i]) return set_err(c, PHJ_ERR_STATE, "RCCL communicator aborted by an earlier failure");
        auto* d = static_cast<uint64_t*>(B.cnt.p);
        if (!d) return abort_comm(G, i, set_err(c, PHJ_ERR_STATE, "count buffer missing"));
        // this rank's words of phj_count_contribution: {count, 0}, or {0, 1} when it failed
        uint64_t w[2];
        phj_count_contribution(0, failed ? 1 : 0, w);
        PHJ_HIP(c, hipMemsetAsync(d + 2, 0, 16, c->ks));
        if (failed) PHJ_HIP(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d + 3), static_cast<uint32_t>(w[1]), 1, c->ks));
        else PHJ_HIP(c, hipMemcpyAsync(d + 2, local_count, pair ? 16 : 8, hipMemcpyDeviceToDevice, c->ks));
        PHJ_NCCL(c, rccl().AllReduce(d + 2, d, 2, ncclUint64, ncclSum, G.comm[i], c->ks));
    } else {
        if (failed) return PHJ_OK;
        PHJ_HIP(c, hipMemcpyAsync(B.cnt.p, local_count, pair ? 16 : 8, hipMemcpyDeviceToDevice, c->ks));
    }
    c->since_ev++;
    return PHJ_OK;
}

int read_count(Group& G, int i, uint64_t* out, bool pair = false) {
    phj_ctx* c = G.mem[i];
    if (!c->count_host && hipHostMalloc(reinterpret_cast<void**>(&c->count_host), 16, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        c->count_host = nullptr;
    }
    unsigned long long hs[2] = {0, 0};
    unsigned long long* h = c->count_host ? c->count_host : hs;   // pinned when it could be allocated
    PHJ_HIP(c, hipMemcpyAsync(h, G.buf[i].cnt.p, 16, hipMemcpyDeviceToHost, c->ks));
    PHJ_HIP(c, hipStreamSynchronize(c->ks));
    if (G.kind == Xchg::kLocal) {
        *out = h[0];
        if (pair && h[1]) return chunk_table_error(c, 0);   // this member's probe folded its pass-1 error
        return PHJ_OK;
    }
    const uint64_t words[2] = {h[0], h[1]};
    if (phj_count_verdict(words, out) != PHJ_OK) {
        // some rank failed, this one's own probe perhaps by a pass-1 error
        // folded into its pair: its chunk tables are cleared before their next
        // pass either way (as chunk_table_error does on the local path)
        for (SideState& S : c->side) {
            S.ctab_dirty = true;
            S.chunk_check = false;
        }
        return set_err(c, PHJ_ERR_STATE, std::to_string(h[1]) + " rank(s) failed during the join");
    }
    return PHJ_OK;
}

// The exchange block carries the pass-1 codes and digit bounds of the on-chip
// join (R's pass 2 happens inside the table build), or the fully partitioned
// keys and final bounds of the fused join.
// A cluster plan (pl.cluster: the LDS join, phj_cluster.h) ships each rank's
// R codes contiguous per cluster + the nb1 + 1 cluster bounds.
bool member_p2(const Group& G, const phj_ctx* c, const Plan& pl) {
    return pl.cluster || use_p2probe(c, pl, c->side[PHJ_SIDE_PROBE].n, total(G.n[PHJ_SIDE_BUILD]));
}

PackLayout member_layout(const Group& G, const Plan& pl, bool p2) {
    (void)p2;   // every form ships codes / keys in partition (or cluster) order + bounds
    uint64_t maxn = 0;
    for (uint64_t x : G.n[PHJ_SIDE_BUILD]) maxn = std::max(maxn, x);
    return pack_layout(maxn, pl.cluster ? pl.nb1 : pl.Ppad);
}

int member_alloc_radix(Group& G, int i, const Plan& pl, bool p2) {
    phj_ctx* c = G.mem[i];
    MemberBufs& B = G.buf[i];
    const PackLayout L = member_layout(G, pl, p2);
    PHJ_TRY(ensure(c, B.recv, static_cast<size_t>(G.world) * L.elems * 8));
    PHJ_TRY(ensure(c, B.cnt, cnt_bytes(G)));
    if (!B.packed) PHJ_HIP(c, hipEventCreateWithFlags(&B.packed, hipEventDisableTiming));
    return PHJ_OK;
}

// Build segments of the gathered blocks (keys only, bounds).
void gathered_segments(const Group& G, int i, const PackLayout& L, uint32_t P, phj_partitioned* segs) {
    const int64_t* base = static_cast<const int64_t*>(G.buf[i].recv.p);
    for (int g = 0; g < G.world; g++) {
        segs[g] = phj_partitioned{};
        segs[g].keys = base + static_cast<size_t>(g) * L.elems;
        segs[g].payloads = nullptr;
        segs[g].bounds = reinterpret_cast<const uint32_t*>(base + static_cast<size_t>(g) * L.elems + L.maxn);
        segs[g].n = G.n[PHJ_SIDE_BUILD][g];
        segs[g].num_partitions = P;
    }
}

// The gathered blocks as build_ht segments: codes and partition bounds per rank.
void gathered_codes(const Group& G, int i, const PackLayout& L, const int64_t** codes, const uint32_t** b1) {
    const int64_t* base = static_cast<const int64_t*>(G.buf[i].recv.p);
    for (int g = 0; g < G.world; g++) {
        codes[g] = base + static_cast<size_t>(g) * L.elems;
        b1[g] = reinterpret_cast<const uint32_t*>(base + static_cast<size_t>(g) * L.elems + L.maxn);
    }
}

int member_prepare_radix(Group& G, int i, const Plan& pl) {
    phj_ctx* c = G.mem[i];
    PHJ_HIP(c, hipSetDevice(c->device));
    PHJ_TRY(reserve_events(c, kPrepEvents));
    const bool p2 = member_p2(G, c, pl);
    PHJ_TRY(member_alloc_radix(G, i, pl, p2));
    struct DryScope {
        phj_ctx* c;
        ~DryScope() { c->dry = false; }
    } scope{c};
    c->dry = true;
    PHJ_TRY(partition_side(c, PHJ_SIDE_PROBE, pl, p2));
    const PackLayout L = member_layout(G, pl, p2);
    if (pl.cluster) {
        PHJ_TRY(partition_build(c, pl, nullptr, nullptr));
        PHJ_TRY(cluster_big_fill(c, pl, G.world, nullptr, nullptr, total(G.n[PHJ_SIDE_BUILD])));
    } else if (p2) {
        PHJ_TRY(partition_build(c, pl, nullptr, nullptr));
        PHJ_TRY(build_ht(c, pl, G.world, nullptr, nullptr, total(G.n[PHJ_SIDE_BUILD])));
    } else {
        PHJ_TRY(partition_side(c, PHJ_SIDE_BUILD, pl));
        std::vector<phj_partitioned> segs(G.world);
        gathered_segments(G, i, L, pl.Ppad, segs.data());
        hipEvent_t b0, b1, p1;
        PHJ_TRY(build_and_probe(c, pl, G.world, segs.data(), &b0, &b1, &p1));
    }
    PHJ_HIP(c, hipStreamSynchronize(c->stream));
    return PHJ_OK;
}

int member_radix(Group& G, int i, const Plan& pl, phj_join_result* r) {
    phj_ctx* c = G.mem[i];
    MemberBufs& B = G.buf[i];
    std::memset(r, 0, sizeof(*r));
    const uint32_t P = pl.Ppad;
    SideState& R = c->side[PHJ_SIDE_BUILD];
    // the probe side's pass 2 on-chip (k_probe_ht) against code tables built
    // over the gathered pass-1 blocks on the aux stream, beside the S pass 1
    const bool p2 = member_p2(G, c, pl);
    const PackLayout L = member_layout(G, pl, p2);
    std::vector<phj_partitioned> segs(G.world);   // filled once the exchange buffers exist
    hipEvent_t t0 = nullptr, x0 = nullptr, x1 = nullptr, t1, b0 = nullptr, b1 = nullptr, p1, te, sdone = nullptr;
    // up to the exchange every step runs even after an error (no early
    // return): the local exchange's barrier must see every member
    int rc = hipSetDevice(c->device) == hipSuccess ? PHJ_OK : set_err(c, PHJ_ERR_HIP, "hipSetDevice");
    if (rc == PHJ_OK) {
        if (!c->defer_timers || c->timers.size() > kMaxTimerRecs) reset_timers(c);
        rc = member_alloc_radix(G, i, pl, p2);
    }
    if (rc == PHJ_OK && G.fail_member == i) rc = set_err(c, PHJ_ERR_STATE, "injected failure (phj_debug_fail_member)");
    if (rc == PHJ_OK) rc = mark(c, &t0);
    // R shard, pack and all-gather on the aux stream (S goes beside them);
    // a rehearsal's members > 0 pack their (unchanging) block once and from
    // then on only take part in the exchange, so member 0 has the GPU
    c->ks = c->aux;
    const bool quiet = G.rehearse && i > 0 && B.rehearsal_packed;
    if (quiet) {
        c->ks = c->stream;
        const int rx = allgather_blocks(G, i, L.elems, rc == PHJ_OK, false);
        if (rc == PHJ_OK) rc = rx;
        PHJ_TRY(rc);
        r->total_ms = 0;
        return PHJ_OK;
    }
    // the S shard's pass 1 goes out first, on the main stream (it needs nothing
    // from R): neither the exchange's host-side wait (the local rehearsal's
    // barrier, a blocking collective) nor the host time of issuing R's chain
    // may hold it back (measured W=8 rehearsal: S.p1 started after R's
    // partition, 0.3 ms in, when it was issued after it)
    // The on-chip join then probes on the aux stream right after the tables
    // (one cross-stream wait fewer on the critical path: S's pass 1, and the
    // count reset behind it, are long done by then)
    const bool s_early = !(G.rehearse && i > 0);
    if (rc == PHJ_OK && s_early) {
        c->ks = c->stream;
        if (p2) rc = ensure(c, c->count, 32);
        // the code pass's bookkeeping kernel clears the count (hcoded); else a memset
        if (rc == PHJ_OK)
            rc = partition_side(c, PHJ_SIDE_PROBE, pl, p2, p2 ? static_cast<unsigned long long*>(c->count.p) : nullptr);
        if (rc == PHJ_OK && p2 && !c->side[PHJ_SIDE_PROBE].hcoded && hipMemsetAsync(c->count.p, 0, 32, c->stream) != hipSuccess)
            rc = set_err(c, PHJ_ERR_HIP, "count reset");
        if (rc == PHJ_OK && p2) rc = mark(c, &sdone);
        c->ks = c->aux;
    }
    // R's chain (aux) waits for t0: the previous step's probe read its tables
    // and exchange block (issued after S's pass 1, so that launch goes out first)
    if (rc == PHJ_OK && hipStreamWaitEvent(c->aux, t0, 0) != hipSuccess) rc = set_err(c, PHJ_ERR_HIP, "wait t0");
    if (p2) {   // the R shard as codes in partition order, straight into the exchange block
        if (rc == PHJ_OK)
            rc = partition_build(c, pl, own_block(G, i, L.elems),
                                 reinterpret_cast<uint32_t*>(own_block(G, i, L.elems) + L.maxn));
    } else {
        if (rc == PHJ_OK) rc = partition_side(c, PHJ_SIDE_BUILD, pl);
        if (rc == PHJ_OK && R.n &&
            hipMemcpyAsync(own_block(G, i, L.elems), R.view.keys, R.n * 8, hipMemcpyDeviceToDevice, c->ks) != hipSuccess)
            rc = set_err(c, PHJ_ERR_HIP, "pack keys");
        if (rc == PHJ_OK &&
            hipMemcpyAsync(own_block(G, i, L.elems) + L.maxn, R.view.bounds, (static_cast<size_t>(P) + 1) * 4,
                           hipMemcpyDeviceToDevice, c->ks) != hipSuccess)
            rc = set_err(c, PHJ_ERR_HIP, "pack bounds");
        c->since_ev += 2;
    }
    if (rc == PHJ_OK) rc = mark(c, &x0);
    if (rc == PHJ_OK) rc = timer_begin(c, "exchange", static_cast<uint64_t>(G.world - 1) * L.elems * 8);
    const int rx = allgather_blocks(G, i, L.elems, rc == PHJ_OK);
    if (rc == PHJ_OK) rc = rx;
    if (rc == PHJ_OK) rc = timer_end(c);
    if (rc == PHJ_OK) rc = mark_shared(c, &x1);
    if (p2) {
        b0 = x1;
        const int64_t* codes[kHtSegs];
        const uint32_t* bnd[kHtSegs];
        gathered_codes(G, i, L, codes, bnd);
        const uint64_t nRall = total(G.n[PHJ_SIDE_BUILD]);
        // the probe (aux, behind the tables) needs S's pass 1: the wait goes
        // before the tables, so the marks between them and the probe are one
        // event (a wait between them would cost another)
        if (rc == PHJ_OK && sdone && hipStreamWaitEvent(c->aux, sdone, 0) != hipSuccess) rc = set_err(c, PHJ_ERR_HIP, "wait S");
        if (pl.cluster) {   // only the big clusters' HBM tables; the LDS tables are built in the probe
            if (rc == PHJ_OK) rc = timer_begin(c, "build.big", 0);
            if (rc == PHJ_OK) rc = cluster_big_fill(c, pl, G.world, codes, bnd, nRall);
        } else {
            if (rc == PHJ_OK) rc = timer_begin(c, "build", nRall * 8 * 3);   // codes read, tables written
            if (rc == PHJ_OK) rc = build_ht(c, pl, G.world, codes, bnd, nRall);
        }
        if (rc == PHJ_OK) rc = timer_end(c);
        if (rc == PHJ_OK) rc = mark_shared(c, &b1);
    } else if (rc == PHJ_OK) {
        gathered_segments(G, i, L, P, segs.data());
    }
    c->ks = c->stream;
    if (G.rehearse && i > 0) {   // rehearsal: only member 0 joins (its time = one rank's device work)
        PHJ_TRY(rc);
        B.rehearsal_packed = true;
        PHJ_HIP(c, hipStreamWaitEvent(c->stream, p2 ? b1 : x1, 0));
        PHJ_HIP(c, hipMemsetAsync(B.cnt.p, 0, 8, c->stream));
        PHJ_HIP(c, hipStreamSynchronize(c->stream));
        r->total_ms = 0;
        return PHJ_OK;
    }
    // (the S shard's pass 1 went out on the main stream before the exchange)
    auto join_local = [&]() -> int {
        if (p2) {   // on the aux stream, behind the tables
            c->ks = c->aux;   // (S's pass 1 waited for before the tables)
            PHJ_TRY(mark_shared(c, &t1));
            if (pl.cluster) {   // one launch: "build" (LDS tables) / "probe" by its clocks
                const int64_t* codes[kHtSegs];
                const uint32_t* bnd[kHtSegs];
                gathered_codes(G, i, L, codes, bnd);
                PHJ_TRY(timer_begin_split(c, total(G.n[PHJ_SIDE_BUILD]) * 8, c->side[PHJ_SIDE_PROBE].n * 8));
                if (c->lean_timers && c->tune.timers) {   // build.big not timed: listed at zero
                    const hipEvent_t e = c->timers.back().a;
                    c->timers.insert(c->timers.end() - 2, TimerRec{"build.big", 0, e, e});
                }
                PHJ_TRY(probe_cluster(c, pl, c->side[PHJ_SIDE_PROBE], G.world, codes, bnd));
                PHJ_TRY(timer_end_split(c));
            } else {
                PHJ_TRY(timer_begin(c, "probe", c->side[PHJ_SIDE_PROBE].n * (c->side[PHJ_SIDE_PROBE].p2.keys_only ? 8 : 16)));
                PHJ_TRY(probe_ht(c, pl, c->side[PHJ_SIDE_PROBE], false));
                PHJ_TRY(timer_end(c));
            }
            PHJ_TRY(mark_shared(c, &p1));
            c->last_fused = false;
            return PHJ_OK;
        }
        PHJ_HIP(c, hipStreamWaitEvent(c->stream, x1, 0));
        PHJ_TRY(mark(c, &t1));
        return build_and_probe(c, pl, G.world, segs.data(), &b0, &b1, &p1);
    };
    if (rc == PHJ_OK) rc = join_local();
    // RCCL: a member that failed still takes part in the count all-reduce
    if (rc == PHJ_OK || G.kind == Xchg::kRccl) {
        const int ra = allreduce_count(G, i, c->count.p, rc != PHJ_OK, p2);
        if (rc == PHJ_OK) rc = ra;
    }
    if (rc != PHJ_OK) {
        c->ks = c->stream;
        return rc;
    }
    PHJ_TRY(mark(c, &te));
    uint64_t m = 0;
    rc = read_count(G, i, &m, p2);
    c->ks = c->stream;
    PHJ_TRY(rc);
    r->matches = m;
    r->partition_ms = elapsed(c, t0, t1);
    r->build_ms = elapsed(c, b0, b1);
    r->probe_ms = p2 ? elapsed(c, t1, p1) : elapsed(c, b1, p1);
    if (pl.cluster && c->tune.timers && !c->defer_timers) {   // the LDS probe launch split by its clocks
        const double t = elapsed(c, t1, p1), fb = fused_build_fraction(c);
        r->build_ms += t * fb;
        r->probe_ms = t * (1.0 - fb);
    }
    if (!p2 && c->last_fused && !c->defer_timers) {
        const double t = elapsed(c, b0, p1), fb = fused_build_fraction(c);
        r->build_ms = t * fb;
        r->probe_ms = t * (1.0 - fb);
    }
    r->exchange_ms = elapsed(c, x0, x1);
    r->total_ms = elapsed(c, t0, te);
    r->num_partitions = P;
    const uint64_t nRall = total(G.n[PHJ_SIDE_BUILD]);
    r->algorithmic_bytes = partition_bytes(pl, R.n) + partition_bytes(pl, c->side[PHJ_SIDE_PROBE].n) + nRall * 8 +
                           c->side[PHJ_SIDE_PROBE].n * 8;
    return fill_timers(c, r);
}

// ---- the NoPartitioning step of one member: replicate R, build, probe ----

int member_nopart(Group& G, int i, const phj_join_params* p, phj_join_result* r, bool dry) {
    phj_ctx* c = G.mem[i];
    MemberBufs& B = G.buf[i];
    std::memset(r, 0, sizeof(*r));
    const std::vector<uint64_t>& nr = G.n[PHJ_SIDE_BUILD];
    const uint64_t nRall = total(nr);
    SideState& R = c->side[PHJ_SIDE_BUILD];
    const phj_tuple* shard = R.rel;
    const uint64_t shard_n = R.n;
    struct Restore {   // the member keeps its R shard as its build relation
        SideState& R;
        const phj_tuple* rel;
        uint64_t n;
        ~Restore() {
            R.rel = rel;
            R.n = n;
            R.partitioned = false;
        }
    } restore{R, shard, shard_n};
    // no early return before the local exchange's barrier (see member_radix)
    int rc = hipSetDevice(c->device) == hipSuccess ? PHJ_OK : set_err(c, PHJ_ERR_HIP, "hipSetDevice");
    if (rc == PHJ_OK) {
        reset_timers(c);
        rc = ensure(c, B.full, std::max<uint64_t>(1, nRall) * sizeof(phj_tuple));
    }
    if (rc == PHJ_OK) rc = ensure(c, B.cnt, cnt_bytes(G));
    if (rc == PHJ_OK && !B.packed && hipEventCreateWithFlags(&B.packed, hipEventDisableTiming) != hipSuccess)
        rc = set_err(c, PHJ_ERR_HIP, "hipEventCreate");
    if (rc == PHJ_OK && !dry && G.fail_member == i) rc = set_err(c, PHJ_ERR_STATE, "injected failure (phj_debug_fail_member)");
    auto* full = static_cast<phj_tuple*>(B.full.p);
    if (dry) {
        PHJ_TRY(rc);
        R.rel = full;
        R.n = nRall;
        c->dry = true;
        rc = join_nopart(c, p, r);
        c->dry = false;
        if (rc == PHJ_OK) PHJ_HIP(c, hipStreamSynchronize(c->stream));
        return rc;
    }
    hipEvent_t t0 = nullptr, t1, te;
    if (rc == PHJ_OK) rc = mark(c, &t0);
    if (rc == PHJ_OK) rc = timer_begin(c, "exchange", (nRall - shard_n) * sizeof(phj_tuple));
    if (G.kind == Xchg::kRccl) {
        // a member that failed still takes part (its peers' broadcasts wait
        // for it) when it has the receive buffer, else it aborts the communicator
        if (rc != PHJ_OK && (!full || B.full.bytes < nRall * sizeof(phj_tuple) || !B.cnt.p)) return abort_comm(G, i, rc);
        if (!G.comm[i]) return set_err(c, PHJ_ERR_STATE, "RCCL communicator aborted by an earlier failure");
        // all-gather-v: one broadcast per root, grouped, straight into the
        // contiguous relation (no padding, no compaction)
        uint64_t off = 0;
        PHJ_NCCL(c, rccl().GroupStart());
        for (int g = 0; g < G.world; g++) {
            if (nr[g]) {
                const ncclResult_t e = rccl().Broadcast(g == G.rank0 + i ? static_cast<const void*>(shard) : nullptr,
                                                        full + off, nr[g] * 2, ncclInt64, g, G.comm[i], c->stream);
                if (e != ncclSuccess && rc == PHJ_OK)
                    rc = set_err(c, PHJ_ERR_HIP, std::string("ncclBroadcast: ") + rccl().GetErrorString(e));
            }
            off += nr[g];
        }
        PHJ_NCCL(c, rccl().GroupEnd());
        c->since_ev++;
    } else {
        // the shards are resident and read-only: every member publishes its
        // shard pointer, then after the barrier copies them all from those
        // snapshots (a peer may already have rebound its SideState to its own
        // replicated relation, which is still being filled)
        B.shard = shard;
        if (rc != PHJ_OK) G.failed.store(1);
        G.barrier->wait();
        if (G.failed.load()) return rc != PHJ_OK ? rc : set_err(c, PHJ_ERR_STATE, "another member failed");
        uint64_t off = 0;
        for (int h = 0; h < G.nlocal(); h++) {
            phj_ctx* ch = G.mem[h];
            const void* src = static_cast<const void*>(G.buf[h].shard);
            if (nr[h]) {
                if (ch->device == c->device)
                    PHJ_HIP(c, hipMemcpyAsync(full + off, src, nr[h] * sizeof(phj_tuple), hipMemcpyDeviceToDevice,
                                              c->stream));
                else
                    PHJ_HIP(c, hipMemcpyPeerAsync(full + off, c->device, src, ch->device, nr[h] * sizeof(phj_tuple),
                                                  c->stream));
            }
            off += nr[h];
        }
        c->since_ev++;
    }
    phj_join_result jr{};
    auto join_local = [&]() -> int {
        PHJ_TRY(timer_end(c));
        PHJ_TRY(mark(c, &t1));
        R.rel = full;
        R.n = nRall;
        R.partitioned = false;
        // join_nopart resets nothing: its timers follow the exchange timer
        return join_nopart(c, p, &jr);
    };
    if (rc == PHJ_OK) rc = join_local();
    // RCCL: a member that failed still takes part in the count all-reduce
    if (rc == PHJ_OK || G.kind == Xchg::kRccl) {
        const int ra = allreduce_count(G, i, c->count.p, rc != PHJ_OK);
        if (rc == PHJ_OK) rc = ra;
    }
    if (rc != PHJ_OK) {
        c->ks = c->stream;
        return rc;
    }
    PHJ_TRY(mark(c, &te));
    uint64_t m = 0;
    rc = read_count(G, i, &m);
    c->ks = c->stream;
    PHJ_TRY(rc);
    *r = jr;
    r->matches = m;
    r->exchange_ms = elapsed(c, t0, t1);
    r->total_ms = elapsed(c, t0, te);
    return PHJ_OK;
}

// The member whose step took longest reports the phases (as the reference
// reports the slowest worker, RadixCluster/HashJoin.hpp:63-87); the count is
// the all-reduced (or, local, summed) total.
void merge_results(Group& G, phj_join_result* r) {
    int slow = 0;
    for (int i = 1; i < G.nlocal(); i++)
        if (G.res[i].total_ms > G.res[slow].total_ms) slow = i;
    *r = G.res[slow];
    if (G.kind == Xchg::kLocal) {
        uint64_t m = 0;
        for (const phj_join_result& x : G.res) m += x.matches;
        r->matches = m;
    }
}

int group_join(phj_ctx* shell, const phj_join_params* p, phj_join_result* r, bool dry) {
    Group& G = *shell->group;
    G.res.assign(G.nlocal(), phj_join_result{});
    // PHJ_DEFER_TIMERS (radix joins): each member keeps its timers for
    // phj_timers_report (a rank context: one member); they accumulate over such joins
    // PHJ_LEAN_TIMERS: the build side's pass-1 timers are not recorded
    for (int i = 0; i < G.nlocal(); i++) {
        G.mem[i]->defer_timers = !dry && p->algo == PHJ_ALGO_RADIX && (p->flags & PHJ_DEFER_TIMERS) != 0;
        G.mem[i]->lean_timers = !dry && p->algo == PHJ_ALGO_RADIX && (p->flags & PHJ_LEAN_TIMERS) != 0;
        G.mem[i]->timer_skipped = false;
    }
    G.failed.store(0);
    struct FailOnce {   // an injected failure applies to one join
        Group& G;
        bool dry;
        ~FailOnce() {
            if (!dry) G.fail_member = -1;
        }
    } once{G, dry};
    if (p->algo == PHJ_ALGO_NO_PARTITIONING) {
        if (total(G.n[PHJ_SIDE_BUILD]) == 0)   // LinearProbing.hpp:295-299
            return set_err(shell, PHJ_ERR_INVALID,
                           "LinearProbingHashTable::LinearProbingHashTable: numberOfObjects must be greater than zero.");
        PHJ_TRY(for_members(shell, G, [&](int i) { return member_nopart(G, i, p, &G.res[i], dry); }));
        if (!dry) merge_results(G, r);
        return PHJ_OK;
    }
    if (p->algo != PHJ_ALGO_RADIX) return set_err(shell, PHJ_ERR_INVALID, "Unrecognized join algorithm");
    if (G.world > kMaxSegs) return set_err(shell, PHJ_ERR_RANGE, "at most 16 ranks");
    Plan pl;
    // planned with member 0's tuning (refine_plan below uses it too), so a
    // group plans exactly as a single-device context would
    if (const int rc = make_plan(G.mem[0], p, pl); rc != PHJ_OK) return set_err(shell, rc, G.mem[0]->err);
    const uint32_t requested = pl.Ppad;
    // every rank plans for the GLOBAL build side (the gathered segments), so all
    // ranks partition by the same function: the LDS join's clusters, or the
    // code tables' refined plan
    Plan cpl;
    uint64_t max_s = 0;   // the largest probe shard: every member's S takes the cluster plan's code pass
    for (uint64_t x : G.n[PHJ_SIDE_PROBE]) max_s = std::max(max_s, x);
    if (use_cluster(G.mem[0], pl, max_s, total(G.n[PHJ_SIDE_BUILD]), cpl)) pl = cpl;
    else refine_plan(G.mem[0], pl, total(G.n[PHJ_SIDE_BUILD]));
    if (dry) return for_members(shell, G, [&](int i) { return member_prepare_radix(G, i, pl); });
    PHJ_TRY(for_members(shell, G, [&](int i) { return member_radix(G, i, pl, &G.res[i]); }));
    merge_results(G, r);
    r->num_partitions = requested;
    return PHJ_OK;
}

int group_create(int ngpus, const int* devs, uint32_t flags, int world, int rank0, const uint8_t* unique_id,
                 phj_ctx** out) {
    *out = nullptr;
    auto* G = new Group();
    G->world = world;
    G->rank0 = rank0;
    G->kind = (flags & PHJ_CTX_LOCAL) ? Xchg::kLocal : Xchg::kRccl;
    phj_ctx* shell = new phj_ctx();
    shell->group = G;
    shell->device = devs[0];
    auto fail = [&](int code, const std::string& msg) {
        std::fprintf(stderr, "phj_ctx_create: %s\n", msg.c_str());
        group_destroy(G);
        shell->group = nullptr;
        delete shell;
        return code;
    };
    for (int i = 0; i < ngpus; i++) {
        phj_ctx* c = nullptr;
        const int rc = ctx_create_device(devs[i], &c);
        if (rc != PHJ_OK) return fail(rc, "device " + std::to_string(devs[i]) + " unavailable");
        G->mem.push_back(c);
        G->buf.emplace_back();
    }
    if (G->kind == Xchg::kLocal) {
        if (world != ngpus) return fail(PHJ_ERR_INVALID, "the local exchange needs every rank in this process");
    } else {
        for (int i = 0; i < ngpus; i++)
            for (int j = 0; j < i; j++)
                if (devs[i] == devs[j])
                    return fail(PHJ_ERR_INVALID, "RCCL needs distinct devices (PHJ_CTX_LOCAL rehearses repeated ones)");
        RcclApi& api = rccl();
        if (!api.loaded) return fail(PHJ_ERR_HIP, api.err);
        G->comm.assign(ngpus, nullptr);
        ncclResult_t e;
        if (world == ngpus) {
            e = api.CommInitAll(G->comm.data(), ngpus, devs);
        } else {
            ncclUniqueId id;
            std::memcpy(&id, unique_id, sizeof(id));
            if (hipSetDevice(devs[0]) != hipSuccess) return fail(PHJ_ERR_HIP, "hipSetDevice");
            e = api.CommInitRank(&G->comm[0], world, id, rank0);
        }
        if (e != ncclSuccess) return fail(PHJ_ERR_HIP, std::string("RCCL communicator: ") + api.GetErrorString(e));
    }
    G->rehearse = G->kind == Xchg::kLocal && env_int("PHJ_REHEARSE", 0) != 0;
    G->barrier.reset(new Barrier(ngpus));   // the local exchange waits on it, even with one member
    if (ngpus > 1) G->threads.reset(new MemberThreads(ngpus));
    for (int s = 0; s < 2; s++) G->n[s].assign(world, 0);
    *out = shell;
    return PHJ_OK;
}

// ---- relation calls on a group: the process's rows, split over its members ----

int group_upload(phj_ctx* shell, int side, const phj_tuple* host, uint64_t n) {
    Group& G = *shell->group;
    PHJ_TRY(for_members(shell, G, [&](int i) {
        uint64_t lo, hi;
        shard_range(n, i, G.nlocal(), &lo, &hi);
        return phj_relation_upload(G.mem[i], side, host ? host + lo : nullptr, hi - lo);
    }));
    return exchange_sizes(shell, G, side);
}

int group_generate(phj_ctx* shell, int side, uint64_t n, uint64_t first_index,
                   const std::function<int(phj_ctx*, uint64_t, uint64_t)>& gen) {
    Group& G = *shell->group;
    PHJ_TRY(for_members(shell, G, [&](int i) {
        uint64_t lo, hi;
        shard_range(n, i, G.nlocal(), &lo, &hi);
        return gen(G.mem[i], hi - lo, first_index + lo);
    }));
    return exchange_sizes(shell, G, side);
}

int group_download(phj_ctx* shell, int side, phj_tuple* host, uint64_t n) {
    Group& G = *shell->group;
    uint64_t have = 0;
    for (phj_ctx* c : G.mem) have += c->side[side].n;
    if (n > have) return set_err(shell, PHJ_ERR_INVALID, "download larger than the relation");
    uint64_t off = 0;
    for (phj_ctx* c : G.mem) {
        const uint64_t k = std::min<uint64_t>(n - off, c->side[side].n);
        if (k) {
            const int rc = phj_relation_download(c, side, host + off, k);
            if (rc != PHJ_OK) return set_err(shell, rc, c->err);
        }
        off += k;
    }
    return PHJ_OK;
}

}  // namespace
