// ks_engine.cpp — host side of the C-ABI declared in include/ks_engine.h.
//
// Host responsibilities (everything that is independent of placements):
//  * FIFO + one-pod-per-tick: the bind tick of pod j is max(bind_tick[j-1] + 1, arrival_j)
//    (kubesim/kubesim.go:105-121 pops at most one pod per tick and always binds it), so bind
//    ticks are fixed at submit time.
//  * expiry schedule: a bound-Ok pod q runs while (t - t0) * tick < Σ phase seconds
//    (kubesim/pod/pod.go:67-69), i.e. for dur = ceil(S / tick) ticks.  Its expiry is attached
//    to the first later pod whose bind tick reaches t0 + dur; the device applies it (if q was
//    bound Ok) right before that pod is scheduled.
//  * resource scale: quantities arrive in milli-units; the device holds resource k in units of
//    g_k = gcd of every capacity and request of k seen so far (exact: every fit / LeastRequested
//    / BalancedAllocation result is unit-free).  A pod whose request g_k does not divide shrinks
//    the unit (rescale_kernel multiplies the device state by g_k / g_k').  When every scaled
//    capacity is < 2^29 the kernels use the narrow (32-bit) evaluator, when moreover every scaled
//    capacity and the largest cpu x memory product are < 2^26 the tiny (int32-only) one, else
//    the 64/128-bit one.
//  * batching: launches (expire_head, scan, merge, resolve) until the device counter says
//    every pod due in [tick+1, tick+ticks] is bound, then copies the binds back.
//  * node sharding (ks_shard): every rank holds the whole node state and runs
//    the identical resolver; rank r scans only its contiguous block range, merges it to a
//    per-pod top-L, and one RCCL all-gather per batch exchanges the [B][L] lists, which a
//    second merge reduces to the exact global top-L (the union of exact per-shard top-L lists
//    contains the global top-L).  Binds are then identical on every rank with no further
//    exchange.  Virtual shards (several parts per rank) run the same merge path on one GPU.
// Placements themselves are decided on the device only.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/ks_engine.h"
#include "ks_device.h"


namespace {

constexpr int64_t kMaxNodes = 1LL << 24;  // node ids fit the packed key; lists stay < 2^31 entries
constexpr int64_t kMaxValue = 1LL << 59;
constexpr int kMaxBatch = 256;
constexpr int kDefaultBatch = 256;
constexpr int kChunkBatch = 192;  // default batch of engines on the chunk resolver (ks_load_nodes)
constexpr int64_t kStageMaxPods = 4096;  // submits of up to this many pods are host-staged
#ifndef KS_PG_MIN_WG
#define KS_PG_MIN_WG 2048  // scan workgroups to keep when raising the pods per workgroup
#endif
constexpr int kProfEv = 11;  // per launch: prep | scan | part merges | exchange | merge | resolve (+ 4 on the
                             // pipelined chain's second stream)
constexpr int kRescanWgs = 1024;  // the pipelined chain's conditional local rescan: workgroups
constexpr int64_t kNever = std::numeric_limits<int64_t>::max();
constexpr int64_t kUBlk = 256;   // usage index: pods per block (= the usage kernels' workgroup)
constexpr int64_t kUSup = 64;    // blocks per super block
constexpr int64_t kMaxDigestTicks = 1 << 20;
// the overlap's limit on a rank's scan blocks (step_body)
#ifndef KS_OVERLAP_MAX_BLOCKS
#define KS_OVERLAP_MAX_BLOCKS 256
#endif
constexpr int kOverlapMaxBlocks = KS_OVERLAP_MAX_BLOCKS;

// Growable device array (stream-ordered copies on growth).
template <typename T>
struct DVec {
    T* p = nullptr;
    int64_t n = 0, cap = 0;
    hipError_t reserve(int64_t want, hipStream_t st) {
        if (want <= cap) return hipSuccess;
        int64_t nc = std::max<int64_t>(want, std::max<int64_t>(cap * 2, 1024));
        T* q = nullptr;
        hipError_t e = hipMalloc(&q, sizeof(T) * nc);
        if (e != hipSuccess) return e;
        if (n) {
            e = hipMemcpyAsync(q, p, sizeof(T) * n, hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return e;
            e = hipStreamSynchronize(st);
            if (e != hipSuccess) return e;
        }
        if (p) (void)hipFree(p);
        p = q;
        cap = nc;
        return hipSuccess;
    }
    hipError_t append(const T* h, int64_t k, hipStream_t st) {
        hipError_t e = reserve(n + k, st);
        if (e != hipSuccess) return e;
        if (k) e = hipMemcpyAsync(p + n, h, sizeof(T) * k, hipMemcpyHostToDevice, st);
        n += k;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = cap = 0;
    }
};

// (finish tick, pod) min-heap whose array can be walked: the entries due by a tick are the heap's
// top subtree (flush_expiries visits them without copying or popping the heap)
struct PendingHeap : std::priority_queue<std::pair<int64_t, int64_t>, std::vector<std::pair<int64_t, int64_t>>,
                                         std::greater<std::pair<int64_t, int64_t>>> {
    template <class F>
    void for_each_due(int64_t t, F&& f) const {
        std::vector<size_t> st;
        if (!c.empty() && c[0].first <= t) st.push_back(0);
        while (!st.empty()) {
            const size_t i = st.back();
            st.pop_back();
            f(c[i].second);
            for (size_t k = 2 * i + 1; k <= 2 * i + 2 && k < c.size(); k++)
                if (c[k].first <= t) st.push_back(k);
        }
    }
};

}  // namespace

struct ks_engine {
    ks_config cfg{};
    ks::Cfg dc{};
    hipStream_t st = nullptr;
    int device = 0;
    bool profiling = false;

    // nodes
    int64_t n = 0, n_pad = 0;
    int nwb = 0;
    bool nodes_loaded = false;
    void* node_mem = nullptr;
    ks::NodeSoA s{};

    // pods (device)
    DVec<ks::PodRec> pods;
    DVec<int32_t> dur, b_node, b_status, phase_off, cum_sec, exp_pod;
    DVec<int64_t> exp_off, t0, fin, use, exp_pos;
    DVec<uint8_t> expired;
    DVec<ks::ScanRec> srec;  // the pods' scan records (ks_device.h scan_rec_micro), rebuilt on a rescale
    // pods (host mirror of placement-independent facts)
    std::vector<int64_t> h_bind_tick, h_fin;
    std::vector<int64_t> h_exp_off{0};
    std::vector<int32_t> h_dur;
    std::vector<int32_t> h_total_sec;  // Σ phase seconds, int32 wrapping (Pod.totalSeconds)
    PendingHeap pending;  // (finish tick, pod) not yet attached to a later pod
    int64_t P = 0, F = 0;
    int64_t last_arrival = 0;
    int64_t scale[3] = {1, 1, 1};   // device unit of cpu / memory / gpu, in milli-units
    int64_t max_alloc[3] = {0, 0, 0};  // largest capacity per resource, milli-units
    int mode = ks::kEvalWide;  // evaluator variant (ks_device.h)
    uint32_t flags = 0;        // KS_ENGINE_*
    std::vector<int64_t> h_exp_pos;  // global exp_pod index holding pod q's own expiry, or -1
    // pod keys (Node.CreatePod's pods.Store(key, pod), kubesim/node/node.go:58)
    std::vector<int64_t> h_key;
    std::unordered_map<int64_t, int64_t> key_end;  // key -> latest run end among pods with it
    // host mirror of the binds (name-keyed queries): node (-1 = not bound) and status
    std::vector<int32_t> h_node;
    std::vector<int8_t> h_status;
    // host mirrors the per-tick path passes by value: device-unit pod records, the expiry CSR's
    // pods, the device's expired flags (exact while err == KS_OK: every expiry attached to a pod
    // < done has been applied, plus the ones a flush applied)
    std::vector<ks::PodRec> h_pods;
    std::vector<int32_t> h_exp_pod;
    std::vector<uint8_t> h_expired;
    // host-staged submits: rows for the device arrays in a pinned, device-visible arena, applied by
    // one scatter (or by the per-tick kernel) before any device work reads them
    uint8_t* stage = nullptr;           // pinned host arena
    uint8_t* stage_dev = nullptr;       // its device address
    int64_t stage_cap = 0, stage_used = 0;
    ks::CopySeg* segs = nullptr;        // pinned segment table
    ks::CopySeg* segs_dev = nullptr;
    int seg_cap = 0, nseg = 0, seg_done = 0;
    int64_t xpos_lo = INT64_MAX;        // exp_pos rows [xpos_lo, P) changed since the last flush
    hipEvent_t stage_ev = nullptr;      // recorded after the launch that consumed the last segments
    // per-tick path (ks_tick.hip)
    ks::TickScratch* d_tick = nullptr;
    ks::TickOut* h_tick = nullptr;      // pinned, device-visible
    ks::TickOut* h_tick_dev = nullptr;
    // name-keyed index over binds [0, idx_upto), extended on each query
    int64_t idx_upto = 0;
    std::vector<std::vector<int64_t>> node_pods;      // per node: every pod bound there, FIFO
    // run-interval index for the usage queries: pod q may run only in [t0, end) (end = t0 when
    // it never runs); per block of kUBlk pods and per super block of kUSup blocks the max end
    std::vector<int64_t> h_end, blk_end, sup_end;
    DVec<uint8_t> preg;  // 1: phases non-negative and no int32 wrap (digest by segments)

    // progress
    int64_t tick = 0, done = 0;
    int err = KS_OK;
    std::string errmsg;

    // batch machinery
    int B = kDefaultBatch, PG = 32;
    uint64_t* lists = nullptr;
    uint64_t* cand = nullptr;
    int nblk = 0;
    // node sharding
    int world = 1, rank = 0, vsh = 1;
    ncclComm_t comm = nullptr;
    ks_allgather_fn xfn = nullptr;  // host exchange (ks_shard_host) instead of RCCL
    void* xuser = nullptr;
    uint64_t* h_xbuf = nullptr;     // pinned [world][vsh][B][L]
    std::vector<int> part_lo;  // [world * vsh + 1] block boundaries of the parts
    int blk_lo = 0, blk_n = 0;  // this rank's scan range
    uint64_t* cand_all = nullptr;  // [world * vsh][B][L]
    // pruned block lists (ks_scan.h): per-pod bitmaps of the blocks that wrote a list and thresholds
    bool prune = false;
    int L = ks::kTopL;  // the block lists' length (kTopLOverlap: the overlap's single-shard engines)
    uint64_t* lbit = nullptr;  // [B][nwl]
    uint64_t* lthr = nullptr;  // [2][kThrCopies][B]
    int nwl = 0;
    int64_t* d_ctr = nullptr;
    int64_t* h_ctr = nullptr;  // pinned
    ks::EngineArgs* d_args = nullptr;  // the kernels' argument record (device)
    ks::EngineArgs* h_args = nullptr;  // its pinned host staging
    // overlap of the next batch's scan with the chunk resolver (chunk class, one shard): the
    // speculative scan's argument records (ctr = d_spec + parity) and counters, its workgroups
    bool overlap = true;
    int scan_workers = 0;
    int64_t* d_spec = nullptr;
    ks::EngineArgs* d_args_spec = nullptr;  // [2]: ctr = d_spec + kSpecStride * parity
    ks::EngineArgs* h_args_spec = nullptr;
    // the pipelined sharded chain (round 6, step_body): the next batch's speculative scan, per-part
    // merges and exchange on a second stream beside the resolve; a rescan scans every block locally
    // (d_args_full: the whole block range, the engine's own list set)
    hipStream_t st2 = nullptr;
    hipEvent_t pev_m = nullptr, pev_x = nullptr;
    ks::EngineArgs* d_args_full = nullptr;
    ks::EngineArgs* h_args_full = nullptr;
    // group membership (ks_group_add): stream, counters and argument slots belong to the group
    ks_group* group = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    std::vector<hipEvent_t> prof_ev;
    ks_step_stats stats{};
    ks_kernel_stats kstats{};

    // scratch for queries
    uint8_t* d_mask = nullptr;
    int64_t* d_score = nullptr;
    ks::WinWS* d_sweep = nullptr;    // batch window workspace and node -> E index (n_pad, -1)
    int32_t* d_eidx = nullptr;
    int32_t* d_nslot = nullptr;      // node -> candidate slot of the batch (ks_cand.hip), -1
    int32_t* d_first = nullptr;      // node -> its first kept entry of the batch, kNoFirst
    unsigned long long* d_usage = nullptr;
    DVec<int32_t> d_blk;                  // usage query: candidate pod blocks
    std::vector<int32_t> h_blk;
    DVec<unsigned long long> d_digest;    // [6][T + 1] difference arrays, then the prefix sums
};

namespace {

void engine_free(ks_engine* e);  // ks_destroy's body; a group frees its members with it

// Pod.passedSeconds is int32(clock.Sub(start).Seconds()) (kubesim/pod/pod.go:148-153): past 2^31
// seconds Go's float -> int32 conversion is implementation-defined (amd64: INT32_MIN, so
// IsRunning, pod.go:67-69, would revive every finished pod).  The engine's domain: every tick at
// which a bound pod is evaluated stays below 2^31 seconds after the run's first bind; steps,
// submits and usage queries past it are refused with KS_ERANGE (the oracle refuses the same).
bool in_passed_domain(const ks_engine* e, int64_t first_bind, int64_t t) {
    return t - first_bind <= (int64_t)INT32_MAX / e->cfg.tick_seconds;
}
ks_status fail(ks_engine* e, ks_status code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (e) e->errmsg = buf;
    return code;
}

#define HIPCHK(e, expr)                                                                     \
    do {                                                                                    \
        hipError_t _r = (expr);                                                             \
        if (_r != hipSuccess)                                                               \
            return fail((e), KS_EDEVICE, "%s failed: %s", #expr, hipGetErrorString(_r));    \
    } while (0)

ks::EngineArgs make_args(ks_engine* e) {
    ks::EngineArgs a{};
    a.c = e->dc;
    a.s = e->s;
    a.pods = e->pods.p;
    a.dur = e->dur.p;
    a.exp_off = e->exp_off.p;
    a.exp_pod = e->exp_pod.p;
    a.exp_pos = e->exp_pos.p;
    a.b_node = e->b_node.p;
    a.b_status = e->b_status.p;
    a.expired = e->expired.p;
    a.lists = e->lists;
    a.cand = e->cand;
    a.nblk = e->nblk;
    a.blk_lo = e->blk_lo;
    a.blk_n = e->blk_n;
    a.ctr = e->d_ctr;
    a.B = e->B;
    a.PG = e->PG;
    a.sw = e->d_sweep;
    a.e_idx = e->d_eidx;
    a.n_slot = e->d_nslot;
    a.n_first = e->d_first;
    a.det_cids = e->world * e->vsh > 1 ? 1 : 0;
    a.spec_ctr = e->d_spec;
    a.lbit = e->prune ? e->lbit : nullptr;
    a.lthr = e->prune ? e->lthr : nullptr;
    a.nwl = e->nwl;
    a.lset = 1;  // the engine's own scans (the speculative scan's record: set 0, step_body)
    a.srec = e->srec.p;
    return a;
}

// ---- host-staged submits ---------------------------------------------------------------------
// Staged rows are applied in submission order by one scatter launch (stage_flush) or by the
// per-tick kernel, always before the device work that reads them (stream order).  The arena is
// reused once the launch that consumed its last segment has completed.
hipError_t stage_copy(ks_engine* e, void* dst, const void* src, int64_t bytes);
// The rows of exp_pos that submits rewrote since the last flush, as one segment from the host
// mirror: per-submit rewrites overlap, and the scatter applies segments in parallel.
hipError_t stage_xpos(ks_engine* e) {
    const int64_t lo = e->xpos_lo;
    if (lo >= e->P) return hipSuccess;
    e->xpos_lo = INT64_MAX;
    return stage_copy(e, e->exp_pos.p + lo, e->h_exp_pos.data() + lo, sizeof(int64_t) * (e->P - lo));
}

hipError_t stage_flush(ks_engine* e) {
    if (hipError_t r = stage_xpos(e); r != hipSuccess) return r;
    if (e->seg_done >= e->nseg) return hipSuccess;
    hipError_t r = ks::launch_scatter(e->segs_dev + e->seg_done, e->nseg - e->seg_done, e->st);
    if (r == hipSuccess) r = hipEventRecord(e->stage_ev, e->st);
    e->seg_done = e->nseg;
    return r;
}

// room for `bytes` more in the arena and one more segment
hipError_t stage_room(ks_engine* e, int64_t bytes) {
    if (e->nseg > 0 && e->seg_done == e->nseg && hipEventQuery(e->stage_ev) == hipSuccess) {
        e->stage_used = 0;
        e->nseg = e->seg_done = 0;
    }
    const int64_t need = e->stage_used + bytes + 16;
    if (need <= e->stage_cap && e->nseg < e->seg_cap) return hipSuccess;
    hipError_t r = stage_flush(e);
    if (r == hipSuccess) r = hipStreamSynchronize(e->st);
    if (r != hipSuccess) return r;
    e->stage_used = 0;
    e->nseg = e->seg_done = 0;
    if (bytes + 16 > e->stage_cap) {
        if (e->stage) (void)hipHostFree(e->stage);
        e->stage = nullptr;
        e->stage_cap = std::max<int64_t>(bytes + 16, std::max<int64_t>(2 * e->stage_cap, 1 << 20));
        r = hipHostMalloc(&e->stage, e->stage_cap, hipHostMallocMapped);
        if (r == hipSuccess) r = hipHostGetDevicePointer((void**)&e->stage_dev, e->stage, 0);
        if (r != hipSuccess) { e->stage = nullptr; e->stage_cap = 0; return r; }
    }
    if (e->seg_cap == 0) {
        e->seg_cap = 1 << 16;
        r = hipHostMalloc(&e->segs, sizeof(ks::CopySeg) * e->seg_cap, hipHostMallocMapped);
        if (r == hipSuccess) r = hipHostGetDevicePointer((void**)&e->segs_dev, e->segs, 0);
        if (r == hipSuccess && !e->stage_ev) r = hipEventCreateWithFlags(&e->stage_ev, hipEventDisableTiming);
        if (r != hipSuccess) { e->seg_cap = 0; return r; }
    }
    return hipSuccess;
}

// one staged copy of `bytes` host bytes to device address dst
hipError_t stage_copy(ks_engine* e, void* dst, const void* src, int64_t bytes) {
    if (bytes <= 0) return hipSuccess;
    hipError_t r = stage_room(e, bytes);
    if (r != hipSuccess) return r;
    std::memcpy(e->stage + e->stage_used, src, bytes);
    e->segs[e->nseg++] = ks::CopySeg{(uint8_t*)dst, e->stage_dev + e->stage_used, bytes};
    e->stage_used += (bytes + 15) / 16 * 16;
    return hipSuccess;
}

// DVec::append through the arena (growth flushes first: the copy of the old contents must
// follow the staged rows written into them)
template <typename T>
hipError_t stage_append(ks_engine* e, DVec<T>& v, const T* h, int64_t k) {
    if (v.n + k > v.cap) {
        hipError_t r = stage_flush(e);
        if (r == hipSuccess) r = v.reserve(v.n + k, e->st);
        if (r != hipSuccess) return r;
    }
    hipError_t r = stage_copy(e, v.p + v.n, h, sizeof(T) * k);
    v.n += k;
    return r;
}

// every total + 1 fits the scan's 16-bit key table (weights and constant values are >= 0)
bool key16(const ks_engine* e) {
    return (int64_t)e->dc.const_total + 10 * ((int64_t)e->dc.w_lr + e->dc.w_ba) + 1 < (1 << 16);
}

// the small (register-table) resolver holds this engine's batches
bool small_resolver(const ks_engine* e) {
    return e->B <= ks::small_resolver_max_batch() && e->dc.n_nodes <= ks::small_resolver_max_nodes();
}

// Resolvers, the same binds: the role-split resolve_kernel (16 waves, ks_kernels.hip) takes any
// engine; the register-table resolver (4 waves, ks_resolve.hip) is lighter — four per CU, so a
// what-if group's resolvers run side by side (C4 2.29e11 against 2.16e11 evals/s with the
// role-split kernel's half-size class); the chunk resolver (ks_chunk.hip) takes one
// engine per launch, batches of <= kWinMaxB pods.
// the chunk resolver: node state in 32-bit words (every scaled capacity < 2^32 - 1: the modes >=
// narrow, and the wide mode's decimal-SI memory class, whose capacities scale to 2^31), totals in
// 16 bits
bool chunk_eligible(const ks_engine* e) {
    bool words = e->mode >= ks::kEvalNarrow;
    if (!words) {
        words = true;
        for (int k = 0; k < 3; k++) words &= e->max_alloc[k] / e->scale[k] < (int64_t)0xFFFFFFFF;
    }
    return e->B <= ks::kWinMaxB && words && key16(e);
}
enum Resolver { kResolveRole = 0, kResolveSmall = 1, kResolveChunk = 4 };
// an explicit resolver flag wins over the size class (every resolver is exact on every engine
// its limits admit; the flags exist to test them against each other)
int resolver_of(const ks_engine* e) {
    if ((e->flags & KS_ENGINE_CHUNK_RESOLVER) && chunk_eligible(e)) return kResolveChunk;
    if (e->flags & KS_ENGINE_ONE_POD_RESOLVER) return kResolveRole;
    // default: the register-table resolver for the small class, else the chunk resolver where
    // its limits admit the engine (C3: 8.8e5 vs 7.2e5 pods/s with the one-pod kernel), else
    // the one-pod kernel
    if (small_resolver(e)) return kResolveSmall;
    return chunk_eligible(e) ? kResolveChunk : kResolveRole;
}
// (the chunk resolver runs fused into the batch chain, step_body)
hipError_t launch_resolver(const ks::EngineArgs* d, int S, int mode, int which, hipStream_t st) {
    return which == kResolveSmall ? ks::launch_resolve_small(d, S, mode, st) : ks::launch_resolve(d, S, mode, st);
}
void update_mode(ks_engine* e) {
    int64_t m[3];
    for (int k = 0; k < 3; k++) m[k] = e->max_alloc[k] / e->scale[k];
    const bool narrow = m[0] < ks::kNarrowCap && m[1] < ks::kNarrowCap && m[2] < ks::kNarrowCap;
    const bool tiny = m[0] < ks::kTinyCap && m[1] < ks::kTinyCap && m[2] < ks::kTinyCap && m[0] * m[1] < ks::kTinyCap;
    const bool micro = m[0] < ks::kMicroCap && m[1] < ks::kMicroCap && m[2] < ks::kMicroCap &&
                       m[0] * m[1] < ks::kMicroProd && e->dc.w_lr < ks::kMicroWeight &&
                       e->dc.w_ba < ks::kMicroWeight;
    const bool no_tiny = (e->flags & KS_ENGINE_NO_TINY) != 0;
    e->mode = (e->flags & KS_ENGINE_FORCE_WIDE) ? ks::kEvalWide
            : (micro && !no_tiny && !(e->flags & KS_ENGINE_NO_MICRO)) ? ks::kEvalMicro
            : (tiny && !no_tiny) ? ks::kEvalTiny
            : narrow ? ks::kEvalNarrow : ks::kEvalWide;
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {

// Validation and host-side construction shared by ks_create and ks_group_add (no HIP calls).
ks_status engine_init(const ks_config* cfg, ks_engine** out) {
    if (!cfg || !out) return KS_EINVAL;
    *out = nullptr;
    if (cfg->abi_version != KS_ABI_VERSION) return KS_EINVAL;
    if (cfg->tick_seconds < 1) return KS_EINVAL;
    if (cfg->filter_mode != KS_FILTER_REFERENCE_LITERAL && cfg->filter_mode != KS_FILTER_FEEDS_SCORE)
        return KS_EINVAL;
    if (cfg->filters & ~7u) return KS_EINVAL;
    if (cfg->n_scorers < 0 || cfg->n_scorers > 8) return KS_EINVAL;
    if (cfg->batch_pods < 0 || cfg->batch_pods > kMaxBatch) return KS_EINVAL;
    if (cfg->engine_flags &
        ~(uint32_t)(KS_ENGINE_FORCE_WIDE | KS_ENGINE_NO_TINY | KS_ENGINE_NO_MICRO | KS_ENGINE_ONE_POD_RESOLVER |
                    KS_ENGINE_CHUNK_RESOLVER | KS_ENGINE_NO_OVERLAP | KS_ENGINE_PRUNED_LISTS))
        return KS_EINVAL;
    int64_t const_total = 0, w_lr = 0, w_ba = 0;
    for (int i = 0; i < cfg->n_scorers; i++) {
        const ks_scorer& sc = cfg->scorers[i];
        if (sc.weight < 0) return KS_EINVAL;
        switch (sc.kind) {
            case KS_SCORER_CONST:
                if (sc.value < 0) return KS_EINVAL;
                const_total += (int64_t)sc.weight * sc.value;
                break;
            case KS_SCORER_LEAST_REQUESTED: w_lr += sc.weight; break;
            case KS_SCORER_BALANCED: w_ba += sc.weight; break;
            default: return KS_EINVAL;
        }
    }
    if (const_total + 10 * (w_lr + w_ba) >= (1LL << 30) - 2) return KS_EINVAL;  // total + 1 < 2^30 (resolver ikey)

    ks_engine* e = new ks_engine();
    e->cfg = *cfg;
    e->device = cfg->device;
    e->B = cfg->batch_pods ? cfg->batch_pods : kDefaultBatch;
    e->flags = cfg->engine_flags;
    e->overlap = !(cfg->engine_flags & KS_ENGINE_NO_OVERLAP);
    e->dc.filter_feeds = cfg->filter_mode == KS_FILTER_FEEDS_SCORE;
    e->dc.filters = cfg->filters;
    e->dc.has_scorers = cfg->n_scorers > 0;
    e->dc.w_lr = (int32_t)w_lr;
    e->dc.w_ba = (int32_t)w_ba;
    e->dc.const_total = (int32_t)const_total;
    e->dc.tick_seconds = cfg->tick_seconds;
    *out = e;
    return KS_OK;
}

}  // namespace

extern "C" {

ks_status ks_create(const ks_config* cfg, ks_engine** out) {
    ks_engine* e = nullptr;
    const ks_status v = engine_init(cfg, &e);
    if (v != KS_OK) return v;
    hipError_t r = hipSetDevice(e->device);
    if (r == hipSuccess) r = hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking);
    if (r == hipSuccess) r = hipMalloc(&e->d_ctr, 32 * sizeof(int64_t));
    if (r == hipSuccess) r = hipHostMalloc(&e->h_ctr, 32 * sizeof(int64_t), hipHostMallocDefault);
    if (r == hipSuccess) r = hipMalloc(&e->d_args, sizeof(ks::EngineArgs));
    if (r == hipSuccess) r = hipHostMalloc(&e->h_args, sizeof(ks::EngineArgs), hipHostMallocDefault);
    for (int i = 0; i < 4 && r == hipSuccess; i++) r = hipEventCreate(&e->ev[i]);
    if (r == hipSuccess) r = hipMemsetAsync(e->d_ctr, 0, 32 * sizeof(int64_t), e->st);
    if (r == hipSuccess) r = hipStreamSynchronize(e->st);
    if (r != hipSuccess) {
        engine_free(e);
        return KS_EDEVICE;
    }
    *out = e;
    return KS_OK;
}

}  // extern "C"

namespace {

void engine_free(ks_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->st) (void)hipStreamSynchronize(e->st);
    e->pods.release(); e->dur.release(); e->b_node.release(); e->b_status.release();
    e->phase_off.release(); e->cum_sec.release(); e->exp_pod.release(); e->exp_off.release();
    e->t0.release(); e->fin.release(); e->use.release(); e->expired.release(); e->exp_pos.release();
    e->preg.release(); e->d_blk.release(); e->d_digest.release(); e->srec.release();
    if (e->node_mem) (void)hipFree(e->node_mem);
    if (e->lists) (void)hipFree(e->lists);
    if (e->cand) (void)hipFree(e->cand);
    if (e->cand_all) (void)hipFree(e->cand_all);
    if (e->lbit) (void)hipFree(e->lbit);
    if (e->lthr) (void)hipFree(e->lthr);
    if (e->comm) (void)ncclCommDestroy(e->comm);
    if (e->h_xbuf) (void)hipHostFree(e->h_xbuf);
    if (!e->group) {
        if (e->d_ctr) (void)hipFree(e->d_ctr);
        if (e->h_ctr) (void)hipHostFree(e->h_ctr);
        if (e->d_args) (void)hipFree(e->d_args);
        if (e->h_args) (void)hipHostFree(e->h_args);
    }
    if (e->d_mask) (void)hipFree(e->d_mask);
    if (e->d_score) (void)hipFree(e->d_score);
    if (e->d_sweep) (void)hipFree(e->d_sweep);
    if (e->d_eidx) (void)hipFree(e->d_eidx);
    if (e->d_nslot) (void)hipFree(e->d_nslot);
    if (e->d_first) (void)hipFree(e->d_first);
    if (e->d_spec) (void)hipFree(e->d_spec);
    if (e->d_args_spec) (void)hipFree(e->d_args_spec);
    if (e->h_args_spec) (void)hipHostFree(e->h_args_spec);
    if (e->st2) (void)hipStreamSynchronize(e->st2);
    if (e->d_args_full) (void)hipFree(e->d_args_full);
    if (e->h_args_full) (void)hipHostFree(e->h_args_full);
    if (e->pev_m) (void)hipEventDestroy(e->pev_m);
    if (e->pev_x) (void)hipEventDestroy(e->pev_x);
    if (e->st2) (void)hipStreamDestroy(e->st2);
    if (e->d_usage) (void)hipFree(e->d_usage);
    if (e->stage) (void)hipHostFree(e->stage);
    if (e->segs) (void)hipHostFree(e->segs);
    if (e->stage_ev) (void)hipEventDestroy(e->stage_ev);
    if (e->d_tick) (void)hipFree(e->d_tick);
    if (e->h_tick) (void)hipHostFree(e->h_tick);
    for (auto ev : e->ev) if (ev) (void)hipEventDestroy(ev);
    for (auto ev : e->prof_ev) (void)hipEventDestroy(ev);
    if (e->st && !e->group) (void)hipStreamDestroy(e->st);
    delete e;
}

}  // namespace

extern "C" {

// a group's members are destroyed with their group (ks_group_destroy)
void ks_destroy(ks_engine* e) {
    if (e && !e->group) engine_free(e);
}

ks_status ks_comm_unique_id(uint8_t* id_out) {
    if (!id_out) return KS_EINVAL;
    ncclUniqueId uid;
    if (ncclGetUniqueId(&uid) != ncclSuccess) return KS_EDEVICE;
    static_assert(sizeof(uid) == KS_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id_out, &uid, sizeof uid);
    return KS_OK;
}

ks_status ks_shard(ks_engine* e, int32_t world, int32_t rank, const uint8_t* id, int32_t vshards) {
    if (!e) return KS_EINVAL;
    if (e->nodes_loaded) return fail(e, KS_EINVAL, "ks_shard must precede ks_load_nodes");
    if (e->comm) return fail(e, KS_EINVAL, "already sharded");
    if (world < 1 || rank < 0 || rank >= world || vshards < 1 || (int64_t)world * vshards > 4096)
        return fail(e, KS_EINVAL, "bad shard geometry world=%d rank=%d vshards=%d", world, rank, vshards);
    if (world > 1 && !id) return fail(e, KS_EINVAL, "world > 1 needs a communicator id");
    HIPCHK(e, hipSetDevice(e->device));
    if (id) {
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof uid);
        const ncclResult_t r = ncclCommInitRank(&e->comm, world, uid, rank);
        if (r != ncclSuccess) {
            e->comm = nullptr;
            return fail(e, KS_EDEVICE, "ncclCommInitRank: %s", ncclGetErrorString(r));
        }
    }
    e->world = world;
    e->rank = rank;
    e->vsh = vshards;
    return KS_OK;
}

ks_status ks_shard_host(ks_engine* e, int32_t world, int32_t rank, int32_t vshards, ks_allgather_fn fn, void* user) {
    if (!e) return KS_EINVAL;
    if (e->nodes_loaded) return fail(e, KS_EINVAL, "ks_shard_host must precede ks_load_nodes");
    if (e->comm || e->xfn) return fail(e, KS_EINVAL, "already sharded");
    if (!fn || world < 1 || rank < 0 || rank >= world || vshards < 1 || (int64_t)world * vshards > 4096)
        return fail(e, KS_EINVAL, "bad host-exchange shard geometry world=%d rank=%d vshards=%d", world, rank, vshards);
    e->world = world;
    e->rank = rank;
    e->vsh = vshards;
    e->xfn = fn;
    e->xuser = user;
    return KS_OK;
}

ks_status ks_merge_candidates(const uint64_t* cand_all, int32_t parts, int32_t B, uint64_t* out) {
    if (!cand_all || !out || parts < 1 || B < 0) return KS_EINVAL;
    constexpr int L = ks::kTopL;
    for (int64_t b = 0; b < B; b++) {
        uint64_t top[L] = {};
        for (int64_t p = 0; p < parts; p++) {
            uint64_t lv[L];
            std::memcpy(lv, cand_all + (p * B + b) * L, sizeof(lv));
            ks::topl_insert(top, lv);
        }
        std::memcpy(out + b * L, top, sizeof(top));
    }
    return KS_OK;
}

ks_status ks_shard_layout(int64_t n_nodes, int32_t world, int32_t vshards, int32_t* part_lo_out) {
    if (!part_lo_out || n_nodes < 0 || n_nodes > kMaxNodes || world < 1 || vshards < 1 || (int64_t)world * vshards > 4096)
        return KS_EINVAL;
    const int64_t n_pad = std::max<int64_t>(64, (n_nodes + 63) / 64 * 64);
    const int64_t nblk = (n_pad + ks::block_nodes() - 1) / ks::block_nodes();
    const int G = world * vshards;
    for (int p = 0; p <= G; p++) part_lo_out[p] = (int32_t)((int64_t)p * nblk / G);
    return KS_OK;
}

ks_status ks_load_nodes(ks_engine* e, int64_t n, const int64_t* alloc, const uint64_t* taint, const uint64_t* label) {
    if (!e) return KS_EINVAL;
    if (e->nodes_loaded) return fail(e, KS_EINVAL, "nodes already loaded");
    if (n < 0 || n > kMaxNodes) return fail(e, KS_EINVAL, "node count %lld outside [0, %lld]", (long long)n, (long long)kMaxNodes);
    if (n && (!alloc || !taint || !label)) return fail(e, KS_EINVAL, "null node buffer");
    for (int64_t i = 0; i < n; i++) {
        for (int k = 0; k < 3; k++)
            if (alloc[i * 4 + k] < -1 || alloc[i * 4 + k] >= kMaxValue)
                return fail(e, KS_EINVAL, "node %lld: capacity %d out of range", (long long)i, k);
        if (alloc[i * 4 + 3] < 0 || alloc[i * 4 + 3] >= kMaxValue)
            return fail(e, KS_EINVAL, "node %lld: pods capacity out of range", (long long)i);
    }
    HIPCHK(e, hipSetDevice(e->device));
    e->n = n;
    e->n_pad = std::max<int64_t>(64, (n + 63) / 64 * 64);
    e->nwb = (int)(e->n_pad / 64);
    const int64_t np = e->n_pad;
    // host staging in SoA order: ac am ag ap rc rm rg nr taint label
    for (int k = 0; k < 3; k++) {
        int64_t g = 0, mx = 0;
        for (int64_t i = 0; i < n; i++) {
            const int64_t v = alloc[i * 4 + k];
            if (v > 0) { g = std::gcd(g, v); mx = std::max(mx, v); }
        }
        e->scale[k] = g > 0 ? g : 1;
        e->max_alloc[k] = mx;
    }
    update_mode(e);
    std::vector<int64_t> h(10 * np, 0);
    for (int64_t i = 0; i < np; i++) {
        const bool real = i < n;
        for (int k = 0; k < 4; k++) h[k * np + i] = real ? alloc[i * 4 + k] : (k == 3 ? 0 : -1);
        for (int k = 0; k < 3; k++)
            if (real && h[k * np + i] > 0) h[k * np + i] /= e->scale[k];
        h[8 * np + i] = real ? (int64_t)taint[i] : 0;
        h[9 * np + i] = real ? (int64_t)label[i] : 0;
    }
    HIPCHK(e, hipMalloc(&e->node_mem, sizeof(int64_t) * 10 * np));
    HIPCHK(e, hipMemcpyAsync(e->node_mem, h.data(), sizeof(int64_t) * 10 * np, hipMemcpyHostToDevice, e->st));
    int64_t* b = (int64_t*)e->node_mem;
    e->s.ac = b; e->s.am = b + np; e->s.ag = b + 2 * np; e->s.ap = b + 3 * np;
    e->s.rc = b + 4 * np; e->s.rm = b + 5 * np; e->s.rg = b + 6 * np; e->s.nr = b + 7 * np;
    e->s.taint = (uint64_t*)(b + 8 * np); e->s.label = (uint64_t*)(b + 9 * np);
    e->dc.n_nodes = (int32_t)n;
    e->dc.nwb = e->nwb;
    // pods per scan workgroup: the most pod reuse per node load that still leaves >= ~2048
    // workgroups (8 per CU) per scan
    e->nblk = (int)((e->n_pad + ks::block_nodes() - 1) / ks::block_nodes());
    const int G = e->world * e->vsh;
    e->part_lo.assign(G + 1, 0);
    (void)ks_shard_layout(n, e->world, e->vsh, e->part_lo.data());
    e->blk_lo = e->part_lo[e->rank * e->vsh];
    e->blk_n = e->part_lo[(e->rank + 1) * e->vsh] - e->blk_lo;
    // default batch: small clusters exhaust a pod's top-L list after fewer binds, so a batch of
    // 256 would mostly commit early and rescan; ~n/16 pods rounded down to a multiple of 32
    // (>= 64) keeps most of each batch (C4's 2,000-node scenarios: 96 pods 2.64e11 evals/s, 128
    // pods 2.57e11, 64 pods 2.56-2.63e11; round 1: 256 pods 6.1e7 pods/s vs 128 pods 7.9e7)
    if (!e->cfg.batch_pods && n < 16 * kDefaultBatch)
        e->B = (int)std::clamp<int64_t>(n / 16 / 32 * 32, 64, kDefaultBatch);
    // the chunk resolver's default batch: three 64-pod chunks.  Its per-chunk cache of earlier
    // binds grows with the chunk's position, and 256-pod batches hit the candidate-id table
    // (~215 pods committed): 192 pods binds more per second on C3 (9.96e5 vs 9.12e5 pods/s,
    // 224: 9.53e5, 176: 9.64e5, 128: 9.49e5) and C5 (3.67e5 vs 3.19e5; tests/dev/ab_resolvers.py)
    if (!e->cfg.batch_pods && !e->group && !small_resolver(e) && chunk_eligible(e) &&
        !(e->flags & KS_ENGINE_ONE_POD_RESOLVER))
        e->B = kChunkBatch;
    // pods per scan workgroup: the most pod reuse per node load that still leaves >= ~2048
    // workgroups (8 per CU) per scan
    int pg = 1;
    while (pg < ks::max_pods_per_scan_wg() && pg < e->B &&
           (int64_t)e->blk_n * ((e->B + pg * 2 - 1) / (pg * 2)) >= KS_PG_MIN_WG)
        pg *= 2;
    e->PG = pg;
    // (the overlap's single-shard engines may scan lists of kTopLOverlap keys: step_body)
    // (and the pipelined sharded engines': every sharded engine may)
    const int lmax = (G == 1 && e->blk_n <= kOverlapMaxBlocks) || G > 1 ? ks::kTopLOverlap : ks::kTopL;
    HIPCHK(e, hipMalloc(&e->lists, sizeof(uint64_t) * (size_t)e->B * e->nblk * lmax));
    HIPCHK(e, hipMalloc(&e->cand, sizeof(uint64_t) * (size_t)e->B * ks::kTopL));
    if (G > 1) HIPCHK(e, hipMalloc(&e->cand_all, sizeof(uint64_t) * (size_t)G * e->B * ks::kTopLOverlap));
    if (G > 1 && e->xfn) HIPCHK(e, hipHostMalloc(&e->h_xbuf, sizeof(uint64_t) * (size_t)G * e->B * ks::kTopLOverlap, hipHostMallocDefault));
    HIPCHK(e, hipMalloc(&e->d_mask, std::max<int64_t>(n, 1)));
    HIPCHK(e, hipMalloc(&e->d_score, sizeof(int64_t) * std::max<int64_t>(n, 1)));
    HIPCHK(e, hipMalloc(&e->d_usage, sizeof(unsigned long long) * 3 * std::max<int64_t>(n, 1)));
    HIPCHK(e, hipStreamSynchronize(e->st));
    e->nodes_loaded = true;
    return KS_OK;
}

ks_status ks_submit_pods(ks_engine* e, int64_t m, const int64_t* arrival, const int64_t* req, const uint8_t* keymask,
                         const uint64_t* tol, const uint64_t* sel, const int32_t* phase_off, const int32_t* phase_sec,
                         const int64_t* phase_use, const uint8_t* flags, const int64_t* key_id) {
    if (!e) return KS_EINVAL;
    if (!e->nodes_loaded) return fail(e, KS_EINVAL, "ks_load_nodes must precede ks_submit_pods");
    if (m < 0) return fail(e, KS_EINVAL, "negative pod count");
    if (m == 0) return KS_OK;
    if (!arrival || !req || !keymask || !tol || !sel || !phase_off) return fail(e, KS_EINVAL, "null pod buffer");
    if (e->P + m >= (1LL << 31)) return fail(e, KS_EINVAL, "too many pods");
    if (phase_off[0] != 0) return fail(e, KS_EINVAL, "phase_off[0] must be 0");
    const int64_t nf = phase_off[m];
    if (nf && (!phase_sec || !phase_use)) return fail(e, KS_EINVAL, "null phase buffer");
    // validate first, mutate after
    int64_t last = e->last_arrival;
    for (int64_t i = 0; i < m; i++) {
        if (arrival[i] < last) return fail(e, KS_EINVAL, "arrival ticks must be non-decreasing (pod %lld)", (long long)(e->P + i));
        last = arrival[i];
        if (phase_off[i + 1] < phase_off[i]) return fail(e, KS_EINVAL, "phase_off must be non-decreasing");
        if (key_id && key_id[i] < 0) return fail(e, KS_EINVAL, "pod %lld: key ids must be >= 0", (long long)(e->P + i));
        for (int k = 0; k < 3; k++)
            if (req[i * 3 + k] < 0 || req[i * 3 + k] >= kMaxValue)
                return fail(e, KS_EINVAL, "pod %lld: request out of range", (long long)(e->P + i));
    }
    for (int64_t f = 0; f < nf * 3; f++)
        if (phase_use[f] < 0 || phase_use[f] >= kMaxValue) return fail(e, KS_EINVAL, "usage out of range");
    // the int32 passed-seconds domain (kubesim/pod/pod.go:148-153): every bind tick must stay
    // within 2^31 seconds of the run's first bind
    {
        int64_t pb = e->P ? e->h_bind_tick[e->P - 1] : e->tick;
        const int64_t first = e->P ? e->h_bind_tick[0] : std::max<int64_t>(pb + 1, std::max<int64_t>(arrival[0], e->tick + 1));
        for (int64_t i = 0; i < m; i++) {
            pb = std::max<int64_t>(pb + 1, std::max<int64_t>(arrival[i], e->tick + 1));
            if (!in_passed_domain(e, first, pb))
                return fail(e, KS_ERANGE, "pod %lld: bind tick %lld is %lld ticks after the first bind (tick %lld): "
                            "(t - t0) * %d s reaches 2^31 and Go's int32(passed seconds) leaves its domain",
                            (long long)(e->P + i), (long long)pb, (long long)(pb - first), (long long)first,
                            e->cfg.tick_seconds);
        }
    }
    // Pod keys: a Store over a same-key pod that is still running on the chosen node would drop
    // that pod from the node's totals (kubesim/node/node.go:58).  Refuse the one case where that
    // can happen — an earlier pod with the key may still run at this pod's bind tick — so every
    // accepted trace schedules exactly as the reference (ks_engine.h, ks_submit_pods).
    std::unordered_map<int64_t, int64_t> new_end;  // this call's keys -> latest run end
    if (key_id) {
        int64_t pb = e->P ? e->h_bind_tick[e->P - 1] : e->tick;
        for (int64_t i = 0; i < m; i++) {
            const int64_t bt = std::max<int64_t>(pb + 1, std::max<int64_t>(arrival[i], e->tick + 1));
            pb = bt;
            int64_t prev = std::numeric_limits<int64_t>::min();
            auto it = new_end.find(key_id[i]);
            if (it != new_end.end()) prev = it->second;
            else if (auto jt = e->key_end.find(key_id[i]); jt != e->key_end.end()) prev = jt->second;
            if (prev > bt)
                return fail(e, KS_ERANGE, "pod %lld: key %lld reused at bind tick %lld while an earlier pod with it may run "
                            "until tick %lld (Store would replace a running pod: outside the exact domain)",
                            (long long)(e->P + i), (long long)key_id[i], (long long)bt, (long long)prev);
            uint32_t acc = 0;
            for (int32_t f = phase_off[i]; f < phase_off[i + 1]; f++) acc += (uint32_t)phase_sec[f];
            const int32_t S = (int32_t)acc;
            const int64_t d = S > 0 ? ((int64_t)S + e->cfg.tick_seconds - 1) / e->cfg.tick_seconds : 0;
            new_end[key_id[i]] = std::max(prev, bt + d);
        }
    }

    {
        int64_t f[3] = {1, 1, 1};
        bool any = false;
        for (int k = 0; k < 3; k++) {
            int64_t g = e->scale[k];
            for (int64_t i = 0; i < m; i++)
                if ((keymask[i] >> k & 1) && req[i * 3 + k] > 0) g = std::gcd(g, req[i * 3 + k]);
            f[k] = e->scale[k] / g;
            any |= f[k] != 1;
            e->scale[k] = g;
        }
        if (any) {
            HIPCHK(e, hipSetDevice(e->device));
            HIPCHK(e, stage_flush(e));
            HIPCHK(e, ks::launch_rescale(e->s, e->n_pad, e->pods.p, e->P, f, e->st));
            HIPCHK(e, hipStreamSynchronize(e->st));
            for (ks::PodRec& r : e->h_pods)
                for (int k = 0; k < 3; k++) r.req[k] *= f[k];
            update_mode(e);
            if (e->P) {  // the scan records of the rescaled requests
                std::vector<ks::ScanRec> sr(e->P);
                for (int64_t q = 0; q < e->P; q++) sr[q] = ks::scan_rec_micro(e->dc, e->h_pods[q]);
                HIPCHK(e, hipMemcpy(e->srec.p, sr.data(), sizeof(ks::ScanRec) * e->P, hipMemcpyHostToDevice));
            }
        }
    }
    std::vector<ks::PodRec> recs(m);
    std::vector<ks::ScanRec> srecs(m);
    std::vector<int32_t> dur(m), poff(m), cum(nf);
    std::vector<int64_t> t0(m), fin(m), eoff(m);
    std::vector<int32_t> tsec(m);
    std::vector<int64_t> run_end(m);
    std::vector<uint8_t> reg(m);
    std::vector<int32_t> epod;
    epod.reserve(m);
    const int64_t epod_base = e->exp_pod.n;
    e->h_exp_pos.resize(e->P + m, -1);
    int64_t pos_lo = e->P;  // lowest pod whose expiry position changed
    int64_t prev_bind = e->P ? e->h_bind_tick[e->P - 1] : e->tick;
    for (int64_t i = 0; i < m; i++) {
        const int64_t j = e->P + i;
        ks::PodRec& r = recs[i];
        const uint8_t km = keymask[i] & 7;
        for (int k = 0; k < 3; k++) r.req[k] = (km >> k & 1) ? req[i * 3 + k] / e->scale[k] : 0;
        r.tol = tol[i];
        r.sel = sel[i];
        r.keymask = km;
        r.flags = flags ? flags[i] : 0;
        srecs[i] = ks::scan_rec_micro(e->dc, r);
        const int64_t arr = std::max<int64_t>(arrival[i], e->tick + 1);
        const int64_t bt = std::max<int64_t>(prev_bind + 1, arr);
        prev_bind = bt;
        uint32_t acc = 0;  // int32 wrapping, kubesim/pod/pod.go:155-162
        int64_t acc64 = 0;
        bool nonneg = true;
        for (int32_t f = phase_off[i]; f < phase_off[i + 1]; f++) {
            acc += (uint32_t)phase_sec[f];
            acc64 += phase_sec[f];
            nonneg &= phase_sec[f] >= 0;
            cum[f] = (int32_t)acc;
        }
        const int32_t S = (int32_t)acc;
        tsec[i] = S;
        const int64_t d = S > 0 ? ((int64_t)S + e->cfg.tick_seconds - 1) / e->cfg.tick_seconds : 0;
        dur[i] = (int32_t)d;
        t0[i] = bt;
        fin[i] = d > 0 ? bt + d : kNever;
        run_end[i] = bt + d;
        // the digest's segment form: cumulative seconds non-decreasing and (t - t0) * tick never
        // wraps int32 while the pod runs (else the exact per-tick form)
        reg[i] = nonneg && acc64 <= (int64_t)INT32_MAX - e->cfg.tick_seconds;
        poff[i] = (int32_t)(e->F + phase_off[i]);
        // expiries due before pod j binds: finish tick in (bind_tick[j-1], bind_tick[j]]
        while (!e->pending.empty() && e->pending.top().first <= bt) {
            const int64_t q = e->pending.top().second;
            e->h_exp_pos[q] = epod_base + (int64_t)epod.size();
            pos_lo = std::min(pos_lo, q);
            epod.push_back((int32_t)q);
            e->pending.pop();
        }
        eoff[i] = e->h_exp_off.back() + (int64_t)epod.size();
        if (d > 0) e->pending.push({fin[i], j});
    }
    // device uploads: small submits (a drop-in's per-tick calls) are staged in pinned memory and
    // applied by the next launch (no copy call, no synchronisation here); large ones are copied
    hipStream_t st = e->st;
    HIPCHK(e, hipSetDevice(e->device));
    std::vector<int32_t> neg(m, -1);
    std::vector<uint8_t> zero(m, 0);
    const int32_t tail = (int32_t)(e->F + nf);
    const int64_t z0 = 0;
    if (!e->group && m <= kStageMaxPods) {
        HIPCHK(e, stage_append(e, e->pods, recs.data(), m));
        HIPCHK(e, stage_append(e, e->srec, srecs.data(), m));
        HIPCHK(e, stage_append(e, e->dur, dur.data(), m));
        HIPCHK(e, stage_append(e, e->t0, t0.data(), m));
        HIPCHK(e, stage_append(e, e->fin, fin.data(), m));
        HIPCHK(e, stage_append(e, e->b_node, neg.data(), m));
        HIPCHK(e, stage_append(e, e->b_status, neg.data(), m));
        HIPCHK(e, stage_append(e, e->expired, zero.data(), m));
        HIPCHK(e, stage_append(e, e->preg, reg.data(), m));
        if (e->phase_off.n) e->phase_off.n -= 1;  // phase_off holds P+1 entries: overwrite the sentinel
        HIPCHK(e, stage_append(e, e->phase_off, poff.data(), m));
        HIPCHK(e, stage_append(e, e->phase_off, &tail, 1));
        HIPCHK(e, stage_append(e, e->cum_sec, cum.data(), nf));
        HIPCHK(e, stage_append(e, e->use, phase_use, nf * 3));
        if (e->exp_off.n == 0) HIPCHK(e, stage_append(e, e->exp_off, &z0, 1));
        HIPCHK(e, stage_append(e, e->exp_off, eoff.data(), m));
        HIPCHK(e, stage_append(e, e->exp_pod, epod.data(), (int64_t)epod.size()));
        if (e->exp_pos.cap < e->P + m) {
            HIPCHK(e, stage_flush(e));
            HIPCHK(e, e->exp_pos.reserve(e->P + m, st));
        }
        e->xpos_lo = std::min(e->xpos_lo, pos_lo);  // staged at the next flush (stage_xpos)
        e->exp_pos.n = e->P + m;
    } else {
        HIPCHK(e, stage_flush(e));
        HIPCHK(e, e->pods.append(recs.data(), m, st));
        HIPCHK(e, e->srec.append(srecs.data(), m, st));
        HIPCHK(e, e->dur.append(dur.data(), m, st));
        HIPCHK(e, e->t0.append(t0.data(), m, st));
        HIPCHK(e, e->fin.append(fin.data(), m, st));
        HIPCHK(e, e->b_node.append(neg.data(), m, st));
        HIPCHK(e, e->b_status.append(neg.data(), m, st));
        HIPCHK(e, e->expired.append(zero.data(), m, st));
        HIPCHK(e, e->preg.append(reg.data(), m, st));
        if (e->phase_off.n) e->phase_off.n -= 1;  // phase_off holds P+1 entries: overwrite the sentinel
        HIPCHK(e, e->phase_off.append(poff.data(), m, st));
        HIPCHK(e, e->phase_off.append(&tail, 1, st));
        HIPCHK(e, e->cum_sec.append(cum.data(), nf, st));
        HIPCHK(e, e->use.append(phase_use, nf * 3, st));
        if (e->exp_off.n == 0) HIPCHK(e, e->exp_off.append(&z0, 1, st));
        HIPCHK(e, e->exp_off.append(eoff.data(), m, st));
        HIPCHK(e, e->exp_pod.append(epod.data(), (int64_t)epod.size(), st));
        HIPCHK(e, e->exp_pos.reserve(e->P + m, st));
        HIPCHK(e, hipMemcpyAsync(e->exp_pos.p + pos_lo, e->h_exp_pos.data() + pos_lo, sizeof(int64_t) * (e->P + m - pos_lo),
                                 hipMemcpyHostToDevice, st));
        e->exp_pos.n = e->P + m;
        HIPCHK(e, hipStreamSynchronize(st));  // host staging vectors die here
    }
    e->h_pods.insert(e->h_pods.end(), recs.begin(), recs.end());
    e->h_exp_pod.insert(e->h_exp_pod.end(), epod.begin(), epod.end());
    e->h_expired.resize(e->P + m, 0);
    e->h_bind_tick.insert(e->h_bind_tick.end(), t0.begin(), t0.end());
    e->h_fin.insert(e->h_fin.end(), fin.begin(), fin.end());
    e->h_dur.insert(e->h_dur.end(), dur.begin(), dur.end());
    e->h_total_sec.insert(e->h_total_sec.end(), tsec.begin(), tsec.end());
    e->h_exp_off.insert(e->h_exp_off.end(), eoff.begin(), eoff.end());
    // default keys (key_id NULL) live in their own namespace: pod j is key -(j + 1), explicit
    // keys are >= 0, so a mix of both on one engine never aliases
    for (int64_t i = 0; i < m; i++) e->h_key.push_back(key_id ? key_id[i] : -(e->P + i) - 1);
    for (const auto& kv : new_end) e->key_end[kv.first] = kv.second;
    e->h_node.resize(e->P + m, -1);
    e->h_status.resize(e->P + m, -1);
    // run-interval index (usage queries)
    e->h_end.insert(e->h_end.end(), run_end.begin(), run_end.end());
    for (int64_t q = e->P; q < e->P + m; q++) {
        const int64_t b = q / kUBlk, s = b / kUSup;
        if ((int64_t)e->blk_end.size() <= b) e->blk_end.push_back(std::numeric_limits<int64_t>::min());
        if ((int64_t)e->sup_end.size() <= s) e->sup_end.push_back(std::numeric_limits<int64_t>::min());
        e->blk_end[b] = std::max(e->blk_end[b], e->h_end[q]);
        e->sup_end[s] = std::max(e->sup_end[s], e->h_end[q]);
    }
    e->P += m;
    e->F += nf;
    e->last_arrival = last;
    return KS_OK;
}

}  // extern "C"

namespace {

// ks_step, first half: the pods whose bind tick falls in (tick, tick + ticks] and the device
// counters for them.  Returns false when there is nothing to schedule (the caller just advances
// the tick once the step as a whole has succeeded).
bool step_prepare(ks_engine* e, int64_t ticks, int64_t* p_hi_out) {
    const int64_t t_end = e->tick + ticks;
    const int64_t p_hi = std::upper_bound(e->h_bind_tick.begin() + e->done, e->h_bind_tick.end(), t_end) -
                         e->h_bind_tick.begin();
    *p_hi_out = p_hi;
    e->stats = ks_step_stats{};
    e->kstats = ks_kernel_stats{};
    e->h_ctr[0] = e->done;
    e->h_ctr[1] = std::max(p_hi, e->done);
    e->h_ctr[2] = 0;
    e->h_ctr[3] = -1;
    e->h_ctr[4] = 0;
    *e->h_args = make_args(e);
    return p_hi > e->done;
}

// A device failure inside a step leaves the device counters and the binds of the step unknown:
// the engine stops (sticky KS_EDEVICE) with its tick and binds at the last completed step.
ks_status device_stop(ks_engine* e, ks_status r) {
    if (r == KS_EDEVICE && e->err == KS_OK) {
        e->err = KS_EDEVICE;
        if (e->errmsg.empty()) e->errmsg = "device failure during a step";
    }
    return r;
}

// ks_step, second half: the binds [done, new_done) (node / status copied back by the caller),
// errors as Run would return them (kubesim.go:114-120, 217-220).
ks_status step_finish(ks_engine* e, int64_t t_end, int64_t new_done, const int32_t* node, const int32_t* status,
                      ks_bind* out, int64_t cap, int64_t* n_out) {
    const int64_t nb = new_done - e->done;
    for (int64_t i = 0; i < nb && i < cap; i++) {
        out[i].pod = e->done + i;
        out[i].node = node[i];
        out[i].status = status[i];
        out[i].tick = e->h_bind_tick[e->done + i];
    }
    for (int64_t i = 0; i < nb; i++) {
        e->h_node[e->done + i] = node[i];
        e->h_status[e->done + i] = (int8_t)status[i];
    }
    *n_out = nb;
    e->done = new_done;
    if (e->h_ctr[2] != 0) {
        const int64_t pod = e->h_ctr[3];
        e->err = (int)e->h_ctr[2];
        e->tick = e->h_bind_tick[pod];
        e->done = pod + 1;  // popped from the queue, not bound
        if (e->err == KS_ENOTFOUND)
            fail(e, KS_ENOTFOUND, "node \"\" not found (pod %lld, tick %lld)", (long long)pod, (long long)e->tick);
        else
            fail(e, KS_EINVAL, "pod %lld: invalid pod key or simSpec (tick %lld)", (long long)pod, (long long)e->tick);
        return (ks_status)e->err;
    }
    e->tick = t_end;
    return KS_OK;
}

}  // namespace

extern "C" {

static ks_status step_body(ks_engine* e, int64_t ticks, ks_bind* out, int64_t cap, int64_t* n_out);

ks_status ks_step(ks_engine* e, int64_t ticks, ks_bind* out, int64_t cap, int64_t* n_out) {
    if (!e || !n_out || ticks < 0 || cap < 0 || (cap > 0 && !out)) return KS_EINVAL;
    *n_out = 0;
    if (e->err) return (ks_status)e->err;
    if (!e->nodes_loaded) return fail(e, KS_EINVAL, "no nodes loaded");
    if (e->P > 0 && !in_passed_domain(e, e->h_bind_tick[0], e->tick + ticks))
        return fail(e, KS_ERANGE, "step to tick %lld: more than 2^31 s after the first bind (tick %lld)",
                    (long long)(e->tick + ticks), (long long)e->h_bind_tick[0]);
    return device_stop(e, step_body(e, ticks, out, cap, n_out));
}

// Expiries attached to pods [lo, hi) have been applied on the device (the batch path applies
// every expiry attached to a processed pod whose pod was bound Ok): mirror them.
static void mirror_expired(ks_engine* e, int64_t lo, int64_t hi) {
    for (int64_t j = lo; j < hi; j++)
        for (int64_t u = e->h_exp_off[j]; u < e->h_exp_off[j + 1]; u++) {
            const int32_t q = e->h_exp_pod[u];
            if (e->h_status[q] == KS_POD_OK) e->h_expired[q] = 1;
        }
}

// The per-tick path (ks_tick.hip): exactly one pod binds in this step — one launch does the
// staged submits, the pod's expiries, the full-cluster evaluation, the argmax and the bind.
// Returns false (nothing done) when the pod's expiries do not fit the launch's by-value list.
static bool tick_step(ks_engine* e, int64_t t_end, ks_bind* out, int64_t cap, int64_t* n_out, ks_status* rc) {
    const int64_t j = e->done;
    ks::TickArgs a{};
    for (int64_t u = e->h_exp_off[j]; u < e->h_exp_off[j + 1]; u++) {
        const int32_t q = e->h_exp_pod[u];
        if (e->h_status[q] != KS_POD_OK || e->h_expired[q]) continue;
        if (a.n_exp == ks::kTickMaxExp) return false;
        ks::TickExp& x = a.exp[a.n_exp++];
        x.node = e->h_node[q];
        x.q = q;
        for (int k = 0; k < 3; k++) x.req[k] = e->h_pods[q].req[k];
    }
    *rc = KS_OK;
    if (!e->d_tick) {
        hipError_t r = hipMalloc(&e->d_tick, sizeof(ks::TickScratch));
        if (r == hipSuccess) r = hipMemsetAsync(e->d_tick, 0, sizeof(ks::TickScratch), e->st);
        if (r == hipSuccess) r = hipHostMalloc(&e->h_tick, sizeof(ks::TickOut), hipHostMallocMapped);
        if (r == hipSuccess) r = hipHostGetDevicePointer((void**)&e->h_tick_dev, e->h_tick, 0);
        if (r == hipSuccess && !e->stage_ev) r = hipEventCreateWithFlags(&e->stage_ev, hipEventDisableTiming);
        if (r != hipSuccess) { *rc = fail(e, KS_EDEVICE, "per-tick path setup: %s", hipGetErrorString(r)); return true; }
    }
    a.c = e->dc;
    a.s = e->s;
    a.pod = e->h_pods[j];
    a.j = j;
    a.run = e->h_dur[j] > 0;
    a.b_node = e->b_node.p;
    a.b_status = e->b_status.p;
    a.expired = e->expired.p;
    a.scr = e->d_tick;
    a.out = e->h_tick_dev;
    if (stage_xpos(e) != hipSuccess) { *rc = fail(e, KS_EDEVICE, "per-tick path: staging failed"); return true; }
    // the pending staged rows inline in the arguments when they fit (one pod's submit does), else
    // one scatter launch ahead of the kernel
    {
        int32_t off = 0;
        bool fits = e->nseg - e->seg_done <= ks::kTickInlSeg;
        for (int k = e->seg_done; fits && k < e->nseg; k++) {
            off += (int32_t)((e->segs[k].bytes + 15) / 16 * 16);
            fits = off <= ks::kTickInl;
        }
        if (fits) {
            off = 0;
            for (int k = e->seg_done; k < e->nseg; k++) {
                const ks::CopySeg& sg = e->segs[k];
                std::memcpy(a.inl + off, e->stage + (sg.src - e->stage_dev), (size_t)sg.bytes);
                a.iseg[a.n_iseg++] = ks::TickSeg{sg.dst, off, (int32_t)sg.bytes};
                off += (int32_t)((sg.bytes + 15) / 16 * 16);
            }
            e->seg_done = e->nseg;
        } else if (stage_flush(e) != hipSuccess) {
            *rc = fail(e, KS_EDEVICE, "per-tick path: staging failed");
            return true;
        }
    }
    __atomic_store_n(&e->h_tick->code, -1, __ATOMIC_RELAXED);
    hipError_t r = ks::launch_tick(a, e->mode, e->st);
    if (r == hipSuccess) r = hipEventRecord(e->stage_ev, e->st);
    // the result: poll the host-mapped code the last workgroup stores (release) after node and
    // status — microseconds sooner than a stream synchronisation; the stream is queried now and
    // then so that a failed launch still ends the wait
    for (uint32_t spin = 1; r == hipSuccess; spin++) {
        if (__atomic_load_n(&e->h_tick->code, __ATOMIC_ACQUIRE) >= 0) break;
        if ((spin & 1023) == 0) {
            const hipError_t q = hipStreamQuery(e->st);
            if (q == hipSuccess) break;  // done: the code is read below
            if (q != hipErrorNotReady) r = q;
        }
        __builtin_ia32_pause();
    }
    if (r != hipSuccess) { *rc = fail(e, KS_EDEVICE, "per-tick launch: %s", hipGetErrorString(r)); return true; }
    ks::TickOut o;
    o.code = __atomic_load_n(&e->h_tick->code, __ATOMIC_ACQUIRE);
    o.node = ((volatile ks::TickOut*)e->h_tick)->node;
    o.status = ((volatile ks::TickOut*)e->h_tick)->status;
    for (int k = 0; k < a.n_exp; k++) e->h_expired[a.exp[k].q] = 1;
    e->stats = ks_step_stats{};
    e->stats.launches = 1;
    e->h_ctr[2] = o.code;
    e->h_ctr[3] = j;
    if (o.code < 0) { *rc = fail(e, KS_EDEVICE, "per-tick kernel wrote no result"); return true; }
    const int32_t node = o.node, status = o.status;
    *rc = step_finish(e, t_end, o.code ? j : j + 1, &node, &status, out, cap, n_out);
    e->stats.pods = *n_out;
    return true;
}

// The batch window workspace (~0.8 MB) and the node -> E index, allocated on the first step that
// runs a resolver using them (what-if group members never do).
// pruned block lists for chunk-resolver engines of >= this many scan blocks (or KS_ENGINE_PRUNED_LISTS)
#ifndef KS_PRUNE_MIN_BLOCKS
#define KS_PRUNE_MIN_BLOCKS 1024  // (A/B: make variant NAME=noprune DEFS=-DKS_PRUNE_MIN_BLOCKS=1000000)
#endif
constexpr int kPruneMinBlocks = KS_PRUNE_MIN_BLOCKS;


static ks_status ensure_window_ws(ks_engine* e) {
    const int r = resolver_of(e);
    e->prune = r == kResolveChunk && !e->group && (e->nblk >= kPruneMinBlocks || (e->flags & KS_ENGINE_PRUNED_LISTS));
    if (e->prune && !e->lbit) {
        e->nwl = (e->nblk + 63) / 64;
        HIPCHK(e, hipMalloc(&e->lbit, sizeof(uint64_t) * 2 * (size_t)e->B * e->nwl));  // two sets (EngineArgs)
        HIPCHK(e, hipMemsetAsync(e->lbit, 0, sizeof(uint64_t) * 2 * (size_t)e->B * e->nwl, e->st));
        HIPCHK(e, hipMalloc(&e->lthr, sizeof(uint64_t) * 2 * ks::kThrCopies * (size_t)e->B));
        HIPCHK(e, hipMemsetAsync(e->lthr, 0, sizeof(uint64_t) * 2 * ks::kThrCopies * (size_t)e->B, e->st));
    }
    if (e->d_sweep || r != kResolveChunk) return KS_OK;
    HIPCHK(e, hipMalloc(&e->d_sweep, sizeof(ks::WinWS)));
    HIPCHK(e, hipMemsetAsync(e->d_sweep, 0, sizeof(ks::WinWS), e->st));
    HIPCHK(e, hipMalloc(&e->d_eidx, sizeof(int32_t) * e->n_pad));
    HIPCHK(e, hipMemsetAsync(e->d_eidx, 0xFF, sizeof(int32_t) * e->n_pad, e->st));
    HIPCHK(e, hipMalloc(&e->d_nslot, sizeof(int32_t) * e->n_pad));
    HIPCHK(e, hipMemsetAsync(e->d_nslot, 0xFF, sizeof(int32_t) * e->n_pad, e->st));
    HIPCHK(e, hipMalloc(&e->d_first, sizeof(int32_t) * e->n_pad));
    HIPCHK(e, hipMemsetAsync(e->d_first, 0x7F, sizeof(int32_t) * e->n_pad, e->st));  // kNoFirst
    HIPCHK(e, hipMalloc(&e->d_spec, 2 * ks::kSpecStride * sizeof(int64_t)));
    HIPCHK(e, hipMemsetAsync(e->d_spec, 0, 2 * ks::kSpecStride * sizeof(int64_t), e->st));
    HIPCHK(e, hipMalloc(&e->d_args_spec, 2 * sizeof(ks::EngineArgs)));
    HIPCHK(e, hipHostMalloc(&e->h_args_spec, 2 * sizeof(ks::EngineArgs), hipHostMallocDefault));
    {   // the fused scan's workgroups: one per CU beside the resolver's (the resolver's LDS
        // footprint allows one workgroup per CU)
        int cus = 0;
        HIPCHK(e, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->device));
#ifndef KS_SCAN_WORKERS_DIV
#define KS_SCAN_WORKERS_DIV 1  // (A/B builds: make variant DEFS=-DKS_SCAN_WORKERS_DIV=2)
#endif
        e->scan_workers = std::max(15, cus / KS_SCAN_WORKERS_DIV - 1);  // (>= 15: every XCD deals its share to at least one)
    }
    if (e->world * e->vsh > 1) {  // the pipelined sharded chain's stream, events and full-range arguments
        HIPCHK(e, hipStreamCreateWithFlags(&e->st2, hipStreamNonBlocking));
        HIPCHK(e, hipEventCreateWithFlags(&e->pev_m, hipEventDisableTiming));
        HIPCHK(e, hipEventCreateWithFlags(&e->pev_x, hipEventDisableTiming));
        HIPCHK(e, hipMalloc(&e->d_args_full, sizeof(ks::EngineArgs)));
        HIPCHK(e, hipHostMalloc(&e->h_args_full, sizeof(ks::EngineArgs), hipHostMallocDefault));
    }
    return KS_OK;
}

// This rank's per-part merges of its block lists into its parts' slices of cand_all (a: the
// argument record whose counters name the batch; lset_fixed >= 0: that list set's bitmaps)
static hipError_t part_merges(ks_engine* e, const ks::EngineArgs* a, hipStream_t s, int lset_fixed) {
    const int64_t L = e->L, BL = (int64_t)e->B * L;
    for (int v = 0; v < e->vsh; v++) {
        const int p = e->rank * e->vsh + v;
        const int nlp = e->part_lo[p + 1] - e->part_lo[p];
        const hipError_t r = ks::launch_merge(a, 1, e->B, e->lists + (int64_t)e->part_lo[p] * L, (int64_t)e->nblk * L, nlp,
                                              L, e->cand_all + p * BL, nlp, s, e->prune ? e->lbit : nullptr, e->nwl,
                                              e->part_lo[p], lset_fixed, (int)L);
        if (r != hipSuccess) return r;
    }
    return hipSuccess;
}

// The all-gather of every rank's parts of cand_all on stream s: RCCL, or the host callback
static ks_status exchange(ks_engine* e, hipStream_t s) {
    const int64_t BL = (int64_t)e->B * e->L;
    if (e->comm) {
        const ncclResult_t nr = ncclAllGather(e->cand_all + (int64_t)e->rank * e->vsh * BL, e->cand_all,
                                              (size_t)e->vsh * BL, ncclUint64, e->comm, s);
        if (nr != ncclSuccess) return fail(e, KS_EDEVICE, "ncclAllGather: %s", ncclGetErrorString(nr));
    } else if (e->xfn) {  // host exchange: this rank's parts out, every rank's parts back
        const int64_t slice = (int64_t)e->vsh * BL, off = (int64_t)e->rank * slice;
        HIPCHK(e, hipMemcpyAsync(e->h_xbuf + off, e->cand_all + off, sizeof(uint64_t) * slice, hipMemcpyDeviceToHost, s));
        HIPCHK(e, hipStreamSynchronize(s));
        const ks_status xr = e->xfn(e->xuser, e->rank, e->world, e->h_xbuf, (int64_t)sizeof(uint64_t) * slice);
        if (xr != KS_OK) return fail(e, KS_EDEVICE, "host exchange failed (%d)", (int)xr);
        HIPCHK(e, hipMemcpyAsync(e->cand_all, e->h_xbuf, sizeof(uint64_t) * slice * e->world, hipMemcpyHostToDevice, s));
    }
    return KS_OK;
}

// One batch of the pipelined sharded chain (step_body).  Main stream: [the pass's first batch: window
// prep, scan of this rank's blocks, part merges, exchange | later batches: wait for the second
// stream's exchange, the conditional local rescan (E overflow only) with the E staging] -> merge_cl
// -> the resolve with the next batch's window in its tail.  Second stream, once merge_cl has read
// the lists and cleared the speculative set: the next batch's speculative scan of this rank's blocks
// (the counters this batch's window prep wrote), its part merges and the exchange — beside the
// resolve.  cand_all and the block lists are single-buffered: each side pass starts after the
// merge_cl that read the previous one.
static ks_status pipe_batch(ks_engine* e, int64_t b, int64_t nbat, hipEvent_t* ev) {
    hipStream_t st = e->st, s2 = e->st2;
    const ks::EngineArgs* d = e->d_args;
    const int G = e->world * e->vsh;
    const int64_t L = e->L, BL = (int64_t)e->B * L;  // (kTopLOverlap: step_body)
    const bool first = b == 0, more = b + 1 < nbat;
    if (ev[0]) HIPCHK(e, hipEventRecord(ev[0], st));
    if (first) {
        HIPCHK(e, ks::launch_window_prep(d, true, false, (int)(b & 1), st));
        if (ev[1]) HIPCHK(e, hipEventRecord(ev[1], st));
        HIPCHK(e, ks::launch_scan(d, 1, e->blk_n, e->B, e->PG, e->mode, key16(e), st, false, e->prune, (int)L, true));
        if (ev[2]) HIPCHK(e, hipEventRecord(ev[2], st));
        HIPCHK(e, part_merges(e, d, st, -1));
        if (ev[5]) HIPCHK(e, hipEventRecord(ev[5], st));
        if (ks_status r = exchange(e, st); r != KS_OK) return r;
        if (ev[6]) HIPCHK(e, hipEventRecord(ev[6], st));
    } else {
        HIPCHK(e, hipStreamWaitEvent(st, e->pev_x, 0));
        if (ev[1]) HIPCHK(e, hipEventRecord(ev[1], st));
        HIPCHK(e, ks::launch_scan(e->d_args_full, 1, e->nblk, e->B, e->PG, e->mode, key16(e), st, true, e->prune, (int)L,
                                  true, kRescanWgs));
        if (ev[2]) HIPCHK(e, hipEventRecord(ev[2], st));
        if (ev[5]) HIPCHK(e, hipEventRecord(ev[5], st));
        if (ev[6]) HIPCHK(e, hipEventRecord(ev[6], st));
    }
    HIPCHK(e, ks::launch_merge_cl(d, e->mode, e->B, e->cand_all, L, G, BL, G, st, (int)L, !first));
    if (ev[3]) HIPCHK(e, hipEventRecord(ev[3], st));
    if (more) {
        HIPCHK(e, hipEventRecord(e->pev_m, st));
        // (no scan workers: the resolver and the next window only; the list length is the workers')
        HIPCHK(e, ks::launch_chunk_scan(d, e->d_args_spec + (b & 1), 0, (int)((b + 1) & 1), e->mode, e->prune, ks::kTopL, st));
    } else {
        HIPCHK(e, ks::launch_chunk_only(d, e->mode, st));
    }
    if (ev[4]) HIPCHK(e, hipEventRecord(ev[4], st));
    if (more) {
        const ks::EngineArgs* ds = e->d_args_spec + (b & 1);
        HIPCHK(e, hipStreamWaitEvent(s2, e->pev_m, 0));
        if (ev[7]) HIPCHK(e, hipEventRecord(ev[7], s2));
        HIPCHK(e, ks::launch_scan(ds, 1, e->blk_n, e->B, e->PG, e->mode, key16(e), s2, false, e->prune, (int)L, false));
        if (ev[8]) HIPCHK(e, hipEventRecord(ev[8], s2));
        HIPCHK(e, part_merges(e, ds, s2, 0));
        if (ev[9]) HIPCHK(e, hipEventRecord(ev[9], s2));
        if (ks_status r = exchange(e, s2); r != KS_OK) return r;
        if (ev[10]) HIPCHK(e, hipEventRecord(ev[10], s2));
        HIPCHK(e, hipEventRecord(e->pev_x, s2));
    }
    return KS_OK;
}

static ks_status step_body(ks_engine* e, int64_t ticks, ks_bind* out, int64_t cap, int64_t* n_out) {
    HIPCHK(e, hipSetDevice(e->device));
    if (ks_status r = ensure_window_ws(e); r != KS_OK) return r;
    const int64_t t_end = e->tick + ticks;
    int64_t p_hi = 0;
    if (!step_prepare(e, ticks, &p_hi)) {
        e->tick = t_end;
        return KS_OK;
    }
    // (an explicitly forced resolver keeps one-pod steps on that resolver: its A/B tests)
    if (p_hi == e->done + 1 && !e->group && e->world * e->vsh == 1 && e->n > 0 && !e->profiling &&
        !(e->flags & (KS_ENGINE_CHUNK_RESOLVER | KS_ENGINE_ONE_POD_RESOLVER))) {
        ks_status rc = KS_OK;
        if (tick_step(e, t_end, out, cap, n_out, &rc)) return rc;
    }
    const int64_t done0 = e->done;
    HIPCHK(e, stage_flush(e));
    hipStream_t st = e->st;
    const int which = resolver_of(e);
    const bool fused = which == kResolveChunk;
    HIPCHK(e, hipMemcpyAsync(e->d_ctr, e->h_ctr, 5 * sizeof(int64_t), hipMemcpyHostToDevice, st));
    HIPCHK(e, hipMemcpyAsync(e->d_args, e->h_args, sizeof(ks::EngineArgs), hipMemcpyHostToDevice, st));
    // the overlap (chunk class, 16-bit keys, not profiling): batch b + 1's scan fused into batch b's
    // chunk kernel, over the pods after batch b (the speculative counters window prep writes) and
    // this rank's scan blocks.  Sharded engines too: every rank's lists are speculative alike and its
    // touched nodes (the same on every rank: the resolvers are identical) join E; the exchange runs
    // every batch whether or not window prep flagged a rescan, so every rank issues the same
    // collectives.  In the fused kernel the scan runs one workgroup per CU (the resolver's LDS fixes
    // the kernel's), ~3 blocks per us: ranks scanning more than kOverlapMaxBlocks blocks keep the
    // plain chain, whose scan runs at full occupancy (C5 on 8 ranks, 512 blocks each: fused kernel
    // 129 us against a 78 us resolve + a 37 us scan; C3: 196 blocks hide under the resolve)
    // (profiling keeps it: the per-kernel events bracket the same launches)
    const bool overlap = fused && e->overlap && e->d_args_spec && key16(e) && e->blk_n <= kOverlapMaxBlocks;
    // The pipelined sharded chain (round 6; sharded engines the fused overlap does not take, e.g. C5 on
    // 8 ranks, 512 blocks each): batch b + 1's speculative scan of this rank's blocks, its per-part
    // merges and the exchange run on a second stream beside batch b's resolve, so only the resolve
    // (with the next window in its tail), the E staging and merge_cl stay on the critical path.  A
    // batch that starts inside its predecessor (an early stop) reuses its merged lists (ks_prep.h),
    // so the exchanged lists always serve; when E overflows, the conditional rescan scans every block
    // locally (no second exchange: every rank holds the whole table) and merge_cl merges those.
    const bool pipe = fused && !overlap && e->overlap && e->st2 && e->world * e->vsh > 1;
    // the overlap's single-shard lists are longer (ks_device.h kTopLOverlap, ks_cand.hip cand_list)
    // (and the pipelined chain's: its speculative lists go stale like the overlap's)
    e->L = (overlap && e->world * e->vsh == 1 && !e->prune) || pipe ? ks::kTopLOverlap : ks::kTopL;
    if (pipe) {
        *e->h_args_full = *e->h_args;
        e->h_args_full->blk_lo = 0;
        e->h_args_full->blk_n = e->nblk;
        HIPCHK(e, hipMemcpyAsync(e->d_args_full, e->h_args_full, sizeof(ks::EngineArgs), hipMemcpyHostToDevice, st));
    }
    if (overlap || pipe) {
        for (int k = 0; k < 2; k++) {
            e->h_args_spec[k] = *e->h_args;
            e->h_args_spec[k].ctr = e->d_spec + ks::kSpecStride * k;
            e->h_args_spec[k].lset = 0;  // pruned lists: the speculative set
        }
        HIPCHK(e, hipMemcpyAsync(e->d_args_spec, e->h_args_spec, 2 * sizeof(ks::EngineArgs), hipMemcpyHostToDevice, st));
    }
    HIPCHK(e, hipEventRecord(e->ev[0], st));
    const ks::EngineArgs* d = e->d_args;
#ifdef KS_MCL_BYVAL
    ks::ks_mcl_host_args = e->h_args;  // (diagnostic build only; one engine per thread at a time is not guaranteed)
#endif
    int64_t start = e->done;
    int64_t launches = 0;
    double scan_ms = 0, res_ms = 0;
    ks_kernel_stats ks{};
    std::vector<uint8_t> kind;  // per launch: 1 window prep launched, 2 fused resolve
    while (true) {
        const int64_t nbat = (p_hi - start + e->B - 1) / e->B;
        for (int64_t b = 0; b < nbat; b++) {
            // profiling: events around the scan kernel alone and the resolve kernel alone (on
            // the engine's stream), so their averages agree with rocprofv3's kernel trace
            hipEvent_t ev[kProfEv] = {};
            if (e->profiling) {
                while ((int64_t)e->prof_ev.size() < kProfEv * (launches + 1)) {
                    hipEvent_t x;
                    HIPCHK(e, hipEventCreate(&x));
                    e->prof_ev.push_back(x);
                }
                for (int k = 0; k < kProfEv; k++) ev[k] = e->prof_ev[kProfEv * launches + k];
            }
            if (pipe) {
                ks_status pr = pipe_batch(e, b, nbat, ev);
                if (pr != KS_OK) return pr;
                if (e->profiling) kind.push_back((uint8_t)(8 | (b == 0 ? 1 : 0) | (b + 1 < nbat ? 2 : 0)));
                launches++;
                continue;
            }
            // the chunk resolver's chain is fused: window prep with the head's expiries, the scan,
            // merge with the candidate lists, the resolver (four launches per batch)
            // overlap: batch b > 0 of this pass takes the speculative scan's lists (a conditional
            // rescan when they do not fit, ks_cand.hip window_prep_kernel)
            const bool spec = overlap && b > 0;
            if (ev[0]) HIPCHK(e, hipEventRecord(ev[0], st));
            // (an overlapped batch's window was computed by the previous chunk kernel after its commit)
            if (!spec) HIPCHK(e, fused ? ks::launch_window_prep(d, true, false, (int)(b & 1), st) : ks::launch_expire_head(d, 1, st));
            if (ev[1]) HIPCHK(e, hipEventRecord(ev[1], st));
            // (chunk class: the scan launch also stages the batch's E records for merge_cl)
            HIPCHK(e, ks::launch_scan(d, 1, e->blk_n, e->B, e->PG, e->mode, key16(e), st, spec, e->prune, e->L, fused));
            if (ev[2]) HIPCHK(e, hipEventRecord(ev[2], st));
            const int G = e->world * e->vsh;
            hipEvent_t evx[2] = {ev[5], ev[6]};  // part merges | exchange | merge (sharded engines)
            const int64_t L = ks::kTopL, BL = (int64_t)e->B * L;
            if (G == 1) {
                HIPCHK(e, fused ? ks::launch_merge_cl(d, e->mode, e->B, nullptr, 0, 0, 0, e->nblk, st, e->L)
                                : ks::launch_merge(d, 1, e->B, nullptr, 0, 0, 0, nullptr, e->nblk, st));
            } else {
                HIPCHK(e, part_merges(e, d, st, -1));
                if (evx[0]) HIPCHK(e, hipEventRecord(evx[0], st));
                if (ks_status r = exchange(e, st); r != KS_OK) return r;
                if (evx[1]) HIPCHK(e, hipEventRecord(evx[1], st));
                HIPCHK(e, fused ? ks::launch_merge_cl(d, e->mode, e->B, e->cand_all, L, G, BL, G, st)
                                : ks::launch_merge(d, 1, e->B, e->cand_all, L, G, BL, e->cand, G, st));
            }
            if (ev[3]) HIPCHK(e, hipEventRecord(ev[3], st));
            if (overlap && b + 1 < nbat)  // the resolver with the next batch's scan beside it
                HIPCHK(e, ks::launch_chunk_scan(d, e->d_args_spec + (b & 1), e->scan_workers, (int)((b + 1) & 1), e->mode,
                                                e->prune, e->L, st));
            else
                HIPCHK(e, fused ? ks::launch_chunk_only(d, e->mode, st) : launch_resolver(d, 1, e->mode, which, st));
            if (ev[4]) HIPCHK(e, hipEventRecord(ev[4], st));
            if (e->profiling) kind.push_back((uint8_t)((!spec ? 1 : 0) | (overlap && b + 1 < nbat ? 2 : 0) | (G > 1 ? 4 : 0)));
            launches++;
        }
        HIPCHK(e, hipMemcpyAsync(e->h_ctr, e->d_ctr, 5 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIPCHK(e, hipStreamSynchronize(st));
        const int64_t prev = start;
        start = e->h_ctr[0];
        if (e->h_ctr[2] != 0 || start >= p_hi) break;
        // every launch commits at least its first pod (resolve_kernel): no progress is a bug
        if (start <= prev) return fail(e, KS_EDEVICE, "scheduling made no progress at pod %lld", (long long)start);
    }
    HIPCHK(e, hipEventRecord(e->ev[1], st));
    const int64_t new_done = start;
    const int64_t nb = new_done - e->done;
    std::vector<int32_t> node(nb), status(nb);
    if (nb) {
        HIPCHK(e, hipMemcpyAsync(node.data(), e->b_node.p + e->done, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, st));
        HIPCHK(e, hipMemcpyAsync(status.data(), e->b_status.p + e->done, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(e, hipStreamSynchronize(st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e->ev[0], e->ev[1]);
    double other_ms = 0;
    if (e->profiling) {
        for (int64_t l = 0; l < launches; l++) {
            float t[4] = {};
            hipEvent_t* E = &e->prof_ev[kProfEv * l];
            if (kind[l] & 8) {  // pipelined: [0,1) exchange wait, [1,2) scan / rescan + staging, [2,5) part merges,
                                // [5,6) exchange (the pass's first batch), [6,3) merge_cl, [3,4) resolve; side [7..10]
                float w = 0, sc = 0, pm = 0, xc = 0, mg = 0, rs = 0;
                (void)hipEventElapsedTime(&w, E[0], E[1]);
                (void)hipEventElapsedTime(&sc, E[1], E[2]);
                (void)hipEventElapsedTime(&pm, E[2], E[5]);
                (void)hipEventElapsedTime(&xc, E[5], E[6]);
                (void)hipEventElapsedTime(&mg, E[6], E[3]);
                (void)hipEventElapsedTime(&rs, E[3], E[4]);
                ks.wait_ms += w;
                ks.scan_ms += sc; ks.scan_n += 1; scan_ms += sc;
                ks.merge_ms += pm + xc + mg; ks.merge_n += 1; other_ms += pm + xc + mg + w;
                if (kind[l] & 1) { ks.part_ms += pm; ks.xchg_ms += xc; ks.xchg_n += 1; }
                if (kind[l] & 2) { ks.fused_ms += rs; ks.fused_n += 1; } else { ks.resolve_ms += rs; ks.resolve_n += 1; }
                res_ms += rs;
                if (kind[l] & 2) {
                    float a0 = 0, a1 = 0, a2 = 0;
                    (void)hipEventElapsedTime(&a0, E[7], E[8]);
                    (void)hipEventElapsedTime(&a1, E[8], E[9]);
                    (void)hipEventElapsedTime(&a2, E[9], E[10]);
                    ks.side_scan_ms += a0; ks.side_part_ms += a1; ks.side_xchg_ms += a2; ks.side_n += 1;
                }
                continue;
            }
            for (int k = 0; k < 4; k++) (void)hipEventElapsedTime(&t[k], E[k], E[k + 1]);
            if (kind[l] & 4) {  // sharded: [2, 5) part merges, [5, 6) exchange, [6, 3) merge
                float pm = 0, xc = 0;
                (void)hipEventElapsedTime(&pm, E[2], E[5]);
                (void)hipEventElapsedTime(&xc, E[5], E[6]);
                ks.part_ms += pm; ks.xchg_ms += xc;
                ks.xchg_n += 1;
            }
            other_ms += t[0] + t[2];
            scan_ms += t[1];
            res_ms += t[3];
            ks.prep_ms += t[0]; ks.prep_n += kind[l] & 1;
            ks.scan_ms += t[1]; ks.scan_n += 1;
            ks.merge_ms += t[2]; ks.merge_n += 1;
            if (kind[l] & 2) { ks.fused_ms += t[3]; ks.fused_n += 1; }
            else { ks.resolve_ms += t[3]; ks.resolve_n += 1; }
        }
    }
    e->kstats = ks;
    e->stats.step_ms = ms;
    e->stats.scan_ms = scan_ms;
    e->stats.resolve_ms = res_ms;
    e->stats.other_ms = other_ms;
    e->stats.launches = launches;
    e->stats.pods = nb;
    const ks_status rc = step_finish(e, t_end, new_done, node.data(), status.data(), out, cap, n_out);
    if (rc == KS_OK) mirror_expired(e, done0, e->done);
    return rc;
}

// ---------------------------------------------------------------------------------------------
// Scenario groups (BASELINE.json configs[3]): independent what-if clusters stepped together, one
// launch per kernel for all of them (scenario = a grid dimension; one resolve workgroup each).
// ---------------------------------------------------------------------------------------------
struct ks_group {
    int device = 0;
    int cap = 0;
    hipStream_t st = nullptr;
    std::vector<ks_engine*> engs;
    int64_t* d_ctr = nullptr;           // [cap][32]
    int64_t* h_ctr = nullptr;           // pinned
    ks::EngineArgs* d_args = nullptr;   // [cap]
    ks::EngineArgs* h_args = nullptr;   // pinned
    ks::BindSeg* d_seg = nullptr;       // [cap]
    ks::BindSeg* h_seg = nullptr;       // pinned
    int32_t* d_out = nullptr;           // packed binds: node, then status
    int32_t* h_out = nullptr;           // pinned mirror of d_out
    int64_t out_cap = 0;
    hipEvent_t ev[2] = {nullptr, nullptr};
    // the second half of the scenarios runs its batch rounds on its own stream: one half's
    // latency-bound resolvers then share the GPU with the other half's throughput-bound scans
    hipStream_t st2 = nullptr;
    hipEvent_t xev = nullptr;  // argument upload done (st -> st2)
    std::string errmsg;
};

ks_status ks_group_create(int32_t device, int32_t max_scenarios, ks_group** out) {
    if (!out || max_scenarios < 1 || max_scenarios > 65535) return KS_EINVAL;
    *out = nullptr;
    ks_group* g = new ks_group();
    g->device = device;
    g->cap = max_scenarios;
    hipError_t r = hipSetDevice(device);
    if (r == hipSuccess) r = hipStreamCreateWithFlags(&g->st, hipStreamNonBlocking);
    if (r == hipSuccess) r = hipStreamCreateWithFlags(&g->st2, hipStreamNonBlocking);
    if (r == hipSuccess) r = hipEventCreateWithFlags(&g->xev, hipEventDisableTiming);
    if (r == hipSuccess) r = hipMalloc(&g->d_ctr, sizeof(int64_t) * 32 * max_scenarios);
    if (r == hipSuccess) r = hipHostMalloc(&g->h_ctr, sizeof(int64_t) * 32 * max_scenarios, hipHostMallocDefault);
    if (r == hipSuccess) r = hipMalloc(&g->d_args, sizeof(ks::EngineArgs) * max_scenarios);
    if (r == hipSuccess) r = hipHostMalloc(&g->h_args, sizeof(ks::EngineArgs) * max_scenarios, hipHostMallocDefault);
    if (r == hipSuccess) r = hipMalloc(&g->d_seg, sizeof(ks::BindSeg) * max_scenarios);
    if (r == hipSuccess) r = hipHostMalloc(&g->h_seg, sizeof(ks::BindSeg) * max_scenarios, hipHostMallocDefault);
    for (int i = 0; i < 2 && r == hipSuccess; i++) r = hipEventCreate(&g->ev[i]);
    if (r == hipSuccess) r = hipMemsetAsync(g->d_ctr, 0, sizeof(int64_t) * 32 * max_scenarios, g->st);
    if (r == hipSuccess) r = hipStreamSynchronize(g->st);
    if (r != hipSuccess) {
        ks_group_destroy(g);
        return KS_EDEVICE;
    }
    *out = g;
    return KS_OK;
}

void ks_group_destroy(ks_group* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->st) (void)hipStreamSynchronize(g->st);
    for (ks_engine* e : g->engs) engine_free(e);
    if (g->d_ctr) (void)hipFree(g->d_ctr);
    if (g->h_ctr) (void)hipHostFree(g->h_ctr);
    if (g->d_args) (void)hipFree(g->d_args);
    if (g->h_args) (void)hipHostFree(g->h_args);
    if (g->d_seg) (void)hipFree(g->d_seg);
    if (g->h_seg) (void)hipHostFree(g->h_seg);
    if (g->d_out) (void)hipFree(g->d_out);
    if (g->h_out) (void)hipHostFree(g->h_out);
    if (g->st2) (void)hipStreamSynchronize(g->st2);
    for (auto ev : g->ev) if (ev) (void)hipEventDestroy(ev);
    if (g->xev) (void)hipEventDestroy(g->xev);
    if (g->st2) (void)hipStreamDestroy(g->st2);
    if (g->st) (void)hipStreamDestroy(g->st);
    delete g;
}

ks_status ks_group_add(ks_group* g, const ks_config* cfg, ks_engine** out) {
    if (!g || !cfg || !out) return KS_EINVAL;
    *out = nullptr;
    if ((int)g->engs.size() >= g->cap) return KS_EINVAL;
    if (cfg->device != g->device) return KS_EINVAL;
    ks_engine* e = nullptr;
    const ks_status v = engine_init(cfg, &e);
    if (v != KS_OK) return v;
    const int idx = (int)g->engs.size();
    e->group = g;
    e->st = g->st;
    e->d_ctr = g->d_ctr + 32 * idx;
    e->h_ctr = g->h_ctr + 32 * idx;
    e->d_args = g->d_args + idx;
    e->h_args = g->h_args + idx;
    hipError_t r = hipSetDevice(g->device);
    for (int i = 0; i < 4 && r == hipSuccess; i++) r = hipEventCreate(&e->ev[i]);
    if (r != hipSuccess) {
        engine_free(e);
        return KS_EDEVICE;
    }
    g->engs.push_back(e);
    *out = e;
    return KS_OK;
}

int32_t ks_group_size(const ks_group* g) { return g ? (int32_t)g->engs.size() : -1; }

// groups of at least this many scenarios run as two halves on two streams
#ifndef KS_GROUP_SPLIT_MIN
#define KS_GROUP_SPLIT_MIN 64
#endif
constexpr int kGroupSplitMin = KS_GROUP_SPLIT_MIN;

ks_status ks_group_step(ks_group* g, int64_t ticks, ks_bind* out, int64_t cap, int64_t* n_out, int32_t* status_out,
                        ks_step_stats* stats) {
    if (!g || !n_out || !status_out || ticks < 0 || cap < 0) return KS_EINVAL;
    const int S = (int)g->engs.size();
    if (S == 0) return KS_OK;
    if (hipSetDevice(g->device) != hipSuccess) return KS_EDEVICE;
    std::vector<int64_t> p_hi(S, 0), t_end(S, 0);
    std::vector<char> live(S, 0), part(S, 0);  // part: takes part in this step
    int mode = ks::kEvalMicro, blk_n = 0, B = 0;  // B: the largest member batch (grid size)
    bool k16 = true, small = true;
    for (ks_engine* e : g->engs) {
        B = std::max(B, e->B);
        k16 = k16 && key16(e);
        small = small && small_resolver(e);
    }
    // (the chunk resolver takes one engine per launch: not in groups)
    const int which = small ? kResolveSmall : kResolveRole;
    int64_t blocks = 0;
    for (int i = 0; i < S; i++) {
        ks_engine* e = g->engs[i];
        n_out[i] = 0;
        status_out[i] = KS_OK;
        const bool out_of_domain = e->P > 0 && !in_passed_domain(e, e->h_bind_tick[0], e->tick + ticks);
        if (e->err || !e->nodes_loaded || e->world * e->vsh != 1 || out_of_domain) {
            status_out[i] = e->err ? e->err : out_of_domain ? KS_ERANGE : KS_EINVAL;
            if (!e->err) {
                if (out_of_domain) fail(e, KS_ERANGE, "step past 2^31 s after the first bind");
                else fail(e, KS_EINVAL, "group step needs loaded, unsharded nodes");
            }
            e->h_ctr[0] = e->h_ctr[1] = e->done;
            e->h_ctr[2] = 0;
            *e->h_args = e->nodes_loaded ? make_args(e) : ks::EngineArgs{};
            e->h_args->ctr = e->d_ctr;
            e->h_args->blk_n = 0;
            continue;
        }
        t_end[i] = e->tick + ticks;
        part[i] = 1;
        live[i] = step_prepare(e, ticks, &p_hi[i]);
        // the widest evaluator any scenario needs (each is exact on every narrower domain)
        mode = std::min(mode, e->mode);
        blk_n = std::max(blk_n, e->blk_n);
        blocks += e->blk_n;
    }
    // pods per scan workgroup for the whole group: the most node-record reuse that still leaves
    // >= ~2048 workgroups per scan
    int pg = 1;
    while (pg < ks::max_pods_per_scan_wg() && pg < B && blocks * ((B + pg * 2 - 1) / (pg * 2)) >= 2048) pg *= 2;
    for (int i = 0; i < S; i++) g->h_args[i].PG = pg;
    hipStream_t st = g->st;
    auto dev = [&](hipError_t r) { return r == hipSuccess; };
    // a device failure leaves every participating member's step unknown: sticky KS_EDEVICE, ticks
    // and binds stay at the last completed step
    auto dev_fail = [&](const char* what) {
        g->errmsg = what;
        for (int i = 0; i < S; i++)
            if (part[i]) {
                ks_engine* e = g->engs[i];
                e->err = KS_EDEVICE;
                e->errmsg = what;
                status_out[i] = KS_EDEVICE;
            }
        return KS_EDEVICE;
    };
    if (!dev(hipMemcpyAsync(g->d_ctr, g->h_ctr, sizeof(int64_t) * 32 * S, hipMemcpyHostToDevice, st)) ||
        !dev(hipMemcpyAsync(g->d_args, g->h_args, sizeof(ks::EngineArgs) * S, hipMemcpyHostToDevice, st)) ||
        !dev(hipEventRecord(g->ev[0], st)))
        return dev_fail("group step: argument upload failed");
    std::vector<int64_t> start(S);
    for (int i = 0; i < S; i++) start[i] = g->engs[i]->done;
    int64_t launches = 0;
    // scenario halves [h_lo[h], h_lo[h + 1]) on streams st / st2 (one stream for small groups)
    const int nh = S >= kGroupSplitMin ? 2 : 1;
    const int h_lo[3] = {0, nh == 2 ? S / 2 : S, S};
    hipStream_t hst[2] = {st, g->st2};
    if (nh == 2 && (!dev(hipEventRecord(g->xev, st)) || !dev(hipStreamWaitEvent(g->st2, g->xev, 0))))
        return dev_fail("group step: stream ordering failed");
    while (true) {
        int64_t nbat[2] = {0, 0};
        for (int h = 0; h < nh; h++)
            for (int i = h_lo[h]; i < h_lo[h + 1]; i++)
                if (live[i]) nbat[h] = std::max(nbat[h], (p_hi[i] - start[i] + B - 1) / B);
        if (nbat[0] == 0 && nbat[1] == 0) break;
        // the halves' rounds issued alternately: independent scenarios, no ordering between them
        // (a token that made the halves' scans take turns measured no better)
        for (int64_t b = 0; b < std::max(nbat[0], nbat[1]); b++) {
            for (int h = 0; h < nh; h++) {
                if (b >= nbat[h]) continue;
                const ks::EngineArgs* d = g->d_args + h_lo[h];
                const int Sh = h_lo[h + 1] - h_lo[h];
                if (!dev(ks::launch_expire_head(d, Sh, hst[h])) ||
                    !dev(ks::launch_scan(d, Sh, blk_n, B, pg, mode, k16, hst[h])) ||
                    !dev(ks::launch_merge(d, Sh, B, nullptr, 0, 0, 0, nullptr, blk_n, hst[h])) ||
                    !dev(launch_resolver(d, Sh, mode, which, hst[h])))
                    return dev_fail("group step: kernel launch failed");
            }
            launches++;
        }
        for (int h = 0; h < nh; h++) {
            const int64_t lo = h_lo[h], n = h_lo[h + 1] - h_lo[h];
            if (n && !dev(hipMemcpyAsync(g->h_ctr + 32 * lo, g->d_ctr + 32 * lo, sizeof(int64_t) * 32 * n,
                                         hipMemcpyDeviceToHost, hst[h])))
                return dev_fail("group step: device synchronisation failed");
        }
        for (int h = 0; h < nh; h++)
            if (!dev(hipStreamSynchronize(hst[h]))) return dev_fail("group step: device synchronisation failed");
        for (int i = 0; i < S; i++) {
            if (!live[i]) continue;
            ks_engine* e = g->engs[i];
            const int64_t prev = start[i];
            start[i] = e->h_ctr[0];
            if (e->h_ctr[2] != 0 || start[i] >= p_hi[i]) live[i] = 0;
            else if (start[i] <= prev)  // every launch commits at least its first pod
                return dev_fail("group step: scheduling made no progress");
        }
    }
    // binds back: one gather into a packed buffer, one copy
    int64_t total = 0, max_n = 0;
    for (int i = 0; i < S; i++) {
        ks_engine* e = g->engs[i];
        const int64_t nb = status_out[i] == KS_OK && part[i] ? start[i] - e->done : 0;
        g->h_seg[i] = ks::BindSeg{e->b_node.p, e->b_status.p, e->done, std::max<int64_t>(nb, 0), total};
        total += std::max<int64_t>(nb, 0);
        max_n = std::max(max_n, nb);
    }
    if (total > g->out_cap) {
        if (g->d_out) (void)hipFree(g->d_out);
        if (g->h_out) (void)hipHostFree(g->h_out);
        g->d_out = g->h_out = nullptr;
        g->out_cap = std::max<int64_t>(total, 2 * g->out_cap);
        if (!dev(hipMalloc(&g->d_out, sizeof(int32_t) * 2 * g->out_cap)) ||
            !dev(hipHostMalloc(&g->h_out, sizeof(int32_t) * 2 * g->out_cap, hipHostMallocDefault))) {
            g->out_cap = 0;
            return dev_fail("group step: bind buffer allocation failed");
        }
    }
    if (total) {
        if (!dev(hipMemcpyAsync(g->d_seg, g->h_seg, sizeof(ks::BindSeg) * S, hipMemcpyHostToDevice, st)) ||
            !dev(ks::launch_gather_binds(g->d_seg, S, max_n, g->d_out, g->d_out + total, st)) ||
            !dev(hipMemcpyAsync(g->h_out, g->d_out, sizeof(int32_t) * 2 * total, hipMemcpyDeviceToHost, st)))
            return dev_fail("group step: bind copy failed");
    }
    if (!dev(hipEventRecord(g->ev[1], st)) || !dev(hipStreamSynchronize(st)))
        return dev_fail("group step: device synchronisation failed");
    float ms = 0;
    (void)hipEventElapsedTime(&ms, g->ev[0], g->ev[1]);
    // unpack into the caller's ks_bind rows: members are independent, so large groups fill them
    // on several host threads (this is host-memory-bound: 24 B written per bind)
    auto finish = [&](int lo, int hi) {
        for (int i = lo; i < hi; i++) {
            ks_engine* e = g->engs[i];
            if (status_out[i] != KS_OK || !part[i]) continue;
            const ks::BindSeg& sg = g->h_seg[i];
            status_out[i] = step_finish(e, t_end[i], start[i], g->h_out + sg.off, g->h_out + total + sg.off,
                                        out ? out + (int64_t)i * cap : nullptr, out ? cap : 0, &n_out[i]);
        }
    };
    // the host's CPU share: OMP_NUM_THREADS when the job sets it (the GPU box does: 16), else the
    // hardware threads, at most 32
    int hw = (int)std::thread::hardware_concurrency();
    if (const char* v = std::getenv("OMP_NUM_THREADS"))
        if (std::atoi(v) > 0) hw = std::atoi(v);
    const int nth = total >= (1 << 18) ? std::min<int>(S, std::clamp<int>(hw, 1, 32)) : 1;
    if (nth <= 1) {
        finish(0, S);
    } else {
        std::vector<std::thread> pool;
        for (int k = 1; k < nth; k++) pool.emplace_back(finish, (int)((int64_t)S * k / nth), (int)((int64_t)S * (k + 1) / nth));
        finish(0, (int)((int64_t)S / nth));
        for (auto& th : pool) th.join();
    }
    if (stats) {
        *stats = ks_step_stats{};
        stats->step_ms = ms;
        stats->launches = launches;
        for (int i = 0; i < S; i++) stats->pods += n_out[i];
    }
    return KS_OK;
}

// Apply every not-yet-applied expiry with finish tick <= the current tick (ks_filter / ks_score
// see the state Run's next scheduleOne would).  While the run is live the host knows them
// exactly: every expiry attached to a pod < done has been applied (mirror_expired), an expiry
// attached to a later pod j > done finishes after bind_tick[j - 1] >= bind_tick[done] > tick, so
// only the next pod's attached expiries and the unattached ones (pending, when every submitted pod
// is bound) can be due — usually none, and no launch is made.
static ks_status flush_expiries(ks_engine* e) {
    if (e->err == KS_OK) {
        std::vector<int32_t> qs;
        auto add = [&](int64_t q) {
            if (e->h_status[q] == KS_POD_OK && !e->h_expired[q] && e->h_fin[q] <= e->tick) qs.push_back((int32_t)q);
        };
        if (e->done < e->P)
            for (int64_t u = e->h_exp_off[e->done]; u < e->h_exp_off[e->done + 1]; u++) add(e->h_exp_pod[u]);
        e->pending.for_each_due(e->tick, add);
        if ((int)qs.size() <= ks::kTickMaxExp) {
            if (!qs.empty()) {
                ks::ExpList L{};
                for (int32_t q : qs) {
                    ks::TickExp& x = L.x[L.n++];
                    x.node = e->h_node[q];
                    x.q = q;
                    for (int k = 0; k < 3; k++) x.req[k] = e->h_pods[q].req[k];
                }
                HIPCHK(e, ks::launch_apply_exp(e->s, e->expired.p, L, e->st));
            }
        } else {
            HIPCHK(e, ks::launch_flush(e->s, e->pods.p, e->fin.p, e->tick, e->done, e->b_node.p, e->b_status.p,
                                       e->expired.p, e->st));
        }
        for (int32_t q : qs) e->h_expired[q] = 1;
        return KS_OK;
    }
    HIPCHK(e, ks::launch_flush(e->s, e->pods.p, e->fin.p, e->tick, e->done, e->b_node.p, e->b_status.p,
                               e->expired.p, e->st));
    return KS_OK;
}

static ks_status eval_pod(ks_engine* e, int64_t pod) {
    if (!e->nodes_loaded) return fail(e, KS_EINVAL, "no nodes loaded");
    if (pod < 0 || pod >= e->P) return fail(e, KS_EINVAL, "pod %lld out of range", (long long)pod);
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, stage_flush(e));
    ks_status r = flush_expiries(e);
    if (r != KS_OK) return r;
    if (e->n == 0) return KS_OK;
    HIPCHK(e, ks::launch_eval_pod(e->dc, e->s, e->pods.p + pod, e->cfg.filters, e->d_mask, e->d_score, e->mode, e->st));
    return KS_OK;
}

ks_status ks_filter(ks_engine* e, int64_t pod, uint8_t* mask_out) {
    if (!e || !mask_out) return KS_EINVAL;
    ks_status r = eval_pod(e, pod);
    if (r != KS_OK) return r;
    if (e->n) HIPCHK(e, hipMemcpyAsync(mask_out, e->d_mask, e->n, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return KS_OK;
}

ks_status ks_score(ks_engine* e, int64_t pod, int64_t* score_out) {
    if (!e || !score_out) return KS_EINVAL;
    ks_status r = eval_pod(e, pod);
    if (r != KS_OK) return r;
    if (e->n)
        HIPCHK(e, hipMemcpyAsync(score_out, e->d_score, sizeof(int64_t) * e->n, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return KS_OK;
}

// Candidate pod blocks of a usage query over ticks >= t_lo: blocks of the pods [0, q_hi) (bind
// ticks are FIFO-monotone, so q_hi bounds the start side) holding a pod whose run end is > t_lo;
// super blocks whose every pod ended by t_lo are skipped whole.
static int64_t usage_blocks(ks_engine* e, int64_t t_lo, int64_t q_hi) {
    e->h_blk.clear();
    const int64_t nblk = (q_hi + kUBlk - 1) / kUBlk;
    for (int64_t s = 0; s * kUSup < nblk; s++) {
        if (e->sup_end[s] <= t_lo) continue;
        const int64_t b1 = std::min(nblk, (s + 1) * kUSup);
        for (int64_t b = s * kUSup; b < b1; b++)
            if (e->blk_end[b] > t_lo) e->h_blk.push_back((int32_t)b);
    }
    return (int64_t)e->h_blk.size();
}

// pods bound at ticks <= t (a FIFO prefix of the binds made so far)
static int64_t bound_by(const ks_engine* e, int64_t t) {
    return std::upper_bound(e->h_bind_tick.begin(), e->h_bind_tick.begin() + e->done, t) - e->h_bind_tick.begin();
}

static_assert(kUBlk == 256, "usage index block = the usage kernels' workgroup");

ks_status ks_usage_at(ks_engine* e, int64_t t, int64_t* usage_out) {
    if (!e || !usage_out) return KS_EINVAL;
    if (!e->nodes_loaded) return fail(e, KS_EINVAL, "no nodes loaded");
    if (t < 0 || t > e->tick) return fail(e, KS_EINVAL, "usage tick %lld outside [0, %lld]", (long long)t, (long long)e->tick);
    if (e->n == 0) return KS_OK;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, stage_flush(e));
    const int64_t q_hi = bound_by(e, t);
    const int64_t nb = usage_blocks(e, t, q_hi);
    HIPCHK(e, hipMemsetAsync(e->d_usage, 0, sizeof(unsigned long long) * 3 * e->n, e->st));
    if (nb) {
        HIPCHK(e, e->d_blk.reserve(nb, e->st));
        HIPCHK(e, hipMemcpyAsync(e->d_blk.p, e->h_blk.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice, e->st));
        // (profiling: HIP events around the usage kernel alone — its roofline in bench.py)
        if (e->profiling && e->ev[2]) HIPCHK(e, hipEventRecord(e->ev[2], e->st));
        HIPCHK(e, ks::launch_usage(e->d_blk.p, nb, q_hi, t, e->cfg.tick_seconds, e->b_node.p, e->b_status.p, e->t0.p,
                                   e->dur.p, e->phase_off.p, e->cum_sec.p, e->use.p, e->d_usage, e->st));
        if (e->profiling && e->ev[3]) HIPCHK(e, hipEventRecord(e->ev[3], e->st));
    }
    HIPCHK(e, hipMemcpyAsync(usage_out, e->d_usage, sizeof(int64_t) * 3 * e->n, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    if (e->profiling && nb && e->ev[2]) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e->ev[2], e->ev[3]);
        e->kstats.usage_ms += ms;
        e->kstats.usage_n += 1;
        e->kstats.usage_pods += (int64_t)nb * ks::usage_block_pods();
    }
    return KS_OK;
}

ks_status ks_usage(ks_engine* e, int64_t* usage_out) {
    if (!e) return KS_EINVAL;
    return ks_usage_at(e, e->tick, usage_out);
}

ks_status ks_usage_digest(ks_engine* e, int64_t t_lo, int64_t t_hi, uint64_t* out) {
    if (!e || !out) return KS_EINVAL;
    if (!e->nodes_loaded) return fail(e, KS_EINVAL, "no nodes loaded");
    if (t_lo < 0 || t_hi <= t_lo || t_hi - 1 > e->tick || t_hi - t_lo > kMaxDigestTicks)
        return fail(e, KS_EINVAL, "digest window [%lld, %lld) outside [0, %lld] or longer than %lld ticks",
                    (long long)t_lo, (long long)t_hi, (long long)e->tick + 1, (long long)kMaxDigestTicks);
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, stage_flush(e));
    const int64_t T = t_hi - t_lo;
    const int64_t q_hi = bound_by(e, t_hi - 1);
    const int64_t nb = usage_blocks(e, t_lo, q_hi);
    HIPCHK(e, e->d_digest.reserve(6 * (T + 1) + 6 * T, e->st));
    unsigned long long* diff = e->d_digest.p;
    unsigned long long* res = diff + 6 * (T + 1);
    HIPCHK(e, hipMemsetAsync(diff, 0, sizeof(unsigned long long) * 6 * (T + 1), e->st));
    if (nb) {
        HIPCHK(e, e->d_blk.reserve(nb, e->st));
        HIPCHK(e, hipMemcpyAsync(e->d_blk.p, e->h_blk.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice, e->st));
    }
    HIPCHK(e, ks::launch_usage_digest(e->d_blk.p, nb, q_hi, t_lo, t_hi, e->cfg.tick_seconds, e->b_node.p, e->b_status.p,
                                      e->t0.p, e->dur.p, e->preg.p, e->phase_off.p, e->cum_sec.p, e->use.p, diff, res,
                                      e->st));
    HIPCHK(e, hipMemcpyAsync(out, res, sizeof(uint64_t) * 6 * T, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return KS_OK;
}

uint64_t ks_node_mix(int64_t node) {
    uint64_t z = (uint64_t)(node + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Name-keyed index: every pod bound per node in FIFO order, extended over the binds
// [idx_upto, done) on each query; a key's stored pod is the last one bound there (Store
// replaces, kubesim/node/node.go:58).
static void index_binds(ks_engine* e) {
    if ((int64_t)e->node_pods.size() < e->n) e->node_pods.resize(e->n);
    for (int64_t q = e->idx_upto; q < e->done; q++) {
        const int32_t nd = e->h_node[q];
        if (nd < 0) continue;  // the pod an aborted run stopped at is never stored
        e->node_pods[nd].push_back(q);
    }
    e->idx_upto = e->done;
}

ks_status ks_pod_lookup(ks_engine* e, int32_t node, int64_t key_id, int64_t* pod_out) {
    if (!e || !pod_out) return KS_EINVAL;
    *pod_out = -1;
    if (node < 0 || node >= e->n) return fail(e, KS_EINVAL, "node %d out of range", node);
    index_binds(e);
    const std::vector<int64_t>& v = e->node_pods[node];
    for (auto it = v.rbegin(); it != v.rend(); ++it)  // the last Store under the key wins
        if (e->h_key[*it] == key_id) {
            *pod_out = *it;
            return KS_OK;
        }
    return fail(e, KS_ENOTFOUND, "pod with key %lld not found on node %d", (long long)key_id, node);
}

ks_status ks_node_pods(ks_engine* e, int32_t node, int64_t* pods_out, int64_t cap, int64_t* n_out) {
    if (!e || !n_out || cap < 0 || (cap > 0 && !pods_out)) return KS_EINVAL;
    *n_out = 0;
    if (node < 0 || node >= e->n) return fail(e, KS_EINVAL, "node %d out of range", node);
    index_binds(e);
    const std::vector<int64_t>& v = e->node_pods[node];
    // one pod per key: the last one bound here (a pod is listed iff no later pod on this node
    // has its key)
    std::unordered_map<int64_t, int64_t> last;
    last.reserve(v.size());
    for (int64_t q : v) last[e->h_key[q]] = q;
    int64_t k = 0;
    for (int64_t q : v)
        if (last[e->h_key[q]] == q) {
            if (k < cap) pods_out[k] = q;
            k++;
        }
    *n_out = k;
    return KS_OK;
}

ks_status ks_pod_status(ks_engine* e, int64_t pod_lo, int64_t n, ks_pod_info* out) {
    if (!e || (n > 0 && !out) || pod_lo < 0 || n < 0 || pod_lo + n > e->P) return KS_EINVAL;
    if (n == 0) return KS_OK;
    const int64_t hi = std::min(pod_lo + n, e->done), nb = std::max<int64_t>(hi - pod_lo, 0);
    std::vector<int32_t> node(nb), status(nb);
    if (nb) {
        HIPCHK(e, hipSetDevice(e->device));
        HIPCHK(e, stage_flush(e));
        HIPCHK(e, hipMemcpyAsync(node.data(), e->b_node.p + pod_lo, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, e->st));
        HIPCHK(e, hipMemcpyAsync(status.data(), e->b_status.p + pod_lo, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
    }
    for (int64_t i = 0; i < n; i++) {
        const int64_t q = pod_lo + i;
        ks_pod_info& o = out[i];
        o.total_seconds = e->h_total_sec[q];
        const bool bound = i < nb && node[i] >= 0;
        o.node = bound ? node[i] : -1;
        o.start_tick = bound ? e->h_bind_tick[q] : -1;
        if (!bound) o.phase = KS_PHASE_PENDING;
        else if (status[i] != KS_POD_OK) o.phase = KS_PHASE_FAILED;  // CapacityExceeded
        else {
            // IsRunning (kubesim/pod/pod.go:67-69): passed = (t - t0) * tick < Σ phase seconds
            const int64_t dt = e->tick - e->h_bind_tick[q];
            o.phase = (dt >= 0 && dt < e->h_dur[q]) ? KS_PHASE_RUNNING : KS_PHASE_SUCCEEDED;
        }
    }
    return KS_OK;
}

int64_t ks_current_tick(const ks_engine* e) { return e ? e->tick : -1; }
int32_t ks_tick_seconds(const ks_engine* e) { return e ? e->cfg.tick_seconds : -1; }
int64_t ks_queued_pods(const ks_engine* e) { return e ? e->P - e->done : -1; }
const char* ks_last_error(const ks_engine* e) { return e ? e->errmsg.c_str() : "null engine"; }

ks_status ks_last_step_stats(const ks_engine* e, ks_step_stats* out) {
    if (!e || !out) return KS_EINVAL;
    *out = e->stats;
    return KS_OK;
}

ks_status ks_last_step_kernels(const ks_engine* e, ks_kernel_stats* out) {
    if (!e || !out) return KS_EINVAL;
    *out = e->kstats;
    return KS_OK;
}

ks_status ks_debug_counters(ks_engine* e, int64_t* out32) {
    if (!e || !out32) return KS_EINVAL;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemcpyAsync(out32, e->d_ctr, 32 * sizeof(int64_t), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return KS_OK;
}

#ifndef KS_SRC_HASH
#define KS_SRC_HASH "unhashed"
#endif
const char* ks_build_id(void) { return KS_SRC_HASH; }

ks_status ks_debug_invariants(ks_engine* e, int64_t* out4) {
    if (!e || !out4) return KS_EINVAL;
    out4[0] = out4[1] = out4[2] = out4[3] = 0;
    if (!e->d_sweep) return KS_OK;  // (no chunk-resolver batch ran: nothing to check)
    HIPCHK(e, hipSetDevice(e->device));
    std::vector<int32_t> ns(e->n_pad), ei(e->n_pad), fi(e->n_pad);
    int32_t hw = 0;
    HIPCHK(e, hipMemcpyAsync(ns.data(), e->d_nslot, sizeof(int32_t) * e->n_pad, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipMemcpyAsync(fi.data(), e->d_first, sizeof(int32_t) * e->n_pad, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipMemcpyAsync(ei.data(), e->d_eidx, sizeof(int32_t) * e->n_pad, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipMemcpyAsync(&hw, &e->d_sweep->nslot_hw, sizeof hw, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    for (int64_t i = 0; i < e->n_pad; i++) {
        out4[0] += ns[i] != -1 || fi[i] != ks::kNoFirst;
        out4[1] += ei[i] != -1;
    }
    out4[2] = hw;
    out4[3] = ks::kSlotMax;
    return KS_OK;
}

ks_status ks_debug_window(ks_engine* e, void* out, int64_t cap, int64_t* size_out) {
    if (!e || !size_out) return KS_EINVAL;
    *size_out = (int64_t)sizeof(ks::WinWS);
    if (!e->d_sweep || !out || cap <= 0) return KS_OK;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemcpyAsync(out, e->d_sweep, std::min<int64_t>(cap, sizeof(ks::WinWS)), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return KS_OK;
}

ks_status ks_debug_watch(ks_engine* e, int64_t pod) {
    if (!e) return KS_EINVAL;
#ifdef KS_BATCH_LOG
    if (ks_status r = ensure_window_ws(e); r != KS_OK) return r;
    const int32_t w[2] = {(int32_t)pod, 0};
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemcpyAsync(&e->d_sweep->watch_pod, w, sizeof w, hipMemcpyHostToDevice, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return KS_OK;
#else
    (void)pod;
    return KS_EINVAL;  // (a KS_BATCH_LOG diagnostic build only)
#endif
}

void ks_set_profiling(ks_engine* e, int enable) {
    if (e) e->profiling = enable != 0;
}

ks_status ks_selftest(int32_t device, int32_t test, int64_t* failures) {
    if (!failures || test != KS_SELFTEST_LR_MICRO) return KS_EINVAL;
    *failures = -1;
    if (hipSetDevice(device) != hipSuccess) return KS_EDEVICE;
    unsigned long long* d = nullptr;
    unsigned long long h = 0;
    bool ok = hipMalloc(&d, sizeof h) == hipSuccess;
    ok = ok && hipMemset(d, 0, sizeof h) == hipSuccess;
    ok = ok && ks::launch_selftest_lr_micro(d, nullptr) == hipSuccess;
    ok = ok && hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost) == hipSuccess;
    if (d) (void)hipFree(d);
    if (!ok) return KS_EDEVICE;
    *failures = (int64_t)h;
    return KS_OK;
}

}  // extern "C"
