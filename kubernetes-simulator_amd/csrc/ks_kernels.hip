// ks_kernels.hip — CDNA4 (gfx950) kernels of the kubesim scheduling engine.
//
// The reference schedules one pod per tick (kubesim/kubesim.go:105-121) and every placement
// depends on the binds before it.  The engine keeps that order exactly, but only a tiny part
// of each pod's decision is sequential.  Per batch of B pods:
//
//   expire_head  applies the expiries due before the batch's first pod.
//   scan         evaluates every (pod, node) pair of the batch against the node state as of
//                the batch start (the "snapshot"): fused Filter + Score + packed key.  Node
//                records are read once per pod group; per pod and per 256-node block it keeps
//                the exact top-L keys.
//   merge        per pod: exact global top-L keys of the snapshot (sorted).
//   resolve      one 1024-thread workgroup walks the batch in FIFO order.  A node's key can
//                differ from the snapshot only if the node was touched in this batch (a bind
//                or an expiry landed on it).  Touched nodes live in an LDS table and are
//                re-evaluated exactly for every pod; the best untouched node is the first
//                untouched entry of the pod's top-L list — exact because any node outside the
//                list scores below every list entry.  winner = max(those).  If all L entries
//                are touched the batch commits early and the next batch rescans.
//
// Every kernel that evaluates exists four times, one per evaluator (ks_device.h): kEvalMicro
// (capacities < 2^16, Ac*Am < 2^24: 24-bit multiplies, correction-free LeastRequested),
// kEvalTiny (int32 math; capacities and Ac*Am < 2^26), kEvalNarrow (capacities < 2^29),
// kEvalWide (64/128-bit, any capacity < 2^59).  The host picks the narrowest that holds.
//
// Packed key: (total + 1) << 32 | (0xFFFFFFFF - node); 0 = no candidate (NotFound).  Max key =
// highest total, ties to the lowest node index.
#include <algorithm>

#include "ks_device.h"
#include "ks_scan.h"

namespace ks {

constexpr int kScanWaves = 4;            // 256-thread scan workgroups, one 256-node block each
constexpr int kBlockNodes = kScanWaves * kWave;
constexpr int kL = kTopL;                // candidate list length per pod
#ifndef KS_MAX_PG
#define KS_MAX_PG 32
#endif
constexpr int kMaxPG = KS_MAX_PG;        // pods per scan workgroup (LDS key table rows)
constexpr int kResolveThreads = 1024;    // 16 waves
constexpr int kOwnerWave0 = 3;           // waves 3..15 own the touched entries, except
#ifndef KS_WRITER_WAVE
#define KS_WRITER_WAVE 5
#endif
#ifndef KS_PRIO
#define KS_PRIO 0
#endif
constexpr int kWriterWave = KS_WRITER_WAVE;  // the bind's bookkeeping writer (off the critical path)
// Resolver size (the LDS footprint): touched-node table entries, open-addressing node -> entry
// map slots (log2), pods per launch, touched filter bits (log2; the filter is exact — no hash
// confirmation — for clusters of at most that many nodes).  RBig: any cluster, 256-pod batches,
// 1024 threads, ~150 KB of LDS (one workgroup per CU).  Small batches of small clusters (what-if
// scenarios) go to the register-table resolver instead (ks_resolve.hip).
template <int THREADS, int TMAX, int HASH_LOG2, int MAXB, int FBITS_LOG2>
struct RCfg {
    static constexpr int kThreads = THREADS;
    static constexpr int kTMax = TMAX;
    static constexpr int kHashLog2 = HASH_LOG2;
    static constexpr int kHash = 1 << HASH_LOG2;
    static constexpr int kMaxBatchR = MAXB;
    static constexpr int kMaxExp = TMAX - MAXB;  // expiries pre-inserted per batch
    static constexpr int kFilterBits = 1 << FBITS_LOG2;
    static_assert(kWriterWave < THREADS / kWave, "the writer wave exists");
    static_assert(TMAX <= (THREADS / kWave - kOwnerWave0 - 1) * kWave, "one touched entry per owner thread");
    static_assert(TMAX - MAXB <= THREADS, "one thread per pre-inserted expiry");
};
using RBig = RCfg<kResolveThreads, 768, 11, 256, 16>;
constexpr int kMaxBatchR = RBig::kMaxBatchR;


// owner slot of a resolve wave, or -1
__device__ __forceinline__ int owner_slot(int wave) {
    if (wave < kOwnerWave0 || wave == kWriterWave) return -1;
    return wave - kOwnerWave0 - (wave > kWriterWave);
}

__device__ __forceinline__ int popc_below(uint64_t mask, int lane) {
    return __popcll(mask & ((1ull << lane) - 1ull));
}

// Every batch kernel takes the device array of its engines' arguments: one engine for ks_step,
// a group's scenarios side by side for ks_group_step (BASELINE configs[3]: independent what-if
// clusters in one launch).  The scenario index is a grid dimension, so every field read is
// uniform (scalar loads).

// ------------------------------------------------------------------------------------------
// expire_head: grid (S).  Expiries due before the batch's first pod, applied straight to the
// node SoA.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void expire_head_kernel(const EngineArgs* __restrict__ A) {
    const EngineArgs a = A[blockIdx.x];
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0 || start >= end) return;
    const int64_t e0 = a.exp_off[start], e1 = a.exp_off[start + 1];
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int32_t q = a.exp_pod[e];
        if (a.b_status[q] != 0 || a.expired[q]) continue;
        const int32_t nd = a.b_node[q];
        const PodRec& p = a.pods[q];
        atomicAdd((unsigned long long*)&a.s.rc[nd], (unsigned long long)(-p.req[0]));
        atomicAdd((unsigned long long*)&a.s.rm[nd], (unsigned long long)(-p.req[1]));
        atomicAdd((unsigned long long*)&a.s.rg[nd], (unsigned long long)(-p.req[2]));
        atomicAdd((unsigned long long*)&a.s.nr[nd], (unsigned long long)(-1ll));
        a.expired[q] = 1;
    }
}

// ------------------------------------------------------------------------------------------
// scan: grid (blk_n, ceil(B / PG), S).  A workgroup owns one 256-node block (lane = node within
// its wave's 64) and PG pods.  Phase 1: every wave evaluates its nodes for all PG pods into an
// LDS key table (one u32 total+1 per pod and node).  Phase 2: one wave per pod extracts the
// block's exact top-L from the 256 keys (4 per lane).  Scores are small integers, so the top-L
// is usually one or two "tie classes": take the max, every node at it in node order, repeat below
// it — a lane max of 4, a 32-bit wave max and 4 ballots per class.
// ------------------------------------------------------------------------------------------
// KT: the key table's word, uint16_t when every total + 1 < 2^16 (the host's check on the scorer
// weights) — half the LDS per workgroup, so more workgroups fit a CU.
constexpr int kStageWgs = 8;  // workgroups staging the E records (grid-stride over n_e <= kEMax)
template <int kMode, typename KT, bool kPrune, int kLL>
__global__ __launch_bounds__(256) void scan_kernel(const EngineArgs* __restrict__ A, int xcd, int cond, int stage,
                                                   int pers) {
    extern __shared__ uint32_t kv_raw[];
    KT* const kv = reinterpret_cast<KT*>(kv_raw);  // [PG][kBlockNodes]: total+1 per (pod, node of the block)
    const EngineArgs& a = A[blockIdx.z];
    // stage: the chunk class — the first kStageWgs workgroups also stage the batch's E records for
    // merge_cl (WinWS::e_rec; one node per thread, grid-stride), before their own work.  launch_scan
    // launches at least kStageWgs workgroups when staging, also for a rank with no scan blocks.
    if (stage && blockIdx.x < kStageWgs) {
        const WinWS& ws = *a.sw;
        const int n_e = ws.n_e;
        for (int k = (int)blockIdx.x * kBlockNodes + (int)threadIdx.x; k < n_e; k += kStageWgs * kBlockNodes)
            put_rec12(a.sw->e_rec[k], load_node(a.s, ws.e_node[k]));
    }
    // cond: the overlap's fallback scan, needed only when window prep flagged a rescan
    if (cond && *(volatile const int32_t*)&a.sw->rescan == 0) return;
    const int64_t start = sload(a.ctr + kCtrStart), end = sload(a.ctr + kCtrEnd);
    if (sload(a.ctr + kCtrErr) != 0) return;
    const int64_t nb = min<int64_t>(a.B, end - start);
    if (nb <= 0) return;
    const int groups = (int)((nb + a.PG - 1) / a.PG);
    // work items (block, pod group), item = block * groups + group, one per workgroup: grid
    // (blk_n, groups, S), or — one engine (xcd) — a 1-D grid dealt XCD-aware: blocks b and b + 8
    // share an XCD (round-robin dispatch, MI355X_MICROARCH.md), so workgroup w takes item
    // (w % 8) * per + w / 8 — each XCD a contiguous item range, the groups of a node block on one
    // XCD back to back: the block's node records come from HBM once and from that XCD's L2 for
    // the other groups (the placement is for speed only; any placement gives the same lists)
    int64_t it_lo;
    if (xcd && pers) {  // (the pipelined engines' rescan: a fixed grid, each workgroup loops over its XCD's items)
        const int64_t tot = (int64_t)a.blk_n * groups, per = (tot + 7) / 8;
        const int64_t lo = (int64_t)(blockIdx.x % 8) * per, hi = min<int64_t>(tot, lo + per);
        for (int64_t it = lo + blockIdx.x / 8; it < hi; it += gridDim.x / 8) {
            if (it != lo + blockIdx.x / 8) __syncthreads();  // (the previous item's extraction has read kv)
            scn::scan_item<kMode, KT, kPrune, kLL>(a, kv, start, nb, groups, it, true, threadIdx.x, (int)(blockIdx.x % kThrCopies));
        }
        return;
    }
    if (xcd) {
        const int64_t tot = (int64_t)a.blk_n * groups, per = (tot + 7) / 8;
        const int64_t k = blockIdx.x / 8;
        if (k >= per) return;
        it_lo = (int64_t)(blockIdx.x % 8) * per + k;
        if (it_lo >= tot) return;
    } else {
        if ((int)blockIdx.x >= a.blk_n || (int)blockIdx.y >= groups) return;  // scenarios may differ in size
        it_lo = (int64_t)blockIdx.x * groups + blockIdx.y;
    }
    scn::scan_item<kMode, KT, kPrune, kLL>(a, kv, start, nb, groups, it_lo, true, threadIdx.x, (int)(blockIdx.x % kThrCopies));
}

// ------------------------------------------------------------------------------------------
// merge: grid (B, S), one workgroup per pod (256 threads, or 1024 for more than 1024 lists);
// exact top-L over nl sorted lists (the scan's block lists of one shard, or the shards'
// all-gathered lists).  src == nullptr: the scenario's own block lists into its candidate lists.
// ------------------------------------------------------------------------------------------
constexpr int kMergeMaxWaves = 16;
// bits != nullptr (a pruned engine's per-part merge, ks_scan.h): only the blocks pod b's bitmap
// bits[b * nwl ...] flags among blocks [blk0, blk0 + nl) (list k = block blk0 + k) are read
// kLL: the lists' length (kTopL; kTopLOverlap for the pipelined sharded engines' per-part merges)
template <int kLL>
__global__ __launch_bounds__(1024) void merge_kernel(const EngineArgs* __restrict__ A, const uint64_t* src,
                                                      int64_t pod_stride, int32_t nl, int64_t list_stride,
                                                      uint64_t* out, const uint64_t* bits, int32_t nwl, int32_t blk0,
                                                      int32_t lset_fixed) {
    const EngineArgs a = A[blockIdx.y];
    if (src == nullptr) {
        src = a.lists;
        pod_stride = (int64_t)a.nblk * kLL;
        nl = a.nblk;
        list_stride = kLL;
        out = a.cand;
    }
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const int64_t nb = min<int64_t>(a.B, end - start);
    const int b = blockIdx.x;
    if (b >= nb) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t top[kLL];  // per-thread sorted (descending) top-L over its blocks
#pragma unroll
    for (int k = 0; k < kLL; ++k) top[k] = 0;
    const uint64_t* lists = src + (int64_t)b * pod_stride;
    const int nthr = blockDim.x, nwav = nthr / kWave;
    __shared__ scn::FlagLDS F;
    // (a sharded chunk engine's per-part merge: bits = the two sets, [2][B][nwl]; the batch's set is
    // the one its window prep named)
    // (lset_fixed >= 0: the pipelined engines' speculative part merges, which run beside the window
    // prep that rewrites a.sw->lset)
    const int lset = lset_fixed >= 0 ? lset_fixed : (bits && a.sw ? a.sw->lset : 1);
    const int nfl = bits ? scn::flagged_index(bits + ((int64_t)lset * a.B + b) * nwl, blk0, nl, F) : nl;
    for (int j = tid; j < nfl; j += nthr) {
        const int blk = bits ? scn::flagged_block(j, blk0, nl, F) : j;
        // the whole list in one round trip (16-byte loads), then the insertions
        const ulonglong2* lp = reinterpret_cast<const ulonglong2*>(lists + (int64_t)blk * list_stride);
        uint64_t lv[kLL];
#pragma unroll
        for (int k = 0; k < kLL / 2; ++k) {
            const ulonglong2 w = lp[k];
            lv[2 * k] = w.x;
            lv[2 * k + 1] = w.y;
        }
        topl_insert<kLL>(top, lv);
    }
    // each wave: L rounds of its max thread head (the owner advances), no barrier; then wave 0
    // merges the wave lists (<= 16 x kLL candidates, kPer per lane) the same way
    __shared__ uint64_t wl[kMergeMaxWaves][kLL];
    int head = 0;
    for (int r = 0; r < kLL; ++r) {
        uint64_t h = 0;
#pragma unroll
        for (int k = 0; k < kLL; ++k) h = (k == head) ? top[k] : h;
        const uint64_t m = wave_max_u64(h);
        const uint64_t hit = __ballot(h == m && m != 0);
        if (lane == 0) wl[wave][r] = m;
        if (hit && lane == __ffsll((unsigned long long)hit) - 1) head++;
    }
    __syncthreads();
    if (wave != 0) return;
    constexpr int kPer = (kMergeMaxWaves * kLL + kWave - 1) / kWave;
    const int nc = nwav * kLL;
    uint64_t v[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int c = lane + q * kWave;
        v[q] = c < nc ? wl[c / kLL][c % kLL] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kLL; ++r) {
        uint64_t lm = v[0];
#pragma unroll
        for (int q = 1; q < kPer; ++q) lm = lm > v[q] ? lm : v[q];
        const uint64_t m = wave_max_u64(lm);
        if (lane == 0) out[(int64_t)b * kLL + r] = m;
        if (m == 0) continue;
        bool done = false;  // keys are distinct: exactly one holder
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const uint64_t h = __ballot(!done && v[q] == m);
            if (h && lane == __ffsll((unsigned long long)h) - 1) v[q] = 0;
            done = done || h != 0;
        }
    }
}

// merge_small: the same for nl * L <= 64 candidates per pod (clusters of <= 2048 nodes — a
// what-if group's scenarios — or a merge of <= 8 shards): one wave per pod, lane = candidate,
// L rounds of a wave max.  Grid (ceil(B / 4), S).
__global__ __launch_bounds__(256) void merge_small_kernel(const EngineArgs* __restrict__ A, const uint64_t* src,
                                                           int64_t pod_stride, int32_t nl, int64_t list_stride,
                                                           uint64_t* out) {
    const EngineArgs a = A[blockIdx.y];
    if (src == nullptr) {
        src = a.lists;
        pod_stride = (int64_t)a.nblk * kL;
        nl = a.nblk;
        list_stride = kL;
        out = a.cand;
    }
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const int64_t nb = min<int64_t>(a.B, end - start);
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
    const int b = blockIdx.x * (blockDim.x / kWave) + wave;
    if (b >= nb) return;  // wave-uniform: the wave max below needs every lane
    const int li = lane / kL, le = lane % kL;
    uint64_t v = li < nl ? src[(int64_t)b * pod_stride + (int64_t)li * list_stride + le] : 0ull;
#pragma unroll
    for (int r = 0; r < kL; ++r) {
        const uint64_t m = wave_max_u64(v);
        if (lane == 0) out[(int64_t)b * kL + r] = m;
        const uint64_t hit = __ballot(v == m && m != 0);
        if (hit && lane == __ffsll((unsigned long long)hit) - 1) v = 0;
    }
}

// ------------------------------------------------------------------------------------------
// resolve: one workgroup, sequential over the batch in FIFO order (one bind per tick).
//
// One barrier per pod.  Pod i's winner is a single LDS word ctl[i % 3].best: every contributor of
// pod i (list candidate, re-evaluated touched entries) folds its key in with an LDS atomic max
// during iteration i-1, so after the barrier every wave reads the decision (and the NotFound /
// InvalidArgument / exhausted-list stops) with one load.  Internal key (ikey):
//     (total + 1) << 34 | (2^24 - 1 - node) << 10 | entry          (entry 1023 = untouched)
// orders exactly like the packed key (node < 2^24, total + 1 < 2^30: ks_engine.cpp) and carries
// the winner's table entry.  Between two barriers the waves split the bind of pod i and the
// evaluation of pod i+1:
//   wave 0    table insert of an untouched winner; pod i+1's best untouched list node (chosen
//             from two prefetched candidates, see below) staged in LDS; pod i+2's list walk and
//             HBM prefetch
//   wave 1    CreatePod admission + bind on the winner's entry (and pod i+1's expiries that
//             land on it); outputs; pod i+1's exact key on that entry
//   wave 2    pod i+1's other expiries; pod i+1's exact keys on those entries
//   3..15     owner threads: thread r keeps touched entry r in registers (reloading the
//             mutable fields when an entry was modified the iteration before) and computes pod
//             i+1's exact key on it, unless wave 1 or 2 owns the entry this iteration
// Writers (waves 1, 2) touch disjoint entries and every reader of those skips them.
//
// Prefetch: pod i+2's list is walked in iteration i; its first two untouched entries' records
// are loaded into wave 0's registers (lane = slot * 10 + field).  In iteration i+1 exactly one
// node can join the table (pod i+1's winner), so pod i+2's first untouched entry is the first
// prefetched one unless that node just won, else the second.
//
// Pruning (exact): pod i+1's winner is >= its first untouched list entry >= its L-th list
// entry (lists are sorted; a full list with every entry touched stops the batch before the
// winner matters; wave 0 publishes a tighter bound, see prefetch_issue).  A touched entry whose
// float upper bound (prune_tmax) is below it is not evaluated, and exact keys below it are not
// folded into best.
// ------------------------------------------------------------------------------------------
// Per-pod control read by every wave right after the barrier: one 16/32-byte LDS load each,
// issued together (a chain of dependent reads here costs ~150 cycles per link).
struct alignas(16) Ctl {
    uint64_t best;   // pod's winner (ikey), folded during the previous iteration
    uint64_t lbk_next;  // lower bound of the NEXT pod's winner key (prefetch_issue), read with best
    int32_t kfull;   // every entry of a full list touched: the batch must stop
    int32_t ntab;    // table size when the pod is evaluated
    int32_t pad[2];
};
// Per-pod control read by every wave each iteration: one 16-byte LDS load (pod i's flags, run
// ticks and own expiry slot; pod i+1's expiry window)
struct alignas(16) PodCC {
    uint32_t w0;     // flags | (exp_slot + 1) << 2
    int32_t dur;     // ticks the pod runs if bound Ok
    int32_t ex_lo1;  // pod i+1's expiry window [ex_lo1, ex_hi1) (empty for the batch's last pod)
    int32_t ex_hi1;
};

template <class C>
struct ResolveShared {
    using Cfg = C;
    static constexpr int kTMax = C::kTMax, kHash = C::kHash, kMaxBatchR = C::kMaxBatchR, kMaxExp = C::kMaxExp,
                         kFilterBits = C::kFilterBits;
    int64_t ts[8][kTMax];       // touched-node state: ac am ag ap rc rm rg nr
    uint64_t tu[2][kTMax];      // taint label
    int32_t tnode[kTMax];
    int32_t dirty[kTMax];       // iteration at which the owner must reload the mutable fields
    int32_t hkey[kHash];        // node id or -1
    int32_t hval[kHash];        // entry index
    uint32_t tfilt[kFilterBits / 32];
    PodRec pod[kMaxBatchR + 1];  // +1: pod i + 1 is read unconditionally
    float podf[kMaxBatchR][2];  // cpu / memory requests as float (prune_tmax)
    PodCC pcc[kMaxBatchR];
    uint64_t cand[kMaxBatchR][kL];
    int32_t ex_q[kMaxExp];
    int32_t ex_node[kMaxExp];
    int32_t ex_ok[kMaxExp];     // the expiring pod was bound Ok and has not expired yet
    int32_t ex_entry[kMaxExp];  // table entry of its node (set at the bind for in-batch pods)
    int64_t ex_req[kMaxExp][3];
    Ctl ctl[3];                 // pod i's decision state, slot i % 3
    int64_t stage[2][10];       // snapshot fields of the pod's best untouched list node
    int32_t n_t, committed, err_code, err_pod, nb, e_cnt;
};

constexpr int kEntUntouched = 1023;
static_assert(RBig::kTMax < kEntUntouched, "entry index fits 10 bits");

__device__ __forceinline__ uint64_t ikey(uint64_t key, int ent) {
    const uint32_t node = 0xFFFFFFFFu - (uint32_t)key;
    return ((key >> 32) << 34) | ((uint64_t)(0xFFFFFFu - node) << 10) | (uint64_t)(uint32_t)ent;
}
__device__ __forceinline__ int32_t ikey_node(uint64_t b) { return (int32_t)(0xFFFFFFu - (uint32_t)((b >> 10) & 0xFFFFFFu)); }
__device__ __forceinline__ int ikey_ent(uint64_t b) {
    const int e = (int)(b & 1023u);
    return e == kEntUntouched ? -1 : e;
}
__device__ __forceinline__ void fold_best(uint64_t* slot, uint64_t k) {
    atomicMax((unsigned long long*)slot, (unsigned long long)k);
}

// Diagnostic build only (-DKS_STAMPS): per-iteration cycle sums and lane counts, accumulated in
// ctr[16..31] (layout: tests/dev/diag_resolve.py); the real kernel executes no stamp.
#ifndef KS_ABL
#define KS_ABL 0  // diagnostic ablations (timing only, results invalid); 0 in every real build
#endif
#ifdef KS_STAMPS
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define KS_STAMP(var) uint64_t var = stamp()
#else
#define KS_STAMP(var)
#endif

template <class SH>
__device__ __forceinline__ uint32_t hslot(int32_t node) {
    return ((uint32_t)node * 2654435761u) >> (32 - SH::Cfg::kHashLog2);
}

// entry index of `node` in the touched table, or -1
template <class SH>
__device__ __forceinline__ int h_find(const SH& sh, int32_t node) {
    constexpr int kHash = SH::kHash;
    uint32_t s = hslot<SH>(node);
    for (int i = 0; i < kHash; ++i) {
        const int32_t k = sh.hkey[s];
        if (k == node) return sh.hval[s];
        if (k == -1) return -1;
        s = (s + 1) & (kHash - 1);
    }
    return -1;
}

// single-lane insert of a node known to be absent
template <class SH>
__device__ __forceinline__ void h_insert(SH& sh, int32_t node, int32_t idx) {
    constexpr int kHash = SH::kHash, kFilterBits = SH::kFilterBits;
    uint32_t s = hslot<SH>(node);
    while (sh.hkey[s] != -1) s = (s + 1) & (kHash - 1);
    sh.hkey[s] = node;
    sh.hval[s] = idx;
    const uint32_t f = (uint32_t)node & (kFilterBits - 1);
    sh.tfilt[f >> 5] |= 1u << (f & 31);
}

// touched? — one LDS read; the filter is exact (node & 0xFFFF is injective) when the cluster has
// at most kFilterBits nodes, otherwise a set bit is confirmed in the hash
template <class SH>
__device__ __forceinline__ bool is_touched(const SH& sh, int32_t node, bool exact) {
    constexpr int kFilterBits = SH::kFilterBits;
    const uint32_t f = (uint32_t)node & (kFilterBits - 1);
    if (!((sh.tfilt[f >> 5] >> (f & 31)) & 1u)) return false;
    return exact || h_find(sh, node) >= 0;
}

// table insert of an in-loop winner: with an exact filter only the filter bit (the hash is
// consulted only by the batch-start pre-insert and by inexact filters)
template <class SH>
__device__ __forceinline__ void t_insert(SH& sh, int32_t node, int32_t idx, bool exact) {
    constexpr int kFilterBits = SH::kFilterBits;
    if (exact) {
        const uint32_t f = (uint32_t)node & (kFilterBits - 1);
        atomicOr(&sh.tfilt[f >> 5], 1u << (f & 31));
    } else {
        h_insert(sh, node, idx);
    }
}

template <class SH>
__device__ __forceinline__ NodeV t_node(const SH& sh, int e) {
    NodeV v;
    v.ac = sh.ts[0][e]; v.am = sh.ts[1][e]; v.ag = sh.ts[2][e]; v.ap = sh.ts[3][e];
    v.rc = sh.ts[4][e]; v.rm = sh.ts[5][e]; v.rg = sh.ts[6][e]; v.nr = sh.ts[7][e];
    v.taint = sh.tu[0][e]; v.label = sh.tu[1][e];
    return v;
}

template <class SH>
__device__ __forceinline__ NodeV stage_node(const SH& sh, int b) {
    NodeV v;
    v.ac = sh.stage[b][0]; v.am = sh.stage[b][1]; v.ag = sh.stage[b][2]; v.ap = sh.stage[b][3];
    v.rc = sh.stage[b][4]; v.rm = sh.stage[b][5]; v.rg = sh.stage[b][6]; v.nr = sh.stage[b][7];
    v.taint = (uint64_t)sh.stage[b][8]; v.label = (uint64_t)sh.stage[b][9];
    return v;
}

// field f (0..9, NodeV order) of node i: the SoA is one allocation with a fixed field stride
__device__ __forceinline__ int64_t node_field(const NodeSoA& s, int f, int64_t i) {
    return gptr(s.ac)[(int64_t)f * (s.am - s.ac) + i];
}

__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }

// A pod record read from LDS as three 16-byte loads issued together, pinned in registers by an
// empty asm use (otherwise the compiler sinks each field's load into the config branch that
// uses it, turning one LDS round trip into several dependent ones).
__device__ __forceinline__ PodRec pod_regs(const PodRec* src) {
    const uint4* w = reinterpret_cast<const uint4*>(src);
    const uint4 w0 = w[0], w1 = w[1], w2 = w[2];
    asm volatile("" ::"v"(w0.x), "v"(w0.y), "v"(w0.z), "v"(w0.w), "v"(w1.x), "v"(w1.y), "v"(w1.z), "v"(w1.w),
                 "v"(w2.x), "v"(w2.y), "v"(w2.z), "v"(w2.w));
    PodRec p;
    static_assert(sizeof(PodRec) == 3 * sizeof(uint4), "PodRec is three 16-byte words");
    __builtin_memcpy(&p, &w0, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p) + 16, &w1, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p) + 32, &w2, 16);
    return p;
}

// two records, all six loads issued before the single pin
__device__ __forceinline__ void pod_regs2(const PodRec* s0, const PodRec* s1, PodRec& p0, PodRec& p1) {
    const uint4* a = reinterpret_cast<const uint4*>(s0);
    const uint4* b = reinterpret_cast<const uint4*>(s1);
    const uint4 a0 = a[0], a1 = a[1], a2 = a[2], b0 = b[0], b1 = b[1], b2 = b[2];
    asm volatile("" ::"v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a0.w), "v"(a1.x), "v"(a1.y), "v"(a1.z), "v"(a1.w),
                 "v"(a2.x), "v"(a2.y), "v"(a2.z), "v"(a2.w), "v"(b0.x), "v"(b0.y), "v"(b0.z), "v"(b0.w),
                 "v"(b1.x), "v"(b1.y), "v"(b1.z), "v"(b1.w), "v"(b2.x), "v"(b2.y), "v"(b2.z), "v"(b2.w));
    __builtin_memcpy(&p0, &a0, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p0) + 16, &a1, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p0) + 32, &a2, 16);
    __builtin_memcpy(&p1, &b0, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p1) + 16, &b1, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p1) + 32, &b2, 16);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Wave 0 prefetch state for one pod: its first two list entries whose node is untouched
// (key1, key2; 0 = none), whether the list holds L candidates (so "none" means exhausted, not
// "no candidates"), and their records: lanes 0..19 hold field (lane % 10) of entry lane / 10.
struct Prefetch {
    int64_t val;
    uint64_t key1, key2;
    bool full;
};

// Walk pod p's list against the table and issue the record loads.  Also publishes pod p's
// winner lower bound: the first untouched entry when pod p is decided is key1 or key2 (or none:
// then the batch stops at a full list, or the list is short and the bound is 0), so key2 — or
// key1 when the list is full and has no second — is <= it.
template <class SH>
__device__ __forceinline__ void prefetch_issue(const EngineArgs& a, SH& sh, int p, int lane, bool exact,
                                               Prefetch& pf) {
    const uint64_t c = lane < kL ? sh.cand[p][lane] : 0ull;
    const bool ok = c != 0 && !is_touched(sh, key_node(c), exact);
    uint64_t m = __ballot(ok);
    pf.full = __popcll(__ballot(c != 0)) == kL;
    const int pa1 = m ? __ffsll((unsigned long long)m) - 1 : -1;
    m &= m - 1;
    const int pa2 = m ? __ffsll((unsigned long long)m) - 1 : -1;
    pf.key1 = pa1 >= 0 ? readlane64(c, pa1) : 0ull;
    pf.key2 = pa2 >= 0 ? readlane64(c, pa2) : 0ull;
    // into pod p-1's slot: read by every wave together with pod p-1's decision
    if (lane == 0) sh.ctl[(p + 2) % 3].lbk_next = pf.key2 ? pf.key2 : (pf.full ? pf.key1 : 0ull);
    const uint64_t ks = lane < 10 ? pf.key1 : pf.key2;
    if (lane < 20 && ks != 0) pf.val = node_field(a.s, lane % 10, key_node(ks));
}

// Wave 0: pod p's best untouched list node given that `winner` just joined the table (-1:
// none): stage its record, fold its key into ctl[bslot].best, set kfull.
template <class SH>
__device__ __forceinline__ void prefetch_commit(SH& sh, int lane, const Prefetch& pf, int32_t winner,
                                                int stage_buf, int bslot) {
    const int slot = (pf.key1 != 0 && key_node(pf.key1) == winner) ? 1 : 0;
    const uint64_t key = slot ? pf.key2 : pf.key1;
    if (key != 0 && lane < 20 && lane / 10 == slot) sh.stage[stage_buf][lane % 10] = pf.val;
    if (lane == 0) {
        if (key != 0) fold_best(&sh.ctl[bslot].best, ikey(key, kEntUntouched));
        sh.ctl[bslot].kfull = key == 0 && pf.full;
    }
}

// The expiries due before pod j + 1 binds (window range [e0, e1)) that land on entry t — pod
// j's own included when it was bound Ok and runs one tick — subtracted from n.  Lane-parallel:
// one LDS round for the whole range; the (usually zero or one) hits are folded via a ballot.
// Marks them expired when `expired` is given (the writer wave).
template <class SH>
__device__ __forceinline__ void expire_on(const SH& sh, int e0, int e1, int t, int64_t j, bool ok,
                                          int lane, NodeV& n, uint8_t* expired) {
    for (int x0 = e0; x0 < e1; x0 += kWave) {
        const int x = x0 + lane;
        bool hit = false;
        int32_t q = 0;
        int64_t r0 = 0, r1 = 0, r2 = 0;
        if (x < e1) {
            q = sh.ex_q[x];
            hit = q == j ? ok : (sh.ex_entry[x] == t && sh.ex_ok[x] != 0);
            r0 = sh.ex_req[x][0]; r1 = sh.ex_req[x][1]; r2 = sh.ex_req[x][2];
        }
        if (hit && expired) gptr(expired)[q] = 1;
        uint64_t m = __ballot(hit);
        while (m) {
            const int l = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            n.rc -= (int64_t)readlane64((uint64_t)r0, l);
            n.rm -= (int64_t)readlane64((uint64_t)r1, l);
            n.rg -= (int64_t)readlane64((uint64_t)r2, l);
            n.nr -= 1;
        }
    }
}

template <int kMode, class C>
__global__ __launch_bounds__(C::kThreads) void resolve_kernel(const EngineArgs* __restrict__ A) {
    constexpr int kTMax = C::kTMax, kHash = C::kHash, kMaxBatchR = C::kMaxBatchR, kMaxExp = C::kMaxExp,
                  kFilterBits = C::kFilterBits, kResolveThreads = C::kThreads;
    __shared__ ResolveShared<C> sh;
    const EngineArgs a = A[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const bool exact = a.c.n_nodes <= kFilterBits;  // touched filter needs no hash confirmation
    int nb = (int)min<int64_t>(min<int64_t>(a.B, kMaxBatchR), end - start);
    if (nb <= 0) return;
    KS_STAMP(g0);

    // window: expiries of pods start+1 .. start+nb-1 (pod start's were applied by expire_head);
    // shrink the batch so that they fit the pre-insert budget
    // largest nb' <= nb whose window fits: exp_off is non-decreasing, so the count of fitting
    // prefixes is nb' (one HBM round trip for all candidates instead of a serial bisection)
    const int64_t e_base = a.exp_off[start + 1];
    const int64_t off_mid = tid < nb ? a.exp_off[start + tid + 1] : 0;
    const bool fits_win = tid < nb && off_mid - e_base <= kMaxExp;
    if (tid == 0) {
        sh.n_t = 0; sh.err_code = 0; sh.err_pod = -1;
        for (int b = 0; b < 3; ++b) sh.ctl[b] = Ctl{0, 0, 0, 0, {0, 0}};
    }
    for (int h = tid; h < kHash; h += kResolveThreads) sh.hkey[h] = -1;
    for (int w = tid; w < kFilterBits / 32; w += kResolveThreads) sh.tfilt[w] = 0;
    nb = __syncthreads_count(fits_win);
    if (tid == nb - 1) { sh.nb = nb; sh.committed = nb; sh.e_cnt = nb > 1 ? (int32_t)(off_mid - e_base) : 0; }
    __syncthreads();
    const int64_t e_cnt = sh.e_cnt;
    KS_STAMP(g1);

    for (int i = tid; i < nb; i += kResolveThreads) {
        sh.pod[i] = a.pods[start + i];
        sh.podf[i][0] = (float)a.pods[start + i].req[0];
        sh.podf[i][1] = (float)a.pods[start + i].req[1];
        const int64_t pos = a.exp_pos[start + i];
        const int32_t exp_slot = (pos >= e_base && pos - e_base < e_cnt) ? (int32_t)(pos - e_base) : -1;
        PodCC pc;
        pc.w0 = a.pods[start + i].flags | (uint32_t)(exp_slot + 1) << 2;
        pc.dur = a.dur[start + i];
        // pod i+1's window: the expiries due before it binds (pod start's were applied by expire_head)
        const bool nx = i + 1 < nb;
        pc.ex_lo1 = !nx || i + 1 <= 1 ? 0 : (int32_t)(a.exp_off[start + i + 1] - e_base);
        pc.ex_hi1 = !nx ? 0 : (int32_t)(a.exp_off[start + i + 2] - e_base);
        sh.pcc[i] = pc;
    }
    for (int i = tid; i < nb * kL; i += kResolveThreads) sh.cand[i / kL][i % kL] = a.cand[i];
    for (int e = tid; e < e_cnt; e += kResolveThreads) {
        const int32_t q = a.exp_pod[e_base + e];
        const PodRec& pq = a.pods[q];
        sh.ex_q[e] = q;
        sh.ex_entry[e] = -1;
        sh.ex_req[e][0] = pq.req[0]; sh.ex_req[e][1] = pq.req[1]; sh.ex_req[e][2] = pq.req[2];
        if (q < start) {
            sh.ex_node[e] = a.b_node[q];
            sh.ex_ok[e] = (a.b_status[q] == 0) && !a.expired[q];
        } else {
            sh.ex_node[e] = -1;
            sh.ex_ok[e] = 0;  // set when the pod binds
        }
    }
    __syncthreads();
    KS_STAMP(g2);
    // pre-insert every node an expiry of this batch lands on (q bound before the batch): the
    // per-pod expiry step then never waits on HBM.  One thread per expiry (e_cnt <= kMaxExp <
    // kResolveThreads): claim the node's hash slot with a CAS (duplicates find it), number the
    // claimed slots, then read the entry back.  Entry numbering order is immaterial: an entry
    // index only names a node, it never takes part in a comparison between distinct nodes.
    const bool pre_want = tid < e_cnt && sh.ex_ok[tid];
    int pre_slot = -1;
    bool pre_claim = false;
    if (pre_want) {
        const int32_t nd = sh.ex_node[tid];
        uint32_t hs = hslot<ResolveShared<C>>(nd);
        for (;;) {  // the table holds <= kMaxExp < kHash nodes: terminates
            const int32_t prev = atomicCAS(&sh.hkey[hs], -1, nd);
            if (prev == -1 || prev == nd) { pre_slot = (int)hs; pre_claim = prev == -1; break; }
            hs = (hs + 1) & (kHash - 1);
        }
    }
    __syncthreads();
    if (pre_claim) {
        const int32_t nd = sh.ex_node[tid];
        const int idx = atomicAdd(&sh.n_t, 1);
        sh.hval[pre_slot] = idx;
        sh.tnode[idx] = nd;
        const uint32_t f = (uint32_t)nd & (kFilterBits - 1);
        atomicOr(&sh.tfilt[f >> 5], 1u << (f & 31));
    }
    __syncthreads();
    if (pre_want) sh.ex_entry[tid] = sh.hval[pre_slot];
    __syncthreads();
    KS_STAMP(g3);
    for (int e = tid; e < kTMax; e += kResolveThreads) sh.dirty[e] = -1;
    for (int e = tid; e < sh.n_t; e += kResolveThreads) {
        const NodeV v = load_node(a.s, sh.tnode[e]);
        sh.ts[0][e] = v.ac; sh.ts[1][e] = v.am; sh.ts[2][e] = v.ag; sh.ts[3][e] = v.ap;
        sh.ts[4][e] = v.rc; sh.ts[5][e] = v.rm; sh.ts[6][e] = v.rg; sh.ts[7][e] = v.nr;
        sh.tu[0][e] = v.taint; sh.tu[1][e] = v.label;
    }
    __syncthreads();
    KS_STAMP(g4);

    // owner registers (waves 3..15): entry r = tid - 192
    const int oslot = owner_slot(wave);
    const int r = oslot >= 0 ? oslot * kWave + lane : kTMax;
    bool loaded = false;
    NodeV own{};
    int32_t own_node = 0;
    PruneF own_pf{};      // prune_tmax state of the entry
    Prefetch pf{};        // wave 0

    // ---- prologue: pod 0's contributions into ctl[0].best; pod 1's prefetch
    if (wave == 0) {
        Prefetch p0;
        prefetch_issue(a, sh, 0, lane, exact, p0);
        prefetch_commit(sh, lane, p0, -1, 0, 0);
        // Pod 0 never stops on an exhausted list: its own expiries were applied before the scan
        // and nothing else has changed yet, so every touched entry still holds its snapshot key
        // and is evaluated exactly below — a node outside the list cannot beat them.  (Stopping
        // here would commit nothing, and the next launch would rescan the same state forever.)
        if (lane == 0) { sh.ctl[0].ntab = sh.n_t; sh.ctl[0].kfull = 0; }
        if (nb > 1) prefetch_issue(a, sh, 1, lane, exact, pf);
    } else if (oslot >= 0 && r < sh.n_t) {
        own = t_node(sh, r);
        own_node = sh.tnode[r];
        own_pf = prune_prep_t<kMode>(a.c, own);
        loaded = true;
        const uint64_t k = make_key(eval_t<kMode>(a.c, sh.pod[0], own), (uint32_t)own_node);
        if (k != 0 && k >= sh.cand[0][kL - 1]) fold_best(&sh.ctl[0].best, ikey(k, r));
    }
    __syncthreads();
    KS_STAMP(g5);
#if !KS_KEEP_IDLE_OWNERS
    // The table grows by at most one entry per pod, so owner waves whose first entry lies past
    // n_t + nb can never own one: they end here.  s_barrier waits only for the surviving waves of
    // the workgroup (CDNA ISA, S_BARRIER), and their threads have no share in the write-back
    // (tid >= 64 * (oslot + 3) > n_t + nb >= the final table size).
    if (oslot >= 0 && oslot * kWave >= sh.n_t + nb) return;
#endif

#ifdef KS_STAMPS
    uint64_t acc_work = 0, acc_wait = 0, acc_sub[8] = {0, 0, 0, 0, 0, 0, 0, 0}, acc_cnt[4] = {0, 0, 0, 0};
#endif
#if KS_PRIO
    // static issue priority for the waves on the per-pod critical path (the bind wave first,
    // then the list walker and the expiry wave) over the owner waves sharing their SIMDs
    if (wave == 1) __builtin_amdgcn_s_setprio(2);
    else if (wave == 0 || wave == 2) __builtin_amdgcn_s_setprio(1);
#endif
    int i = 0;
    for (; i < nb; ++i) {
        KS_STAMP(s0);
        const int64_t j = start + i;
        const int cur = i & 1, nxt = cur ^ 1;
        const int b_cur = i % 3, b_nxt = (i + 1) % 3;
        // ---- every wave: pod i's winner and the stop decision (identical in all waves)
        const Ctl cc = sh.ctl[b_cur];
        const PodCC pci = sh.pcc[i];
        const uint64_t lbk = cc.lbk_next;
        const uint64_t bw = cc.best;
        int stop = 0;
        if (cc.kfull) stop = 1;                                       // list exhausted: rescan
        else if (bw == 0) stop = 2;                                   // NotFound
        else if (pci.w0 & (kFlagBadKey | kFlagBadSpec)) stop = 3;     // InvalidArgument
        if (stop) {
            if (tid == 0) {
                sh.committed = i;
                if (stop > 1) { sh.err_code = stop == 2 ? kErrNotFound : kErrEinval; sh.err_pod = (int32_t)j; }
            }
            break;
        }
        const int went = ikey_ent(bw);
        const int32_t nd = ikey_node(bw);
        const int nt = cc.ntab;
        const int t = went >= 0 ? went : nt;  // an untouched winner becomes entry nt
        const bool has_next = i + 1 < nb;
        const int e0 = pci.ex_lo1, e1 = pci.ex_hi1;
        KS_STAMP(sw);
#ifdef KS_STAMPS
        acc_sub[0] += sw - s0;
#endif

        if (oslot >= 0) {
            if (has_next && oslot * kWave < nt && !(KS_ABL & 16)) {
                // one round of independent LDS reads, then the (rare) reload
                const int32_t dr = sh.dirty[r < kTMax ? r : 0];
                const float qfc = sh.podf[i + 1][0], qfm = sh.podf[i + 1][1];
                const PodRec pn = pod_regs(&sh.pod[i + 1]);
                if (r < nt) {
                    if (!loaded) {
                        own = t_node(sh, r);
                        own_node = sh.tnode[r];
                        own_pf = prune_prep_t<kMode>(a.c, own);
                        loaded = true;
                    } else if (dr == i) {
                        own.rc = sh.ts[4][r]; own.rm = sh.ts[5][r]; own.rg = sh.ts[6][r]; own.nr = sh.ts[7][r];
                        own_pf = prune_prep_t<kMode>(a.c, own);
                    }
                }
                bool want = r < nt && own_pf.live && r != went;
#ifdef KS_STAMPS
                acc_cnt[0] += __popcll(__ballot(r < nt));
                acc_cnt[1] += __popcll(__ballot(want));
#endif
                if (lbk != 0 && want) {
                    const uint32_t tm = prune_tmax(a.c, own_pf, qfc, qfm);
                    want = make_key(tm + 1u, (uint32_t)own_node) >= lbk;
                }
#ifdef KS_STAMPS
                acc_cnt[2] += __popcll(__ballot(want));
                acc_cnt[3] += __ballot(want) != 0;
#endif
                KS_STAMP(sa);
                if (__ballot(want)) {
                    for (int x = e0; x < e1; ++x)  // wave 2 owns the entries pod i+1's expiries land on
                        want &= !(sh.ex_entry[x] == r && sh.ex_q[x] != j);
                    KS_STAMP(sb);
                    if (want && !(KS_ABL & 1)) {
                        const uint64_t k = make_key(eval_t<kMode>(a.c, pn, own), (uint32_t)own_node);
                        if (k != 0 && k >= lbk) fold_best(&sh.ctl[b_nxt].best, ikey(k, r));
                    }
                    KS_STAMP(sc);
#ifdef KS_STAMPS
                    if (wave == 3) { acc_sub[2] += sb - sa; acc_sub[3] += sc - sb; }
#endif
                }
#ifdef KS_STAMPS
                if (wave == 3) acc_sub[1] += sa - sw;
#endif
            }
        } else if (wave == 0) {
            if (lane == 0) {
                if (went < 0) { sh.tnode[t] = nd; t_insert(sh, nd, t, exact); }
                sh.ctl[b_nxt].ntab = went < 0 ? nt + 1 : nt;
                sh.ctl[(i + 2) % 3].best = 0;  // read in iteration i-1, folded into in iteration i+1
            }
            KS_STAMP(t0a);
            if (has_next) prefetch_commit(sh, lane, pf, went < 0 ? nd : -1, nxt, b_nxt);
            KS_STAMP(t0b);
            if (i + 2 < nb) prefetch_issue(a, sh, i + 2, lane, exact, pf);
            KS_STAMP(t0c);
#ifdef KS_STAMPS
            acc_cnt[0] += t0a - sw; acc_cnt[1] += t0b - t0a; acc_cnt[2] += t0c - t0b;
#endif
        } else if (wave == 1 || wave == kWriterWave) {
            // the bind of pod i on entry t: wave 1 computes pod i+1's key on the new state (the
            // critical path), the writer wave stores the state and the outputs
            PodRec p, pnext;  // pod i + 1 <= nb: a readable slot
            pod_regs2(&sh.pod[i], &sh.pod[i + 1], p, pnext);
            NodeV n = went >= 0 ? t_node(sh, t) : stage_node(sh, cur);
            const bool ok = fits(p, n);  // CreatePod admission (kubesim/node/node.go:44-47)
            if (ok && pci.dur > 0) { n.rc += p.req[0]; n.rm += p.req[1]; n.rg += p.req[2]; n.nr += 1; }
            KS_STAMP(t1a);
            expire_on(sh, e0, e1, t, j, ok, lane, n, wave == 1 ? nullptr : a.expired);
            KS_STAMP(t1b);
            if (wave == 1) {
                if (lane == 0 && has_next && !(KS_ABL & 2)) {
                    const uint64_t k = make_key(eval_t<kMode>(a.c, pnext, n), (uint32_t)nd);
                    if (k != 0) fold_best(&sh.ctl[b_nxt].best, ikey(k, t));
                }
                KS_STAMP(t1d);
#ifdef KS_STAMPS
                acc_sub[4] += t1a - sw; acc_sub[5] += t1b - t1a; acc_sub[7] += t1d - t1b;
#endif
            } else if (lane == 0) {
                if (went < 0) {
                    sh.ts[0][t] = n.ac; sh.ts[1][t] = n.am; sh.ts[2][t] = n.ag; sh.ts[3][t] = n.ap;
                    sh.tu[0][t] = n.taint; sh.tu[1][t] = n.label;
                }
                sh.ts[4][t] = n.rc; sh.ts[5][t] = n.rm; sh.ts[6][t] = n.rg; sh.ts[7][t] = n.nr;
                sh.dirty[t] = i + 1;
                const int slot = (int)(pci.w0 >> 2) - 1;
                if (slot >= 0) { sh.ex_entry[slot] = t; sh.ex_ok[slot] = ok ? 1 : 0; }
                gptr(a.b_node)[j] = nd;
                gptr(a.b_status)[j] = ok ? 0 : 1;
            }
        } else if (wave == 2) {
            if (has_next && e1 > e0 && !(KS_ABL & 4)) {
                // pod i+1's other expiries, lane-parallel: LDS atomics apply them (several may hit
                // one entry), then each lane evaluates its expiry's entry on the final state
                // (LDS operations of one wave complete in order)
                const PodRec pn = pod_regs(&sh.pod[i + 1]);
                for (int x0 = e0; x0 < e1; x0 += kWave) {  // apply every expiry first ...
                    const int x = x0 + lane;
                    if (x < e1) {
                        const int32_t q = sh.ex_q[x];
                        const int tq = sh.ex_entry[x];
                        const int okx = sh.ex_ok[x];
                        const int64_t r0 = sh.ex_req[x][0], r1 = sh.ex_req[x][1], r2 = sh.ex_req[x][2];
                        if (q != j && tq >= 0 && tq != t && okx) {
                            atomicAdd((unsigned long long*)&sh.ts[4][tq], (unsigned long long)-r0);
                            atomicAdd((unsigned long long*)&sh.ts[5][tq], (unsigned long long)-r1);
                            atomicAdd((unsigned long long*)&sh.ts[6][tq], (unsigned long long)-r2);
                            atomicAdd((unsigned long long*)&sh.ts[7][tq], (unsigned long long)-1ll);
                            sh.dirty[tq] = i + 1;
                            gptr(a.expired)[q] = 1;
                        }
                    }
                }
                for (int x0 = e0; x0 < e1; x0 += kWave) {  // ... then evaluate their entries
                    const int x = x0 + lane;
                    if (x < e1) {
                        const int tq = sh.ex_entry[x];
                        if (sh.ex_q[x] != j && tq >= 0 && tq != t) {
                            const uint64_t k = make_key(eval_t<kMode>(a.c, pn, t_node(sh, tq)), (uint32_t)sh.tnode[tq]);
                            if (k != 0) fold_best(&sh.ctl[b_nxt].best, ikey(k, tq));
                        }
                    }
                }
            }
        }
        KS_STAMP(s1);
        __syncthreads();
        KS_STAMP(s2);
#ifdef KS_STAMPS
        acc_work += s1 - s0;
        acc_wait += s2 - s1;
#endif
    }
    __syncthreads();
#ifdef KS_STAMPS
    {
        unsigned long long* d = (unsigned long long*)a.ctr + 16;
        if (lane == 0 && wave <= 3) atomicAdd(&d[wave == 3 ? 15 : (wave == 0 ? 0 : wave + 1)], acc_work);
        if (lane == 0 && wave == 0) atomicAdd(&d[1], acc_wait);
        if (tid == 0) atomicAdd(&d[4], (unsigned long long)i);
        if (lane == 0 && wave == 3)
            for (int k = 0; k < 4; ++k) atomicAdd(&d[5 + k], acc_sub[k]);       // top, load, excl, eval
        if (lane == 0 && wave == 1)
            for (int k = 0; k < 4; ++k) atomicAdd(&d[11 + k], acc_sub[4 + k]);  // fetch+fit, expiries, writes, eval
        if (lane == 0 && wave == 3) atomicAdd(&d[3 + 0], 0ull);
        if (tid == 0) atomicAdd(&d[4 + 0], 0ull);
        if (lane == 0 && wave == 0)
            for (int k = 0; k < 3; ++k) atomicAdd((unsigned long long*)a.ctr + 5 + k, acc_cnt[k]);  // w0 insert/commit/issue
        if (lane == 0 && oslot >= 0) {
            atomicAdd(&d[9], acc_cnt[2]);   // lanes passing prune_tmax
            atomicAdd(&d[10], acc_cnt[3]);  // owner waves evaluating
        }
    }
#endif

    // ---- write back the mutable fields of every touched node
    KS_STAMP(g6);
    const int n_final = sh.ctl[sh.committed % 3].ntab;
    for (int e = tid; e < n_final; e += kResolveThreads) {
        const int64_t ndx = sh.tnode[e];
        a.s.rc[ndx] = sh.ts[4][e];
        a.s.rm[ndx] = sh.ts[5][e];
        a.s.rg[ndx] = sh.ts[6][e];
        a.s.nr[ndx] = sh.ts[7][e];
    }
    if (tid == 0) {
        a.ctr[kCtrStart] = start + sh.committed;
        if (sh.committed < a.B && sh.err_code == 0 && start + sh.committed < end) a.ctr[kCtrEarly] += 1;
        if (sh.err_code) { a.ctr[kCtrErr] = sh.err_code; a.ctr[kCtrErrPod] = sh.err_pod; }
    }
#ifdef KS_STAMPS
    __syncthreads();
    KS_STAMP(g7);
    if (tid == 0) {  // setup / writeback phases, ctr[8..14]
        unsigned long long* d = (unsigned long long*)a.ctr;
        atomicAdd(&d[8], g1 - g0);   // init + expiry-window search
        atomicAdd(&d[9], g2 - g1);   // pod / list / expiry loads
        atomicAdd(&d[10], g3 - g2);  // expiry-node pre-insert
        atomicAdd(&d[11], g4 - g3);  // table record loads
        atomicAdd(&d[12], g5 - g4);  // prologue (pod 0)
        atomicAdd(&d[13], g7 - g6);  // writeback
        atomicAdd(&d[14], 1ull);     // launches
        atomicAdd(&d[15], (unsigned long long)e_cnt);  // expiries in windows
    }
#endif
}

// ------------------------------------------------------------------------------------------
// Filter mask / score of one pod against every node (api.Filter / api.Scorer shims).
// ------------------------------------------------------------------------------------------
template <int kMode>
__global__ __launch_bounds__(256) void eval_pod_kernel(Cfg c, NodeSoA s, const PodRec* pod, uint32_t filters,
                                                        uint8_t* mask, int64_t* score) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= c.n_nodes) return;
    const NodeV n = load_node(s, i);
    const PodRec p = *pod;
    bool ok = true;
    if (filters & kFilterFit) ok &= fits(p, n);
    if (filters & kFilterTaint) ok &= (n.taint & ~p.tol) == 0;
    if (filters & kFilterSelector) ok &= (n.label & p.sel) == p.sel;
    mask[i] = ok ? 1 : 0;
    const uint32_t t1 = eval_t<kMode>(c, p, n);
    score[i] = t1 ? (int64_t)t1 - 1 : -1;
}

// Apply every not-yet-applied expiry with finish tick <= t (before ks_filter / ks_score).
__global__ __launch_bounds__(256) void flush_kernel(NodeSoA s, const PodRec* pods, const int64_t* fin, int64_t t,
                                                     int64_t n_done, const int32_t* b_node, const int32_t* b_status,
                                                     uint8_t* expired) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n_done; q += (int64_t)gridDim.x * blockDim.x) {
        if (fin[q] > t || b_status[q] != 0 || expired[q]) continue;
        const int32_t nd = b_node[q];
        const PodRec& p = pods[q];
        atomicAdd((unsigned long long*)&s.rc[nd], (unsigned long long)(-p.req[0]));
        atomicAdd((unsigned long long*)&s.rm[nd], (unsigned long long)(-p.req[1]));
        atomicAdd((unsigned long long*)&s.rg[nd], (unsigned long long)(-p.req[2]));
        atomicAdd((unsigned long long*)&s.nr[nd], (unsigned long long)(-1ll));
        expired[q] = 1;
    }
}

// Per-node usage at tick t: Σ over running pods of the current simSpec phase's usage
// (kubesim/pod/pod.go:47-63; int32 passed seconds vs int32 cumulative phase seconds), scattered
// into the node rows with 64-bit atomic adds (exact).  Grid: the host's candidate blocks of
// kUsageBlk pods (only blocks holding a pod that may still run at t), pods < q_hi (bound by t).
constexpr int kUsageBlk = 256;
__global__ __launch_bounds__(kUsageBlk) void usage_kernel(const int32_t* __restrict__ blocks, int64_t q_hi, int64_t t,
                                                           int32_t tick_s, const int32_t* b_node, const int32_t* b_status,
                                                           const int64_t* t0, const int32_t* dur,
                                                           const int32_t* phase_off, const int32_t* cum_sec,
                                                           const int64_t* use, unsigned long long* usage) {
    const int64_t q = (int64_t)blocks[blockIdx.x] * kUsageBlk + threadIdx.x;
    if (q >= q_hi || b_status[q] != 0) return;
    const int64_t dt = t - t0[q];
    if (dt < 0 || dt >= dur[q]) return;
    const int32_t passed = (int32_t)(dt * tick_s);
    for (int32_t f = phase_off[q]; f < phase_off[q + 1]; ++f) {
        if (passed < cum_sec[f]) {
            const int64_t nd = b_node[q];
            atomicAdd(&usage[nd * 3 + 0], (unsigned long long)use[(int64_t)f * 3 + 0]);
            atomicAdd(&usage[nd * 3 + 1], (unsigned long long)use[(int64_t)f * 3 + 1]);
            atomicAdd(&usage[nd * 3 + 2], (unsigned long long)use[(int64_t)f * 3 + 2]);
            break;
        }
    }
}

// Per-tick usage digest over ticks [t_lo, t_hi) (ks_usage_digest): each running pod's phases
// are piecewise constant in t, so a phase active over ticks [a, b) adds +u at a and -u at b
// of a difference array (six of them: Σ usage[k] and Σ mix(node) * usage[k], mod 2^64), and
// one prefix sum gives every tick.  Regular pods (non-negative phases, no int32 wrap): phase f
// is active iff c_{f-1} <= (t - t0) * tick < c_f, i.e. t - t0 in [ceil(c_{f-1}/tick),
// ceil(c_f/tick)); others are evaluated tick by tick with the reference's int32 arithmetic.
__device__ __forceinline__ uint64_t node_mix(int64_t node) {
    uint64_t z = (uint64_t)(node + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ void digest_add(unsigned long long* diff, int64_t T1, int64_t lo, int64_t hi,
                                           const int64_t* u, uint64_t w) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint64_t v = (uint64_t)u[k];
        if (!v) continue;
        atomicAdd(&diff[k * T1 + lo], (unsigned long long)v);
        atomicAdd(&diff[k * T1 + hi], (unsigned long long)(0ull - v));
        const uint64_t vw = v * w;
        atomicAdd(&diff[(3 + k) * T1 + lo], (unsigned long long)vw);
        atomicAdd(&diff[(3 + k) * T1 + hi], (unsigned long long)(0ull - vw));
    }
}
__global__ __launch_bounds__(kUsageBlk) void usage_digest_kernel(
    const int32_t* __restrict__ blocks, int64_t q_hi, int64_t t_lo, int64_t t_hi, int32_t tick_s,
    const int32_t* b_node, const int32_t* b_status, const int64_t* t0, const int32_t* dur, const uint8_t* preg,
    const int32_t* phase_off, const int32_t* cum_sec, const int64_t* use, unsigned long long* diff) {
    const int64_t q = (int64_t)blocks[blockIdx.x] * kUsageBlk + threadIdx.x;
    if (q >= q_hi || b_status[q] != 0) return;
    const int64_t d = dur[q];
    if (d <= 0) return;
    const int64_t s = t0[q];
    const int64_t a0 = max(s, t_lo), a1 = min(s + d, t_hi);
    if (a0 >= a1) return;
    const uint64_t w = node_mix(b_node[q]);
    const int64_t T1 = t_hi - t_lo + 1;
    const int32_t f0 = phase_off[q], f1 = phase_off[q + 1];
    if (preg[q]) {
        int64_t c_prev = 0;
        for (int32_t f = f0; f < f1; ++f) {
            const int64_t c = cum_sec[f];
            if (c > c_prev) {
                const int64_t lo = max(a0, s + (c_prev + tick_s - 1) / tick_s);
                const int64_t hi = min(a1, s + (c + tick_s - 1) / tick_s);
                if (lo < hi) digest_add(diff, T1, lo - t_lo, hi - t_lo, use + (int64_t)f * 3, w);
                c_prev = c;
            }
        }
    } else {
        for (int64_t t = a0; t < a1; ++t) {
            const int32_t passed = (int32_t)((t - s) * tick_s);
            for (int32_t f = f0; f < f1; ++f)
                if (passed < cum_sec[f]) {
                    digest_add(diff, T1, t - t_lo, t - t_lo + 1, use + (int64_t)f * 3, w);
                    break;
                }
        }
    }
}

// Prefix sums of the six difference arrays ([6][T + 1]) into out[T][6]: one workgroup per
// array, each thread a contiguous chunk, a workgroup scan of the chunk sums.
__global__ __launch_bounds__(1024) void digest_scan_kernel(const unsigned long long* __restrict__ diff, int64_t T,
                                                            unsigned long long* __restrict__ out) {
    __shared__ unsigned long long part[1024];
    const int k = blockIdx.x, tid = threadIdx.x;
    const unsigned long long* d = diff + (int64_t)k * (T + 1);
    const int64_t chunk = (T + 1023) / 1024, lo = min<int64_t>(T, tid * chunk), hi = min<int64_t>(T, lo + chunk);
    unsigned long long s = 0;
    for (int64_t i = lo; i < hi; ++i) s += d[i];
    part[tid] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const unsigned long long v = tid >= off ? part[tid - off] : 0ull;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    unsigned long long run = tid ? part[tid - 1] : 0ull;
    for (int64_t i = lo; i < hi; ++i) {
        run += d[i];
        out[i * 6 + k] = run;
    }
}

// Multiply every device quantity of resource k by f[k] (node capacity unless absent, requested
// totals, pod requests): the unit of resource k shrinks to a divisor of the old one when a pod
// brings a quantity the old unit does not divide (see ks_engine.cpp, resource scale).
__global__ __launch_bounds__(256) void rescale_kernel(NodeSoA s, int64_t n_pad, PodRec* pods, int64_t P,
                                                      int64_t f0, int64_t f1, int64_t f2) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += stride) {
        if (s.ac[i] >= 0) s.ac[i] *= f0;
        if (s.am[i] >= 0) s.am[i] *= f1;
        if (s.ag[i] >= 0) s.ag[i] *= f2;
        s.rc[i] *= f0; s.rm[i] *= f1; s.rg[i] *= f2;
    }
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < P; q += stride) {
        pods[q].req[0] *= f0; pods[q].req[1] *= f1; pods[q].req[2] *= f2;
    }
}

// ---------------------------------------------------------------------------------------------
// Launchers, called by ks_engine.cpp.
// ---------------------------------------------------------------------------------------------
int max_batch_pods() { return kMaxBatchR; }
int max_pods_per_scan_wg() { return kMaxPG; }
int block_nodes() { return kBlockNodes; }

hipError_t launch_expire_head(const EngineArgs* d, int S, hipStream_t st) {
    hipLaunchKernelGGL(expire_head_kernel, dim3(S), dim3(256), 0, st, d);
    return hipGetLastError();
}

template <typename KT, bool kPrune, int kLL>
static void launch_scan_t(const EngineArgs* d, const dim3& g, size_t lds, int mode, int xcd, int cond, int stage, int pers,
                          hipStream_t st) {
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL((scan_kernel<kEvalMicro, KT, kPrune, kLL>), g, dim3(kBlockNodes), lds, st, d, xcd, cond, stage, pers); break;
        case kEvalTiny: hipLaunchKernelGGL((scan_kernel<kEvalTiny, KT, kPrune, kLL>), g, dim3(kBlockNodes), lds, st, d, xcd, cond, stage, pers); break;
        case kEvalNarrow: hipLaunchKernelGGL((scan_kernel<kEvalNarrow, KT, kPrune, kLL>), g, dim3(kBlockNodes), lds, st, d, xcd, cond, stage, pers); break;
        default: hipLaunchKernelGGL((scan_kernel<kEvalWide, KT, kPrune, kLL>), g, dim3(kBlockNodes), lds, st, d, xcd, cond, stage, pers); break;
    }
}

hipError_t launch_scan(const EngineArgs* d, int S, int blk_n, int B, int PG, int mode, bool key16, hipStream_t st,
                       bool cond, bool prune, int L, bool stage, int pw) {
    // (a staging launch runs even when this rank scans no blocks: merge_cl reads the E records)
    if ((blk_n > 0 || (stage && S == 1)) && S > 0) {
        // one (block, pod group) item per workgroup; one engine: the XCD-aware 1-D deal
        const int groups = (B + PG - 1) / PG;
        const size_t lds = (key16 ? sizeof(uint16_t) : sizeof(uint32_t)) * kBlockNodes * PG;
        const bool xcd = S == 1;
        int64_t wgs = std::max<int64_t>(((int64_t)blk_n * groups + 7) / 8 * 8, stage ? kStageWgs : 0);
        if (pw > 0 && S == 1) wgs = std::max<int64_t>(std::min<int64_t>(wgs, pw / 8 * 8), kStageWgs);  // (persistent)
        const dim3 g = xcd ? dim3((unsigned)wgs, 1, 1) : dim3(blk_n, groups, S);
        const int x = xcd ? 1 : 0, c = cond ? 1 : 0, sg = stage && xcd ? 1 : 0;
        if (L != kTopL) {  // the overlap's single-shard lists and the pipelined sharded engines' (ks_engine.cpp)
            if (L != kTopLOverlap) return hipErrorInvalidValue;
            if (key16) {
                if (prune) launch_scan_t<uint16_t, true, kTopLOverlap>(d, g, lds, mode, x, c, sg, pw > 0 ? 1 : 0, st);
                else launch_scan_t<uint16_t, false, kTopLOverlap>(d, g, lds, mode, x, c, sg, pw > 0 ? 1 : 0, st);
            } else {
                if (prune) launch_scan_t<uint32_t, true, kTopLOverlap>(d, g, lds, mode, x, c, sg, pw > 0 ? 1 : 0, st);
                else launch_scan_t<uint32_t, false, kTopLOverlap>(d, g, lds, mode, x, c, sg, pw > 0 ? 1 : 0, st);
            }
        } else if (key16) {
            if (prune) launch_scan_t<uint16_t, true, kTopL>(d, g, lds, mode, x, c, sg, pw > 0 ? 1 : 0, st);
            else launch_scan_t<uint16_t, false, kTopL>(d, g, lds, mode, x, c, sg, pw > 0 ? 1 : 0, st);
        } else {
            if (prune) launch_scan_t<uint32_t, true, kTopL>(d, g, lds, mode, x, c, sg, pw > 0 ? 1 : 0, st);
            else launch_scan_t<uint32_t, false, kTopL>(d, g, lds, mode, x, c, sg, pw > 0 ? 1 : 0, st);
        }
    }
    return hipGetLastError();
}

hipError_t launch_merge(const EngineArgs* d, int S, int B, const uint64_t* lists, int64_t pod_stride, int32_t nl,
                        int64_t list_stride, uint64_t* out, int nl_max, hipStream_t st, const uint64_t* bits,
                        int32_t nwl, int32_t blk0, int32_t lset_fixed, int L) {
    const dim3 g(B, S), t(nl_max > 1024 ? 1024 : 256);
    if (L == kTopLOverlap && L != kTopL) {
        hipLaunchKernelGGL(merge_kernel<kTopLOverlap>, g, t, 0, st, d, lists, pod_stride, nl, list_stride, out, bits,
                           nwl, blk0, lset_fixed);
    } else if (L != kTopL) {
        return hipErrorInvalidValue;
    } else if ((int64_t)nl_max * kL <= kWave && !bits) {
        hipLaunchKernelGGL(merge_small_kernel, dim3((B + 3) / 4, S), dim3(256), 0, st, d, lists, pod_stride, nl,
                           list_stride, out);
    } else {
        hipLaunchKernelGGL(merge_kernel<kTopL>, g, t, 0, st, d, lists, pod_stride, nl, list_stride, out, bits, nwl, blk0,
                           lset_fixed);
    }
    return hipGetLastError();
}

template <class C>
static void launch_resolve_t(const EngineArgs* d, int S, int mode, hipStream_t st) {
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL((resolve_kernel<kEvalMicro, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        case kEvalTiny: hipLaunchKernelGGL((resolve_kernel<kEvalTiny, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        case kEvalNarrow: hipLaunchKernelGGL((resolve_kernel<kEvalNarrow, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        default: hipLaunchKernelGGL((resolve_kernel<kEvalWide, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
    }
}

hipError_t launch_resolve(const EngineArgs* d, int S, int mode, hipStream_t st) {
    launch_resolve_t<RBig>(d, S, mode, st);
    return hipGetLastError();
}

// Packed copy of each scenario's new binds (ks_group_step): one D2H copy for the whole group.
__global__ __launch_bounds__(256) void gather_binds_kernel(const BindSeg* __restrict__ segs, int32_t* node,
                                                            int32_t* status) {
    const BindSeg g = segs[blockIdx.y];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g.n; i += (int64_t)gridDim.x * blockDim.x) {
        node[g.off + i] = g.node[g.lo + i];
        status[g.off + i] = g.status[g.lo + i];
    }
}

hipError_t launch_gather_binds(const BindSeg* segs, int S, int64_t max_n, int32_t* node, int32_t* status,
                               hipStream_t st) {
    if (S <= 0 || max_n <= 0) return hipSuccess;
    const unsigned bx = (unsigned)std::min<int64_t>((max_n + 255) / 256, 64);
    hipLaunchKernelGGL(gather_binds_kernel, dim3(bx, S), dim3(256), 0, st, segs, node, status);
    return hipGetLastError();
}

hipError_t launch_rescale(const NodeSoA& s, int64_t n_pad, PodRec* pods, int64_t P, const int64_t f[3], hipStream_t st) {
    hipLaunchKernelGGL(rescale_kernel, dim3(1024), dim3(256), 0, st, s, n_pad, pods, P, f[0], f[1], f[2]);
    return hipGetLastError();
}

hipError_t launch_eval_pod(const Cfg& c, const NodeSoA& s, const PodRec* pod, uint32_t filters, uint8_t* mask,
                           int64_t* score, int mode, hipStream_t st) {
    const dim3 g((c.n_nodes + 255) / 256);
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL(eval_pod_kernel<kEvalMicro>, g, dim3(256), 0, st, c, s, pod, filters, mask, score); break;
        case kEvalTiny: hipLaunchKernelGGL(eval_pod_kernel<kEvalTiny>, g, dim3(256), 0, st, c, s, pod, filters, mask, score); break;
        case kEvalNarrow: hipLaunchKernelGGL(eval_pod_kernel<kEvalNarrow>, g, dim3(256), 0, st, c, s, pod, filters, mask, score); break;
        default: hipLaunchKernelGGL(eval_pod_kernel<kEvalWide>, g, dim3(256), 0, st, c, s, pod, filters, mask, score); break;
    }
    return hipGetLastError();
}

// Self-test of the micro evaluator's correction-free LeastRequested floor: every (x, A) pair with
// 0 <= x <= A < 2^16 against the exact integer floor (one thread per A).
__global__ __launch_bounds__(256) void selftest_lr_micro_kernel(unsigned long long* bad) {
    const int32_t A = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x) + 1;
    if (A >= kMicroCap) return;
    const float r = 10.f * rcp_est((float)A);
    unsigned long long nbad = 0;
    for (int32_t x = 0; x <= A; ++x) {
        const int64_t q = lr10_micro(x, r), y = 10ll * x;
        nbad += (q * A <= y && y < (q + 1) * A) ? 0ull : 1ull;
    }
    if (nbad) atomicAdd(bad, nbad);
}

hipError_t launch_selftest_lr_micro(unsigned long long* bad, hipStream_t st) {
    hipLaunchKernelGGL(selftest_lr_micro_kernel, dim3((unsigned)((kMicroCap + 255) / 256)), dim3(256), 0, st, bad);
    return hipGetLastError();
}

hipError_t launch_flush(const NodeSoA& s, const PodRec* pods, const int64_t* fin, int64_t t, int64_t n_done,
                        const int32_t* b_node, const int32_t* b_status, uint8_t* expired, hipStream_t st) {
    if (n_done <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n_done + 255) / 256, 2048);
    hipLaunchKernelGGL(flush_kernel, dim3((unsigned)blocks), dim3(256), 0, st, s, pods, fin, t, n_done, b_node,
                       b_status, expired);
    return hipGetLastError();
}

int usage_block_pods() { return kUsageBlk; }

hipError_t launch_usage(const int32_t* blocks, int64_t nblocks, int64_t q_hi, int64_t t, int32_t tick_s,
                        const int32_t* b_node, const int32_t* b_status, const int64_t* t0, const int32_t* dur,
                        const int32_t* phase_off, const int32_t* cum_sec, const int64_t* use,
                        unsigned long long* usage, hipStream_t st) {
    if (nblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(usage_kernel, dim3((unsigned)nblocks), dim3(kUsageBlk), 0, st, blocks, q_hi, t, tick_s, b_node,
                       b_status, t0, dur, phase_off, cum_sec, use, usage);
    return hipGetLastError();
}

hipError_t launch_usage_digest(const int32_t* blocks, int64_t nblocks, int64_t q_hi, int64_t t_lo, int64_t t_hi,
                               int32_t tick_s, const int32_t* b_node, const int32_t* b_status, const int64_t* t0,
                               const int32_t* dur, const uint8_t* preg, const int32_t* phase_off,
                               const int32_t* cum_sec, const int64_t* use, unsigned long long* diff,
                               unsigned long long* out, hipStream_t st) {
    if (nblocks > 0)
        hipLaunchKernelGGL(usage_digest_kernel, dim3((unsigned)nblocks), dim3(kUsageBlk), 0, st, blocks, q_hi, t_lo,
                           t_hi, tick_s, b_node, b_status, t0, dur, preg, phase_off, cum_sec, use, diff);
    hipLaunchKernelGGL(digest_scan_kernel, dim3(6), dim3(1024), 0, st, diff, t_hi - t_lo, out);
    return hipGetLastError();
}
}  // namespace ks
