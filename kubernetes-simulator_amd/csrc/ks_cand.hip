// ks_cand.hip — a batch's expiry window and static candidate lists (gfx950), the chunk resolver's
// inputs (ks_chunk.hip).
//
// The reference binds one pod per tick in FIFO order (kubesim/kubesim.go:105-121, 143-166): pod i
// takes the argmax of its key over every node, on the state that the binds of the pods before it
// (admitted per kubesim/node/node.go:36-60) and the expiries due by its tick leave.  After the scan
// (ks_kernels.hip) every pod of the batch has per-block top-L lists; this file turns them into
// what the resolver needs, in two launches around the scan:
//
//   window_prep_kernel   (before the scan) the expiries due before the batch's first pod, applied to
//                        the node state (expire_head's work); the batch's expiry window: the
//                        expiries due before pods 1 .. nb-1 (slots), the distinct nodes E of the
//                        pre-batch pods among them, each pod's own slot.
//   merge_cl_kernel      (after the scan, one workgroup per pod) the exact top-L of the pod's block
//                        lists (the merge kernel's algorithm), then its static candidates cl_i: the
//                        top-L entries outside E (their snapshot key is exact while the node is
//                        unbound) and every E node whose exact key at pod i's tick (the pre-batch
//                        expiries due by then applied) reaches thr_i, the list's last key — sorted,
//                        <= kChR.  Any node outside cl_i that no earlier pod of the batch bound
//                        scores below thr_i.  Every distinct candidate node of the batch gets one
//                        slot (claimed through node_slot) with its record at the batch start.
#include <climits>

#include "ks_device.h"
#include "ks_prep.h"
#include "ks_scan.h"

namespace ks {
namespace sq {

constexpr int kR = kChR;
constexpr int kPrepThreads = 1024;
constexpr int kClBuf = 256;
static_assert(kR <= kWave, "one candidate per lane");
static_assert(kWinSlots <= kPrepThreads, "one window slot per prep thread");

__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }
__device__ __forceinline__ int32_t clamp32(int64_t v) { return (int32_t)(v > INT_MAX ? INT_MAX : v); }

template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* cg(const T* p) {
    return (const __attribute__((address_space(1))) T*)p;
}

// ---------------------------------------------------------------------------------------------
// Window (ks_prep.h prep_body): the expiries attached to pods start+1 .. start+nb-1, the node set E,
// the head expiries, the overlap's touched nodes and rescan flag.  This kernel runs it for the first
// batch of each ks_step pass (and for every batch of the plain chain); an overlapped batch's window
// is computed by the previous chunk kernel's resolver workgroup right after its commit.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kPrepThreads) void window_prep_kernel(const EngineArgs* __restrict__ A, int head, int spec,
                                                                    int slot) {
    const EngineArgs& a = A[0];
    __shared__ prep::PrepLDS L;
    prep::prep_body<kPrepThreads>(a, a.ctr[kCtrStart], a.ctr[kCtrEnd], a.ctr[kCtrErr], head, spec, slot, L);
}

// ---------------------------------------------------------------------------------------------
// Candidate slots.  Every distinct node in the batch's candidate lists gets one slot (the first
// workgroup to meet it claims it through node_slot) and its record at the batch start: ac am ag ap
// rc rm rg nr in 32-bit words (capacities / usage as uint32, -1 = absent; ap clamped), taint,
// label — 12 dwords (ks_chunk.hip NS32; the engine routes an engine here only when its scaled
// capacities are < 2^32 - 1).  The resolver stages all slots in LDS, so a pod's winner is one LDS
// read away.
// ---------------------------------------------------------------------------------------------
#ifdef KS_MCL_DIAG  // (merge_cl sections, thread 0's cycles: ctr[6..12], workgroups ctr[5])
#define MDG_AT(I, T)                                                                      \
    do {                                                                                  \
        const uint64_t t_ = prep::pstamp();                                               \
        if (threadIdx.x == 0) atomicAdd((unsigned long long*)&a.ctr[(I)], t_ - (T));      \
        (T) = t_;                                                                         \
    } while (0)
using prep::pstamp;
#endif
constexpr int kRecWords = 12;
static_assert(kRecWords <= kRecDw, "record size");
constexpr int kSlotPending = -2;
static_assert(kSlotIds <= 65535, "slot ids in 16 bits");

__device__ __forceinline__ void put_rec(uint32_t* o, const NodeV& v) {
    o[0] = (uint32_t)v.ac; o[1] = (uint32_t)v.am; o[2] = (uint32_t)v.ag;
    o[3] = (uint32_t)clamp32(v.ap);
    o[4] = (uint32_t)v.rc; o[5] = (uint32_t)v.rm; o[6] = (uint32_t)v.rg;
    o[7] = (uint32_t)v.nr;
    o[8] = (uint32_t)v.taint; o[9] = (uint32_t)(v.taint >> 32); o[10] = (uint32_t)v.label; o[11] = (uint32_t)(v.label >> 32);
}

// E-node keys per merge_cl thread (E node tid + q * threads)
constexpr int kEPer = kEMax / 256;

// Pod i's static candidates from its merged top-L `cand` (LDS or global, kLL entries), by one
// workgroup: the kept entries (sorted, <= kR) with their slots.  ek: this thread's E-node keys
// (computed before the merge, so their dependent reads overlap the block lists'), 0 = none.
// The list's entries on no E node (their snapshot key is exact) are kept up to kTopL of them; the
// threshold thr is the last kept one when kTopL are kept, else the list's last key (1 when the list
// is not full: no other node is a candidate at all); an E node is kept when its exact key reaches
// thr.  Any other node scores below thr: an untouched node outside the kept entries is below them
// in the snapshot order, and the list's own order bounds every node outside it.  (kLL = kTopL: the
// list's entries outside E and thr = its last key; the overlap's longer lists keep kTopL exact
// entries even when the previous batch bound some of the top ones.)
static_assert(kTopLOverlap >= kTopL, "merged lists kept at the longest list length");
template <int kMode, int kLL>
__device__ __forceinline__ void cand_list(const EngineArgs& a, WinWS& ws, int i, const uint64_t* cand,
                                          const uint64_t* ek, int n_e) {
    static_assert(kLL >= kTopL && kLL <= kWave, "one list entry per lane");
    const int tid = threadIdx.x;
    PDG(uint64_t pt = pstamp();)
    __shared__ uint64_t buf[kClBuf];
    __shared__ int cnt;
    __shared__ uint64_t s_thr;
    __shared__ int s_full;
    if (tid == 0) cnt = 0;
    __syncthreads();
    if (tid < kWave) {  // wave 0, lane k: list entry k
        const int lane = tid;
        const uint64_t x = lane < kLL ? cand[lane] : 0ull;
        const bool un = x != 0 && a.e_idx[key_node(x)] < 0;
        const uint64_t um = __ballot(un);
        const int rank = __popcll(um & ((1ull << lane) - 1ull));
        if (un && rank < kTopL) {
            const int pos = atomicAdd(&cnt, 1);
            if (pos < kClBuf) buf[pos] = x;
        }
        const uint64_t last = cand[kLL - 1];
        const bool enough = __popcll(um) >= kTopL;
        if (enough && un && rank == kTopL - 1) s_thr = x;
        if (!enough && lane == 0) s_thr = last != 0 ? last : 1ull;
        if (lane == 0) s_full = enough || last != 0;
    }
    __syncthreads();
    PDG(MDG_AT(9, pt);)
    const uint64_t thr = s_thr;
    const bool full = s_full != 0;
    for (int k = tid; k < n_e; k += blockDim.x)
        if (ek[k] != 0 && ek[k] >= thr) {
            const int pos = atomicAdd(&cnt, 1);
            if (pos < kClBuf) buf[pos] = ek[k];
        }
    __syncthreads();
    PDG(MDG_AT(10, pt);)
    const int c = cnt, n = c < kClBuf ? c : kClBuf;
    __shared__ uint64_t kept[kR];
    if (tid < n) {  // rank by counting (keys are distinct: the node is in the low bits)
        const uint64_t me = buf[tid];
        int r = 0;
        for (int u = 0; u < n; ++u) r += buf[u] > me;
        if (r < kR) kept[r] = me;
    }
    __syncthreads();
    PDG(MDG_AT(11, pt);)
    if (tid < kWave) {  // the kept entries' slots: one wave, one counter update for its claims
        const int lane = tid;
        const bool valid = lane < (n < kR ? n : kR);
        const uint64_t me = valid ? kept[lane] : 0ull;
        const int32_t nd = key_node(me);
        // the record and E index read before the claim (a claimer needs them; the reads overlap
        // the claim's round trip)
        NodeV rec{};
        int32_t eix = -1;
        if (valid) { rec = load_node(a.s, nd); eix = a.e_idx[nd]; }
        // the node's first kept entry in pod order (the chunk kernel numbers the batch's candidates by
        // it: deterministic ids, so every rank cuts a batch at the same pod)
        if (valid && a.det_cids) atomicMin(&a.n_first[nd], i * kR + lane);
        int sl = valid ? atomicCAS(&a.n_slot[nd], -1, kSlotPending) : 0;
        const bool claim = valid && sl == -1;
        const uint64_t cm = __ballot(claim);
        int base = 0;
        if (cm) {
            const int first = __ffsll((unsigned long long)cm) - 1;
            if (lane == first) base = atomicAdd(&ws.nslot, __popcll(cm));
            base = __shfl(base, first);
        }
        if (claim) {  // number it, stage its record, publish
            sl = base + __popcll(cm & ((1ull << lane) - 1ull));
            ws.slot_node[sl] = nd;
            if (sl < kSlotMax) {
                put_rec(ws.slot_rec[sl], rec);
                ws.slot_eix[sl] = eix;
            }
            atomicExch(&a.n_slot[nd], sl);
        }
        // a node another workgroup claimed: wait for its number (every workgroup publishes its own
        // claims before it waits, and the claimer is running: it executed its CAS)
        bool wait = valid && sl == kSlotPending;
        while (__ballot(wait)) {
            if (wait) {
                sl = __hip_atomic_load(&a.n_slot[nd], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                wait = sl < 0;
            }
            if (__ballot(wait)) __builtin_amdgcn_s_sleep(1);
        }
        if (valid) {
            ws.cl_key[i][lane] = me;
            ws.cl_slot[i][lane] = sl;
        }
    }
    PDG(__syncthreads(); MDG_AT(12, pt);)
    if (tid == 0) {
        ws.cl_info[i] = (c < kR ? c : kR) | (c > kR ? kClTrunc : 0) | (full ? kClFull : 0) | (c > kClBuf ? kClOvf : 0);
        ws.cl_thr[i] = thr;
    }
}

// merge + candidate list of pod b in one workgroup (the merge kernel's exact top-L over nl sorted
// lists lists[b * pod_stride + k * list_stride] of kLL keys, ks_kernels.hip, then cand_list) — one
// launch fewer per batch.  src == nullptr: the engine's own block lists (pruned: only the blocks its
// bitmap flags, ks_scan.h).  Every launch clears the pods' bitmaps and thresholds for the next scan.
constexpr int kMergeMaxWaves = 16;
}  // namespace sq
#ifdef KS_MCL_BYVAL
thread_local const EngineArgs* ks_mcl_host_args = nullptr;  // (diagnostic build: set by step_body before each launch)
#endif
namespace sq {
template <int kMode, int kLL>
#ifdef KS_MCL_BYVAL  // (diagnostic build only: the engine arguments by value, VERDICT r5 item 1's A/B)
__global__ __launch_bounds__(1024) void merge_cl_kernel(const EngineArgs av, const uint64_t* src,
                                                         int64_t pod_stride, int32_t nl, int64_t list_stride, int own_fb) {
    const EngineArgs& a = av;
#else
__global__ __launch_bounds__(1024) void merge_cl_kernel(const EngineArgs* __restrict__ A, const uint64_t* src,
                                                         int64_t pod_stride, int32_t nl, int64_t list_stride, int own_fb) {
    const EngineArgs& a = A[0];
#endif
    WinWS& ws = *a.sw;
    // (own_fb: a pipelined engine's rescan scanned every block locally — its own lists, not src)
    const bool own = src == nullptr || (own_fb && ws.rescan);
    if (own) {
        src = a.lists;
        pod_stride = (int64_t)a.nblk * kLL;
        nl = a.nblk;
        list_stride = kLL;
    }
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nthr = blockDim.x, nwav = nthr / kWave;
    const bool prn = a.lbit != nullptr;
    const int lset = prn ? ws.lset : 1;
    const bool pruned = own && prn;
    // the previous batch stopped early (ks_prep.h): pods b < split take the merged lists kept for
    // them, the others the speculative scan's lists at slot sb = b - split
    const int nbw = ws.nb, split = ws.split, moff = ws.moff, mpar = ws.mpar;
    const bool reuse = b < split;
    const int sb = b - split;
    // pruned: the flagged blocks of the batch's set (one round trip for the bitmap words); then both
    // sets' bitmaps and thresholds of one pod slot are cleared for the next scans — every slot once:
    // this workgroup's own slot sb, the slots no pod reads ([nb - split, B)) by the others
    __shared__ scn::FlagLDS F;
    int nfl = reuse ? 0 : nl;
    if (b < nbw && !reuse && pruned) nfl = scn::flagged_index(lbit_of(a, lset, sb), 0, nl, F);
    if (prn) {
        const int cs = b < split ? nbw - split + b : (b < nbw ? sb : b);
        for (int w = tid; w < 2 * a.nwl; w += nthr) lbit_of(a, w / a.nwl, cs)[w % a.nwl] = 0;
        if (tid < 2 * kThrCopies) *lthr_of(a, tid / kThrCopies, tid % kThrCopies, cs) = 0;
    }
    if (b >= nbw) return;  // (the window prep cut the batch; errors left nb = 0)
    PDG(uint64_t pt = pstamp(); if (tid == 0) atomicAdd((unsigned long long*)&a.ctr[5], 1ull);)
    uint64_t top[kLL];
#pragma unroll
    for (int k = 0; k < kLL; ++k) top[k] = 0;
    const uint64_t* lists = src + (int64_t)(reuse ? 0 : sb) * pod_stride;
    // independent reads first: this thread's first block list, then the E nodes' keys (dependent
    // chains: node, slots, expiring requests) while it is in flight
    uint64_t lv0[kLL];
    const bool has0 = tid < nfl;
    {
        const int l0 = has0 ? (pruned ? scn::flagged_block(tid, 0, nl, F) : tid) : 0;
        const ulonglong2* lp = reinterpret_cast<const ulonglong2*>(lists + (int64_t)l0 * list_stride);
#pragma unroll
        for (int k = 0; k < kLL / 2; ++k) {
            const ulonglong2 w = has0 ? lp[k] : make_ulonglong2(0, 0);
            lv0[2 * k] = w.x;
            lv0[2 * k + 1] = w.y;
        }
    }
    // The E nodes' keys, into LDS, from the records the window prep staged (ws.e_rec: three 16-byte
    // words per E node).  The first two per thread (E nodes tid, tid + nthr) have their reads issued
    // with the counts (unconditionally, clamped into the arrays: one dependent round trip fewer);
    // any further ones (more than 2 nthr E nodes) in a plain loop.
    __shared__ uint64_t ek[kEMax];
    const int n_e = ws.n_e;
    {
        const int64_t start = a.ctr[kCtrStart];
        const int hi = ws.win_hi[b], n_es = ws.n_es;
        uint4 er[2][3];
        int32_t en[2], eu[2], ue[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int k = tid + q * nthr;
            const int kc = k < kEMax ? k : kEMax - 1;
            const int ks = k < kWinSlots ? k : kWinSlots;
            en[q] = ws.e_node[kc];
            const uint4* r = reinterpret_cast<const uint4*>(ws.e_rec[kc]);
            er[q][0] = r[0]; er[q][1] = r[1]; er[q][2] = r[2];
            eu[q] = ws.e_off[ks];
            ue[q] = ws.e_off[ks < kWinSlots ? ks + 1 : ks];
        }
#if defined(KS_MCL_DIAG) && KS_MCL_DIAG == 2
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        uint64_t t_e0 = pstamp();
        if (tid == 0) atomicAdd((unsigned long long*)&a.ctr[13], t_e0 - pt);
#endif
        const PodRec p = a.pods[start + b];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int k = tid + q * nthr;
            if (k >= n_e) continue;
            NodeV v = get_rec12(er[q]);
            if (k < n_es) {
                for (int u = eu[q]; u < ue[q]; ++u) {
                    const int x = ws.e_slot[u];
                    if (x >= hi) break;  // ascending
                    v.rc -= ws.ex_req[x][0]; v.rm -= ws.ex_req[x][1]; v.rg -= ws.ex_req[x][2]; v.nr -= 1;
                }
            }
            ek[k] = make_key(eval_t<kMode>(a.c, p, v), (uint32_t)en[q]);
        }
#pragma unroll 1
        for (int k = tid + 2 * nthr; k < n_e; k += nthr) {
            const int32_t n = ws.e_node[k];
            const uint4* r = reinterpret_cast<const uint4*>(ws.e_rec[k]);
            const uint4 w3[3] = {r[0], r[1], r[2]};
            NodeV w = get_rec12(w3);
            const int ue1 = k < n_es ? ws.e_off[k + 1] : 0;
            for (int u = k < n_es ? ws.e_off[k] : 0; u < ue1; ++u) {
                const int x = ws.e_slot[u];
                if (x >= hi) break;  // ascending
                w.rc -= ws.ex_req[x][0]; w.rm -= ws.ex_req[x][1]; w.rg -= ws.ex_req[x][2]; w.nr -= 1;
            }
            ek[k] = make_key(eval_t<kMode>(a.c, p, w), (uint32_t)n);
        }
#if defined(KS_MCL_DIAG) && KS_MCL_DIAG == 2
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if (tid == 0) { atomicAdd((unsigned long long*)&a.ctr[14], pstamp() - t_e0); atomicAdd((unsigned long long*)&a.ctr[24], (unsigned long long)(n_e > tid) + (n_e > tid + nthr)); }
        if (tid == 0) atomicAdd((unsigned long long*)&a.ctr[25], (unsigned long long)n_e);
#endif
    }
    if (has0) {  // (the first list is the thread's top as it is: sorted)
#pragma unroll
        for (int k = 0; k < kLL; ++k) top[k] = lv0[k];
    }
    for (int j = tid + nthr; j < nfl; j += nthr) {
        const int blk = pruned ? scn::flagged_block(j, 0, nl, F) : j;
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
    __shared__ uint64_t wl[kMergeMaxWaves][kLL];
    __shared__ uint64_t pc[kLL];
    PDG(MDG_AT(6, pt);)
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
    PDG(MDG_AT(7, pt);)
    if (wave == 0 && nthr <= 256) {  // the wave lists' top kLL: one candidate per lane (4 waves)
        static_assert(4 * kLL <= kWave, "one candidate per lane");
        uint64_t v = lane < nwav * kLL ? wl[lane / kLL][lane % kLL] : 0ull;
        for (int r = 0; r < kLL; ++r) {
            const uint64_t m = wave_max_u64(v);
            if (lane == 0) pc[r] = m;
            if (m == 0) continue;
            const uint64_t h = __ballot(v == m);  // keys are distinct: one holder
            if (lane == __ffsll((unsigned long long)h) - 1) v = 0;
        }
    } else if (wave == 0) {  // up to kPer candidates per lane
        constexpr int kPer = (kMergeMaxWaves * kLL + kWave - 1) / kWave;
        const int nc = nwav * kLL;
        uint64_t v[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int c = lane + q * kWave;
            v[q] = c < nc ? wl[c / kLL][c % kLL] : 0ull;
        }
        for (int r = 0; r < kLL; ++r) {
            uint64_t lm = v[0];
#pragma unroll
            for (int q = 1; q < kPer; ++q) lm = lm > v[q] ? lm : v[q];
            const uint64_t m = wave_max_u64(lm);
            if (lane == 0) pc[r] = m;
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
    __syncthreads();
    // a reused pod's merged list as merge_cl kept it for the previous batch; every pod's merged list
    // kept for the next (its possible reuse)
    if (reuse && tid < kLL) pc[tid] = ws.mrg[mpar ^ 1][b + moff][tid];
    if (reuse) __syncthreads();
    if (tid < kLL) ws.mrg[mpar][b][tid] = pc[tid];
    PDG(MDG_AT(8, pt);)
    cand_list<kMode, kLL>(a, ws, b, pc, ek, n_e);
}

}  // namespace sq

hipError_t launch_window_prep(const EngineArgs* d, bool head, bool spec, int slot, hipStream_t st) {
    hipLaunchKernelGGL(sq::window_prep_kernel, dim3(1), dim3(sq::kPrepThreads), 0, st, d, head ? 1 : 0, spec ? 1 : 0,
                       slot & 1);
    return hipGetLastError();
}

hipError_t launch_merge_cl(const EngineArgs* d, int mode, int B, const uint64_t* lists, int64_t pod_stride,
                           int32_t nl, int64_t list_stride, int nl_max, hipStream_t st, int L, bool own_fallback) {
    const int fb = own_fallback ? 1 : 0;
    static_assert(sq::kEPer * 256 >= kEMax, "E keys per thread at 256 threads");
    const dim3 g(B), t(nl_max > 1024 ? 1024 : 256);
#ifdef KS_MCL_BYVAL
    if (!ks_mcl_host_args) return hipErrorInvalidValue;
    const EngineArgs hv = *ks_mcl_host_args;  // (diagnostic: the host copy, as commit 63524d5 passed it)
#define d hv
#endif
#define KS_MCL(LL)                                                                                                   \
    switch (mode) {                                                                                                  \
        case kEvalMicro: hipLaunchKernelGGL((sq::merge_cl_kernel<kEvalMicro, LL>), g, t, 0, st, d, lists, pod_stride, nl, list_stride, fb); break; \
        case kEvalTiny: hipLaunchKernelGGL((sq::merge_cl_kernel<kEvalTiny, LL>), g, t, 0, st, d, lists, pod_stride, nl, list_stride, fb); break;   \
        case kEvalNarrow: hipLaunchKernelGGL((sq::merge_cl_kernel<kEvalNarrow, LL>), g, t, 0, st, d, lists, pod_stride, nl, list_stride, fb); break; \
        default: hipLaunchKernelGGL((sq::merge_cl_kernel<kEvalWide, LL>), g, t, 0, st, d, lists, pod_stride, nl, list_stride, fb); break;          \
    }
    if (L == kTopL) { KS_MCL(kTopL) }
    else if (L == kTopLOverlap) { KS_MCL(kTopLOverlap) }
    else return hipErrorInvalidValue;
#undef KS_MCL
#ifdef KS_MCL_BYVAL
#undef d
#endif
    return hipGetLastError();
}

}  // namespace ks
