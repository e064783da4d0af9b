// ks_seq.hip — the sequential resolver (gfx950): a batch's binds one pod at a time in ONE wave.
//
// The reference binds one pod per tick in FIFO order (kubesim/kubesim.go:105-121, 143-166): pod i
// takes the argmax of its key over every node, on the state that the binds of the pods before it
// (admitted per kubesim/node/node.go:36-60) and the expiries due by its tick leave.  After the scan
// and merge (ks_kernels.hip) every pod of the batch has its exact snapshot top-L list; this file
// turns those lists into the batch's binds in three kernels:
//
//   window_prep_kernel   the batch's expiry window: the expiries due before pods 1 .. nb-1 (slots),
//                        the distinct nodes E of the pre-batch pods among them, each pod's own slot.
//   seq_cl_kernel        per pod i (one workgroup each): its static candidates cl_i — the top-L
//                        entries outside E (their snapshot key is exact while the node is unbound)
//                        and every E node whose exact key at pod i's tick (the pre-batch expiries
//                        due by then applied) reaches thr_i, the list's last key — sorted, <= kChR,
//                        with each candidate's node record staged for the resolver.  Any node
//                        outside cl_i that no earlier pod of the batch bound scores below thr_i.
//   resolve_seq_kernel   the FIFO loop.  Pod i's winner is max(S_i, D_i): S_i = the first cl_i
//                        entry that no earlier pod bound; D_i = the best exact key over the nodes
//                        the earlier pods bound ("entries", their states replayed exactly: binds
//                        with admission, the pre-batch expiries, the bound pods' own expiries).
//                        With no S_i the exhausted-list rule applies (D must beat the list's last
//                        key or the batch commits before pod i and the next launch rescans).
//
// The loop has no barrier.  Entries live in the registers of wave 0 (entry e: lane e % 64, slot
// e / 64); per pod the wave prunes its entries against S_i with the float upper bound prune_tmax
// (exact: only entries that might beat S_i are evaluated), evaluates the rest, and takes a wave
// maximum only when one beats S_i (C3: ~5 of ~190 pods per batch land on a node bound earlier in
// the batch).  Everything the next pods need — their candidate keys, the bound test of those keys
// (an LDS hash of the entries' nodes), their staged records, their pod records — is fetched one to
// three pods ahead, so the per-pod chain is: prune, (evaluate), decide, bind.
#include <climits>

#include "ks_device.h"

namespace ks {
namespace sq {

constexpr int kL = kTopL;
constexpr int kB = kWinMaxB;
constexpr int kR = kChR;
constexpr int kThreads = 256;              // setup and commit; the loop runs in wave 0 alone
constexpr int kES = kB / kWave;            // entry register slots (one entry per bind at most)
constexpr int kPend = 4;                   // pending own expiries per entry
constexpr int kPrepThreads = 1024;
constexpr int kEHashLog2 = 11, kEHash = 1 << kEHashLog2;
constexpr int kClBuf = 256;
static_assert(kR <= kWave, "one candidate per lane");
static_assert(kWinSlots <= kPrepThreads, "one window slot per prep thread");
static_assert(kES * kWave < 1023, "entry index fits the ikey's 10 bits");

__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }
__device__ __forceinline__ uint32_t ehslot(int32_t n) { return ((uint32_t)n * 2654435761u) >> (32 - kEHashLog2); }
__device__ __forceinline__ int32_t clamp32(int64_t v) { return (int32_t)(v > INT_MAX ? INT_MAX : v); }

template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* cg(const T* p) {
    return (const __attribute__((address_space(1))) T*)p;
}

// ---------------------------------------------------------------------------------------------
// Window: the expiries attached to pods start+1 .. start+nb-1 (exp_off CSR), one slot each; the
// batch shrinks to the largest prefix whose window fits kWinSlots.  E = the distinct nodes of the
// slots whose pod was bound Ok before the batch and has not expired; e_idx marks them.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kPrepThreads) void window_prep_kernel(const EngineArgs* __restrict__ A, int head) {
    const EngineArgs& a = A[0];
    WinWS& ws = *a.sw;
    const int tid = threadIdx.x;
    __shared__ int32_t hk[kEHash], hv[kEHash];
    __shared__ int32_t cnt[kWinSlots], fill[kWinSlots];
    __shared__ int32_t s_ne;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    int nb = (int)min<int64_t>(min<int64_t>(a.B, kWinMaxB), end - start);
    if (a.ctr[kCtrErr] != 0 || nb <= 0) {
        if (tid == 0) { ws.nb = 0; ws.e_cnt = 0; ws.n_e = 0; }
        return;
    }
    if (head) {  // expire_head's work: the expiries due before the batch's first pod
        const int64_t e0 = a.exp_off[start], e1 = a.exp_off[start + 1];
        for (int64_t e = e0 + tid; e < e1; e += kPrepThreads) {
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
    const int64_t e_base = a.exp_off[start + 1];
    const bool fits_win = tid < nb && a.exp_off[start + tid + 1] - e_base <= kWinSlots;
    for (int h = tid; h < kEHash; h += kPrepThreads) hk[h] = -1;
    if (tid == 0) s_ne = 0;
    nb = __syncthreads_count(fits_win);  // exp_off is non-decreasing: a prefix of the pods
    const int e_cnt = (int)(a.exp_off[start + nb] - e_base);
    if (tid < nb) {
        ws.win_hi[tid] = tid >= 1 ? (int32_t)(a.exp_off[start + tid + 1] - e_base) : 0;
        const int64_t pos = a.exp_pos[start + tid];
        ws.own[tid] = (pos >= e_base && pos - e_base < e_cnt) ? (int32_t)(pos - e_base) : -1;
    }
    int32_t my_node = -1, my_k = -1;
    if (tid < e_cnt) {
        const int32_t q = a.exp_pod[e_base + tid];
        const PodRec& pq = a.pods[q];
        ws.ex_q[tid] = q;
        ws.ex_req[tid][0] = pq.req[0]; ws.ex_req[tid][1] = pq.req[1]; ws.ex_req[tid][2] = pq.req[2];
        const bool ok = q < start && a.b_status[q] == 0 && !a.expired[q];
        ws.ex_ok[tid] = ok ? 1 : 0;
        if (ok) my_node = a.b_node[q];
    }
    bool claimed = false;
    if (my_node >= 0) {
        uint32_t h = ehslot(my_node);
        for (;;) {  // <= kWinSlots distinct nodes < kEHash slots: terminates
            const int32_t prev = atomicCAS(&hk[h], -1, my_node);
            if (prev == -1) { claimed = true; break; }
            if (prev == my_node) break;
            h = (h + 1) & (kEHash - 1);
        }
        my_k = (int32_t)h;  // hash slot; the claiming thread numbers the node
        if (claimed) hv[h] = atomicAdd(&s_ne, 1);
    }
    __syncthreads();
    const int n_e = s_ne;
    if (tid < n_e) { cnt[tid] = 0; fill[tid] = 0; }
    __syncthreads();
    int k_of = -1;
    if (my_node >= 0) {
        k_of = hv[my_k];
        ws.e_node[k_of] = my_node;
        atomicAdd(&cnt[k_of], 1);
    }
    __syncthreads();
    {  // exclusive prefix of the counts (n_e <= kPrepThreads: one per thread)
        __shared__ int32_t wsum[kPrepThreads / 64];
        const int lane = tid & 63, wv = tid >> 6;
        const int v = tid < n_e ? cnt[tid] : 0;
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int base = 0;
        for (int g = 0; g < wv; ++g) base += wsum[g];
        if (tid < n_e) ws.e_off[tid] = base + incl - v;
        if (tid == n_e - 1) ws.e_off[n_e] = base + incl;
        if (n_e == 0 && tid == 0) ws.e_off[0] = 0;
    }
    __syncthreads();
    if (my_node >= 0) ws.e_slot[ws.e_off[k_of] + atomicAdd(&fill[k_of], 1)] = tid;  // slot x == tid
    __syncthreads();
    if (tid < n_e) {  // each node's few slots ascending
        const int lo = ws.e_off[tid], hi = ws.e_off[tid + 1];
        for (int u = lo + 1; u < hi; ++u) {
            const int32_t x = ws.e_slot[u];
            int v = u - 1;
            while (v >= lo && ws.e_slot[v] > x) { ws.e_slot[v + 1] = ws.e_slot[v]; --v; }
            ws.e_slot[v + 1] = x;
        }
        a.e_idx[ws.e_node[tid]] = tid;
    }
    if (tid == 0) { ws.nb = nb; ws.e_cnt = e_cnt; ws.n_e = n_e; ws.nslot = 0; }
}

// ---------------------------------------------------------------------------------------------
// Candidate slots.  Every distinct node in the batch's candidate lists gets one slot (the first
// workgroup to meet it claims it through node_slot) and its record at the batch start: ac am ag ap
// rc rm rg nr as int32 (ap clamped), taint, label — 12 dwords; the wide mode the ten int64 fields
// (20 dwords).  The resolver stages all slots in LDS, so a pod's winner is one LDS read away.
// ---------------------------------------------------------------------------------------------
template <int kMode> struct Fmt {
    static constexpr int kDw = 12;
    static constexpr int kCap = kSlotMax;  // slots the resolver stages
};
template <> struct Fmt<kEvalWide> {
    static constexpr int kDw = 20;
    static constexpr int kCap = 896;
};
static_assert(Fmt<kEvalWide>::kDw <= kRecDw && Fmt<kEvalWide>::kCap <= kSlotMax, "record size");
constexpr int kSlotsAll = kWinMaxB * kChR;  // claims a batch can make (slot_node holds every one)
constexpr int kSlotPending = -2;
static_assert(kSlotsAll <= 65535, "slot ids in 16 bits");

template <int kMode>
__device__ __forceinline__ void put_rec(uint32_t* o, const NodeV& v) {
    if constexpr (kMode == kEvalWide) {
        const int64_t f[10] = {v.ac, v.am, v.ag, v.ap, v.rc, v.rm, v.rg, v.nr, (int64_t)v.taint, (int64_t)v.label};
#pragma unroll
        for (int k = 0; k < 10; ++k) { o[2 * k] = (uint32_t)f[k]; o[2 * k + 1] = (uint32_t)((uint64_t)f[k] >> 32); }
    } else {
        o[0] = (uint32_t)(int32_t)v.ac; o[1] = (uint32_t)(int32_t)v.am; o[2] = (uint32_t)(int32_t)v.ag;
        o[3] = (uint32_t)clamp32(v.ap);
        o[4] = (uint32_t)(int32_t)v.rc; o[5] = (uint32_t)(int32_t)v.rm; o[6] = (uint32_t)(int32_t)v.rg;
        o[7] = (uint32_t)(int32_t)v.nr;
        o[8] = (uint32_t)v.taint; o[9] = (uint32_t)(v.taint >> 32); o[10] = (uint32_t)v.label; o[11] = (uint32_t)(v.label >> 32);
    }
}

// Pod i's static candidates from its merged top-L `cand` (LDS or global), by one workgroup: the
// kept entries (sorted, <= kR) with their slots
template <int kMode>
__device__ __forceinline__ void cand_list(const EngineArgs& a, WinWS& ws, int i, const uint64_t* cand) {
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int64_t start = a.ctr[kCtrStart];
    __shared__ uint64_t buf[kClBuf];
    __shared__ int cnt;
    if (tid == 0) cnt = 0;
    __syncthreads();
    const PodRec p = a.pods[start + i];
    const uint64_t last = cand[kL - 1];
    const bool full = last != 0;
    const uint64_t thr = full ? last : 1ull;
    const int hi = ws.win_hi[i], n_e = ws.n_e;
    for (int k = tid; k < n_e; k += nthr) {
        const int32_t n = ws.e_node[k];
        NodeV v = load_node(a.s, n);
        for (int u = ws.e_off[k], ue = ws.e_off[k + 1]; u < ue; ++u) {
            const int x = ws.e_slot[u];
            if (x >= hi) break;  // ascending
            v.rc -= ws.ex_req[x][0]; v.rm -= ws.ex_req[x][1]; v.rg -= ws.ex_req[x][2]; v.nr -= 1;
        }
        const uint64_t key = make_key(eval_t<kMode>(a.c, p, v), (uint32_t)n);
        if (key >= thr) {
            const int pos = atomicAdd(&cnt, 1);
            if (pos < kClBuf) buf[pos] = key;
        }
    }
    if (tid < kL) {
        const uint64_t x = cand[tid];
        if (x != 0 && a.e_idx[key_node(x)] < 0) {
            const int pos = atomicAdd(&cnt, 1);
            if (pos < kClBuf) buf[pos] = x;
        }
    }
    __syncthreads();
    const int c = cnt, n = c < kClBuf ? c : kClBuf;
    __shared__ uint64_t kept[kR];
    if (tid < n) {  // rank by counting (keys are distinct: the node is in the low bits)
        const uint64_t me = buf[tid];
        int r = 0;
        for (int u = 0; u < n; ++u) r += buf[u] > me;
        if (r < kR) kept[r] = me;
    }
    __syncthreads();
    if (tid < kWave) {  // the kept entries' slots: one wave, one counter update for its claims
        const int lane = tid;
        const bool valid = lane < (n < kR ? n : kR);
        const uint64_t me = valid ? kept[lane] : 0ull;
        const int32_t nd = key_node(me);
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
            if (sl < Fmt<kMode>::kCap) {
                put_rec<kMode>(ws.slot_rec[sl], load_node(a.s, nd));
                ws.slot_eix[sl] = a.e_idx[nd];
            }
            atomicExch(&a.n_slot[nd], sl);
        }
        if (valid) {
            ws.cl_key[i][lane] = me;
            ws.cl_slot[i][lane] = sl;  // kSlotPending: read node_slot in the resolver
        }
    }
    if (tid == 0) {
        ws.cl_info[i] = (c < kR ? c : kR) | (c > kR ? kClTrunc : 0) | (full ? kClFull : 0) | (c > kClBuf ? kClOvf : 0);
        ws.cl_thr[i] = thr;
    }
}

template <int kMode>
__global__ __launch_bounds__(256) void seq_cl_kernel(const EngineArgs* __restrict__ A) {
    const EngineArgs& a = A[0];
    WinWS& ws = *a.sw;
    const int i = blockIdx.x;
    if (i >= ws.nb) return;
    cand_list<kMode>(a, ws, i, a.cand + (int64_t)i * kL);
}

// merge + candidate list of pod b in one workgroup (the merge kernel's exact top-L over nl sorted
// lists lists[b * pod_stride + k * list_stride], ks_kernels.hip, then cand_list) — one launch
// fewer per batch.  src == nullptr: the engine's own block lists.
constexpr int kMergeMaxWaves = 16;
template <int kMode>
__global__ __launch_bounds__(1024) void merge_cl_kernel(const EngineArgs* __restrict__ A, const uint64_t* src,
                                                         int64_t pod_stride, int32_t nl, int64_t list_stride) {
    const EngineArgs& a = A[0];
    WinWS& ws = *a.sw;
    if (src == nullptr) {
        src = a.lists;
        pod_stride = (int64_t)a.nblk * kL;
        nl = a.nblk;
        list_stride = kL;
    }
    const int b = blockIdx.x;
    if (b >= ws.nb) return;  // (the window prep cut the batch; errors left nb = 0)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t top[kL];
#pragma unroll
    for (int k = 0; k < kL; ++k) top[k] = 0;
    const uint64_t* lists = src + (int64_t)b * pod_stride;
    const int nthr = blockDim.x, nwav = nthr / kWave;
    for (int blk = tid; blk < nl; blk += nthr) {
        const ulonglong2* lp = reinterpret_cast<const ulonglong2*>(lists + (int64_t)blk * list_stride);
        uint64_t lv[kL];
#pragma unroll
        for (int k = 0; k < kL / 2; ++k) {
            const ulonglong2 w = lp[k];
            lv[2 * k] = w.x;
            lv[2 * k + 1] = w.y;
        }
        topl_insert(top, lv);
    }
    __shared__ uint64_t wl[kMergeMaxWaves][kL];
    __shared__ uint64_t pc[kL];
    int head = 0;
    for (int r = 0; r < kL; ++r) {
        uint64_t h = 0;
#pragma unroll
        for (int k = 0; k < kL; ++k) h = (k == head) ? top[k] : h;
        const uint64_t m = wave_max_u64(h);
        const uint64_t hit = __ballot(h == m && m != 0);
        if (lane == 0) wl[wave][r] = m;
        if (hit && lane == __ffsll((unsigned long long)hit) - 1) head++;
    }
    __syncthreads();
    if (wave == 0) {
        const int nc = nwav * kL;
        uint64_t v0 = lane < nc ? wl[lane / kL][lane % kL] : 0ull;
        uint64_t v1 = lane + kWave < nc ? wl[(lane + kWave) / kL][(lane + kWave) % kL] : 0ull;
#pragma unroll
        for (int r = 0; r < kL; ++r) {
            const uint64_t m = wave_max_u64(v0 > v1 ? v0 : v1);
            if (lane == 0) pc[r] = m;
            if (m == 0) continue;
            const uint64_t h0 = __ballot(v0 == m), h1 = __ballot(v1 == m);
            if (h0 && lane == __ffsll((unsigned long long)h0) - 1) v0 = 0;
            if (!h0 && h1 && lane == __ffsll((unsigned long long)h1) - 1) v1 = 0;
        }
    }
    __syncthreads();
    cand_list<kMode>(a, ws, b, pc);
}

// ---------------------------------------------------------------------------------------------
// Entries: the nodes bound in this batch, state in registers.  Every entry type carries the two
// reciprocals of its capacities (node invariants); the micro type also the product the micro
// evaluator reuses (ks_device.h micro_ic / micro_im / micro_d, found by overload).
// ---------------------------------------------------------------------------------------------
struct E32 {
    int32_t ac, am, ag, ap, rc, rm, rg, nr;
    uint64_t taint, label;
    float ic, im;  // 1 / max(A, 1)
};
struct EM : E32 {
    int32_t d;
};
struct EW : NodeV {
    float ic, im;
};
__device__ __forceinline__ float micro_ic(const EM& n, int32_t) { return n.ic; }
__device__ __forceinline__ float micro_im(const EM& n, int32_t) { return n.im; }
__device__ __forceinline__ int32_t micro_d(const EM& n, int32_t, int32_t) { return n.d; }

template <int kMode> struct EntSel { using T = E32; };
template <> struct EntSel<kEvalMicro> { using T = EM; };
template <> struct EntSel<kEvalWide> { using T = EW; };

__device__ __forceinline__ void from_rec(const uint32_t* w, E32& o) {
    o.ac = (int32_t)w[0]; o.am = (int32_t)w[1]; o.ag = (int32_t)w[2]; o.ap = (int32_t)w[3];
    o.rc = (int32_t)w[4]; o.rm = (int32_t)w[5]; o.rg = (int32_t)w[6]; o.nr = (int32_t)w[7];
    o.taint = w[8] | ((uint64_t)w[9] << 32); o.label = w[10] | ((uint64_t)w[11] << 32);
    o.ic = rcp_est((float)(o.ac > 0 ? o.ac : 1));
    o.im = rcp_est((float)(o.am > 0 ? o.am : 1));
}
__device__ __forceinline__ void from_rec(const uint32_t* w, EM& o) {
    from_rec(w, static_cast<E32&>(o));
    o.d = mul24(o.ac > 0 ? o.ac : 1, o.am > 0 ? o.am : 1);
}
__device__ __forceinline__ void from_rec(const uint32_t* w, EW& o) {
    auto f = [&](int k) { return (int64_t)(w[2 * k] | ((uint64_t)w[2 * k + 1] << 32)); };
    o.ac = f(0); o.am = f(1); o.ag = f(2); o.ap = f(3); o.rc = f(4); o.rm = f(5); o.rg = f(6); o.nr = f(7);
    o.taint = (uint64_t)f(8); o.label = (uint64_t)f(9);
    o.ic = rcp_est((float)(o.ac > 0 ? o.ac : 1));
    o.im = rcp_est((float)(o.am > 0 ? o.am : 1));
}

// CreatePod admission (kubesim/node/node.go:44-47) in 64-bit whatever the entry type
template <class NS>
__device__ __forceinline__ bool admits(const PodRec& p, const NS& n) {
    bool ok = (int64_t)n.nr < (int64_t)n.ap;
    if (p.keymask & 1) ok &= (int64_t)n.rc + p.req[0] <= (int64_t)n.ac;
    if (p.keymask & 2) ok &= (int64_t)n.rm + p.req[1] <= (int64_t)n.am;
    if (p.keymask & 4) ok &= (int64_t)n.rg + p.req[2] <= (int64_t)n.ag;
    return ok;
}

// prune_tmax's per-entry state from the cached reciprocals (the values prune_prep computes)
template <class NS>
__device__ __forceinline__ PruneF prune_of(const Cfg& c, const NS& n) {
    PruneF f;
    f.ic = n.ac > 0 ? n.ic : 0.f;
    f.bc = n.ac > 0 ? (float)(n.ac - n.rc) * n.ic : -1.f;
    f.im = n.am > 0 ? n.im : 0.f;
    f.bm = n.am > 0 ? (float)(n.am - n.rm) * n.im : -1.f;
    f.live = c.has_scorers && !(c.filter_feeds && (c.filters & kFilterFit) && n.nr >= n.ap);
    return f;
}

// Internal key: (total + 1) << 34 | (2^24 - 1 - node) << 10 | entry — orders exactly like the
// packed key (node < 2^24, total + 1 < 2^30: ks_engine.cpp) and carries the entry.
__device__ __forceinline__ uint64_t ikey(uint64_t key, int ent) {
    const uint32_t node = 0xFFFFFFFFu - (uint32_t)key;
    return ((key >> 32) << 34) | ((uint64_t)(0xFFFFFFu - node) << 10) | (uint64_t)(uint32_t)ent;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
// wave-uniform copies of values read from LDS (every lane read the same address): scalar registers,
// so the loop's control flow and the evaluator's pod operands stay uniform
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int32_t rfl(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl(uint64_t v) { return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v); }
__device__ __forceinline__ PodRec rfl(const PodRec& p) {
    PodRec q;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&p);
    uint32_t* d = reinterpret_cast<uint32_t*>(&q);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(PodRec) / 4); ++k) d[k] = rfl(s[k]);
    return q;
}
__device__ __forceinline__ int4 rfl(const int4& v) { return make_int4(rfl(v.x), rfl(v.y), rfl(v.z), rfl(v.w)); }

// per-pod control: x own slot (-1 none), y win_hi, z flags (kRun | cl_info bits), w kept count
constexpr int32_t kRun = 1;
constexpr uint32_t kNoSlot = 0xFFFFu;  // an entry whose node got no staged slot (overflow)

template <int kMode>
struct Shared {
    using NS = typename EntSel<kMode>::T;
    using Q = decltype(NS{}.rc);
    static constexpr int kCap = Fmt<kMode>::kCap, kDw = Fmt<kMode>::kDw;
    PodRec pod[kB + 2];
    int4 px[kB + 2];
    uint64_t thr[kB + 2];
    uint32_t ent[kB + 1][kR];   // pod i's candidate r: slot << 16 | total + 1 (0: none)
    uint32_t rec[kCap][kDw];    // slot records
    int32_t snode[kCap];
    int16_t seix[kCap];
    uint8_t bnd[kCap];          // the slot's node is bound in this batch (an entry)
    int32_t bnode[kB];
    int8_t bstat[kB];
    int8_t brun[kB];            // bound Ok with a positive run: its own expiry counts
    int16_t xeff[kWinSlots];    // slot x is applied from pod xeff[x] on
    int16_t exk[kWinSlots];     // E index of a pre-batch Ok slot, -1 otherwise
    int32_t ex_q[kWinSlots];
    Q ex_req[kWinSlots][3];
    int32_t e_node[kWinSlots];
    int16_t e_off[kWinSlots + 1], e_slot[kWinSlots];
    int16_t ek_ent[kWinSlots];  // E node k's entry, -1 none
    int32_t pend[kB][kPend];    // pending own expiries of entry e: xeff << 16 | pod, -1 empty
    int32_t rbp[kB];            // rollback: the pod whose expiries the slow path applied last ...
    Q rb[kB][4];                // ... and the entry's rc rm rg nr before them
};

template <int kMode, class NS>
__device__ __forceinline__ void sub_req(NS& n, const typename Shared<kMode>::Q* r) {
    n.rc -= r[0]; n.rm -= r[1]; n.rg -= r[2]; n.nr -= 1;
}

// The next effective pod of entry e's pending expiries: its E cursor's slot, its own pending
template <int kMode>
__device__ __forceinline__ int next_eff(const Shared<kMode>& sh, int e, int ecur, int eend) {
    int nx = ecur < eend ? sh.xeff[sh.e_slot[ecur]] : INT_MAX;
#pragma unroll
    for (int q = 0; q < kPend; ++q) {
        const int32_t w = sh.pend[e][q];
        if (w >= 0) nx = min(nx, w >> 16);
    }
    return nx;
}

#ifdef KS_SEQ_DIAG  // counters in ctr[5..15], phase cycles in ctr[16..23] (tests/dev/ab_resolvers.py)
#define SQ_DIAG(...) __VA_ARGS__
__device__ __forceinline__ uint64_t sq_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#else
#define SQ_DIAG(...)
#endif

template <int kMode>
__global__ __launch_bounds__(kThreads) void resolve_seq_kernel(const EngineArgs* __restrict__ A) {
    using NS = typename EntSel<kMode>::T;
    using SH = Shared<kMode>;
    constexpr int kCap = SH::kCap, kDw = SH::kDw;
    __shared__ SH sh;
    const EngineArgs& a = A[0];
    const WinWS& ws = *a.sw;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    const int nb = ws.nb;
    if (a.ctr[kCtrErr] != 0 || nb <= 0) return;
    const int n_e = ws.n_e, e_cnt = ws.e_cnt;
    const int nslot = ws.nslot < kSlotsAll ? ws.nslot : kSlotsAll;
    const int nstage = nslot < kCap ? nslot : kCap;

    SQ_DIAG(const uint64_t t_setup = sq_stamp();)
    // ---- setup (4 waves): pods, per-pod control, candidate entries, slot records, the window
    for (int i = tid; i < kB + 2; i += kThreads) {
        if (i < nb) {
            sh.pod[i] = a.pods[start + i];
            const int info = ws.cl_info[i];
            sh.px[i] = make_int4(ws.own[i], ws.win_hi[i], (a.dur[start + i] > 0 ? kRun : 0) | (info & ~0xFF), info & 0xFF);
            sh.thr[i] = ws.cl_thr[i];
        } else {
            sh.pod[i] = PodRec{};
            sh.px[i] = make_int4(-1, 0, 0, 0);
            sh.thr[i] = 0;
        }
    }
    for (int k = tid; k < (nb + 1) * kR; k += kThreads) {
        const int i = k / kR, r = k % kR;
        uint32_t v = 0;
        if (i < nb && r < (ws.cl_info[i] & 0xFF)) {
            const uint64_t key = ws.cl_key[i][r];
            int sl = ws.cl_slot[i][r];
            if (sl == kSlotPending) sl = a.n_slot[key_node(key)];  // published by the claimer
            v = ((sl >= 0 && sl < kCap) ? (uint32_t)sl : kNoSlot) << 16 | (uint32_t)(key >> 32);
        }
        sh.ent[i][r] = v;
    }
    for (int k = tid; k < nstage * kDw; k += kThreads) sh.rec[k / kDw][k % kDw] = ws.slot_rec[k / kDw][k % kDw];
    for (int k = tid; k < nstage; k += kThreads) {
        sh.snode[k] = ws.slot_node[k];
        sh.seix[k] = (int16_t)ws.slot_eix[k];
        sh.bnd[k] = 0;
    }
    for (int x = tid; x < e_cnt; x += kThreads) {
        sh.ex_q[x] = ws.ex_q[x];
        sh.exk[x] = -1;
#pragma unroll
        for (int k = 0; k < 3; ++k) sh.ex_req[x][k] = (typename SH::Q)(kMode == kEvalWide ? ws.ex_req[x][k] : clamp32(ws.ex_req[x][k]));
    }
    for (int i = tid + 1; i < nb; i += kThreads)  // slot x is applied from the first pod i >= 1 with win_hi[i] > x
        for (int x = ws.win_hi[i - 1]; x < ws.win_hi[i]; ++x) sh.xeff[x] = (int16_t)i;
    for (int k = tid; k <= n_e; k += kThreads) {
        sh.e_off[k] = (int16_t)ws.e_off[k];
        if (k < n_e) { sh.e_node[k] = ws.e_node[k]; sh.ek_ent[k] = -1; }
    }
    for (int u = tid; u < e_cnt; u += kThreads) sh.e_slot[u] = (int16_t)ws.e_slot[u];
    for (int e = tid; e < kB; e += kThreads) {
        sh.rbp[e] = -1;
#pragma unroll
        for (int q = 0; q < kPend; ++q) sh.pend[e][q] = -1;
    }
    __syncthreads();
    for (int k = tid; k < n_e; k += kThreads)
        for (int u = sh.e_off[k]; u < sh.e_off[k + 1]; ++u) sh.exk[sh.e_slot[u]] = (int16_t)k;
    __syncthreads();
    if (wave != 0) {  // the other waves reset the node -> slot map and leave
        for (int k = tid - kWave; k < nslot; k += kThreads - kWave) a.n_slot[ws.slot_node[k]] = -1;
        return;
    }

    // ---- the FIFO loop: wave 0 alone, no barrier, no global memory access
    NS st[kES];
    int32_t nd[kES];
    PruneF pf[kES];
    int nx[kES], ecu[kES], esl[kES];
#pragma unroll
    for (int s = 0; s < kES; ++s) { st[s] = NS{}; nd[s] = 0; pf[s] = PruneF{}; nx[s] = INT_MAX; ecu[s] = 0; esl[s] = 0; }
    int T = 0;  // entries (uniform)
    // pod i's candidates, lane r = entry r: entry word, node, bound (as of the fetch: before pod
    // i - 1's bind, which (A) patches)
    auto fetch = [&](int p, uint32_t& ce, int32_t& cn, bool& cb) {
        ce = lane < kR ? sh.ent[p][lane] : 0u;
        const uint32_t sl = ce >> 16;
        const bool ok = ce != 0 && sl < (uint32_t)kCap;
        cn = ok ? sh.snode[sl] : -1;
        cb = ok && sh.bnd[sl];
    };
    uint32_t ce;
    int32_t cn;
    bool cb;
    fetch(0, ce, cn, cb);
    PodRec P = rfl(sh.pod[0]);
    int4 X = rfl(sh.px[0]);
    uint64_t thr = rfl(sh.thr[0]);
    uint32_t wslot = kNoSlot;  // the previous pod's winner's slot
    int pstop = INT_MAX;       // a pending-expiry overflow at pod j stops the batch before pod j + 1
    int i = 0, code = 0;
    SQ_DIAG(int64_t n_dwin = 0, n_eval = 0, n_slow = 0, n_sdepth = 0; uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            uint64_t t_loop = sq_stamp(); ph[7] = t_loop - t_setup;)
    for (; i < nb; ++i) {
        SQ_DIAG(uint64_t q0 = sq_stamp();)
        // (A) S_i: the first static candidate no earlier pod bound
        const int cnt = X.w;
        const uint32_t fl = (uint32_t)X.z;
        const uint32_t csl = ce >> 16;
        const uint64_t ckey = ce ? (((uint64_t)(ce & 0xFFFFu) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)cn)) : 0ull;
        const uint64_t um = __ballot(lane < cnt && ce != 0 && !cb && csl != wslot);
        const int jpos = um ? __ffsll((unsigned long long)um) - 1 : -1;
        const uint64_t skey = jpos >= 0 ? readlane64(ckey, jpos) : 0ull;
        const uint32_t ssl = jpos >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)csl, jpos) : kNoSlot;
        const uint64_t lbk = jpos >= 0 ? skey : (fl & kClTrunc) ? readlane64(ckey, kR - 1) : (fl & kClFull) ? thr : 0ull;
        SQ_DIAG(n_sdepth += jpos; uint64_t q1 = sq_stamp(); ph[0] += q1 - q0;)
        // (B) the next pod's candidates, pod record and control; S_i's record
        uint32_t ce1;
        int32_t cn1;
        bool cb1;
        fetch(i + 1, ce1, cn1, cb1);
        const PodRec Pn = sh.pod[i + 1];
        const int4 Xn = sh.px[i + 1];
        const uint64_t thrn = sh.thr[i + 1];
        const bool srec = ssl < (uint32_t)kCap;
        uint32_t w[kDw];
#pragma unroll
        for (int d = 0; d < kDw; ++d) w[d] = srec ? sh.rec[ssl][d] : 0u;
        const int eix = srec ? sh.seix[ssl] : -1;
        SQ_DIAG(uint64_t q2 = sq_stamp(); ph[1] += q2 - q1;)
        // (C) expiries due at pod i on the entries (rare: the slow path)
        bool due = false;
#pragma unroll
        for (int s = 0; s < kES; ++s) due |= (s * kWave + lane < T) && nx[s] <= i;
        if (__ballot(due)) {
            SQ_DIAG(++n_slow;)
#pragma unroll
            for (int s = 0; s < kES; ++s) {
                const int e = s * kWave + lane;
                if (e < T && nx[s] <= i) {
                    sh.rbp[e] = i;
                    sh.rb[e][0] = st[s].rc; sh.rb[e][1] = st[s].rm; sh.rb[e][2] = st[s].rg; sh.rb[e][3] = st[s].nr;
                    const int eend = ecu[s] >> 16;
                    int ec = ecu[s] & 0xFFFF;
                    while (ec < eend && sh.xeff[sh.e_slot[ec]] <= i) { sub_req<kMode>(st[s], sh.ex_req[sh.e_slot[ec]]); ++ec; }
                    ecu[s] = ec | (eend << 16);
#pragma unroll
                    for (int q = 0; q < kPend; ++q) {
                        const int32_t pw = sh.pend[e][q];
                        if (pw >= 0 && (pw >> 16) <= i) {
                            const PodRec& pj = sh.pod[pw & 0xFFFF];
                            st[s].rc -= (decltype(st[s].rc))pj.req[0]; st[s].rm -= (decltype(st[s].rm))pj.req[1];
                            st[s].rg -= (decltype(st[s].rg))pj.req[2]; st[s].nr -= 1;
                            sh.pend[e][q] = -1;
                        }
                    }
                    nx[s] = next_eff<kMode>(sh, e, ec, eend);
                    pf[s] = prune_of(a.c, st[s]);
                }
            }
        }
        SQ_DIAG(uint64_t q3 = sq_stamp(); ph[2] += q3 - q2;)
        // (D) D_i: the entries whose upper bound reaches past lbk, evaluated exactly
        uint64_t bk = 0;
        {
            const float qfc = (float)P.req[0], qfm = (float)P.req[1];
#pragma unroll
            for (int s = 0; s < kES; ++s) {
                if (T > s * kWave) {
                    const int e = s * kWave + lane;
                    const bool want = e < T && pf[s].live != 0 &&
                                      make_key(prune_tmax(a.c, pf[s], qfc, qfm) + 1u, (uint32_t)nd[s]) > lbk;
                    if (__ballot(want)) {
                        SQ_DIAG(++n_eval;)
                        const uint64_t k = make_key(eval_t<kMode>(a.c, P, st[s]), (uint32_t)nd[s]);
                        if (want && k > lbk) { const uint64_t ik = ikey(k, e); bk = ik > bk ? ik : bk; }
                    }
                }
            }
        }
        const bool dh = __ballot(bk != 0) != 0;
        const uint64_t dk = dh ? wave_max_u64(bk) : 0ull;
        SQ_DIAG(uint64_t q4 = sq_stamp(); ph[3] += q4 - q3;)
        // (E) decision (the order of the other resolvers' stops: exhausted list / overflow, then
        // NotFound, then a bad pod key or simSpec)
        bool dwin = false;
        if (i >= pstop || (fl & kClOvf)) code = 1;
        else if (jpos >= 0) { dwin = dh; if (!dh && !srec) code = 1; }  // (S_i's node has no staged slot)
        else if (fl & (kClTrunc | kClFull)) { if (dh) dwin = true; else code = 1; }
        else if (dh) dwin = true;
        else code = 2;  // no static candidate, no entry: NotFound
        if (code == 0 && (P.flags & (kFlagBadKey | kFlagBadSpec))) code = 3;
        if (code != 0) break;
        SQ_DIAG(n_dwin += dwin; uint64_t q5 = sq_stamp(); ph[4] += q5 - q4;)
        // (F) bind pod i (CreatePod admission) on the winner's entry — a new one for S_i
        const int e = dwin ? (int)(dk & 1023u) : T;
        const int32_t wnode = dwin ? (int32_t)(0xFFFFFFu - (uint32_t)((dk >> 10) & 0xFFFFFFu)) : key_node(skey);
        const int ol = e & (kWave - 1), os = e / kWave;
        const bool run = (X.z & kRun) != 0;
        const int own = X.x;
        bool okb = false;
        int wsl = 0;
        if (!dwin) {
            T += 1;
            wsl = (int)ssl;
#pragma unroll
            for (int s = 0; s < kES; ++s) {
                if (os == s && lane == ol) {
                    NS n;
                    from_rec(w, n);
                    int ec = 0, eend = 0;
                    if (eix >= 0) {  // an E node: the pre-batch expiries due by pod i
                        ec = sh.e_off[eix];
                        eend = sh.e_off[eix + 1];
                        while (ec < eend && sh.xeff[sh.e_slot[ec]] <= i) { sub_req<kMode>(n, sh.ex_req[sh.e_slot[ec]]); ++ec; }
                        sh.ek_ent[eix] = (int16_t)e;
                    }
                    okb = admits(P, n);
                    if (okb && run) {
                        n.rc += (decltype(n.rc))P.req[0]; n.rm += (decltype(n.rm))P.req[1];
                        n.rg += (decltype(n.rg))P.req[2]; n.nr += 1;
                    }
                    st[s] = n;
                    nd[s] = wnode;
                    esl[s] = wsl;
                    ecu[s] = ec | (eend << 16);
                    if (okb && run && own >= 0) sh.pend[e][0] = ((int32_t)sh.xeff[own] << 16) | i;
                    nx[s] = next_eff<kMode>(sh, e, ec, eend);
                    pf[s] = prune_of(a.c, n);
                    sh.bnd[ssl] = 1;
                }
            }
        } else {
#pragma unroll
            for (int s = 0; s < kES; ++s) {
                if (os == s) {
                    wsl = __builtin_amdgcn_readlane(esl[s], ol);
                    if (lane == ol) {
                        NS n = st[s];
                        okb = admits(P, n);
                        if (okb && run) {
                            n.rc += (decltype(n.rc))P.req[0]; n.rm += (decltype(n.rm))P.req[1];
                            n.rg += (decltype(n.rg))P.req[2]; n.nr += 1;
                            if (own >= 0) {
                                int q = 0;
                                while (q < kPend && sh.pend[e][q] >= 0) ++q;
                                if (q < kPend) sh.pend[e][q] = ((int32_t)sh.xeff[own] << 16) | i;
                                else pstop = i + 1;  // untracked: the state is unknown from pod i + 1 on
                            }
                        }
                        st[s] = n;
                        nx[s] = next_eff<kMode>(sh, e, ecu[s] & 0xFFFF, ecu[s] >> 16);
                        pf[s] = prune_of(a.c, n);
                    }
                }
            }
        }
        okb = __ballot(okb) != 0;
        pstop = __builtin_amdgcn_readlane(pstop, ol);
        if (lane == 0) {
            sh.bnode[i] = wnode;
            sh.bstat[i] = okb ? 0 : 1;
            sh.brun[i] = (okb && run) ? 1 : 0;
        }
        wslot = (uint32_t)wsl;
        SQ_DIAG(uint64_t q6 = sq_stamp(); ph[5] += q6 - q5;)
        ce = ce1; cn = cn1; cb = cb1;
        P = rfl(Pn); X = rfl(Xn); thr = rfl(thrn);
        SQ_DIAG(ph[6] += sq_stamp() - q6;)
    }
    const int c = i;  // committed pods

    // ---- commit (wave 0): a stop at pod c undoes the expiries applied for it
    if (c < nb) {
#pragma unroll
        for (int s = 0; s < kES; ++s) {
            const int e = s * kWave + lane;
            if (e < T && sh.rbp[e] == c) {
                st[s].rc = sh.rb[e][0]; st[s].rm = sh.rb[e][1]; st[s].rg = sh.rb[e][2]; st[s].nr = sh.rb[e][3];
            }
        }
    }
    const int h_end = c >= 1 ? sh.px[c - 1].y : 0;  // slots applied: < win_hi[c - 1]
#pragma unroll
    for (int s = 0; s < kES; ++s) {
        const int e = s * kWave + lane;
        if (e < T) {
            const int64_t n = nd[s];
            gptr(a.s.rc)[n] = (int64_t)st[s].rc; gptr(a.s.rm)[n] = (int64_t)st[s].rm;
            gptr(a.s.rg)[n] = (int64_t)st[s].rg; gptr(a.s.nr)[n] = (int64_t)st[s].nr;
        }
    }
    for (int j = lane; j < c; j += kWave) {
        gptr(a.b_node)[start + j] = sh.bnode[j];
        gptr(a.b_status)[start + j] = sh.bstat[j];
        const int x = sh.px[j].x;
        if (sh.brun[j] && x >= 0 && x < h_end) gptr(a.expired)[start + j] = 1;
    }
    for (int x = lane; x < h_end; x += kWave) {
        const int k = sh.exk[x];
        if (k < 0) continue;  // (in-batch pods: above)
        gptr(a.expired)[sh.ex_q[x]] = 1;
        if (sh.ek_ent[k] < 0) {  // an E node no pod of the batch bound: its expiries here
            const int32_t n = sh.e_node[k];
            atomicAdd((unsigned long long*)&a.s.rc[n], (unsigned long long)(-ws.ex_req[x][0]));
            atomicAdd((unsigned long long*)&a.s.rm[n], (unsigned long long)(-ws.ex_req[x][1]));
            atomicAdd((unsigned long long*)&a.s.rg[n], (unsigned long long)(-ws.ex_req[x][2]));
            atomicAdd((unsigned long long*)&a.s.nr[n], (unsigned long long)(-1ll));
        }
    }
    for (int k = lane; k < n_e; k += kWave) a.e_idx[sh.e_node[k]] = -1;
    if (lane == 0) {
        a.ctr[kCtrStart] = start + c;
        const bool err = code == 2 || code == 3;
        if (err) {
            a.ctr[kCtrErr] = code == 2 ? kErrNotFound : kErrEinval;
            a.ctr[kCtrErrPod] = start + c;
        }
        if (c < a.B && !err && start + c < end) a.ctr[kCtrEarly] += 1;
#ifdef KS_SEQ_DIAG
        unsigned long long* dg = (unsigned long long*)a.ctr;
        atomicAdd(&dg[5], 1ull);
        atomicAdd(&dg[6], (unsigned long long)c);
        atomicAdd(&dg[7], (unsigned long long)n_dwin);
        atomicAdd(&dg[8], (unsigned long long)n_eval);
        atomicAdd(&dg[9], (unsigned long long)n_slow);
        atomicAdd(&dg[10], (unsigned long long)nslot);
        atomicAdd(&dg[11], (unsigned long long)n_sdepth);
        atomicAdd(&dg[12], (unsigned long long)T);
        atomicAdd(&dg[13 + (code < 2 ? code : 2)], 1ull);
        for (int q = 0; q < 8; ++q) atomicAdd(&dg[16 + q], ph[q]);
#endif
    }
}

}  // namespace sq

hipError_t launch_window_prep(const EngineArgs* d, bool head, hipStream_t st) {
    hipLaunchKernelGGL(sq::window_prep_kernel, dim3(1), dim3(sq::kPrepThreads), 0, st, d, head ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_merge_cl(const EngineArgs* d, int mode, int B, const uint64_t* lists, int64_t pod_stride,
                           int32_t nl, int64_t list_stride, int nl_max, hipStream_t st) {
    const dim3 g(B), t(nl_max > 1024 ? 1024 : 256);
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL(sq::merge_cl_kernel<kEvalMicro>, g, t, 0, st, d, lists, pod_stride, nl, list_stride); break;
        case kEvalTiny: hipLaunchKernelGGL(sq::merge_cl_kernel<kEvalTiny>, g, t, 0, st, d, lists, pod_stride, nl, list_stride); break;
        case kEvalNarrow: hipLaunchKernelGGL(sq::merge_cl_kernel<kEvalNarrow>, g, t, 0, st, d, lists, pod_stride, nl, list_stride); break;
        default: hipLaunchKernelGGL(sq::merge_cl_kernel<kEvalWide>, g, t, 0, st, d, lists, pod_stride, nl, list_stride); break;
    }
    return hipGetLastError();
}

hipError_t launch_seq_only(const EngineArgs* d, int mode, hipStream_t st) {
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL(sq::resolve_seq_kernel<kEvalMicro>, dim3(1), dim3(sq::kThreads), 0, st, d); break;
        case kEvalTiny: hipLaunchKernelGGL(sq::resolve_seq_kernel<kEvalTiny>, dim3(1), dim3(sq::kThreads), 0, st, d); break;
        case kEvalNarrow: hipLaunchKernelGGL(sq::resolve_seq_kernel<kEvalNarrow>, dim3(1), dim3(sq::kThreads), 0, st, d); break;
        default: hipLaunchKernelGGL(sq::resolve_seq_kernel<kEvalWide>, dim3(1), dim3(sq::kThreads), 0, st, d); break;
    }
    return hipGetLastError();
}

template <int kMode>
static void launch_seq_t(const EngineArgs* d, hipStream_t st) {
    hipLaunchKernelGGL(sq::seq_cl_kernel<kMode>, dim3(kWinMaxB), dim3(256), 0, st, d);
    hipLaunchKernelGGL(sq::resolve_seq_kernel<kMode>, dim3(1), dim3(sq::kThreads), 0, st, d);
}

hipError_t launch_resolve_seq(const EngineArgs* d, int mode, hipStream_t st) {
    hipError_t r = launch_window_prep(d, false, st);
    if (r != hipSuccess) return r;
    switch (mode) {
        case kEvalMicro: launch_seq_t<kEvalMicro>(d, st); break;
        case kEvalTiny: launch_seq_t<kEvalTiny>(d, st); break;
        case kEvalNarrow: launch_seq_t<kEvalNarrow>(d, st); break;
        default: launch_seq_t<kEvalWide>(d, st); break;
    }
    return hipGetLastError();
}

}  // namespace ks
