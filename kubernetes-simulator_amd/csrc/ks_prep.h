// ks_prep.h — a batch's expiry window (gfx950): the body of ks_cand.hip's window_prep_kernel, shared
// with the chunk kernel, whose resolver workgroup runs it for the next batch right after its commit
// (ks_chunk.hip chunk_scan_kernel: one launch and one kernel boundary fewer per overlapped batch).
//
// The reference binds one pod per tick in FIFO order (kubesim/kubesim.go:105-121); before pod j is
// scheduled, every pod whose run ended by its tick stops counting toward its node's totals
// (kubesim/node/node.go:97-118 over kubesim/pod/pod.go:67-69).  Per batch this computes:
//   * head: the expiries due before the batch's first pod, applied to the node state;
//   * the window: the expiries attached to pods start+1 .. start+nb-1 (exp_off CSR), one slot each;
//     the batch shrinks to the largest prefix whose window fits kWinSlots;
//   * E: the distinct nodes of the window's slots whose pod was bound Ok before the batch and has
//     not expired (e_idx marks them), and — `spec`, the overlap — the nodes the previous batch
//     changed (its commit's `touched`) and the head expiries' nodes, with no slots: the batch's
//     block lists come from the speculative scan that ran beside the previous batch's resolve, on
//     the node table as it was then — exact for every other node.  The speculative scan covered the
//     pods after the previous batch; if that batch stopped early (this batch starts elsewhere) or the
//     changed nodes overflow E, `rescan` asks the conditional scan to redo the lists;
//   * the speculative counters for the next scan (the pods after this batch), double-buffered by
//     batch parity `slot`.
#pragma once
#include "ks_device.h"

namespace ks {
namespace prep {

constexpr int kEHashLog2 = 12, kEHash = 1 << kEHashLog2;

// Diagnostic build only (-DKS_MCL_DIAG, tests/dev/diag_mcl.py): section cycles of thread 0 in
// ctr[16..22] (the window prep) — the product executes none of it.
#ifdef KS_MCL_DIAG
__device__ __forceinline__ uint64_t pstamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define PDG(...) __VA_ARGS__
#define PDG_AT(I, T)                                                                      \
    do {                                                                                  \
        const uint64_t t_ = pstamp();                                                     \
        if (threadIdx.x == 0) atomicAdd((unsigned long long*)&a.ctr[16 + (I)], t_ - (T)); \
        (T) = t_;                                                                         \
    } while (0)
#else
#define PDG(...)
#define PDG_AT(I, T)
#endif
static_assert(2 * kEMax <= kEHash, "E hash load <= 1/2");

__device__ __forceinline__ uint32_t ehslot(int32_t n) { return ((uint32_t)n * 2654435761u) >> (32 - kEHashLog2); }

// LDS scratch of one window prep (~44 KB)
struct PrepLDS {
    int32_t hk[kEHash], hv[kEHash];
    int32_t cnt[kWinSlots], fill[kWinSlots];
    int32_t xn[kEMax];  // touched nodes to insert (overlap)
    int64_t off[kWinMaxB];  // exp_off[start + 1 + i]
    int32_t wsum[16];
    int32_t s_ne, s_nx;
};

// One workgroup of NT threads (tid = threadIdx.x).  start / end / err: the batch's counters (the
// caller read them; the chunk kernel passes its commit's values through LDS).
template <int NT>
__device__ __forceinline__ void prep_body(const EngineArgs& a, int64_t start, int64_t end, int64_t err, int head,
                                          int spec, int slot, PrepLDS& L) {
    static_assert(kWinSlots <= NT && kWinMaxB <= NT, "one window slot and one pod per thread");
    static_assert(NT / 64 <= 16, "wave sums");
    WinWS& ws = *a.sw;
    const int tid = threadIdx.x;
    PDG(uint64_t pt = pstamp();)
    int64_t* const spec_out = a.spec_ctr + kSpecStride * slot;
    const int64_t* const spec_in = a.spec_ctr + kSpecStride * (slot ^ 1);
    int nb = (int)min<int64_t>(min<int64_t>(a.B, kWinMaxB), end - start);
    if (err != 0 || nb <= 0) {
        if (tid == 0) {
            ws.nb = 0; ws.e_cnt = 0; ws.n_e = 0; ws.n_es = 0; ws.rescan = 0; ws.lset = 1;
            ws.split = 0; ws.moff = 0; ws.mpar = slot;
            spec_out[kCtrStart] = end; spec_out[kCtrEnd] = end; spec_out[kCtrErr] = 0; spec_out[kSpecPrev] = start;
        }
        return;
    }
    // Three dependent global round trips: (1) the CSR offsets and positions of the batch's pods, the
    // speculative counters and the touched nodes (read speculatively, bounded by their arrays);
    // (2) the expiring pods of the head and of the window; (3) their records and bind state.  (Every
    // read is issued before the head's atomics and stores: the compiler cannot move a read across
    // them.)  A head pod and a window pod are never the same pod (one expiry per pod).
    const int64_t e0 = a.exp_off[start], e1 = a.exp_off[start + 1];
    const int64_t e_base = e1;
    const int64_t myoff = tid < nb ? a.exp_off[start + tid + 1] : 0;
    const int64_t mypos = tid < nb ? a.exp_pos[start + tid] : 0;
    const int64_t sp_start = spec ? spec_in[kCtrStart] : 0;
    const int64_t prev_start = spec ? spec_in[kSpecPrev] : 0;
    const int n_touched = spec ? ws.n_touched : 0;
    // the previous batch's E (its nodes join this batch's E when this batch reuses its lists)
    const int n_eold = spec ? ws.n_e : 0;
    constexpr int kOPer = (kEMax + NT - 1) / NT;
    int32_t eold[kOPer];
#pragma unroll
    for (int q = 0; q < kOPer; ++q) {
        const int t = tid + q * NT;
        eold[q] = spec && t < kEMax ? ws.e_node[t] : -1;
    }
    constexpr int kTPer = (kTouchMax + NT - 1) / NT;
    int32_t tch[kTPer];
#pragma unroll
    for (int q = 0; q < kTPer; ++q) {
        const int t = tid + q * NT;
        tch[q] = spec && t < kTouchMax ? ws.touched[t] : -1;
    }
    const bool fits_win = tid < nb && myoff - e_base <= kWinSlots;
    if (tid < nb) L.off[tid] = myoff;
    for (int h = tid; h < kEHash; h += NT) L.hk[h] = -1;
    if (tid == 0) { L.s_ne = 0; L.s_nx = 0; }
    nb = __syncthreads_count(fits_win);  // exp_off is non-decreasing: a prefix of the pods
    PDG_AT(0, pt);
    const int e_cnt = (int)(L.off[nb - 1] - e_base);  // exp_off[start + nb] - e_base (nb >= 1: pod 0 fits)
    // reuse: the previous batch stopped early (this batch starts inside it): its unbound pods keep
    // the merged lists merge_cl kept for them, the rest take the speculative scan's (which covered
    // the pods after the previous batch) — no rescan.  Every node changed since either scan read the
    // table is in the previous batch's E or was changed by that batch (touched) or this batch's head.
    const bool reuse = spec && start != sp_start && start > prev_start && start < sp_start;
    int rescan = 0;
    if (spec) rescan = (start != sp_start && !reuse) ||
                       (int64_t)e_cnt + (e1 - e0) + n_touched + (reuse ? n_eold : 0) > kEMax;
    const bool touch = spec && !rescan;
    const int32_t hq = head && tid < e1 - e0 ? a.exp_pod[e0 + tid] : -1;
    const int32_t wq = tid < e_cnt ? a.exp_pod[e_base + tid] : -1;
    int32_t hst = 1, hex = 1, hnd = 0, wst = 1, wex = 1, wnd = 0;
    int64_t hr0 = 0, hr1 = 0, hr2 = 0, wr0 = 0, wr1 = 0, wr2 = 0;
    if (hq >= 0) {
        hst = a.b_status[hq]; hex = a.expired[hq]; hnd = a.b_node[hq];
        const PodRec& p = a.pods[hq];
        hr0 = p.req[0]; hr1 = p.req[1]; hr2 = p.req[2];
    }
    if (wq >= 0) {
        wst = a.b_status[wq]; wex = a.expired[wq]; wnd = a.b_node[wq];
        const PodRec& p = a.pods[wq];
        wr0 = p.req[0]; wr1 = p.req[1]; wr2 = p.req[2];
    }
    if (head) {  // expire_head's work: the expiries due before the batch's first pod
        if (hq >= 0 && hst == 0 && !hex) {
            atomicAdd((unsigned long long*)&a.s.rc[hnd], (unsigned long long)(-hr0));
            atomicAdd((unsigned long long*)&a.s.rm[hnd], (unsigned long long)(-hr1));
            atomicAdd((unsigned long long*)&a.s.rg[hnd], (unsigned long long)(-hr2));
            atomicAdd((unsigned long long*)&a.s.nr[hnd], (unsigned long long)(-1ll));
            a.expired[hq] = 1;
            if (touch) L.xn[atomicAdd(&L.s_nx, 1)] = hnd;
        }
        for (int64_t e = e0 + NT + tid; e < e1; e += NT) {  // (more head expiries than threads)
            const int32_t q = a.exp_pod[e];
            if (a.b_status[q] != 0 || a.expired[q]) continue;
            const int32_t nd = a.b_node[q];
            const PodRec& p = a.pods[q];
            atomicAdd((unsigned long long*)&a.s.rc[nd], (unsigned long long)(-p.req[0]));
            atomicAdd((unsigned long long*)&a.s.rm[nd], (unsigned long long)(-p.req[1]));
            atomicAdd((unsigned long long*)&a.s.rg[nd], (unsigned long long)(-p.req[2]));
            atomicAdd((unsigned long long*)&a.s.nr[nd], (unsigned long long)(-1ll));
            a.expired[q] = 1;
            if (touch) L.xn[atomicAdd(&L.s_nx, 1)] = nd;
        }
    }
    if (touch) {
#pragma unroll
        for (int q = 0; q < kTPer; ++q)
            if (tid + q * NT < n_touched) L.xn[atomicAdd(&L.s_nx, 1)] = tch[q];
        if (reuse) {
#pragma unroll
            for (int q = 0; q < kOPer; ++q)
                if (tid + q * NT < n_eold) L.xn[atomicAdd(&L.s_nx, 1)] = eold[q];
        }
    }
    if (tid < nb) {
        ws.win_hi[tid] = tid >= 1 ? (int32_t)(myoff - e_base) : 0;
        ws.own[tid] = (mypos >= e_base && mypos - e_base < e_cnt) ? (int32_t)(mypos - e_base) : -1;
    }
    int32_t my_node = -1, my_k = -1;
    if (tid < e_cnt) {
        ws.ex_q[tid] = wq;
        ws.ex_req[tid][0] = wr0; ws.ex_req[tid][1] = wr1; ws.ex_req[tid][2] = wr2;
        const bool ok = wq < start && wst == 0 && !wex;
        ws.ex_ok[tid] = ok ? 1 : 0;
        if (ok) my_node = wnd;
    }
    if (my_node >= 0) {
        uint32_t h = ehslot(my_node);
        bool claimed = false;
        for (;;) {  // <= kEMax distinct nodes < kEHash slots: terminates
            const int32_t prev = atomicCAS(&L.hk[h], -1, my_node);
            if (prev == -1) { claimed = true; break; }
            if (prev == my_node) break;
            h = (h + 1) & (kEHash - 1);
        }
        my_k = (int32_t)h;  // hash slot; the claiming thread numbers the node
        if (claimed) L.hv[h] = atomicAdd(&L.s_ne, 1);
    }
    __syncthreads();
    PDG_AT(1, pt);
    const int n_es = L.s_ne;  // the slot nodes; the touched nodes after them (no slots)
    __syncthreads();
    const int n_x = L.s_nx;
    for (int t = tid; t < n_x; t += NT) {
        const int32_t nd = L.xn[t];
        uint32_t h = ehslot(nd);
        for (;;) {
            const int32_t prev = atomicCAS(&L.hk[h], -1, nd);
            if (prev == -1) { const int k = atomicAdd(&L.s_ne, 1); L.hv[h] = k; ws.e_node[k] = nd; break; }
            if (prev == nd) break;
            h = (h + 1) & (kEHash - 1);
        }
    }
    __syncthreads();
    PDG_AT(2, pt);
    const int n_e = L.s_ne;
    if (tid < n_es) { L.cnt[tid] = 0; L.fill[tid] = 0; }
    __syncthreads();
    int k_of = -1;
    if (my_node >= 0) {
        k_of = L.hv[my_k];
        ws.e_node[k_of] = my_node;
        atomicAdd(&L.cnt[k_of], 1);
    }
    __syncthreads();
    PDG_AT(3, pt);
    {  // exclusive prefix of the slot nodes' counts (n_es <= kWinSlots: one per thread)
        const int lane = tid & 63, wv = tid >> 6;
        const int v = tid < n_es ? L.cnt[tid] : 0;
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        if (lane == 63) L.wsum[wv] = incl;
        __syncthreads();
        int base = 0;
        for (int g = 0; g < wv; ++g) base += L.wsum[g];
        if (tid < n_es) ws.e_off[tid] = base + incl - v;
        if (tid == n_es - 1) ws.e_off[n_es] = base + incl;
        if (n_es == 0 && tid == 0) ws.e_off[0] = 0;
    }
    __syncthreads();
    PDG_AT(4, pt);
    if (my_node >= 0) ws.e_slot[ws.e_off[k_of] + atomicAdd(&L.fill[k_of], 1)] = tid;  // slot x == tid
    __syncthreads();
    PDG_AT(5, pt);
    if (tid < n_es) {  // each node's few slots ascending
        const int lo = ws.e_off[tid], hi = ws.e_off[tid + 1];
        for (int u = lo + 1; u < hi; ++u) {
            const int32_t x = ws.e_slot[u];
            int v = u - 1;
            while (v >= lo && ws.e_slot[v] > x) { ws.e_slot[v + 1] = ws.e_slot[v]; --v; }
            ws.e_slot[v + 1] = x;
        }
    }
    for (int k = tid; k < n_e; k += NT) a.e_idx[ws.e_node[k]] = k;
    if (tid == 0) {
        ws.nb = nb; ws.e_cnt = e_cnt; ws.n_e = n_e; ws.n_es = n_es; ws.nslot = 0; ws.rescan = rescan;
        ws.lset = touch ? 0 : 1;  // pruned lists: the speculative scan's set, or the engine's own scan's
        if (rescan) a.ctr[kCtrRescan] += 1;  // (diagnostics: ks_debug_counters [5])
        if (touch && reuse) a.ctr[kCtrReuse] += 1;
        ws.split = touch && reuse ? (int32_t)(sp_start - start) : 0;
        ws.moff = (int32_t)(start - prev_start);
        ws.mpar = slot;
        // the next speculative scan: the pods after this batch, if it commits them all
        spec_out[kCtrStart] = start + nb; spec_out[kCtrEnd] = end; spec_out[kCtrErr] = 0;
        spec_out[kSpecPrev] = start;
    }
    PDG(__syncthreads(); PDG_AT(6, pt); if (tid == 0) atomicAdd((unsigned long long*)&a.ctr[23], 1ull);)
}

}  // namespace prep
}  // namespace ks
