// ks_sweep.hip — the sweep resolver (gfx950): a batch's binds as the fixed point of parallel
// (Jacobi) sweeps instead of one pod per barrier.
//
// The reference binds one pod per tick in FIFO order (kubesim/kubesim.go:105-121, 143-166):
// pod i takes the argmax of its key over every node on the state that the binds of pods < i
// (admitted per kubesim/node/node.go:36-60) and the expiries due by its tick leave.  Write
// f_i(w_0 .. w_{i-1}) for that argmax: the batch's winners are the unique w with w_i = f_i(w_{<i})
// for every i.  A sweep computes w'_i = f_i(w_{<i}) for ALL pods at once from the previous
// sweep's w; after sweep t the first t pods are exact (induction on i), and a prefix that two
// consecutive sweeps agree on is already the fixed point (w'_{<m} = w_{<m} makes every later
// sweep repeat it).  On the C3 workload a 256-pod batch reaches the fixed point in 7-9 sweeps
// (tests/dev/jacobi_model.py, exact integer model checked against the sequential loop).
//
// One sweep = one workgroup per pod, no communication inside the sweep: pod i's candidates are
//   * the nodes the batch's earlier pods bound in the previous sweep's w (their states replayed
//     bind by bind with exact admission and the expiries between),
//   * E, the nodes on which an expiry of a pod bound before the batch falls inside the batch's
//     expiry window (states with the expiries due by pod i's tick), and
//   * the first entry of pod i's snapshot top-L list (merge kernel) that is neither: its state is
//     the snapshot's, so its list key is exact, and every node outside the list scores below the
//     list's last entry.  If the whole list is covered and no candidate beats the list's last
//     snapshot key, the winner may lie outside the list: the pod stops the batch (the next launch
//     rescans from it), as the other resolvers' exhausted lists do.
// Kernels per launch: sweep_prep (window, E), up to `sweeps` sweep kernels (each exits at once
// when the previous sweep left nothing to change before the first stop), sweep_commit (statuses,
// node state write-back, expiry marks, the committed count).
#include <climits>

#include "ks_device.h"

namespace ks {
namespace sw {

constexpr int kThreads = 256;
constexpr int kPrepThreads = 1024;
constexpr int kHashLog2 = 10, kHash = 1 << kHashLog2;  // LDS hash of a sweep's earlier winners
constexpr int kEHashLog2 = 11, kEHash = 1 << kEHashLog2;
constexpr int kL = kTopL;
constexpr int kMaxPend = 32;  // counted in-batch binds on one node with an in-window expiry pending
static_assert(kSweepMaxB <= kThreads, "one thread per earlier pod");

__device__ __forceinline__ uint32_t hslot(int32_t n, int lg) { return ((uint32_t)n * 2654435761u) >> (32 - lg); }
__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }
__device__ __forceinline__ bool converged(int32_t fc, int32_t fs) { return fc == INT_MAX || fc > fs; }
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void sub_req(NodeV& v, const int64_t* r) {
    v.rc -= r[0]; v.rm -= r[1]; v.rg -= r[2]; v.nr -= 1;
}

// Replays node n from the snapshot through the binds of pods < i_end, with the expiry slots
// < h_final applied at the end (h_final = win_hi[i_end]: the moment before pod i_end binds):
// the pre-batch expiries of n (E slots) and the binds of the batch's pods j < i_end that w names
// n, each admitted on the state at its own bind (CreatePod, kubesim/node/node.go:44-47), a bind of
// a pod with a positive run counted until its own expiry slot (when that falls in the window).
// bind_ok (optional) receives each replayed bind's admission.  Returns -1, or the pod whose bind
// would have made more than kMaxPend counted binds with a pending in-window expiry on n (the
// state is then unknown from that pod on).
template <class W>
__device__ int replay(const EngineArgs& a, const SweepWS& ws, int32_t n, int e_idx, const W& w, int j0, int cnt,
                      int i_end, int h_final, int64_t start, NodeV& v, int32_t* bind_ok) {
    v = load_node(a.s, n);
    int ep = 0, ee = 0;
    if (e_idx >= 0) { ep = ws.e_off[e_idx]; ee = ws.e_off[e_idx + 1]; }
    int32_t pj[kMaxPend];  // counted binds whose own expiry lies in the window, not yet due
    int np = 0;
    auto expire_to = [&](int h) {
        while (ep < ee && ws.e_slot[ep] < h) {
            sub_req(v, ws.ex_req[ws.e_slot[ep]]);
            ++ep;
        }
        int keep = 0;
        for (int q = 0; q < np; ++q) {
            const int j = pj[q];
            if (ws.own[j] < h) sub_req(v, a.pods[start + j].req);
            else pj[keep++] = j;
        }
        np = keep;
    };
    int seen = 0;
    for (int j = j0; j >= 0 && j < i_end && seen < cnt; ++j) {
        if (w(j) != n) continue;
        ++seen;
        expire_to(ws.win_hi[j]);
        const PodRec& p = a.pods[start + j];
        const bool ok = fits(p, v);
        if (bind_ok) bind_ok[j] = ok ? 1 : 0;
        if (ok && a.dur[start + j] > 0) {
            v.rc += p.req[0]; v.rm += p.req[1]; v.rg += p.req[2]; v.nr += 1;
            if (ws.own[j] >= 0) {
                if (np >= kMaxPend) return j;
                pj[np++] = j;
            }
        }
    }
    expire_to(h_final);
    return -1;
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kPrepThreads) void sweep_prep_kernel(const EngineArgs* __restrict__ A, int max_slots) {
    const EngineArgs& a = A[0];
    SweepWS& ws = *a.sw;
    const int tid = threadIdx.x;
    __shared__ int32_t hk[kEHash], hv[kEHash];
    __shared__ int32_t cnt[kSweepMaxSlots], fill[kSweepMaxSlots];
    __shared__ int32_t s_ne;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    for (int s = tid; s < kSweepMaxSweeps; s += kPrepThreads) {
        ws.fc[s] = INT_MAX; ws.fs[s] = INT_MAX; ws.ran[s] = 0;
    }
    int nb = (int)min<int64_t>(min<int64_t>(a.B, kSweepMaxB), end - start);
    if (a.ctr[kCtrErr] != 0 || nb <= 0) {
        if (tid == 0) { ws.nb = 0; ws.e_cnt = 0; ws.n_e = 0; }
        return;
    }
    const int64_t e_base = a.exp_off[start + 1];
    const bool fits_win = tid < nb && a.exp_off[start + tid + 1] - e_base <= max_slots;
    for (int h = tid; h < kEHash; h += kPrepThreads) hk[h] = -1;
    if (tid == 0) s_ne = 0;
    nb = __syncthreads_count(fits_win);  // exp_off is non-decreasing: a prefix of the pods
    const int e_cnt = (int)(a.exp_off[start + nb] - e_base);
    for (int i = tid; i < kSweepMaxB; i += kPrepThreads) {
        if (i < nb) {
            ws.win_hi[i] = i >= 1 ? (int32_t)(a.exp_off[start + i + 1] - e_base) : 0;
            const int64_t pos = a.exp_pos[start + i];
            ws.own[i] = (pos >= e_base && pos - e_base < e_cnt) ? (int32_t)(pos - e_base) : -1;
        }
        ws.w[0][i] = -1;
        ws.code[0][i] = 0;
    }
    // the window's slots; E = distinct nodes of the pre-batch pods' pending expiries
    int32_t my_node = -1, my_k = -1;
    for (int x = tid; x < e_cnt; x += kPrepThreads) {
        const int32_t q = a.exp_pod[e_base + x];
        const PodRec& pq = a.pods[q];
        ws.ex_q[x] = q;
        ws.ex_req[x][0] = pq.req[0]; ws.ex_req[x][1] = pq.req[1]; ws.ex_req[x][2] = pq.req[2];
        const bool ok = q < start && a.b_status[q] == 0 && !a.expired[q];
        ws.ex_ok[x] = ok ? 1 : 0;
        if (ok && x < kPrepThreads) my_node = a.b_node[q];  // e_cnt <= kSweepMaxSlots = kPrepThreads
    }
    static_assert(kSweepMaxSlots <= kPrepThreads, "one thread per window slot");
    bool claimed = false;
    if (my_node >= 0) {
        uint32_t h = hslot(my_node, kEHashLog2);
        for (;;) {  // <= kSweepMaxSlots distinct nodes < kEHash slots: terminates
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
    for (int k = tid; k < n_e; k += kPrepThreads) { cnt[k] = 0; fill[k] = 0; }
    __syncthreads();
    int k_of = -1;
    if (my_node >= 0) {
        k_of = hv[my_k];
        ws.e_node[k_of] = my_node;
        atomicAdd(&cnt[k_of], 1);
    }
    __syncthreads();
    {  // exclusive prefix of the counts (n_e <= kPrepThreads: one per thread; wave scans + wave sums)
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
    static_assert(kSweepMaxSlots <= kPrepThreads, "one E node per thread");
    __syncthreads();
    if (my_node >= 0) ws.e_slot[ws.e_off[k_of] + atomicAdd(&fill[k_of], 1)] = tid;  // slot x == tid here
    __syncthreads();
    for (int k = tid; k < n_e; k += kPrepThreads) {  // each node's few slots ascending
        const int lo = ws.e_off[k], hi = ws.e_off[k + 1];
        for (int u = lo + 1; u < hi; ++u) {
            const int32_t x = ws.e_slot[u];
            int v = u - 1;
            while (v >= lo && ws.e_slot[v] > x) { ws.e_slot[v + 1] = ws.e_slot[v]; --v; }
            ws.e_slot[v + 1] = x;
        }
        a.e_idx[ws.e_node[k]] = k;
    }
    if (tid == 0) { ws.nb = nb; ws.e_cnt = e_cnt; ws.n_e = n_e; }
}

// ---------------------------------------------------------------------------------------------
template <int kMode>
__global__ __launch_bounds__(kThreads) void sweep_kernel(const EngineArgs* __restrict__ A, int s) {
    const EngineArgs& a = A[0];
    SweepWS& ws = *a.sw;
    const int i = blockIdx.x, tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int nb = ws.nb;
    if (i >= nb) return;
    if (s > 0 && (!ws.ran[s - 1] || converged(ws.fc[s - 1], ws.fs[s - 1]))) return;
    if (i == 0 && tid == 0) ws.ran[s] = 1;
    const int64_t start = a.ctr[kCtrStart];
    const int32_t* wc = ws.w[s & 1];
    const int32_t* cc = ws.code[s & 1];
    __shared__ int32_t wl[kSweepMaxB];
    __shared__ int32_t hk[kHash], hfirst[kHash], hcnt[kHash];
    __shared__ uint64_t red[kThreads / kWave];
    for (int h = tid; h < kHash; h += kThreads) { hk[h] = -1; hfirst[h] = INT_MAX; hcnt[h] = 0; }
    if (tid < i) wl[tid] = wc[tid];
    __syncthreads();
    // the earlier pods' winners of the previous sweep: first pod and count per node
    if (tid < i && wl[tid] >= 0) {
        const int32_t n = wl[tid];
        uint32_t h = hslot(n, kHashLog2);
        for (;;) {  // <= kSweepMaxB nodes in kHash slots: terminates
            const int32_t prev = atomicCAS(&hk[h], -1, n);
            if (prev == -1 || prev == n) break;
            h = (h + 1) & (kHash - 1);
        }
        atomicMin(&hfirst[h], tid);
        atomicAdd(&hcnt[h], 1);
    }
    __syncthreads();
    auto find = [&](int32_t n) -> int {
        uint32_t h = hslot(n, kHashLog2);
        for (int t = 0; t < kHash; ++t) {
            const int32_t k = hk[h];
            if (k == n) return (int)h;
            if (k == -1) return -1;
            h = (h + 1) & (kHash - 1);
        }
        return -1;
    };
    const PodRec p = a.pods[start + i];
    uint64_t best = 0;
    bool overflow = false;
    auto wfun = [&](int j) { return wl[j]; };
    // (1) nodes the earlier pods bound: one thread per node (its first binder)
    if (tid < i && wl[tid] >= 0) {
        const int32_t n = wl[tid];
        const int h = find(n);
        if (hfirst[h] == tid) {
            NodeV v;
            if (replay(a, ws, n, a.e_idx[n], wfun, tid, hcnt[h], i, ws.win_hi[i], start, v, nullptr) < 0) {
                const uint64_t k = make_key(eval_t<kMode>(a.c, p, v), (uint32_t)n);
                best = k > best ? k : best;
            } else {
                overflow = true;
            }
        }
    }
    // (2) the pre-batch expiry nodes no earlier pod bound
    for (int e = tid; e < ws.n_e; e += kThreads) {
        const int32_t n = ws.e_node[e];
        if (find(n) >= 0) continue;
        NodeV v;
        replay(a, ws, n, e, wfun, -1, 0, i, ws.win_hi[i], start, v, nullptr);
        const uint64_t k = make_key(eval_t<kMode>(a.c, p, v), (uint32_t)n);
        best = k > best ? k : best;
    }
    // (3) the first list entry no earlier pod bound and no pre-batch expiry touches (wave 0)
    uint64_t lk = 0, last = 0;
    bool all_cov = false;
    if (wave == 0) {
        const uint64_t x = lane < kL ? a.cand[(int64_t)i * kL + lane] : 0ull;
        const int32_t xn = key_node(x);
        const bool cov = x != 0 && (find(xn) >= 0 || a.e_idx[xn] >= 0);
        const uint64_t bx = __ballot(x != 0), bu = __ballot(x != 0 && !cov);
        all_cov = __popcll(bx) == kL && bu == 0;
        if (bu) lk = shfl64(x, __ffsll((unsigned long long)bu) - 1);
        last = shfl64(x, kL - 1);
    }
    // workgroup max of the exact candidates
    const bool ovf = __syncthreads_or(overflow);
    {
        const uint64_t m = wave_max_u64(best);
        if (lane == 0) red[wave] = m;
    }
    __syncthreads();
    if (tid == 0) {
        uint64_t m = 0;
        for (int q = 0; q < kThreads / kWave; ++q) m = red[q] > m ? red[q] : m;
        int code = 0;
        uint64_t win = 0;
        if (ovf || (all_cov && m < last)) {
            code = 1;  // the winner may lie outside the list (or too many binds on one node)
        } else {
            win = m > lk ? m : lk;
            if (win == 0) code = 2;                                        // NotFound
            else if (p.flags & (kFlagBadKey | kFlagBadSpec)) code = 3;     // InvalidArgument
        }
        const int32_t wn = code == 0 ? key_node(win) : -1;
        ws.w[(s + 1) & 1][i] = wn;
        ws.code[(s + 1) & 1][i] = code;
        if (wn != wc[i] || code != cc[i]) atomicMin(&ws.fc[s], i);
        if (code != 0) atomicMin(&ws.fs[s], i);
    }
}

// ---------------------------------------------------------------------------------------------
template <int kMode>
__global__ __launch_bounds__(kPrepThreads) void sweep_commit_kernel(const EngineArgs* __restrict__ A, int sweeps) {
    const EngineArgs& a = A[0];
    SweepWS& ws = *a.sw;
    const int tid = threadIdx.x;
    const int nb = ws.nb;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (nb <= 0) return;
    __shared__ int32_t wl[kSweepMaxB], okl[kSweepMaxB];
    __shared__ int32_t hk[kHash], hfirst[kHash], hcnt[kHash];
    int last = 0;
    for (int s = 0; s < sweeps; ++s)
        if (ws.ran[s]) last = s;
    const int r = (last + 1) & 1;
    const int32_t fc = ws.fc[last], fs = ws.fs[last];
    const bool conv = converged(fc, fs);
    const int c0 = conv ? min(fs, nb) : min(fc, nb);  // the committed prefix
    int stop_code = (conv && fs < nb) ? ws.code[r][fs] : 0;
    __shared__ int32_t s_ovf;
    __shared__ int64_t fst[4][kSweepMaxB];  // final state of the node each leader replayed
    auto wfun = [&](int j) { return wl[j]; };
    auto find = [&](int32_t n) -> int {
        uint32_t h = hslot(n, kHashLog2);
        for (int t = 0; t < kHash; ++t) {
            const int32_t k = hk[h];
            if (k == n) return (int)h;
            if (k == -1) return -1;
            h = (h + 1) & (kHash - 1);
        }
        return -1;
    };
    // the state a batch that commits c pods leaves: binds of pods < c, the expiry windows of pods
    // 1 .. c - 1 (slots < win_hi[c - 1]); the next launch's expire_head applies pod c's window.
    // A second pass only when a replay overflowed (kMaxPend): the prefix is then cut before it.
    int c = c0;
    for (int pass = 0; pass < 2; ++pass) {
        for (int h = tid; h < kHash; h += kPrepThreads) { hk[h] = -1; hfirst[h] = INT_MAX; hcnt[h] = 0; }
        if (tid < kSweepMaxB) { wl[tid] = tid < c ? ws.w[r][tid] : -1; okl[tid] = 0; }
        if (tid == 0) s_ovf = INT_MAX;
        __syncthreads();
        if (tid < c) {
            const int32_t n = wl[tid];
            uint32_t h = hslot(n, kHashLog2);
            for (;;) {
                const int32_t prev = atomicCAS(&hk[h], -1, n);
                if (prev == -1 || prev == n) break;
                h = (h + 1) & (kHash - 1);
            }
            atomicMin(&hfirst[h], tid);
            atomicAdd(&hcnt[h], 1);
        }
        __syncthreads();
        const int h_end = c >= 1 ? ws.win_hi[c - 1] : 0;
        if (tid < c) {
            const int32_t n = wl[tid];
            const int h = find(n);
            if (hfirst[h] == tid) {
                NodeV v;
                const int ov = replay(a, ws, n, a.e_idx[n], wfun, tid, hcnt[h], c, h_end, start, v, okl);
                if (ov >= 0) atomicMin(&s_ovf, ov);
                fst[0][tid] = v.rc; fst[1][tid] = v.rm; fst[2][tid] = v.rg; fst[3][tid] = v.nr;
            }
        }
        __syncthreads();
        if (s_ovf >= c) break;
        c = s_ovf;  // >= kMaxPend: progress is kept
        stop_code = 1;
        __syncthreads();
    }
    const int h_end = c >= 1 ? ws.win_hi[c - 1] : 0;
    if (tid < c) {
        const int32_t n = wl[tid];
        const int64_t j = start + tid;
        if (hfirst[find(n)] == tid) {
            a.s.rc[n] = fst[0][tid]; a.s.rm[n] = fst[1][tid]; a.s.rg[n] = fst[2][tid]; a.s.nr[n] = fst[3][tid];
        }
        gptr(a.b_node)[j] = n;
        gptr(a.b_status)[j] = okl[tid] ? 0 : 1;
        const int own = ws.own[tid];
        if (okl[tid] && a.dur[j] > 0 && own >= 0 && own < h_end) gptr(a.expired)[j] = 1;
    }
    // the pre-batch expiry nodes no committed pod bound: their expiries up to pod c - 1
    for (int e = tid; e < ws.n_e; e += kPrepThreads) {
        const int32_t n = ws.e_node[e];
        if (find(n) < 0) {
            NodeV v;
            replay(a, ws, n, e, wfun, -1, 0, c, h_end, start, v, nullptr);
            a.s.rc[n] = v.rc; a.s.rm[n] = v.rm; a.s.rg[n] = v.rg; a.s.nr[n] = v.nr;
        }
    }
    for (int x = tid; x < h_end; x += kPrepThreads)
        if (ws.ex_ok[x]) gptr(a.expired)[ws.ex_q[x]] = 1;
    __syncthreads();
    for (int e = tid; e < ws.n_e; e += kPrepThreads) a.e_idx[ws.e_node[e]] = -1;
    if (tid == 0) {
        a.ctr[kCtrStart] = start + c;
        const bool err = stop_code == 2 || stop_code == 3;
        if (err) {
            a.ctr[kCtrErr] = stop_code == 2 ? kErrNotFound : kErrEinval;
            a.ctr[kCtrErrPod] = start + c;
        }
        if (c < a.B && !err && start + c < end) a.ctr[kCtrEarly] += 1;
    }
}

}  // namespace sw

hipError_t launch_resolve_sweep(const EngineArgs* d, int mode, int sweeps, hipStream_t st) {
    // at least two sweeps: sweep 0 starts from "no binds", so only from sweep 1 on is a prefix
    // (pod 0 at least) stable and committable
    sweeps = sweeps < 2 ? 2 : (sweeps > kSweepMaxSweeps ? kSweepMaxSweeps : sweeps);
    hipLaunchKernelGGL(sw::sweep_prep_kernel, dim3(1), dim3(sw::kPrepThreads), 0, st, d, kSweepMaxSlots);
    for (int s = 0; s < sweeps; ++s) {
        switch (mode) {
            case kEvalMicro: hipLaunchKernelGGL(sw::sweep_kernel<kEvalMicro>, dim3(kSweepMaxB), dim3(sw::kThreads), 0, st, d, s); break;
            case kEvalTiny: hipLaunchKernelGGL(sw::sweep_kernel<kEvalTiny>, dim3(kSweepMaxB), dim3(sw::kThreads), 0, st, d, s); break;
            case kEvalNarrow: hipLaunchKernelGGL(sw::sweep_kernel<kEvalNarrow>, dim3(kSweepMaxB), dim3(sw::kThreads), 0, st, d, s); break;
            default: hipLaunchKernelGGL(sw::sweep_kernel<kEvalWide>, dim3(kSweepMaxB), dim3(sw::kThreads), 0, st, d, s); break;
        }
    }
    hipLaunchKernelGGL(sw::sweep_commit_kernel<kEvalWide>, dim3(1), dim3(sw::kPrepThreads), 0, st, d, sweeps);
    return hipGetLastError();
}

hipError_t launch_sweep_prep(const EngineArgs* d, int max_slots, hipStream_t st) {
    hipLaunchKernelGGL(sw::sweep_prep_kernel, dim3(1), dim3(sw::kPrepThreads), 0, st, d, max_slots);
    return hipGetLastError();
}

}  // namespace ks
