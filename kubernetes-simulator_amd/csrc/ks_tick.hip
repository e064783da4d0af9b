// ks_tick.hip — the per-tick drop-in path (gfx950): one launch per scheduleOne.
//
// The reference's Run loop (kubesim/kubesim.go:101-122) submits and schedules one pod per tick;
// a drop-in host (the Go shim's Run, go/kubesim/engine/kubesim.go) calls ks_submit_pods and
// ks_step(1) every tick.  The batch machinery (expire_head, scan, merge, window, candidates,
// resolver; two host round trips) is built for thousands of pods per call; for one pod it is pure
// latency.  This file is the one-pod path:
//
//   tick_kernel   grid = the cluster's 1024-node blocks.  Every workgroup evaluates its nodes for the
//                 pod (fused Filter + Score, the expiries due before the pod applied on the fly from
//                 a by-value list), reduces its block maximum of the packed key and folds it into one
//                 u64 with a device-scope atomicMax.  The last workgroup to arrive (atomic counter)
//                 applies the expiries to the node state, binds the pod on the winner (CreatePod
//                 admission, kubesim/node/node.go:36-60; NotFound and bad-pod stops as
//                 kubesim.go:217-220), and writes the result to host-mapped memory, which the host
//                 polls (no stream synchronisation).  One extra workgroup applies the call's staged
//                 submits, passed inline in the kernel arguments, beside the evaluation.
//   scatter_kernel  the host-staged submits alone (before any other device work reads them).
#include "ks_device.h"

namespace ks {

constexpr int kTickThreads = 256;
constexpr int kTickNodes = 4;  // nodes per thread

__device__ __forceinline__ void copy_segs(const CopySeg* segs, int n, int tid, int nthr) {
    for (int k = 0; k < n; ++k) {
        const CopySeg sg = segs[k];
        if (((sg.bytes | (int64_t)(uintptr_t)sg.dst | (int64_t)(uintptr_t)sg.src) & 3) == 0) {
            const uint32_t* s = reinterpret_cast<const uint32_t*>(sg.src);
            uint32_t* d = reinterpret_cast<uint32_t*>(sg.dst);
            for (int64_t w = tid; w < sg.bytes / 4; w += nthr) d[w] = s[w];
        } else {
            for (int64_t b = tid; b < sg.bytes; b += nthr) sg.dst[b] = sg.src[b];
        }
    }
}

__global__ __launch_bounds__(kTickThreads) void scatter_kernel(const CopySeg* segs, int n) {
    if ((int)blockIdx.x < n) copy_segs(segs + blockIdx.x, 1, threadIdx.x, kTickThreads);
}

template <int kMode>
__global__ __launch_bounds__(kTickThreads) void tick_kernel(const TickArgs A) {
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    // the extra (last) workgroup applies this call's staged submits (inline in the arguments)
    // beside the evaluation; it arrives like the others, so the bind — which writes the pod's own
    // submitted rows (b_node, b_status) — follows the copy
    const bool copier = (int)blockIdx.x == (int)gridDim.x - 1;
    uint64_t key = 0;
    if (copier) {
        const uint8_t* base = A.inl;
        for (int k = 0; k < A.n_iseg; ++k) {
            const TickSeg sg = A.iseg[k];
            const uint8_t* src = base + sg.off;
            if ((((uintptr_t)sg.dst | (uint32_t)sg.bytes) & 3) == 0) {
                const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
                uint32_t* d4 = reinterpret_cast<uint32_t*>(sg.dst);
                for (int w = tid; w < sg.bytes / 4; w += kTickThreads) d4[w] = s4[w];
            } else {
                for (int w = tid; w < sg.bytes; w += kTickThreads) sg.dst[w] = src[w];
            }
        }
        __threadfence();
    } else {
        // kTickNodes nodes per thread, their loads issued together (fewer workgroups: fewer
        // arrivals on the two grid-wide atomics)
        NodeV v[kTickNodes];
#pragma unroll
        for (int q = 0; q < kTickNodes; ++q) {
            const int64_t i = ((int64_t)blockIdx.x * kTickNodes + q) * kTickThreads + tid;
            v[q] = NodeV{};
            if (i < A.c.n_nodes) v[q] = load_node(A.s, i);
        }
#pragma unroll
        for (int q = 0; q < kTickNodes; ++q) {
            const int64_t i = ((int64_t)blockIdx.x * kTickNodes + q) * kTickThreads + tid;
            if (i >= A.c.n_nodes) continue;
            for (int e = 0; e < A.n_exp; ++e)
                if (A.exp[e].node == i) {
                    v[q].rc -= A.exp[e].req[0]; v[q].rm -= A.exp[e].req[1]; v[q].rg -= A.exp[e].req[2]; v[q].nr -= 1;
                }
            const uint64_t k = make_key(eval_t<kMode>(A.c, A.pod, v[q]), (uint32_t)i);
            key = k > key ? k : key;
        }
    }
    __shared__ uint64_t wmax[kTickThreads / kWave];
    __shared__ int last;
    const uint64_t m = wave_max_u64(key);
    if (lane == 0) wmax[wave] = m;
    __syncthreads();
    if (tid == 0) {
        uint64_t b = wmax[0];
#pragma unroll
        for (int w = 1; w < kTickThreads / kWave; ++w) b = wmax[w] > b ? wmax[w] : b;
        if (b) atomicMax((unsigned long long*)&A.scr->best, (unsigned long long)b);
        __threadfence();
        last = atomicAdd(&A.scr->count, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    // ---- the last workgroup: every other one has folded its maximum
    __threadfence();
    if (tid < A.n_exp) {
        const TickExp& x = A.exp[tid];
        atomicAdd((unsigned long long*)&A.s.rc[x.node], (unsigned long long)(-x.req[0]));
        atomicAdd((unsigned long long*)&A.s.rm[x.node], (unsigned long long)(-x.req[1]));
        atomicAdd((unsigned long long*)&A.s.rg[x.node], (unsigned long long)(-x.req[2]));
        atomicAdd((unsigned long long*)&A.s.nr[x.node], (unsigned long long)(-1ll));
        A.expired[x.q] = 1;
    }
    __threadfence();
    __syncthreads();
    if (tid == 0) {
        const uint64_t best = __hip_atomic_load((unsigned long long*)&A.scr->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int32_t code = 0, node = -1, status = -1;
        if (best == 0) code = (int32_t)kErrNotFound;  // kubesim.go:217-220
        else if (A.pod.flags & (kFlagBadKey | kFlagBadSpec)) code = (int32_t)kErrEinval;
        else {
            node = (int32_t)(0xFFFFFFFFu - (uint32_t)best);
            auto ld = [](int64_t* p) { return (int64_t)__hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
            NodeV v;
            v.ac = A.s.ac[node]; v.am = A.s.am[node]; v.ag = A.s.ag[node]; v.ap = A.s.ap[node];
            v.rc = ld(&A.s.rc[node]); v.rm = ld(&A.s.rm[node]); v.rg = ld(&A.s.rg[node]); v.nr = ld(&A.s.nr[node]);
            const bool ok = fits(A.pod, v);
            if (ok && A.run) {
                A.s.rc[node] = v.rc + A.pod.req[0]; A.s.rm[node] = v.rm + A.pod.req[1];
                A.s.rg[node] = v.rg + A.pod.req[2]; A.s.nr[node] = v.nr + 1;
            }
            status = ok ? 0 : 1;
            A.b_node[A.j] = node;
            A.b_status[A.j] = status;
        }
        A.scr->best = 0;
        A.scr->count = 0;
        // the result to host-mapped memory: node and status, then (release, system scope) the code
        // the host polls on
        A.out->node = node;
        A.out->status = status;
        __hip_atomic_store(&A.out->code, code, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(64) void apply_exp_kernel(NodeSoA s, uint8_t* expired, const ExpList L) {
    const int t = threadIdx.x;
    if (t >= L.n) return;
    const TickExp& x = L.x[t];
    atomicAdd((unsigned long long*)&s.rc[x.node], (unsigned long long)(-x.req[0]));
    atomicAdd((unsigned long long*)&s.rm[x.node], (unsigned long long)(-x.req[1]));
    atomicAdd((unsigned long long*)&s.rg[x.node], (unsigned long long)(-x.req[2]));
    atomicAdd((unsigned long long*)&s.nr[x.node], (unsigned long long)(-1ll));
    expired[x.q] = 1;
}

hipError_t launch_apply_exp(const NodeSoA& s, uint8_t* expired, const ExpList& l, hipStream_t st) {
    hipLaunchKernelGGL(apply_exp_kernel, dim3(1), dim3(64), 0, st, s, expired, l);
    return hipGetLastError();
}

hipError_t launch_tick(const TickArgs& a, int mode, hipStream_t st) {
    const int64_t per = (int64_t)kTickThreads * kTickNodes;
    const int grid = (int)((a.c.n_nodes + per - 1) / per) + 1;  // + the copy workgroup
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL(tick_kernel<kEvalMicro>, dim3(grid), dim3(kTickThreads), 0, st, a); break;
        case kEvalTiny: hipLaunchKernelGGL(tick_kernel<kEvalTiny>, dim3(grid), dim3(kTickThreads), 0, st, a); break;
        case kEvalNarrow: hipLaunchKernelGGL(tick_kernel<kEvalNarrow>, dim3(grid), dim3(kTickThreads), 0, st, a); break;
        default: hipLaunchKernelGGL(tick_kernel<kEvalWide>, dim3(grid), dim3(kTickThreads), 0, st, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_scatter(const CopySeg* segs, int n, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(scatter_kernel, dim3(n), dim3(kTickThreads), 0, st, segs, n);
    return hipGetLastError();
}

}  // namespace ks
