// ks_kernels.hip — CDNA4 (gfx950) kernels of the kubesim scheduling engine.
//
// The reference schedules one pod per tick (kubesim/kubesim.go:105-121): every pod's
// placement depends on the binds before it.  The engine keeps that order exactly but does
// not pay one full-cluster pass per pod on the critical path.  Per batch of B pods:
//
//   expire_head  applies the expiries due at the batch's first pod (tiny)
//   scan         every (pod, node) pair of the batch against the node state as of the batch
//                start ("snapshot"); per pod and per wave-block of 64 nodes it keeps the best
//                packed key.  Node records are read once per pod group, not once per pod.
//   resolve      one 1024-thread workgroup walks the batch in FIFO order.  Only wave-blocks
//                touched since the snapshot (a bind or an expiry landed in them) can differ
//                from the scan; they are cached in LDS and re-evaluated exactly, every other
//                wave-block's scan key is still exact.  The max over both is the reference's
//                argmax; the admission test and the bind update the LDS cache; the cache is
//                written back at the end.  This is exact, not approximate.
//
// Packed key: (total + 1) << 32 | (0xFFFFFFFF - node); 0 = no candidate (NotFound).
#include "ks_device.h"

namespace ks {

constexpr int kScanWaves = 4;          // 256-thread scan workgroups
constexpr int kResolveThreads = 1024;  // 16 waves
constexpr int kResolveWaves = kResolveThreads / kWave;
constexpr int kMaxTW = 16;             // wave-blocks cached by the resolver
constexpr int kMaxWbPerThread = 16;    // nwb <= 16384 wave-blocks (1,048,576 nodes) per launch
constexpr int kMaxNwb = kMaxWbPerThread * kResolveThreads;
constexpr int kMaxBatch = 512;
constexpr int kMaxExp = 1024;          // expiries prefetched into LDS per batch

enum : int64_t { kCtrStart = 0, kCtrEnd = 1, kCtrErr = 2, kCtrErrPod = 3, kCtrEarly = 4 };
enum : uint32_t { kFlagBadKey = 1, kFlagBadSpec = 2 };
enum : int64_t { kErrEinval = 1, kErrNotFound = 2 };


// ------------------------------------------------------------------------------------------
// expire_head: expiries due at the batch's first pod, applied straight to the node SoA so the
// resolver's first pod never needs cache space for them.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void expire_head_kernel(EngineArgs a) {
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0 || start >= end) return;
    const int64_t e0 = a.exp_off[start], e1 = a.exp_off[start + 1];
    for (int64_t e = e0 + blockIdx.x * blockDim.x + threadIdx.x; e < e1; e += (int64_t)gridDim.x * blockDim.x) {
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
// scan: grid (ceil(nwb / 4), ceil(B / PG)); each wave owns one wave-block (lane = node) and
// evaluates PG pods against it; lane 0 stores the wave-block's best key per pod.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void scan_kernel(EngineArgs a) {
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const int64_t nb = min<int64_t>(a.B, end - start);
    const int pg0 = blockIdx.y * a.PG;
    if (pg0 >= nb) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int wb = blockIdx.x * kScanWaves + (threadIdx.x >> 6);
    if (wb >= a.c.nwb) return;
    const uint32_t base = (uint32_t)wb * kWave;
    const int64_t node = (int64_t)base + lane;
    const NodeV n = load_node(a.s, node);
    const bool valid = node < a.c.n_nodes;
    const int pg1 = (int)min<int64_t>(pg0 + a.PG, nb);
    for (int b = pg0; b < pg1; ++b) {
        const PodRec p = a.pods[start + b];
        const uint32_t t1 = valid ? eval_total1(a.c, p, n) : 0u;
        const uint64_t key = wave_best_key(t1, base);
        if (lane == 0) a.wbkey[(int64_t)b * a.c.nwb + wb] = key;
    }
}

// ------------------------------------------------------------------------------------------
// resolve: one workgroup, sequential over the batch in FIFO order (one bind per tick).
// ------------------------------------------------------------------------------------------
struct ResolveShared {
    int64_t ci[kMaxTW][8][kWave];   // ac am ag ap rc rm rg nr of cached wave-blocks
    uint64_t cu[kMaxTW][2][kWave];  // taint label
    int32_t tw_wb[kMaxTW];
    uint32_t touched[kMaxNwb / 32];
    int32_t lb_node[kMaxBatch];
    int32_t lb_stat[kMaxBatch];
    int32_t ex_off[kMaxBatch + 1];
    int32_t ex_q[kMaxExp];
    int32_t ex_node[kMaxExp];
    int32_t ex_ok[kMaxExp];
    int64_t ex_req[kMaxExp][3];
    uint64_t red[kResolveWaves];
    int32_t tw_count, stop, committed, err_code, err_pod;
};

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Wave 0 only: slot of wave-block wb in the LDS cache, loading it from HBM if needed.
__device__ __forceinline__ int cache_slot(ResolveShared& sh, const EngineArgs& a, int wb, int lane) {
    const int twc = sh.tw_count;
    const bool hit = lane < twc && sh.tw_wb[lane] == wb;
    const uint64_t m = __ballot(hit);
    if (m) return __ffsll((unsigned long long)m) - 1;
    const int slot = twc;
    const int64_t node = (int64_t)wb * kWave + lane;
    const NodeV v = load_node(a.s, node);
    sh.ci[slot][0][lane] = v.ac; sh.ci[slot][1][lane] = v.am;
    sh.ci[slot][2][lane] = v.ag; sh.ci[slot][3][lane] = v.ap;
    sh.ci[slot][4][lane] = v.rc; sh.ci[slot][5][lane] = v.rm;
    sh.ci[slot][6][lane] = v.rg; sh.ci[slot][7][lane] = v.nr;
    sh.cu[slot][0][lane] = v.taint; sh.cu[slot][1][lane] = v.label;
    if (lane == 0) {
        sh.tw_wb[slot] = wb;
        sh.tw_count = twc + 1;
        sh.touched[wb >> 5] |= 1u << (wb & 31);
    }
    lds_fence();
    return slot;
}

__device__ __forceinline__ NodeV cached_node(const ResolveShared& sh, int slot, int l) {
    NodeV v;
    v.ac = sh.ci[slot][0][l]; v.am = sh.ci[slot][1][l]; v.ag = sh.ci[slot][2][l]; v.ap = sh.ci[slot][3][l];
    v.rc = sh.ci[slot][4][l]; v.rm = sh.ci[slot][5][l]; v.rg = sh.ci[slot][6][l]; v.nr = sh.ci[slot][7][l];
    v.taint = sh.cu[slot][0][l]; v.label = sh.cu[slot][1][l];
    return v;
}

__global__ __launch_bounds__(kResolveThreads) void resolve_kernel(EngineArgs a) {
    __shared__ ResolveShared sh;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const int nb = (int)min<int64_t>(a.B, end - start);
    if (nb <= 0) return;
    const int nwb = a.c.nwb;
    const int nper = (nwb + kResolveThreads - 1) / kResolveThreads;
    const int64_t e_base = a.exp_off[start];
    const int64_t e_cnt = a.exp_off[start + nb] - e_base;

    for (int w = tid; w < (nwb + 31) / 32; w += kResolveThreads) sh.touched[w] = 0;
    for (int i = tid; i <= nb; i += kResolveThreads) sh.ex_off[i] = (int32_t)(a.exp_off[start + i] - e_base);
    for (int64_t e = tid; e < e_cnt && e < kMaxExp; e += kResolveThreads) {
        const int32_t q = a.exp_pod[e_base + e];
        sh.ex_q[e] = q;
        const PodRec& pq = a.pods[q];
        sh.ex_req[e][0] = pq.req[0]; sh.ex_req[e][1] = pq.req[1]; sh.ex_req[e][2] = pq.req[2];
        if (q < start) {
            sh.ex_node[e] = a.b_node[q];
            sh.ex_ok[e] = (a.b_status[q] == 0) && !a.expired[q];
        } else {
            sh.ex_node[e] = -1;
            sh.ex_ok[e] = 0;
        }
    }
    if (tid == 0) { sh.tw_count = 0; sh.stop = 0; sh.committed = nb; sh.err_code = 0; sh.err_pod = -1; }

    uint64_t pre[kMaxWbPerThread];
#pragma unroll
    for (int k = 0; k < kMaxWbPerThread; ++k) {
        const int w = tid + k * kResolveThreads;
        pre[k] = (k < nper && w < nwb) ? a.wbkey[w] : 0ull;
    }
    __syncthreads();

    for (int i = 0; i < nb; ++i) {
        const int64_t j = start + i;
        // ---- phase A (wave 0): cache budget, then the expiries due before pod j binds
        if (wave == 0 && i > 0 && !sh.stop) {
            const int e0 = sh.ex_off[i], e1 = sh.ex_off[i + 1];
            if (sh.tw_count + (e1 - e0) + 1 > kMaxTW) {
                if (lane == 0) { sh.stop = 1; sh.committed = i; }
            } else {
                for (int e = e0; e < e1; ++e) {
                    int32_t q, nd, ok;
                    int64_t r0, r1, r2;
                    if (e < kMaxExp) {
                        q = sh.ex_q[e]; r0 = sh.ex_req[e][0]; r1 = sh.ex_req[e][1]; r2 = sh.ex_req[e][2];
                        nd = sh.ex_node[e]; ok = sh.ex_ok[e];
                    } else {  // beyond the prefetch window: read HBM directly
                        q = a.exp_pod[e_base + e];
                        const PodRec& pq = a.pods[q];
                        r0 = pq.req[0]; r1 = pq.req[1]; r2 = pq.req[2];
                        nd = q < start ? a.b_node[q] : -1;
                        ok = q < start ? (a.b_status[q] == 0 && !a.expired[q]) : 0;
                    }
                    if (q >= start) {
                        nd = sh.lb_node[q - start];
                        ok = sh.lb_stat[q - start] == 0;
                    }
                    if (!ok) continue;
                    const int slot = cache_slot(sh, a, nd >> 6, lane);
                    if (lane == 0) {
                        const int l = nd & 63;
                        sh.ci[slot][4][l] -= r0; sh.ci[slot][5][l] -= r1;
                        sh.ci[slot][6][l] -= r2; sh.ci[slot][7][l] -= 1;
                        a.expired[q] = 1;
                    }
                    lds_fence();
                }
            }
        }
        __syncthreads();
        if (sh.stop) break;

        // ---- phase B (all waves): best untouched scan key + exact keys of cached wave-blocks
        const PodRec p = a.pods[j];
        uint64_t best = 0;
#pragma unroll
        for (int k = 0; k < kMaxWbPerThread; ++k) {
            const int w = tid + k * kResolveThreads;
            if (k < nper && w < nwb && !((sh.touched[w >> 5] >> (w & 31)) & 1u)) best = best > pre[k] ? best : pre[k];
        }
        if (i + 1 < nb) {
            const uint64_t* row = a.wbkey + (int64_t)(i + 1) * nwb;
#pragma unroll
            for (int k = 0; k < kMaxWbPerThread; ++k) {
                const int w = tid + k * kResolveThreads;
                if (k < nper && w < nwb) pre[k] = row[w];
            }
        }
        const int twc = sh.tw_count;
        for (int s = wave; s < twc; s += kResolveWaves) {
            const uint32_t base = (uint32_t)sh.tw_wb[s] * kWave;
            const NodeV n = cached_node(sh, s, lane);
            const uint32_t t1 = (base + lane < (uint32_t)a.c.n_nodes) ? eval_total1(a.c, p, n) : 0u;
            const uint64_t key = wave_best_key(t1, base);
            best = best > key ? best : key;
        }
        best = wave_max_u64(best);
        if (lane == 0) sh.red[wave] = best;
        __syncthreads();

        // ---- phase C (wave 0): global argmax, CreatePod admission, bind
        if (wave == 0) {
            uint64_t v = lane < kResolveWaves ? sh.red[lane] : 0ull;
            v = wave_max_u64(v);
            if (v == 0) {
                if (lane == 0) { sh.stop = 1; sh.committed = i; sh.err_code = kErrNotFound; sh.err_pod = (int32_t)j; }
            } else if (p.flags & kFlagBadKey) {
                if (lane == 0) { sh.stop = 1; sh.committed = i; sh.err_code = kErrEinval; sh.err_pod = (int32_t)j; }
            } else {
                const int32_t nd = (int32_t)(0xFFFFFFFFu - (uint32_t)v);
                const int slot = cache_slot(sh, a, nd >> 6, lane);
                const int l = nd & 63;
                const NodeV n = cached_node(sh, slot, l);
                const bool ok = fits(p, n);
                if (p.flags & kFlagBadSpec) {
                    if (lane == 0) { sh.stop = 1; sh.committed = i; sh.err_code = kErrEinval; sh.err_pod = (int32_t)j; }
                } else if (lane == 0) {
                    if (ok && a.dur[j] > 0) {
                        sh.ci[slot][4][l] += p.req[0]; sh.ci[slot][5][l] += p.req[1];
                        sh.ci[slot][6][l] += p.req[2]; sh.ci[slot][7][l] += 1;
                    }
                    sh.lb_node[i] = nd;
                    sh.lb_stat[i] = ok ? 0 : 1;
                    a.b_node[j] = nd;
                    a.b_status[j] = ok ? 0 : 1;
                }
                lds_fence();
            }
        }
        // phase A of the next pod runs on wave 0 too; its barrier publishes this bind.
    }
    __syncthreads();

    // ---- write back the mutable fields of every cached wave-block
    for (int s = wave; s < sh.tw_count; s += kResolveWaves) {
        const int64_t node = (int64_t)sh.tw_wb[s] * kWave + lane;
        a.s.rc[node] = sh.ci[s][4][lane];
        a.s.rm[node] = sh.ci[s][5][lane];
        a.s.rg[node] = sh.ci[s][6][lane];
        a.s.nr[node] = sh.ci[s][7][lane];
    }
    if (tid == 0) {
        a.ctr[kCtrStart] = start + sh.committed;
        if (sh.committed < nb && sh.err_code == 0) a.ctr[kCtrEarly] += 1;
        if (sh.err_code) { a.ctr[kCtrErr] = sh.err_code; a.ctr[kCtrErrPod] = sh.err_pod; }
    }
}

// ------------------------------------------------------------------------------------------
// Filter mask / score of one pod against every node (api.Filter / api.Scorer shims).
// ------------------------------------------------------------------------------------------
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
    const uint32_t t1 = eval_total1(c, p, n);
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
// (kubesim/pod/pod.go:47-63; int32 passed seconds vs int32 cumulative phase seconds).
__global__ __launch_bounds__(256) void usage_kernel(int64_t q_lo, int64_t q_hi, int64_t t, int32_t tick_s,
                                                     const int32_t* b_node, const int32_t* b_status,
                                                     const int64_t* t0, const int32_t* dur, const int32_t* phase_off,
                                                     const int32_t* cum_sec, const int64_t* use,
                                                     unsigned long long* usage) {
    for (int64_t q = q_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < q_hi;
         q += (int64_t)gridDim.x * blockDim.x) {
        if (b_status[q] != 0) continue;
        const int64_t dt = t - t0[q];
        if (dt < 0 || dt >= dur[q]) continue;
        const int32_t passed = (int32_t)(dt * tick_s);
        for (int32_t f = phase_off[q]; f < phase_off[q + 1]; ++f) {
            if (passed < cum_sec[f]) {
                const int32_t nd = b_node[q];
                atomicAdd(&usage[nd * 3 + 0], (unsigned long long)use[(int64_t)f * 3 + 0]);
                atomicAdd(&usage[nd * 3 + 1], (unsigned long long)use[(int64_t)f * 3 + 1]);
                atomicAdd(&usage[nd * 3 + 2], (unsigned long long)use[(int64_t)f * 3 + 2]);
                break;
            }
        }
    }
}

}  // namespace ks

// ---------------------------------------------------------------------------------------------
// Launchers (host side of this translation unit), called by ks_engine.cpp.
// ---------------------------------------------------------------------------------------------
namespace ks {
hipError_t launch_batch(const EngineArgs& a, hipStream_t st, hipEvent_t e_scan0, hipEvent_t e_scan1,
                        hipEvent_t e_res1) {
    hipLaunchKernelGGL(expire_head_kernel, dim3(1), dim3(256), 0, st, a);
    if (e_scan0) (void)hipEventRecord(e_scan0, st);
    dim3 g((a.c.nwb + kScanWaves - 1) / kScanWaves, (a.B + a.PG - 1) / a.PG);
    hipLaunchKernelGGL(scan_kernel, g, dim3(kScanWaves * kWave), 0, st, a);
    if (e_scan1) (void)hipEventRecord(e_scan1, st);
    hipLaunchKernelGGL(resolve_kernel, dim3(1), dim3(kResolveThreads), 0, st, a);
    if (e_res1) (void)hipEventRecord(e_res1, st);
    return hipGetLastError();
}

hipError_t launch_eval_pod(const Cfg& c, const NodeSoA& s, const PodRec* pod, uint32_t filters, uint8_t* mask,
                           int64_t* score, hipStream_t st) {
    hipLaunchKernelGGL(eval_pod_kernel, dim3((c.n_nodes + 255) / 256), dim3(256), 0, st, c, s, pod, filters, mask, score);
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

hipError_t launch_usage(int64_t q_lo, int64_t q_hi, int64_t t, int32_t tick_s, const int32_t* b_node,
                        const int32_t* b_status, const int64_t* t0, const int32_t* dur, const int32_t* phase_off,
                        const int32_t* cum_sec, const int64_t* use, unsigned long long* usage, hipStream_t st) {
    if (q_hi <= q_lo) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((q_hi - q_lo + 255) / 256, 2048);
    hipLaunchKernelGGL(usage_kernel, dim3((unsigned)blocks), dim3(256), 0, st, q_lo, q_hi, t, tick_s, b_node, b_status,
                       t0, dur, phase_off, cum_sec, use, usage);
    return hipGetLastError();
}
}  // namespace ks
