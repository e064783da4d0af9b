// Microbenchmark (diagnostic): the floor of a resolver whose per-pod chain runs in ONE wave with
// no barrier — read the winner's state from LDS (index from the previous iteration's key), the
// CreatePod admission + bind, write the state back, the micro evaluator for the next pod on the
// bound state, the key.  Variants add busy waves (VALU loops) on the other SIMDs / the same SIMD
// to see what sharing costs.   hipcc -O3 --offload-arch=gfx950 ub_chain.hip -o ub_chain
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../../kubernetes-simulator_amd/csrc/ks_device.h"

using namespace ks;

// the micro evaluator's per-node invariants carried by the state (as the register-table
// resolver's NodeM does): found by overload, so eval_total1_micro skips 2 v_rcp + a multiply
struct NodeC : NodeV {
    float ic, im;
    int32_t d;
};
__device__ __forceinline__ float micro_ic(const NodeC& n, int32_t) { return n.ic; }
__device__ __forceinline__ float micro_im(const NodeC& n, int32_t) { return n.im; }
__device__ __forceinline__ int32_t micro_d(const NodeC& n, int32_t, int32_t) { return n.d; }

// kVar: 0 the whole chain; 1 without the evaluator (key from the state); 2 the evaluator alone
// (state kept in registers, no LDS round trip); 3 as 2 with the invariants cached (NodeC);
// 4 as 2 with a different state in every lane (vector code, as the resolver's waves run it)
template <int kThreads, int kVar>
__global__ __launch_bounds__(kThreads) void chain(int iters, Cfg c, const PodRec* gp, const NodeV* gn,
                                                  unsigned long long* out, int* stop) {
    __shared__ PodRec pods[256];
    __shared__ int64_t tab[8][256];
    __shared__ uint64_t tu[2][256];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int i = tid; i < 256; i += kThreads) {
        pods[i] = gp[i];
        const NodeV v = gn[i];
        tab[0][i] = v.ac; tab[1][i] = v.am; tab[2][i] = v.ag; tab[3][i] = v.ap;
        tab[4][i] = v.rc; tab[5][i] = v.rm; tab[6][i] = v.rg; tab[7][i] = v.nr;
        tu[0][i] = v.taint; tu[1][i] = v.label;
    }
    __syncthreads();
    if (wave != 0) {  // busy waves: dependent VALU work until wave 0 is done
        float x = (float)tid;
        int n = 0;
        // the flag is polled every 4,096 dependent FMAs (its load would otherwise idle the wave)
        while (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 && n < (1 << 22)) {
            for (int r = 0; r < 64; ++r) {
#pragma unroll
                for (int k = 0; k < 64; ++k) x = fmaf(x, 1.0001f, 0.5f);
            }
            ++n;
        }
        out[tid] = (unsigned long long)x;
        return;
    }
    uint64_t key = 0;
    NodeV r;
    r.ac = tab[0][0]; r.am = tab[1][0]; r.ag = tab[2][0]; r.ap = tab[3][0];
    r.rc = tab[4][0]; r.rm = tab[5][0]; r.rg = tab[6][0]; r.nr = tab[7][0];
    r.taint = tu[0][0]; r.label = tu[1][0];
    const float ic0 = rcp_est((float)(r.ac > 0 ? r.ac : 1)), im0 = rcp_est((float)(r.am > 0 ? r.am : 1));
    for (int it = 0; it < iters; ++it) {
        const int t = (int)(key & 255u) ^ (it & 255);
        const PodRec p = pods[it & 255], pn = pods[(it + 1) & 255];
        if (kVar == 2) {
            r.rc = (r.rc + (int64_t)(key & 7)) & 1023;  // a dependence on the previous key
            key = make_key(eval_t<kEvalMicro>(c, pn, r), (uint32_t)t);
            continue;
        }
        if (kVar == 4) {
            r.rc = (r.rc + (int64_t)(key & 7) + lane) & 1023;  // per-lane state: no scalarization
            key = make_key(eval_t<kEvalMicro>(c, pn, r), (uint32_t)t);
            key = (uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)key) | (key & 0xFFFFFFFF00000000ull);
            continue;
        }
        if (kVar == 3) {
            NodeC rc;
            static_cast<NodeV&>(rc) = r;
            rc.rc = (r.rc + (int64_t)(key & 7)) & 1023;
            r.rc = rc.rc;
            const int32_t acs = rc.ac > 0 ? (int32_t)rc.ac : 1, ams = rc.am > 0 ? (int32_t)rc.am : 1;
            rc.ic = ic0; rc.im = im0; rc.d = mul24(acs, ams);
            key = make_key(eval_t<kEvalMicro>(c, pn, rc), (uint32_t)t);
            continue;
        }
        NodeV n;
        n.ac = tab[0][t]; n.am = tab[1][t]; n.ag = tab[2][t]; n.ap = tab[3][t];
        n.rc = tab[4][t]; n.rm = tab[5][t]; n.rg = tab[6][t]; n.nr = tab[7][t];
        n.taint = tu[0][t]; n.label = tu[1][t];
        const bool ok = fits(p, n);
        if (ok) { n.rc += p.req[0]; n.rm += p.req[1]; n.rg += p.req[2]; n.nr += 1; }
        if (n.nr > 100) { n.rc = 0; n.rm = 0; n.rg = 0; n.nr = 0; }  // keep the state bounded
        if (lane == 0) { tab[4][t] = n.rc; tab[5][t] = n.rm; tab[6][t] = n.rg; tab[7][t] = n.nr; }
        key = kVar == 1 ? (uint64_t)(n.rc ^ n.nr) : make_key(eval_t<kEvalMicro>(c, pn, n), (uint32_t)t);
    }
    if (lane == 0) {
        out[0] = key;
        __hip_atomic_store(stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int T, int V = 0>
void run(const char* name, Cfg c, const PodRec* p, const NodeV* n, unsigned long long* d, int* stop) {
    const int iters = 200000;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipMemset(stop, 0, 4);
    hipLaunchKernelGGL((chain<T, V>), dim3(1), dim3(T), 0, 0, 1000, c, p, n, d, stop);
    hipMemset(stop, 0, 4);
    hipEventRecord(a);
    hipLaunchKernelGGL((chain<T, V>), dim3(1), dim3(T), 0, 0, iters, c, p, n, d, stop);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-44s %8.1f ns/iter (%6.0f cycles at 2.4 GHz)\n", name, ms * 1e6 / iters, ms * 1e6 / iters * 2.4);
}

int main() {
    PodRec hp[256];
    NodeV hn[256];
    for (int i = 0; i < 256; ++i) {
        hp[i] = PodRec{{100 + i % 7 * 50, 200 + i % 5 * 100, 0}, ~0ull, 0ull, 3u, 0u};
        hn[i] = NodeV{4000 + i % 3 * 1000, 8000 + i % 4 * 1000, 0, 110, i % 9 * 100, i % 11 * 200, 0, i % 5, 0ull, 0ull};
    }
    PodRec* p; NodeV* n; unsigned long long* d; int* stop;
    hipMalloc(&p, sizeof(hp)); hipMalloc(&n, sizeof(hn)); hipMalloc(&d, 1024 * 8); hipMalloc(&stop, 4);
    hipMemcpy(p, hp, sizeof(hp), hipMemcpyHostToDevice);
    hipMemcpy(n, hn, sizeof(hn), hipMemcpyHostToDevice);
    Cfg c{};
    c.n_nodes = 256; c.nwb = 4; c.filter_feeds = 1; c.filters = 7; c.has_scorers = 1; c.w_lr = 1; c.w_ba = 1;
    c.const_total = 0; c.tick_seconds = 10;
    run<64>("1 wave (alone)", c, p, n, d, stop);
    run<256>("1 wave + 3 busy waves (other SIMDs)", c, p, n, d, stop);
    run<512>("1 wave + 7 busy waves (1 shares its SIMD)", c, p, n, d, stop);
    run<1024>("1 wave + 15 busy waves (3 share its SIMD)", c, p, n, d, stop);
    run<64, 1>("1 wave: LDS state + admission, no evaluator", c, p, n, d, stop);
    run<64, 2>("1 wave: evaluator alone (registers)", c, p, n, d, stop);
    run<64, 3>("1 wave: evaluator alone, invariants cached", c, p, n, d, stop);
    run<64, 4>("1 wave: evaluator alone, per-lane state", c, p, n, d, stop);
    return 0;
}
