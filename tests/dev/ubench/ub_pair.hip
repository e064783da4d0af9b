// Microbenchmark (diagnostic): fixed cost of the two-pods-per-barrier decision
// against the one-pod iteration skeleton of ub_iter.hip.  Each iteration every wave reads the
// pair's control word (pod i's folded best, the non-candidate maximum of pod i+1, the candidate
// count) and the candidate array lane-parallel (ikey_i, K1, K2 per candidate), takes pod i's
// winner and pod i+1's winner (K2 for the entry that won pod i, K1 for the others) with uniform
// readlane loops, then kFolds waves append one candidate each into the next slot and fold the
// maximum; one barrier.
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-atomic-optimizer-strategy=None ub_pair.hip -o ub_pair
// (the engine's flags: the atomic optimizer would turn each LDS atomic into a readlane loop)
#include <hip/hip_runtime.h>
#include <cstdio>

struct alignas(16) Ctl { unsigned long long best, m2; int cnt, pad[3]; };
struct alignas(8) Cand { unsigned long long ki, k1, k2; };

__device__ __forceinline__ unsigned long long rl64(unsigned long long v, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

template <int kThreads, int kFolds>
__global__ __launch_bounds__(kThreads) void pair(int iters, unsigned long long* out) {
    __shared__ Ctl ctl[3];
    __shared__ Cand cand[3][64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if (tid < 3) ctl[tid] = Ctl{1, 1, 0, {0, 0, 0}};
    __syncthreads();
    unsigned long long acc = 0;
    int it = 0;
    for (; it < iters; ++it) {
        const int s = it % 3;
        const Ctl c = ctl[s];
        if (c.cnt < 0) break;
        const Cand e = lane < c.cnt ? cand[s][lane] : Cand{0, 0, 0};
        unsigned long long w = c.best;
        for (int l = 0; l < c.cnt; ++l) { const unsigned long long k = rl64(e.ki, l); w = k > w ? k : w; }
        const unsigned long long v = (e.ki & 1023u) == (w & 1023u) ? e.k2 : e.k1;
        unsigned long long w1 = c.m2;
        for (int l = 0; l < c.cnt; ++l) { const unsigned long long k = rl64(v, l); w1 = k > w1 ? k : w1; }
        acc += w ^ w1;
        if (wave >= 1 && wave <= kFolds && lane == 0) {
            const int n = atomicAdd(&ctl[(it + 1) % 3].cnt, 1);
            cand[(it + 1) % 3][n & 63] = Cand{acc + wave, acc * 3 + wave, acc * 5 + wave};
            atomicMax(&ctl[(it + 1) % 3].m2, acc + 7 * wave);
        }
        if (wave == 0 && lane == 0) ctl[(it + 2) % 3] = Ctl{1, 1, 0, {0, 0, 0}};
        __syncthreads();
    }
    out[tid] = acc;
}

// the atomics-only decision: one 32-byte control read (best_i, the non-candidate
// maximum M2', MC = max K1 over the candidates, the list candidate's K2), then — for a touched
// winner — its K2 from a per-entry slot; kFolds waves fold best_i, MC and M2' and store a K2
struct alignas(16) CtlA { unsigned long long best, m2, mc, k2l; };
template <int kThreads, int kFolds, bool kPacked = false, bool kLanes = false>
__global__ __launch_bounds__(kThreads) void pair_atomic(int iters, unsigned long long* out) {
    __shared__ CtlA ctl[3];
    __shared__ unsigned long long k2[1024];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if (tid < 3) ctl[tid] = CtlA{1, 1, 1, 1};
    k2[tid] = tid;
    __syncthreads();
    unsigned long long acc = 0;
    for (int it = 0; it < iters; ++it) {
        // both 16-byte halves issued together and pinned (otherwise the compiler reads `best`,
        // branches on it, and only then reads the rest: two dependent LDS round trips)
        const uint4* q = reinterpret_cast<const uint4*>(&ctl[it % 3]);
        const uint4 h0 = q[0], h1 = q[1];
        asm volatile("" ::"v"(h0.x), "v"(h0.y), "v"(h0.z), "v"(h0.w), "v"(h1.x), "v"(h1.y), "v"(h1.z), "v"(h1.w));
        CtlA c;
        __builtin_memcpy(&c, &h0, 16);
        __builtin_memcpy(reinterpret_cast<char*>(&c) + 16, &h1, 16);
        if (c.best == 0) break;
        const int e = (int)(c.best & 1023u);
        // kPacked: the winner's K2 total rides in best_i's low bits (no dependent read)
        const unsigned long long kw = kPacked ? (c.best >> 10) & 0xFFFFu : e == 1023 ? c.k2l : k2[e];
        unsigned long long w1 = c.m2 > kw ? c.m2 : kw;
        const bool mc_is_w = (c.mc & 1023u) == (c.best & 1023u);
        if (!mc_is_w) w1 = c.mc > w1 ? c.mc : w1;
        acc += c.best ^ w1;
        if (kLanes && wave >= 1 && wave <= kFolds && lane < 3) {
            // the three folds as ONE ds_max_u64 over lanes 0..2 (three addresses of the slot)
            const int s = (it + 1) % 3;
            const unsigned long long ent = (unsigned long long)((acc + wave) & 511u);
            const unsigned long long v = lane == 0 ? ((acc + wave) << 10) | ent
                                       : lane == 1 ? ((acc * 3 + wave) << 10) | ent : acc + 7 * wave;
            unsigned long long* dst = lane == 0 ? &ctl[s].best : lane == 1 ? &ctl[s].mc : &ctl[s].m2;
            atomicMax(dst, v);
        } else if (!kLanes && wave >= 1 && wave <= kFolds && lane == 0) {
            const int s = (it + 1) % 3;
            const unsigned long long ent = (unsigned long long)((acc + wave) & 511u);
            atomicMax(&ctl[s].best, ((acc + wave) << 10) | ent);
            atomicMax(&ctl[s].mc, ((acc * 3 + wave) << 10) | ent);
            atomicMax(&ctl[s].m2, acc + 7 * wave);
            k2[ent] = acc * 5 + wave;
        }
        if (wave == 0 && lane == 0) ctl[(it + 2) % 3] = CtlA{1, 1, 1, 1};
        __syncthreads();
    }
    out[tid] = acc;
}

// the one-pod skeleton (as ub_iter.hip) for the side-by-side figure
struct alignas(16) C1 { unsigned long long best; int kfull; int pad; };
template <int kThreads, int kFolds>
__global__ __launch_bounds__(kThreads) void single(int iters, unsigned long long* out) {
    __shared__ C1 ctl[3];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if (tid < 3) ctl[tid] = C1{1, 0, 0};
    __syncthreads();
    unsigned long long acc = 0;
    for (int it = 0; it < iters; ++it) {
        const C1 c = ctl[it % 3];
        if (c.kfull) break;
        acc += c.best;
        if (wave >= 1 && wave <= kFolds && lane == 0) atomicMax(&ctl[(it + 1) % 3].best, acc + wave);
        if (wave == 0 && lane == 0) ctl[(it + 2) % 3] = C1{0, 0, 0};
        __syncthreads();
    }
    out[tid] = acc;
}

template <class K>
void run(const char* name, K kern, int threads, unsigned long long* d, int pods_per_iter) {
    const int iters = 100000;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, 100, d);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, iters, d);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double ns = ms * 1e6 / iters;
    printf("%-44s %8.1f ns/iter %8.1f ns/pod (%5.0f cycles/iter at 2.4 GHz)\n", name, ns, ns / pods_per_iter, ns * 2.4);
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 1024 * 8);
    run("single: 16 waves, 3 folds", single<1024, 3>, 1024, d, 1);
    run("pair:   16 waves, 1 candidate", pair<1024, 1>, 1024, d, 2);
    run("pair:   16 waves, 3 candidates", pair<1024, 3>, 1024, d, 2);
    run("pair:   16 waves, 8 candidates", pair<1024, 8>, 1024, d, 2);
    run("pair, atomics only: 16 waves, 1 candidate", pair_atomic<1024, 1>, 1024, d, 2);
    run("pair, atomics only: 16 waves, 3 candidates", pair_atomic<1024, 3>, 1024, d, 2);
    run("pair, atomics only: 16 waves, 8 candidates", pair_atomic<1024, 8>, 1024, d, 2);
    run("pair, K2 packed in best: 16 waves, 1 candidate", pair_atomic<1024, 1, true>, 1024, d, 2);
    run("pair, K2 packed in best: 16 waves, 3 candidates", pair_atomic<1024, 3, true>, 1024, d, 2);
    run("pair, packed, folds across lanes: 1 cand", pair_atomic<1024, 1, true, true>, 1024, d, 2);
    run("pair, packed, folds across lanes: 3 cands", pair_atomic<1024, 3, true, true>, 1024, d, 2);
    run("single: 8 waves, 3 folds", single<512, 3>, 512, d, 1);
    run("pair:   8 waves, 3 candidates", pair<512, 3>, 512, d, 2);
    return 0;
}
