// Microbenchmark (diagnostic): fixed cost of one resolver iteration skeleton vs workgroup size.
// Each iteration: every wave reads a 32-byte control word from LDS, branches on it (uniform), one
// lane of wave 1 folds an atomic max into the next slot, then a workgroup barrier.
#include <hip/hip_runtime.h>
#include <cstdio>

struct alignas(16) C { unsigned long long best; int kfull; int pad; };

template <int kThreads, int kFolds>
__global__ __launch_bounds__(kThreads) void k(int iters, unsigned long long* out) {
    __shared__ C ctl[3];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if (tid < 3) ctl[tid] = C{1, 0, 0};
    __syncthreads();
    unsigned long long acc = 0;
    int it = 0;
    for (; it < iters; ++it) {
        const C c = ctl[it % 3];
        if (c.kfull) break;
        acc += c.best;
        if (wave >= 1 && wave <= kFolds && lane == 0) atomicMax(&ctl[(it + 1) % 3].best, acc + wave);
        if (wave == 0 && lane == 0) ctl[(it + 2) % 3] = C{0, 0, 0};
        __syncthreads();
    }
    out[tid] = acc;
}

template <int T, int F>
void run(const char* name, unsigned long long* d) {
    const int iters = 100000;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((k<T, F>), dim3(1), dim3(T), 0, 0, 100, d);
    hipEventRecord(a);
    hipLaunchKernelGGL((k<T, F>), dim3(1), dim3(T), 0, 0, iters, d);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-36s %8.1f ns/iter\n", name, ms * 1e6 / iters);
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 1024 * 8);
    run<256, 1>("4 waves, 1 fold", d);
    run<512, 1>("8 waves, 1 fold", d);
    run<1024, 1>("16 waves, 1 fold", d);
    run<1024, 3>("16 waves, 3 folds", d);
    run<1024, 8>("16 waves, 8 folds", d);
    run<256, 3>("4 waves, 3 folds", d);
    return 0;
}
