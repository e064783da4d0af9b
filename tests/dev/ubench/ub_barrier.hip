// Microbenchmark (diagnostic): cost of one resolver-like iteration skeleton on gfx950.
// 1024 threads, one barrier per iteration; variant adds k dependent LDS round trips per wave,
// an LDS atomic max, or VALU work.  Prints ns/iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int kReads, int kValu, bool kAtomic, int kWaves>
__global__ __launch_bounds__(1024) void k(int iters, unsigned long long* out) {
    __shared__ unsigned long long buf[4096];
    __shared__ unsigned long long best[4];
    const int tid = threadIdx.x;
    for (int i = tid; i < 4096; i += blockDim.x) buf[i] = i * 7;
    if (tid < 4) best[tid] = 0;
    __syncthreads();
    unsigned long long acc = tid;
    const int wave = tid >> 6;
    for (int it = 0; it < iters; ++it) {
        if (wave < kWaves) {
            unsigned idx = (unsigned)(acc + it) & 4095u;
#pragma unroll
            for (int r = 0; r < kReads; ++r) idx = (unsigned)(buf[idx] + r) & 4095u;  // dependent chain
            unsigned v = idx;
#pragma unroll
            for (int q = 0; q < kValu; ++q) v = v * 1664525u + 1013904223u;
            acc += v;
            if (kAtomic && (tid & 63) == 0) atomicMax(&best[it & 3], acc);
        }
        __syncthreads();
    }
    out[tid] = acc + best[0];
}

template <int R, int V, bool A, int W>
void run(const char* name, unsigned long long* d) {
    const int iters = 100000;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((k<R, V, A, W>), dim3(1), dim3(1024), 0, 0, 100, d);
    hipEventRecord(a);
    hipLaunchKernelGGL((k<R, V, A, W>), dim3(1), dim3(1024), 0, 0, iters, d);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-40s %8.1f ns/iter\n", name, ms * 1e6 / iters);
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 1024 * 8);
    run<0, 0, false, 16>("barrier only", d);
    run<1, 0, false, 16>("1 LDS round trip x16 waves", d);
    run<3, 0, false, 16>("3 LDS round trips x16 waves", d);
    run<6, 0, false, 16>("6 LDS round trips x16 waves", d);
    run<3, 0, false, 1>("3 LDS round trips x1 wave", d);
    run<0, 0, true, 16>("LDS atomic x16 waves", d);
    run<0, 100, false, 16>("100 dependent VALU x16 waves", d);
    run<0, 100, false, 4>("100 dependent VALU x4 waves", d);
    run<0, 100, false, 1>("100 dependent VALU x1 wave", d);
    run<0, 400, false, 16>("400 dependent VALU x16 waves", d);
    run<0, 400, false, 1>("400 dependent VALU x1 wave", d);
    run<3, 100, true, 16>("3 LDS + 100 VALU + atomic x16", d);
    return 0;
}
