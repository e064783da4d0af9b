// ks_scan.h — one item of the scan (gfx950): a 256-node block against a group of <= PG pods.
//
// Shared by the scan kernel (ks_kernels.hip: one item per 256-thread workgroup) and the chunk
// kernel's fused form (ks_chunk.hip: 512-thread workgroups beside the resolver, two items at a
// time, one per half).  The snapshot key of every (pod, node) pair — fused Filter + Score,
// kubesim/kubesim.go:168-215 restated in ks_device.h — goes into an LDS table of total+1 words,
// then one wave per pod extracts the block's exact top-L (L = kTopL) to the block list.
#pragma once
#include "ks_device.h"

namespace ks {
namespace scn {

constexpr int kWaves = 4;               // a group of four waves: one node per thread
constexpr int kNodes = kWaves * kWave;  // 256
constexpr int kL = kTopL;
constexpr int kUnroll = 4;              // pods evaluated together per loop step

__device__ __forceinline__ int popc_below(uint64_t mask, int lane) { return __popcll(mask & ((1ull << lane) - 1ull)); }

// Item `it` (= node block * groups + pod group) of the batch [start, start + nb) on the 256
// threads lt = 0..255 of one group; kv: the group's [PG][256] table.  has == false: this group has
// no item this round — it only takes part in the workgroup barrier (one, between the evaluation
// and the extraction; the caller separates items by another).
// excl (nullable): nodes with excl[n] >= 0 are left out of the lists (the overlap's speculative
// scan: the current batch's candidate slots, which join the next batch's E instead)
template <int kMode, typename KT>
__device__ __forceinline__ void scan_item(const EngineArgs& a, KT* kv, int64_t start, int64_t nb, int groups, int64_t it,
                                          bool has, int lt, const int32_t* excl = nullptr) {
    const int lane = lt & (kWave - 1), wave = lt >> 6;
    int pg0 = 0, np = 0, blk = 0;
    uint32_t blk_base = 0;
    if (has) {
        const int bx = (int)(it / groups);
        pg0 = (int)(it - (int64_t)bx * groups) * a.PG;
        blk = a.blk_lo + bx;
        blk_base = (uint32_t)blk * kNodes;
        const int64_t node = (int64_t)blk_base + lt;
        bool valid = node < a.c.n_nodes;
        NodeV n{};
        if (node < (int64_t)a.c.nwb * kWave) n = load_node(a.s, node);
        if (excl && valid && excl[node] >= 0) valid = false;
        np = (int)min<int64_t>(a.PG, nb - pg0);
        const PodRec* pp = a.pods + start + pg0;
        int b = 0;
        // kUnroll pods at a time: their scalar loads share one wait and the independent
        // evaluations interleave (instruction-level parallelism within the wave)
        for (; b + kUnroll <= np; b += kUnroll) {
            PodRec p[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) p[u] = sload(pp + b + u);  // uniform: SGPRs, scalar cache
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t t = eval_t<kMode>(a.c, p[u], n);  // branch-free; padding lanes discarded
                kv[(b + u) * kNodes + lt] = (KT)(valid ? t : 0u);
            }
        }
        for (; b < np; ++b) {
            const PodRec p = sload(pp + b);
            const uint32_t t = eval_t<kMode>(a.c, p, n);
            kv[b * kNodes + lt] = (KT)(valid ? t : 0u);
        }
    }
    __syncthreads();
    if (!has) return;
    // one wave per pod: score tie classes from the top — a lane max of 4, a 32-bit wave max and
    // four ballots per class, ranks by popcount
    for (int b = wave; b < np; b += kWaves) {
        uint32_t v[kWaves];
#pragma unroll
        for (int u = 0; u < kWaves; ++u) v[u] = (uint32_t)kv[b * kNodes + u * kWave + lane];  // node u*64 + lane
        auto out = gptr(a.lists) + ((int64_t)(pg0 + b) * a.nblk + blk) * kL;  // global_: not in lgkmcnt
        int cnt = 0;
        for (int r = 0; r < kL && cnt < kL; ++r) {
            uint32_t lm = v[0];
#pragma unroll
            for (int u = 1; u < kWaves; ++u) lm = lm > v[u] ? lm : v[u];
            const uint32_t m = wave_max_u32(lm);
            if (m == 0) break;
            int below = cnt;  // nodes of this class before (u, lane) in node order
#pragma unroll
            for (int u = 0; u < kWaves; ++u) {
                const uint64_t mask = __ballot(v[u] == m);
                if (v[u] == m) {
                    const int rank = below + popc_below(mask, lane);
                    if (rank < kL) out[rank] = make_key(m, blk_base + u * kWave + lane);
                    v[u] = 0;
                }
                below += __popcll(mask);
            }
            cnt = below;
        }
        if (lane >= cnt && lane < kL) out[lane] = 0ull;
    }
}

}  // namespace scn
}  // namespace ks
