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
#ifndef KS_SCAN_UNROLL
#define KS_SCAN_UNROLL 4
#endif
constexpr int kUnroll = KS_SCAN_UNROLL;  // pods evaluated together per loop step

__device__ __forceinline__ int popc_below(uint64_t mask, int lane) { return __popcll(mask & ((1ull << lane) - 1ull)); }

// Item `it` (= node block * groups + pod group) of the batch [start, start + nb) on the 256
// threads lt = 0..255 of one group; kv: the group's [PG][256] table.  has == false: this group has
// no item this round — it only takes part in the workgroup barrier (one, between the evaluation
// and the extraction; the caller separates items by another).
// excl (nullable): nodes with excl[n] >= 0 are left out of the lists (the overlap's speculative
// scan: the current batch's candidate slots, which join the next batch's E instead)
//
// Pruned lists (a.lbit != nullptr, large clusters): per pod a threshold key = the 8th key of some
// full block list written earlier in this scan.  At least L keys of the snapshot reach it, so a key
// below it is in no pod's global top-L: a block writes only its keys >= the threshold it read (a
// prefix of its sorted top-L) and, if any, sets its bit in the pod's bitmap lbit[pod][blk / 64];
// the merge reads only the flagged blocks.  Any such key is a valid threshold, however stale, so
// the thresholds are plain words — one copy per workgroup group `copy` (= the XCD under round-robin
// dispatch; a hot word shared by every workgroup of the chip serialises its atomics: measured C5
// scan 0.33 -> 0.46 ms with one atomicMax word per pod), updated by a plain store when a block's
// 8th key beats the value it read.  Most blocks of a large cluster then write nothing: the ties of
// the top class go to the lowest node indices, which the first blocks of each XCD's range hold.
// kPrune: the pruned form (the engine's a.lbit is set); the plain form is compiled without it.
// kLL: the list length (kTopL, or kTopLOverlap for the overlap's single-shard engines)
template <int kMode, typename KT, bool kPrune, int kLL = kTopL>
__device__ __forceinline__ void scan_item(const EngineArgs& a, KT* kv, int64_t start, int64_t nb, int groups, int64_t it,
                                          bool has, int lt, int copy, const int32_t* excl = nullptr) {
    const int lane = lt & (kWave - 1), wave = lt >> 6;
    int pg0 = 0, np = 0, blk = 0;
    uint32_t blk_base = 0;
    constexpr bool prune = kPrune;
    uint64_t thr_l = 0;  // lane j < PG / 4: the threshold of this wave's j-th pod (loaded early)
    if (has) {
        const int bx = (int)(it / groups);
        pg0 = (int)(it - (int64_t)bx * groups) * a.PG;
        blk = a.blk_lo + bx;
        blk_base = (uint32_t)blk * kNodes;
        np = (int)min<int64_t>(a.PG, nb - pg0);
        if constexpr (prune) {  // issued before the evaluation: its latency hides under it
            const int b = wave + kWaves * lane;
            if (b < np)
                thr_l = *lthr_of(a, a.lset, copy, pg0 + b);
        }
        const int64_t node = (int64_t)blk_base + lt;
        bool valid = node < a.c.n_nodes;
        NodeV n{};
        if (node < (int64_t)a.c.nwb * kWave) n = load_node(a.s, node);
        if (excl && valid && excl[node] >= 0) valid = false;
        int b = 0;
        if constexpr (kMode == kEvalMicro) {  // the scan records (ks_device.h eval_scan_micro)
            const ScanRec* sp = a.srec + start + pg0;
            const int32_t npen = scan_npen(a.c, n);
            for (; b + kUnroll <= np; b += kUnroll) {
                ScanRec p[kUnroll];
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) p[u] = sload(sp + b + u);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const uint32_t t = eval_scan_micro(a.c, p[u], n, npen);
                    kv[(b + u) * kNodes + lt] = (KT)(valid ? t : 0u);
                }
            }
            for (; b < np; ++b) {
                const ScanRec p = sload(sp + b);
                const uint32_t t = eval_scan_micro(a.c, p, n, npen);
                kv[b * kNodes + lt] = (KT)(valid ? t : 0u);
            }
        } else {
            const PodRec* pp = a.pods + start + pg0;
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
    }
    __syncthreads();
    if (!has) return;
    // one wave per pod: score tie classes from the top — a lane max of 4, a 32-bit wave max and
    // four ballots per class, ranks by popcount
    for (int b = wave, j = 0; b < np; b += kWaves, ++j) {
        uint32_t v[kWaves];
#pragma unroll
        for (int u = 0; u < kWaves; ++u) v[u] = (uint32_t)kv[b * kNodes + u * kWave + lane];  // node u*64 + lane
        auto out = gptr(a.lists) + ((int64_t)(pg0 + b) * a.nblk + blk) * kLL;  // global_: not in lgkmcnt
        uint64_t thr = 0;
        if constexpr (prune) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)thr_l, j);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(thr_l >> 32), j);
            thr = ((uint64_t)hi << 32) | lo;
        }
        int cnt = 0, cq = 0;  // ranked entries; of them the ones >= thr (a prefix)
        for (int r = 0; r < kLL && cnt < kLL; ++r) {
            uint32_t lm = v[0];
#pragma unroll
            for (int u = 1; u < kWaves; ++u) lm = lm > v[u] ? lm : v[u];
            const uint32_t m = wave_max_u32(lm);
            if (m == 0) break;
            // the class's best key here is its lowest node's, >= the block's first: if that is below thr,
            // so is this class and every class after it
            if (prune && (((uint64_t)m << 32) | (uint64_t)(0xFFFFFFFFu - blk_base)) < thr) break;
            int below = cnt;  // nodes of this class before (u, lane) in node order
#pragma unroll
            for (int u = 0; u < kWaves; ++u) {
                const uint64_t mask = __ballot(v[u] == m);
                bool w = false;
                if (v[u] == m) {
                    const int rank = below + popc_below(mask, lane);
                    const uint64_t key = make_key(m, blk_base + u * kWave + lane);
                    w = rank < kLL && (!prune || key >= thr);
                    if (w) out[rank] = key;
                    // a full list: its 8th key is a threshold for every later block (fire and forget)
                    if (prune && w && rank == kLL - 1 && key > thr) *lthr_of(a, a.lset, copy, pg0 + b) = key;
                    v[u] = 0;
                }
                if constexpr (prune) cq += __popcll(__ballot(w));
                below += __popcll(mask);
            }
            cnt = below;
        }
        if constexpr (!prune) {
            if (lane >= cnt && lane < kLL) out[lane] = 0ull;
        } else if (cq > 0) {
            if (lane >= cq && lane < kLL) out[lane] = 0ull;
            if (lane == 0)
                atomicOr((unsigned long long*)(lbit_of(a, a.lset, pg0 + b) + (blk >> 6)), 1ull << (blk & 63));
        }
    }
}

// ---- the merge side of the pruned lists ------------------------------------------------------
// The flagged blocks of one pod among blocks [blk0, blk0 + nl), numbered in block order: after
// flagged_index, flagged_block(j, ...) is the j-th one (0 <= j < the returned count).  One
// workgroup; `bits` = the pod's bitmap words; LDS: wds[kFlagMaxW], pre[kFlagMaxW + 1].
constexpr int kFlagMaxW = 1024;  // bitmap words per pod: 65,536 blocks (2^24 nodes)
struct FlagLDS {
    uint64_t wds[kFlagMaxW];
    int32_t pre[kFlagMaxW + 1];
    int32_t wsum[16];
};

__device__ __forceinline__ int select_bit(uint64_t x, int r) {  // the r-th set bit of x (r < popc(x))
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t lo = x & ((1ull << w) - 1ull);
        const int c = __popcll(lo);
        if (r >= c) { r -= c; x >>= w; pos += w; }
        else x = lo;
    }
    return pos;
}

// Loads and indexes the flagged words (one barrier-separated prefix); returns the flagged count.
__device__ __forceinline__ int flagged_index(const uint64_t* bits, int blk0, int nl, FlagLDS& F) {
    const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63, wv = tid >> 6;
    if (nl <= 0) return 0;
    const int w0 = blk0 >> 6, w1 = (blk0 + nl - 1) >> 6, nw = w1 - w0 + 1;
    // thread t: words [t k, t k + k) — consecutive, so one prefix pass covers them
    const int k = (nw + nthr - 1) / nthr;
    int mine = 0;
    for (int q = 0; q < k; ++q) {
        const int w = tid * k + q;
        if (w >= nw) break;
        uint64_t x = bits[w0 + w];
        if (w == 0) x &= ~0ull << (blk0 & 63);
        if (w == nw - 1 && ((blk0 + nl) & 63)) x &= (1ull << ((blk0 + nl) & 63)) - 1ull;
        F.wds[w] = x;
        mine += __popcll(x);
    }
    int incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
    }
    if (lane == 63) F.wsum[wv] = incl;
    __syncthreads();
    int base = 0;
    for (int g = 0; g < wv; ++g) base += F.wsum[g];
    int run = base + incl - mine;
    for (int q = 0; q < k; ++q) {
        const int w = tid * k + q;
        if (w >= nw) break;
        F.pre[w] = run;
        run += __popcll(F.wds[w]);
    }
    int total = 0;
    for (int g = 0; g < nthr / 64; ++g) total += F.wsum[g];
    if (tid == 0) F.pre[nw] = total;
    __syncthreads();
    return total;
}

// the j-th flagged block's list index (block - blk0)
__device__ __forceinline__ int flagged_block(int j, int blk0, int nl, const FlagLDS& F) {
    const int w0 = blk0 >> 6, nw = ((blk0 + nl - 1) >> 6) - w0 + 1;
    int lo = 0, hi = nw - 1;  // the word w with pre[w] <= j < pre[w + 1]
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (F.pre[mid] <= j) lo = mid;
        else hi = mid - 1;
    }
    return (w0 + lo) * 64 + select_bit(F.wds[lo], j - F.pre[lo]) - blk0;
}

}  // namespace scn
}  // namespace ks
