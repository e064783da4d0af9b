// ks_kernels.hip — CDNA4 (gfx950) kernels of the kubesim scheduling engine.
//
// The reference schedules one pod per tick (kubesim/kubesim.go:105-121) and every placement
// depends on the binds before it.  The engine keeps that order exactly, but only a tiny part
// of each pod's decision is sequential.  Per batch of B pods:
//
//   expire_head  applies the expiries due before the batch's first pod.
//   scan         evaluates every (pod, node) pair of the batch against the node state as of
//                the batch start (the "snapshot"): fused Filter + Score + packed key.  Node
//                records are read once per pod group; per pod and per 256-node block it keeps
//                the exact top-L keys.
//   merge        per pod: exact global top-L keys of the snapshot (sorted).
//   resolve      one 1024-thread workgroup walks the batch in FIFO order.  A node's key can
//                differ from the snapshot only if the node was touched in this batch (a bind
//                or an expiry landed on it).  Touched nodes live in an LDS table and are
//                re-evaluated exactly for every pod; the best untouched node is the first
//                untouched entry of the pod's top-L list — exact because any node outside the
//                list scores below every list entry.  winner = max(those).  If all L entries
//                are touched the batch commits early and the next batch rescans.
//
// Every kernel that evaluates exists twice: kNarrow = true is the 32-bit evaluator, used when
// every scaled capacity fits (ks_device.h); kNarrow = false the general 64/128-bit one.
//
// Packed key: (total + 1) << 32 | (0xFFFFFFFF - node); 0 = no candidate (NotFound).  Max key =
// highest total, ties to the lowest node index.
#include "ks_device.h"

namespace ks {

constexpr int kScanWaves = 4;            // 256-thread scan workgroups, one 256-node block each
constexpr int kBlockNodes = kScanWaves * kWave;
constexpr int kL = kTopL;                // candidate list length per pod
constexpr int kMaxPG = 32;               // pods per scan workgroup (LDS list staging)
constexpr int kResolveThreads = 1024;    // 16 waves
constexpr int kResolveWaves = kResolveThreads / kWave;
constexpr int kOwnerWave0 = 3;           // waves 3..15 own the touched entries
constexpr int kOwners = kResolveThreads - kOwnerWave0 * kWave;
constexpr int kTMax = 768;               // touched-node table (LDS); <= kOwners
constexpr int kHash = 2048;              // open-addressing node -> entry map (LDS)
constexpr int kMaxBatchR = 256;          // pods per resolve launch
constexpr int kMaxExp = kTMax - kMaxBatchR;  // expiries pre-inserted per batch
constexpr int kFilterBits = 1 << 16;     // touched filter indexed by node & 0xFFFF (no false
                                         // negatives; exact below 65,536 nodes)
static_assert(kTMax <= kOwners, "one touched entry per owner thread");

enum : int64_t { kCtrStart = 0, kCtrEnd = 1, kCtrErr = 2, kCtrErrPod = 3, kCtrEarly = 4 };
enum : uint32_t { kFlagBadKey = 1, kFlagBadSpec = 2 };
enum : int64_t { kErrEinval = 1, kErrNotFound = 2 };

__device__ __forceinline__ int popc_below(uint64_t mask, int lane) {
    return __popcll(mask & ((1ull << lane) - 1ull));
}

// ------------------------------------------------------------------------------------------
// expire_head: expiries due before the batch's first pod, applied straight to the node SoA.
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
// scan: grid (nblk, ceil(B / PG)).  Each wave owns 64 nodes (lane = node); for each of the
// workgroup's PG pods it extracts its exact top-L keys.  Scores are small integers, so the
// top-L of a wave is usually one or two "tie classes": take the max score, every lane at it
// (lowest lanes first), repeat below it — a 32-bit wave max + ballot per class.  The four
// wave lists are then merged by rank (each list is sorted) into the block's top-L.
// ------------------------------------------------------------------------------------------
template <bool kNarrow>
__global__ __launch_bounds__(256) void scan_kernel(EngineArgs a) {
    __shared__ uint64_t wl[kMaxPG][kScanWaves][kL];  // per-pod, per-wave top-L lists
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const int64_t nb = min<int64_t>(a.B, end - start);
    const int pg0 = blockIdx.y * a.PG;
    if (pg0 >= nb) return;
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
    const int blk = blockIdx.x;
    const uint32_t base = (uint32_t)blk * kBlockNodes + wave * kWave;
    const int64_t node = (int64_t)base + lane;
    const bool valid = node < a.c.n_nodes;
    NodeV n{};
    if (node < (int64_t)a.c.nwb * kWave) n = load_node(a.s, node);
    const int np = (int)min<int64_t>(a.PG, nb - pg0);
    for (int b = 0; b < np; ++b) {
        const PodRec p = a.pods[start + pg0 + b];
        uint32_t rem = valid ? eval_t<kNarrow>(a.c, p, n) : 0u;
        int cnt = 0;
        for (int r = 0; r < kL && cnt < kL; ++r) {
            const uint32_t m = wave_max_u32(rem);
            if (m == 0) break;
            const uint64_t mask = __ballot(rem == m);
            if (rem == m) {
                const int rank = cnt + popc_below(mask, lane);
                if (rank < kL) wl[b][wave][rank] = make_key(m, base + lane);
                rem = 0;
            }
            cnt += __popcll(mask);
        }
        if (lane >= cnt && lane < kL) wl[b][wave][lane] = 0ull;
    }
    __syncthreads();
    // merge: 32 candidates per pod (4 lists x L), two pods per wave pass; the rank of a
    // candidate = its position in its own list + the entries of the other lists above it.
    const int half = lane >> 5, l32 = lane & 31;
    const int li = l32 / kL, le = l32 % kL;
    for (int b0 = wave * 2; b0 < np; b0 += kScanWaves * 2) {
        const int b = b0 + half;
        const uint64_t c = b < np ? wl[b][li][le] : 0ull;
        const uint64_t nz = __ballot(c != 0);
        if (b < np) {
            uint64_t* out = a.lists + ((int64_t)(pg0 + b) * a.nblk + blk) * kL;
            if (c != 0) {
                int rank = le;
#pragma unroll
                for (int o = 0; o < kScanWaves; ++o) {
                    if (o == li) continue;
#pragma unroll
                    for (int k = 0; k < kL; ++k) rank += wl[b][o][k] > c ? 1 : 0;
                }
                if (rank < kL) out[rank] = c;
            }
            const int total = __popcll((nz >> (half * 32)) & 0xFFFFFFFFull);
            if (l32 < kL && l32 >= total) out[l32] = 0ull;
        }
    }
}

// ------------------------------------------------------------------------------------------
// merge: one 256-thread workgroup per pod; exact global top-L over the block lists.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void merge_kernel(EngineArgs a) {
    __shared__ uint64_t red[4];
    __shared__ int32_t owner[4];
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const int64_t nb = min<int64_t>(a.B, end - start);
    const int b = blockIdx.x;
    if (b >= nb) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t top[kL];  // per-thread sorted (descending) top-L over its blocks
#pragma unroll
    for (int k = 0; k < kL; ++k) top[k] = 0;
    const uint64_t* lists = a.lists + (int64_t)b * a.nblk * kL;
    for (int blk = tid; blk < a.nblk; blk += 256) {
#pragma unroll
        for (int k = 0; k < kL; ++k) {
            uint64_t v = lists[(int64_t)blk * kL + k];
            if (v <= top[kL - 1]) break;  // block lists are sorted: nothing further can enter
#pragma unroll
            for (int s = 0; s < kL; ++s) {
                const uint64_t t = top[s];
                const bool gt = v > t;
                top[s] = gt ? v : t;
                v = gt ? t : v;
            }
        }
    }
    // L rounds: the workgroup max of the thread heads; its owner advances
    int head = 0;
    for (int r = 0; r < kL; ++r) {
        uint64_t h = 0;
#pragma unroll
        for (int k = 0; k < kL; ++k) h = (k == head) ? top[k] : h;
        const uint64_t m = wave_max_u64(h);
        const uint64_t hit = __ballot(h == m && m != 0);
        if (lane == 0) {
            red[wave] = m;
            owner[wave] = hit ? wave * 64 + __ffsll((unsigned long long)hit) - 1 : -1;
        }
        __syncthreads();
        uint64_t best = 0;
        int who = -1;
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (red[w] > best) { best = red[w]; who = owner[w]; }
        if (tid == 0) a.cand[(int64_t)b * kL + r] = best;
        if (tid == who) head++;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// resolve: one workgroup, sequential over the batch in FIFO order (one bind per tick).
//
// One barrier per pod.  After the barrier every wave derives pod i's winner from the
// double-buffered partial maxima red[i&1] (identical decision in every wave, including the
// NotFound / InvalidArgument / exhausted-list stops).  Then, until the next barrier, the waves
// split the bind of pod i and the evaluation of pod i+1:
//   wave 0    table insert of an untouched winner; walk pod i+1's top-L list against the
//             table; stage the snapshot fields of its best untouched node in LDS
//   wave 1    CreatePod admission + bind on the winner's entry (and pod i+1's expiries that
//             land on it); outputs; pod i+1's exact key on that entry
//   wave 2    pod i+1's other expiries; pod i+1's exact keys on those entries
//   3..15     owner threads: thread r keeps touched entry r in registers (reloading the
//             mutable fields when an entry was modified the iteration before) and computes pod
//             i+1's exact key on it, unless wave 1 or 2 owns the entry this iteration
// Writers (waves 1, 2) touch disjoint entries and every reader of those skips them.
// ------------------------------------------------------------------------------------------
struct alignas(16) RedSlot {
    uint64_t key;
    int32_t ent;  // touched-table entry, -1 = the list candidate
    int32_t pad;
};

struct ResolveShared {
    int64_t ts[8][kTMax];       // touched-node state: ac am ag ap rc rm rg nr
    uint64_t tu[2][kTMax];      // taint label
    int32_t tnode[kTMax];
    int32_t dirty[kTMax];       // iteration at which the owner must reload the mutable fields
    int32_t hkey[kHash];        // node id or -1
    int32_t hval[kHash];        // entry index
    uint32_t tfilt[kFilterBits / 32];
    PodRec pod[kMaxBatchR];
    int32_t dur[kMaxBatchR];
    int32_t exp_slot[kMaxBatchR];  // window slot of an in-batch pod's own expiry, or -1
    uint64_t cand[kMaxBatchR][kL];
    int32_t ex_off[kMaxBatchR + 1];
    int32_t ex_q[kMaxExp];
    int32_t ex_node[kMaxExp];
    int32_t ex_ok[kMaxExp];     // the expiring pod was bound Ok and has not expired yet
    int32_t ex_entry[kMaxExp];  // table entry of its node (set at the bind for in-batch pods)
    int64_t ex_req[kMaxExp][3];
    RedSlot red[2][kResolveWaves];  // per-pod hand-offs, double-buffered by pod parity
    int64_t stage[2][10];       // snapshot fields of the pod's best untouched list node
    int32_t kfull[2];           // every entry of a full list touched: the batch must stop
    int32_t ntab[2];            // table size when the pod is evaluated
    int32_t n_t, committed, err_code, err_pod, nb;
};

// Diagnostic build only (-DKS_STAMPS): per-iteration cycle sums of waves 0-3, written to
// ctr[8..13]; the real kernel executes no stamp.
#ifdef KS_STAMPS
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define KS_STAMP(var) uint64_t var = stamp()
#else
#define KS_STAMP(var)
#endif

__device__ __forceinline__ uint32_t hslot(int32_t node) { return ((uint32_t)node * 2654435761u) >> (32 - 11); }

// entry index of `node` in the touched table, or -1
__device__ __forceinline__ int h_find(const ResolveShared& sh, int32_t node) {
    uint32_t s = hslot(node);
    for (int i = 0; i < kHash; ++i) {
        const int32_t k = sh.hkey[s];
        if (k == node) return sh.hval[s];
        if (k == -1) return -1;
        s = (s + 1) & (kHash - 1);
    }
    return -1;
}

// single-lane insert of a node known to be absent
__device__ __forceinline__ void h_insert(ResolveShared& sh, int32_t node, int32_t idx) {
    uint32_t s = hslot(node);
    while (sh.hkey[s] != -1) s = (s + 1) & (kHash - 1);
    sh.hkey[s] = node;
    sh.hval[s] = idx;
    const uint32_t f = (uint32_t)node & (kFilterBits - 1);
    sh.tfilt[f >> 5] |= 1u << (f & 31);
}

// touched? — one LDS read unless the filter bit is shared with another node
__device__ __forceinline__ bool is_touched(const ResolveShared& sh, int32_t node) {
    const uint32_t f = (uint32_t)node & (kFilterBits - 1);
    if (!((sh.tfilt[f >> 5] >> (f & 31)) & 1u)) return false;
    return h_find(sh, node) >= 0;
}

__device__ __forceinline__ NodeV t_node(const ResolveShared& sh, int e) {
    NodeV v;
    v.ac = sh.ts[0][e]; v.am = sh.ts[1][e]; v.ag = sh.ts[2][e]; v.ap = sh.ts[3][e];
    v.rc = sh.ts[4][e]; v.rm = sh.ts[5][e]; v.rg = sh.ts[6][e]; v.nr = sh.ts[7][e];
    v.taint = sh.tu[0][e]; v.label = sh.tu[1][e];
    return v;
}

__device__ __forceinline__ NodeV stage_node(const ResolveShared& sh, int b) {
    NodeV v;
    v.ac = sh.stage[b][0]; v.am = sh.stage[b][1]; v.ag = sh.stage[b][2]; v.ap = sh.stage[b][3];
    v.rc = sh.stage[b][4]; v.rm = sh.stage[b][5]; v.rg = sh.stage[b][6]; v.nr = sh.stage[b][7];
    v.taint = (uint64_t)sh.stage[b][8]; v.label = (uint64_t)sh.stage[b][9];
    return v;
}

__device__ __forceinline__ int64_t node_field(const NodeSoA& s, int f, int64_t i) {
    switch (f) {
        case 0: return s.ac[i]; case 1: return s.am[i]; case 2: return s.ag[i]; case 3: return s.ap[i];
        case 4: return s.rc[i]; case 5: return s.rm[i]; case 6: return s.rg[i]; case 7: return s.nr[i];
        case 8: return (int64_t)s.taint[i]; default: return (int64_t)s.label[i];
    }
}

__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }

// Wave 0: first entry of pod i's list whose node is not in the touched table (-1 if none);
// `full` = the list holds L candidates (so "none" means exhausted, not "no candidates").
__device__ __forceinline__ int first_untouched(const ResolveShared& sh, int i, int lane, bool& full) {
    const uint64_t c = lane < kL ? sh.cand[i][lane] : 0ull;
    const bool ok = c != 0 && !is_touched(sh, key_node(c));
    const uint64_t m = __ballot(ok);
    full = __popcll(__ballot(c != 0)) == kL;
    return m ? __ffsll((unsigned long long)m) - 1 : -1;
}

// wave-wide max of (key, entry) pairs: the key decides, the entry follows it
__device__ __forceinline__ RedSlot wave_best_entry(uint64_t key, int ent) {
    RedSlot r;
    r.key = wave_max_u64(key);
    const uint64_t who = __ballot(key == r.key && r.key != 0);
    r.ent = who ? __builtin_amdgcn_readlane(ent, __ffsll((unsigned long long)who) - 1) : -1;
    r.pad = 0;
    return r;
}

template <bool kNarrow>
__global__ __launch_bounds__(kResolveThreads) void resolve_kernel(EngineArgs a) {
    __shared__ ResolveShared sh;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    int nb = (int)min<int64_t>(min<int64_t>(a.B, kMaxBatchR), end - start);
    if (nb <= 0) return;

    // window: expiries of pods start+1 .. start+nb-1 (pod start's were applied by expire_head);
    // shrink the batch so that they fit the pre-insert budget
    const int64_t e_base = a.exp_off[start + 1];
    if (tid == 0) {
        int lo = 1, hi = nb;
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (a.exp_off[start + mid] - e_base <= kMaxExp) lo = mid; else hi = mid - 1;
        }
        sh.nb = lo;
        sh.n_t = 0; sh.committed = lo; sh.err_code = 0; sh.err_pod = -1;
    }
    for (int h = tid; h < kHash; h += kResolveThreads) sh.hkey[h] = -1;
    for (int w = tid; w < kFilterBits / 32; w += kResolveThreads) sh.tfilt[w] = 0;
    __syncthreads();
    nb = sh.nb;
    const int64_t e_cnt = nb > 1 ? a.exp_off[start + nb] - e_base : 0;

    for (int i = tid; i < nb; i += kResolveThreads) {
        sh.pod[i] = a.pods[start + i];
        sh.dur[i] = a.dur[start + i];
        const int64_t pos = a.exp_pos[start + i];
        sh.exp_slot[i] = (pos >= e_base && pos - e_base < e_cnt) ? (int32_t)(pos - e_base) : -1;
    }
    for (int i = tid; i < nb * kL; i += kResolveThreads) sh.cand[i / kL][i % kL] = a.cand[i];
    for (int i = tid; i <= nb; i += kResolveThreads)
        sh.ex_off[i] = i <= 1 ? 0 : (int32_t)(a.exp_off[start + i] - e_base);
    for (int e = tid; e < e_cnt; e += kResolveThreads) {
        const int32_t q = a.exp_pod[e_base + e];
        const PodRec& pq = a.pods[q];
        sh.ex_q[e] = q;
        sh.ex_entry[e] = -1;
        sh.ex_req[e][0] = pq.req[0]; sh.ex_req[e][1] = pq.req[1]; sh.ex_req[e][2] = pq.req[2];
        if (q < start) {
            sh.ex_node[e] = a.b_node[q];
            sh.ex_ok[e] = (a.b_status[q] == 0) && !a.expired[q];
        } else {
            sh.ex_node[e] = -1;
            sh.ex_ok[e] = 0;  // set when the pod binds
        }
    }
    __syncthreads();
    // pre-insert every node an expiry of this batch lands on (q bound before the batch): the
    // per-pod expiry step then never waits on HBM
    if (wave == 0) {
        for (int e0 = 0; e0 < e_cnt; e0 += kWave) {
            const int e = e0 + lane;
            const bool want = e < e_cnt && sh.ex_ok[e];
            const int32_t mine = want ? sh.ex_node[e] : 0;
            uint64_t m = __ballot(want);
            while (m) {
                const int l = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                const int32_t nd = __shfl(mine, l, kWave);
                if (lane == 0) {
                    int idx = h_find(sh, nd);
                    if (idx < 0) {
                        idx = sh.n_t;
                        sh.tnode[idx] = nd;
                        h_insert(sh, nd, idx);
                        sh.n_t = idx + 1;
                    }
                    sh.ex_entry[e0 + l] = idx;
                }
            }
        }
    }
    __syncthreads();
    for (int e = tid; e < kTMax; e += kResolveThreads) sh.dirty[e] = -1;
    for (int e = tid; e < sh.n_t; e += kResolveThreads) {
        const NodeV v = load_node(a.s, sh.tnode[e]);
        sh.ts[0][e] = v.ac; sh.ts[1][e] = v.am; sh.ts[2][e] = v.ag; sh.ts[3][e] = v.ap;
        sh.ts[4][e] = v.rc; sh.ts[5][e] = v.rm; sh.ts[6][e] = v.rg; sh.ts[7][e] = v.nr;
        sh.tu[0][e] = v.taint; sh.tu[1][e] = v.label;
    }
    __syncthreads();

    // owner registers (waves 3..15): entry r = tid - 192
    const int r = tid - kOwnerWave0 * kWave;
    bool loaded = false;
    NodeV own{};
    int32_t own_node = 0;

    // ---- prologue: pod 0's partial maxima
    if (wave == 0) {
        bool full;
        const int pa = first_untouched(sh, 0, lane, full);
        if (pa >= 0 && lane < 10) sh.stage[0][lane] = node_field(a.s, lane, key_node(sh.cand[0][pa]));
        if (lane == 0) {
            sh.red[0][0].key = pa >= 0 ? sh.cand[0][pa] : 0ull;
            sh.red[0][0].ent = -1;
            sh.kfull[0] = pa < 0 && full;
            sh.ntab[0] = sh.n_t;
        }
    } else if (wave < kOwnerWave0) {
        if (lane == 0) { sh.red[0][wave].key = 0; sh.red[0][wave].ent = -1; }
    } else {
        uint64_t k = 0;
        if (r < sh.n_t) {
            own = t_node(sh, r);
            own_node = sh.tnode[r];
            loaded = true;
            k = make_key(eval_t<kNarrow>(a.c, sh.pod[0], own), (uint32_t)own_node);
        }
        const RedSlot w = wave_best_entry(k, r);
        if (lane == 0) sh.red[0][wave] = w;
    }
    __syncthreads();

#ifdef KS_STAMPS
    uint64_t acc_work = 0, acc_wait = 0;
#endif
    int i = 0;
    for (; i < nb; ++i) {
        KS_STAMP(s0);
        const int64_t j = start + i;
        const int cur = i & 1, nxt = cur ^ 1;
        // ---- every wave: pod i's winner and the stop decision (identical in all waves)
        RedSlot rs;
        rs.key = 0; rs.ent = -1;
        if (lane < kResolveWaves) rs = sh.red[cur][lane];
        const uint64_t v = wave_max_u64(rs.key);
        const uint64_t wl = __ballot(rs.key == v && v != 0);
        const int went = wl ? __builtin_amdgcn_readlane(rs.ent, __ffsll((unsigned long long)wl) - 1) : -1;
        const uint32_t pflags = sh.pod[i].flags;
        int stop = 0;
        if (sh.kfull[cur]) stop = 1;                                  // list exhausted: rescan
        else if (v == 0) stop = 2;                                    // NotFound
        else if (pflags & (kFlagBadKey | kFlagBadSpec)) stop = 3;     // InvalidArgument
        if (stop) {
            if (tid == 0) {
                sh.committed = i;
                if (stop > 1) { sh.err_code = stop == 2 ? kErrNotFound : kErrEinval; sh.err_pod = (int32_t)j; }
            }
            break;
        }
        const int nt = sh.ntab[cur];
        const int32_t nd = key_node(v);
        const int t = went >= 0 ? went : nt;  // an untouched winner becomes entry nt
        const bool has_next = i + 1 < nb;
        const int e0 = has_next ? sh.ex_off[i + 1] : 0, e1 = has_next ? sh.ex_off[i + 2] : 0;

        if (wave == 0) {
            if (lane == 0) {
                if (went < 0) { sh.tnode[t] = nd; h_insert(sh, nd, t); }
                sh.ntab[nxt] = went < 0 ? nt + 1 : nt;
            }
            if (has_next) {
                bool full;
                const int pa = first_untouched(sh, i + 1, lane, full);
                if (pa >= 0 && lane < 10) sh.stage[nxt][lane] = node_field(a.s, lane, key_node(sh.cand[i + 1][pa]));
                if (lane == 0) {
                    sh.red[nxt][0].key = pa >= 0 ? sh.cand[i + 1][pa] : 0ull;
                    sh.red[nxt][0].ent = -1;
                    sh.kfull[nxt] = pa < 0 && full;
                }
            }
        } else if (wave == 1) {
            const PodRec p = sh.pod[i];
            NodeV n = went >= 0 ? t_node(sh, t) : stage_node(sh, cur);
            const bool ok = fits(p, n);  // CreatePod admission (kubesim/node/node.go:44-47)
            if (ok && sh.dur[i] > 0) { n.rc += p.req[0]; n.rm += p.req[1]; n.rg += p.req[2]; n.nr += 1; }
            for (int x = e0; x < e1; ++x) {  // pod i+1's expiries on this entry (pod i's own included)
                const int32_t q = sh.ex_q[x];
                const bool hit = q == j ? ok : (sh.ex_entry[x] == t && sh.ex_ok[x] != 0);
                if (!hit) continue;
                n.rc -= sh.ex_req[x][0]; n.rm -= sh.ex_req[x][1]; n.rg -= sh.ex_req[x][2]; n.nr -= 1;
                if (lane == 0) a.expired[q] = 1;
            }
            if (lane == 0) {
                if (went < 0) {
                    sh.ts[0][t] = n.ac; sh.ts[1][t] = n.am; sh.ts[2][t] = n.ag; sh.ts[3][t] = n.ap;
                    sh.tu[0][t] = n.taint; sh.tu[1][t] = n.label;
                }
                sh.ts[4][t] = n.rc; sh.ts[5][t] = n.rm; sh.ts[6][t] = n.rg; sh.ts[7][t] = n.nr;
                sh.dirty[t] = i + 1;
                const int slot = sh.exp_slot[i];
                if (slot >= 0) { sh.ex_entry[slot] = t; sh.ex_ok[slot] = ok ? 1 : 0; }
                a.b_node[j] = nd;
                a.b_status[j] = ok ? 0 : 1;
            }
            if (has_next) {
                const uint32_t t1 = eval_t<kNarrow>(a.c, sh.pod[i + 1], n);
                if (lane == 0) { sh.red[nxt][1].key = make_key(t1, (uint32_t)nd); sh.red[nxt][1].ent = t; }
            }
        } else if (wave == 2) {
            if (has_next) {
                if (lane == 0) {
                    for (int x = e0; x < e1; ++x) {
                        const int tq = sh.ex_entry[x];
                        if (sh.ex_q[x] == j || tq < 0 || tq == t || !sh.ex_ok[x]) continue;
                        sh.ts[4][tq] -= sh.ex_req[x][0]; sh.ts[5][tq] -= sh.ex_req[x][1];
                        sh.ts[6][tq] -= sh.ex_req[x][2]; sh.ts[7][tq] -= 1;
                        sh.dirty[tq] = i + 1;
                        a.expired[sh.ex_q[x]] = 1;
                    }
                }
                const PodRec pn = sh.pod[i + 1];
                uint64_t best = 0;
                int bent = -1;
                for (int x = e0 + lane; x < e1; x += kWave) {
                    const int tq = sh.ex_entry[x];
                    if (sh.ex_q[x] == j || tq < 0 || tq == t) continue;
                    const uint64_t k = make_key(eval_t<kNarrow>(a.c, pn, t_node(sh, tq)), (uint32_t)sh.tnode[tq]);
                    if (k > best) { best = k; bent = tq; }
                }
                const RedSlot w = wave_best_entry(best, bent);
                if (lane == 0) sh.red[nxt][2] = w;
            }
        } else if (has_next) {
            uint64_t k = 0;
            if (r < nt) {
                if (!loaded) {
                    own = t_node(sh, r);
                    own_node = sh.tnode[r];
                    loaded = true;
                } else if (sh.dirty[r] == i) {
                    own.rc = sh.ts[4][r]; own.rm = sh.ts[5][r]; own.rg = sh.ts[6][r]; own.nr = sh.ts[7][r];
                }
                bool mine = r != went;  // wave 1 owns the winner's entry this iteration
                for (int x = e0; x < e1; ++x)  // wave 2 owns the entries pod i+1's expiries land on
                    mine &= !(sh.ex_entry[x] == r && sh.ex_q[x] != j);
                if (mine) k = make_key(eval_t<kNarrow>(a.c, sh.pod[i + 1], own), (uint32_t)own_node);
            }
            const RedSlot w = wave_best_entry(k, r);
            if (lane == 0) sh.red[nxt][wave] = w;
        }
        KS_STAMP(s1);
        __syncthreads();
        KS_STAMP(s2);
#ifdef KS_STAMPS
        acc_work += s1 - s0;
        acc_wait += s2 - s1;
#endif
    }
    __syncthreads();
#ifdef KS_STAMPS
    if (lane == 0 && wave <= 3) {
        const int slot = wave == 0 ? 8 : (wave == 1 ? 10 : (wave == 2 ? 13 : 11));
        atomicAdd((unsigned long long*)&a.ctr[slot], (unsigned long long)acc_work);
        if (wave == 0) atomicAdd((unsigned long long*)&a.ctr[9], (unsigned long long)acc_wait);
    }
    if (tid == 0) atomicAdd((unsigned long long*)&a.ctr[12], (unsigned long long)i);
#endif

    // ---- write back the mutable fields of every touched node
    const int n_final = sh.ntab[sh.committed & 1];
    for (int e = tid; e < n_final; e += kResolveThreads) {
        const int64_t ndx = sh.tnode[e];
        a.s.rc[ndx] = sh.ts[4][e];
        a.s.rm[ndx] = sh.ts[5][e];
        a.s.rg[ndx] = sh.ts[6][e];
        a.s.nr[ndx] = sh.ts[7][e];
    }
    if (tid == 0) {
        a.ctr[kCtrStart] = start + sh.committed;
        if (sh.committed < a.B && sh.err_code == 0 && start + sh.committed < end) a.ctr[kCtrEarly] += 1;
        if (sh.err_code) { a.ctr[kCtrErr] = sh.err_code; a.ctr[kCtrErrPod] = sh.err_pod; }
    }
}

// ------------------------------------------------------------------------------------------
// Filter mask / score of one pod against every node (api.Filter / api.Scorer shims).
// ------------------------------------------------------------------------------------------
template <bool kNarrow>
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
    const uint32_t t1 = eval_t<kNarrow>(c, p, n);
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

// Multiply every device quantity of resource k by f[k] (node capacity unless absent, requested
// totals, pod requests): the unit of resource k shrinks to a divisor of the old one when a pod
// brings a quantity the old unit does not divide (see ks_engine.cpp, resource scale).
__global__ __launch_bounds__(256) void rescale_kernel(NodeSoA s, int64_t n_pad, PodRec* pods, int64_t P,
                                                      int64_t f0, int64_t f1, int64_t f2) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += stride) {
        if (s.ac[i] >= 0) s.ac[i] *= f0;
        if (s.am[i] >= 0) s.am[i] *= f1;
        if (s.ag[i] >= 0) s.ag[i] *= f2;
        s.rc[i] *= f0; s.rm[i] *= f1; s.rg[i] *= f2;
    }
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < P; q += stride) {
        pods[q].req[0] *= f0; pods[q].req[1] *= f1; pods[q].req[2] *= f2;
    }
}

// ---------------------------------------------------------------------------------------------
// Launchers, called by ks_engine.cpp.
// ---------------------------------------------------------------------------------------------
int max_batch_pods() { return kMaxBatchR; }
int max_pods_per_scan_wg() { return kMaxPG; }
int block_nodes() { return kBlockNodes; }

template <bool kNarrow>
static void launch_batch_t(const EngineArgs& a, hipStream_t st, hipEvent_t e_scan0, hipEvent_t e_scan1,
                           hipEvent_t e_res1) {
    hipLaunchKernelGGL(expire_head_kernel, dim3(1), dim3(256), 0, st, a);
    if (e_scan0) (void)hipEventRecord(e_scan0, st);
    dim3 g(a.nblk, (a.B + a.PG - 1) / a.PG);
    hipLaunchKernelGGL(scan_kernel<kNarrow>, g, dim3(kBlockNodes), 0, st, a);
    hipLaunchKernelGGL(merge_kernel, dim3(a.B), dim3(256), 0, st, a);
    if (e_scan1) (void)hipEventRecord(e_scan1, st);
    hipLaunchKernelGGL(resolve_kernel<kNarrow>, dim3(1), dim3(kResolveThreads), 0, st, a);
    if (e_res1) (void)hipEventRecord(e_res1, st);
}

hipError_t launch_batch(const EngineArgs& a, bool narrow, hipStream_t st, hipEvent_t e_scan0, hipEvent_t e_scan1,
                        hipEvent_t e_res1) {
    if (narrow) launch_batch_t<true>(a, st, e_scan0, e_scan1, e_res1);
    else launch_batch_t<false>(a, st, e_scan0, e_scan1, e_res1);
    return hipGetLastError();
}

hipError_t launch_rescale(const NodeSoA& s, int64_t n_pad, PodRec* pods, int64_t P, const int64_t f[3], hipStream_t st) {
    hipLaunchKernelGGL(rescale_kernel, dim3(1024), dim3(256), 0, st, s, n_pad, pods, P, f[0], f[1], f[2]);
    return hipGetLastError();
}

hipError_t launch_eval_pod(const Cfg& c, const NodeSoA& s, const PodRec* pod, uint32_t filters, uint8_t* mask,
                           int64_t* score, bool narrow, hipStream_t st) {
    const dim3 g((c.n_nodes + 255) / 256);
    if (narrow) hipLaunchKernelGGL(eval_pod_kernel<true>, g, dim3(256), 0, st, c, s, pod, filters, mask, score);
    else hipLaunchKernelGGL(eval_pod_kernel<false>, g, dim3(256), 0, st, c, s, pod, filters, mask, score);
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
