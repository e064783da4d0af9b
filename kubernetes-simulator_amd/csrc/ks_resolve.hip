// ks_resolve.hip — the FIFO resolver of a batch (gfx950): one 4-wave workgroup per engine.
//
// A pod's placement depends on every bind before it (kubesim/kubesim.go:105-121, one pod per
// tick), so this part of the batch is sequential.  The exactness argument is the scan's (see
// ks_kernels.hip): a node's key for pod i can differ from the batch snapshot only if a bind or an
// expiry of this batch touched it.  Touched nodes are table entries, re-evaluated exactly for
// every pod; the best untouched node is the first untouched entry of the pod's snapshot top-L
// list (every node outside the list scores below every list entry).  winner = max of the two.
// When every entry of a full list is touched the batch commits early and the next one rescans.
//
// Layout for latency: the chain from one decision to the next is short and has no hand-off
// between waves except one barrier per pod.
//   * Table entry e lives in the REGISTERS of one lane: wave (e / 64) % W, lane e % 64, slot
//     e / (64 W).  The four waves sit on the four SIMDs, so a pod's re-evaluation of up to 256
//     entries is one pass of the evaluator per wave.
//   * Every wave makes every decision itself: after the barrier each wave reads the W per-wave
//     maxima of pod i, adds pod i's list candidate (it computed pod i's untouched-entry mask
//     itself in the previous iteration) and arrives at the same winner.  Only the lane that owns
//     the winner's entry binds (CreatePod admission, kubesim/node/node.go:36-60); pod i+1's
//     expiries are applied by the lanes owning their entries; every lane then evaluates pod i+1
//     on its entries and the wave maximum goes to LDS for the next barrier.
//   * An untouched winner becomes a new entry: its snapshot record is staged in LDS, gathered
//     one iteration ahead (plain loads into registers at the end of an iteration, written to LDS
//     at the end of the next, so the HBM latency hides behind a whole iteration).
//   * No global store inside the loop: binds, statuses and expiry marks are kept in LDS and
//     written out after it, with the touched nodes' state.
#include "ks_device.h"

namespace ks {
namespace {

constexpr int kL = kTopL;
constexpr int kEntNone = 1023;  // ikey entry field of an untouched (list) node
constexpr int kRecDw = 20;      // a node record in dwords: 10 int64 fields, NodeV order

// W waves, S register slots per lane (TMAX <= 64 W S entries), batches of <= MAXB pods, node ->
// entry hash of 2^HASH_LOG2 slots, touched filter of 2^FBITS_LOG2 bits (exact — no hash
// confirmation — for clusters of at most that many nodes).
template <int W, int S, int TMAX, int MAXB, int HASH_LOG2, int FBITS_LOG2>
struct Cfg4 {
    static constexpr int kWaves = W, kThreads = W * kWave, kSlots = S, kTMax = TMAX;
    static_assert(TMAX <= W * kWave * S && TMAX > W * kWave * (S - 1), "S register slots hold TMAX entries");
    static constexpr int kMaxB = MAXB, kMaxExp = kTMax - MAXB;
    static constexpr int kHashLog2 = HASH_LOG2, kHash = 1 << HASH_LOG2, kFilterBits = 1 << FBITS_LOG2;
    static constexpr int kRecPerWave = kL / W;  // staged list records gathered per wave
    static_assert(kL % W == 0 && kRecPerWave * kRecDw <= kWave, "staging: one dword per lane");
    static_assert(kTMax < kEntNone, "entry index fits the ikey's 10 bits");
    static_assert(kMaxExp < kHash, "the hash never fills");
    static_assert(MAXB <= kThreads, "one thread per pod in the window search");
};
// The small class: batches of <= 128 pods of clusters of <= 8,192 nodes (what-if scenarios),
// 256 entries, ~34 KB of LDS and <= 88 VGPRs, so four resolvers share a CU.  (A 768-entry class
// of the same kernel — 3 register slots — was exact but slower than the role-split resolver on
// 256-pod batches: DESIGN.md §4.)
using RSmall = Cfg4<4, 1, 256, 128, 10, 13>;

// Entry state in registers: 32-bit fields for the narrow evaluators (every capacity < 2^29 and
// usage <= capacity; the pods capacity is clamped, nr < 2^31 either way), NodeV for the wide one.
struct NodeS32 {
    int32_t ac, am, ag, ap, rc, rm, rg, nr;
    uint64_t taint, label;
};
// The micro evaluator's entries also carry its per-node invariants (ks_device.h, micro_ic): the
// capacities never change, so they are computed once, when the entry is filled.
struct NodeM : NodeS32 {
    float ic, im;
    int32_t d;
};
__device__ __forceinline__ float micro_ic(const NodeM& n, int32_t) { return n.ic; }
__device__ __forceinline__ float micro_im(const NodeM& n, int32_t) { return n.im; }
__device__ __forceinline__ int32_t micro_d(const NodeM& n, int32_t, int32_t) { return n.d; }

template <int kMode> struct NodeSel { using T = NodeS32; };
template <> struct NodeSel<kEvalMicro> { using T = NodeM; };
template <> struct NodeSel<kEvalWide> { using T = NodeV; };

__device__ __forceinline__ void conv(const NodeV& v, NodeV& o) { o = v; }
__device__ __forceinline__ void conv(const NodeV& v, NodeS32& o) {
    o.ac = (int32_t)v.ac; o.am = (int32_t)v.am; o.ag = (int32_t)v.ag;
    o.ap = (int32_t)(v.ap < 0x7FFFFFFF ? v.ap : 0x7FFFFFFF);
    o.rc = (int32_t)v.rc; o.rm = (int32_t)v.rm; o.rg = (int32_t)v.rg; o.nr = (int32_t)v.nr;
    o.taint = v.taint; o.label = v.label;
}
__device__ __forceinline__ void conv(const NodeV& v, NodeM& o) {
    conv(v, static_cast<NodeS32&>(o));
    const int32_t acs = o.ac > 0 ? o.ac : 1, ams = o.am > 0 ? o.am : 1;  // eval_total1_micro's guards
    o.ic = rcp_est((float)acs);
    o.im = rcp_est((float)ams);
    o.d = mul24(acs, ams);
}

// Admission (kubesim/node/node.go:44-47) in 64-bit whatever the state type.
template <class NS>
__device__ __forceinline__ bool fits_t(const PodRec& p, const NS& n) {
    bool ok = (int64_t)n.nr < (int64_t)n.ap;
    if (p.keymask & 1) ok &= (int64_t)n.rc + p.req[0] <= (int64_t)n.ac;
    if (p.keymask & 2) ok &= (int64_t)n.rm + p.req[1] <= (int64_t)n.am;
    if (p.keymask & 4) ok &= (int64_t)n.rg + p.req[2] <= (int64_t)n.ag;
    return ok;
}

// A record staged as 20 dwords (LDS), five 16-byte reads.
template <class NS>
__device__ __forceinline__ NS rec_from(const uint32_t* w) {
    const uint4* q = reinterpret_cast<const uint4*>(w);
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
    auto f = [](uint32_t lo, uint32_t hi) { return (int64_t)(((uint64_t)hi << 32) | lo); };
    NodeV v;
    v.ac = f(a.x, a.y); v.am = f(a.z, a.w); v.ag = f(b.x, b.y); v.ap = f(b.z, b.w);
    v.rc = f(c.x, c.y); v.rm = f(c.z, c.w); v.rg = f(d.x, d.y); v.nr = f(d.z, d.w);
    v.taint = (uint64_t)f(e.x, e.y); v.label = (uint64_t)f(e.z, e.w);
    NS o;
    conv(v, o);
    return o;
}

// dword d (0..19) of node i's record: the SoA is one allocation with a fixed field stride
__device__ __forceinline__ uint32_t rec_dword(const NodeSoA& s, int d, int64_t i) {
    const uint32_t* base = reinterpret_cast<const uint32_t*>(s.ac);
    const int64_t stride = (int64_t)(s.am - s.ac) * 2;  // dwords per field
    return gptr(base)[(int64_t)(d >> 1) * stride + 2 * i + (d & 1)];
}

// Internal key: (total + 1) << 34 | (2^24 - 1 - node) << 10 | entry — orders exactly like the
// packed key (node < 2^24, total + 1 < 2^30: ks_engine.cpp) and carries the winner's entry.
__device__ __forceinline__ uint64_t ikey(uint64_t key, int ent) {
    const uint32_t node = 0xFFFFFFFFu - (uint32_t)key;
    return ((key >> 32) << 34) | ((uint64_t)(0xFFFFFFu - node) << 10) | (uint64_t)(uint32_t)ent;
}
__device__ __forceinline__ int32_t ikey_node(uint64_t b) { return (int32_t)(0xFFFFFFu - (uint32_t)((b >> 10) & 0xFFFFFFu)); }
__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Diagnostic build only (-DKS_R4_STAMPS): per-phase cycle sums per wave, accumulated in
// ctr[8 + 6 * wave + phase] (waves 0..3), iterations in ctr[5], launches in ctr[6]
// (tests/dev/diag_r4.py); the product kernel executes no stamp.
#ifdef KS_R4_STAMPS
__device__ __forceinline__ uint64_t r4_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define R4_STAMP(var) const uint64_t var = r4_stamp()
#define R4_ACC(k, d) acc[k] += (d)
#else
#define R4_STAMP(var)
#define R4_ACC(k, d)
#endif

template <class C>
struct Shared4 {
    PodRec pod[C::kMaxB + 1];              // +1: pod i + 1 is read unconditionally
    int4 pctl[C::kMaxB + 1];               // ex_lo, ex_hi, dur, (exp_slot + 1) | flags << 16
    uint64_t cand[C::kMaxB + 1][kL];       // snapshot top-L lists (row nb zero)
    uint32_t stage[2][kL * kRecDw];        // snapshot records of pod p's list, buffer p & 1
    uint64_t best[2][C::kWaves];           // per-wave maximum ikey of pod p's entries, buffer p & 1
    int32_t hkey[C::kHash];                // node id or -1
    int32_t hval[C::kHash];                // entry index (pre-inserted nodes)
    uint32_t tfilt[C::kFilterBits / 32];
    int32_t pre_node[C::kMaxExp];          // node of pre-inserted entry e
    int32_t ex_q[C::kMaxExp];              // expiry window: the expiring pod
    int32_t ex_node[C::kMaxExp];
    int32_t ex_ok[C::kMaxExp];             // bound Ok and not expired yet (set at the bind in-batch)
    int32_t ex_entry[C::kMaxExp];          // table entry of its node
    int64_t ex_req[C::kMaxExp][3];
    int32_t bnode[C::kMaxB], bstat[C::kMaxB];
    int32_t n_pre, nb, e_cnt;
};

template <class SH>
__device__ __forceinline__ uint32_t hslot(int32_t node) {
    return ((uint32_t)node * 2654435761u) >> (32 - SH::kHashLog2);
}

template <class C>
__device__ __forceinline__ bool is_touched(const Shared4<C>& sh, int32_t node, bool exact) {
    const uint32_t f = (uint32_t)node & (C::kFilterBits - 1);
    if (!((sh.tfilt[f >> 5] >> (f & 31)) & 1u)) return false;
    if (exact) return true;
    uint32_t s = hslot<C>(node);
    for (int k = 0; k < C::kHash; ++k) {
        const int32_t h = sh.hkey[s];
        if (h == node) return true;
        if (h == -1) return false;
        s = (s + 1) & (C::kHash - 1);
    }
    return false;
}

// single-lane insert of an untouched winner (absent from the table)
template <class C>
__device__ __forceinline__ void t_insert(Shared4<C>& sh, int32_t node, bool exact) {
    const uint32_t f = (uint32_t)node & (C::kFilterBits - 1);
    atomicOr(&sh.tfilt[f >> 5], 1u << (f & 31));
    if (exact) return;
    uint32_t s = hslot<C>(node);
    while (sh.hkey[s] != -1) s = (s + 1) & (C::kHash - 1);
    sh.hkey[s] = node;
}

template <int kMode, class C>
__global__ __launch_bounds__(C::kThreads) void resolve_kernel(const EngineArgs* __restrict__ A) {
    using NS = typename NodeSel<kMode>::T;
    constexpr int W = C::kWaves, S = C::kSlots, kThreads = C::kThreads, kMaxB = C::kMaxB, kMaxExp = C::kMaxExp;
    __shared__ Shared4<C> sh;
    const EngineArgs a = A[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const bool exact = a.c.n_nodes <= C::kFilterBits;
    int nb = (int)min<int64_t>(min<int64_t>(a.B, kMaxB), end - start);
    if (nb <= 0) return;

    // ---- expiry window: expiries of pods start+1 .. start+nb-1 (pod start's were applied by
    // expire_head); the batch shrinks to the largest prefix whose window fits the table
    // (exp_off is non-decreasing: the fitting prefixes are counted in one round trip)
    const int64_t e_base = a.exp_off[start + 1];
    const int64_t off_mid = tid < nb ? a.exp_off[start + tid + 1] : 0;
    const bool fits_win = tid < nb && off_mid - e_base <= kMaxExp;
    if (tid == 0) sh.n_pre = 0;
    for (int h = tid; h < C::kHash; h += kThreads) sh.hkey[h] = -1;
    for (int w = tid; w < C::kFilterBits / 32; w += kThreads) sh.tfilt[w] = 0;
    nb = __syncthreads_count(fits_win);
    if (tid == nb - 1) { sh.nb = nb; sh.e_cnt = nb > 1 ? (int32_t)(off_mid - e_base) : 0; }
    __syncthreads();
    const int e_cnt = sh.e_cnt;

    for (int i = tid; i < nb; i += kThreads) {
        const PodRec p = a.pods[start + i];
        sh.pod[i] = p;
        const int64_t pos = a.exp_pos[start + i];
        const int ex_lo = i <= 1 ? 0 : (int)(a.exp_off[start + i] - e_base);
        const int ex_hi = i == 0 ? 0 : (int)(a.exp_off[start + i + 1] - e_base);
        const int slot = (pos >= e_base && pos - e_base < e_cnt) ? (int)(pos - e_base) : -1;
        sh.pctl[i] = make_int4(ex_lo, ex_hi, a.dur[start + i], (slot + 1) | (int)((p.flags & 0xFFFFu) << 16));
    }
    if (tid == 0) sh.pctl[nb] = make_int4(0, 0, 0, 0);
    for (int k = tid; k < nb * kL; k += kThreads) sh.cand[k / kL][k % kL] = a.cand[k];
    if (tid < kL) sh.cand[nb][tid] = 0;
    for (int x = tid; x < e_cnt; x += kThreads) {
        const int32_t q = a.exp_pod[e_base + x];
        const PodRec& pq = a.pods[q];
        sh.ex_q[x] = q;
        sh.ex_entry[x] = -1;
        sh.ex_req[x][0] = pq.req[0]; sh.ex_req[x][1] = pq.req[1]; sh.ex_req[x][2] = pq.req[2];
        if (q < start) {
            sh.ex_node[x] = a.b_node[q];
            sh.ex_ok[x] = (a.b_status[q] == 0) && !a.expired[q];
        } else {
            sh.ex_node[x] = -1;
            sh.ex_ok[x] = 0;  // set when the pod binds
        }
    }
    __syncthreads();
    // ---- pre-insert every node an expiry of the window lands on (pod bound before the batch):
    // claim its hash slot with a CAS (duplicates find it), number the claims, then read the entry
    // back.  Entry numbering order is immaterial: an entry only names a node.
    for (int x = tid; x < e_cnt; x += kThreads) {
        if (!sh.ex_ok[x]) continue;
        const int32_t nd = sh.ex_node[x];
        uint32_t hs = hslot<C>(nd);
        for (;;) {  // the hash holds <= kMaxExp < kHash nodes: terminates
            const int32_t prev = atomicCAS(&sh.hkey[hs], -1, nd);
            if (prev == -1 || prev == nd) {
                if (prev == -1) {
                    const int idx = atomicAdd(&sh.n_pre, 1);
                    sh.hval[hs] = idx;
                    sh.pre_node[idx] = nd;
                    const uint32_t f = (uint32_t)nd & (C::kFilterBits - 1);
                    atomicOr(&sh.tfilt[f >> 5], 1u << (f & 31));
                }
                sh.ex_entry[x] = (int)hs;  // the slot for now, its entry below
                break;
            }
            hs = (hs + 1) & (C::kHash - 1);
        }
    }
    __syncthreads();
    for (int x = tid; x < e_cnt; x += kThreads)
        if (sh.ex_ok[x]) sh.ex_entry[x] = sh.hval[sh.ex_entry[x]];
    // pod 0's list records, synchronously
    for (int k = tid; k < kL * kRecDw; k += kThreads) {
        const uint64_t key = sh.cand[0][k / kRecDw];
        sh.stage[0][k] = key ? rec_dword(a.s, k % kRecDw, key_node(key)) : 0u;
    }
    __syncthreads();

    // ---- registers: the pre-inserted entries' records
    int T = sh.n_pre;  // table size (identical in every wave)
    NS own[S];
    int32_t onode[S];
    PruneF opf[S];  // prune_tmax state of each entry (refreshed by the lane whenever the entry changes)
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int e = (s * W + wave) * kWave + lane;
        onode[s] = 0;
        NodeV v{};
        if (e < T) {
            onode[s] = sh.pre_node[e];
            v = load_node(a.s, onode[s]);
        }
        conv(v, own[s]);
        opf[s] = prune_prep(a.c, own[s]);
    }
    // staging registers: this wave's share of pod p+1's list records (lane < kRecPerWave * 20)
    const int st_r = wave * C::kRecPerWave + lane / kRecDw, st_d = lane % kRecDw;
    const bool st_lane = lane < C::kRecPerWave * kRecDw;
    uint32_t st_v = 0;
    if (nb > 1 && st_lane) {
        const uint64_t key = sh.cand[1][st_r];
        if (key) st_v = rec_dword(a.s, st_d, key_node(key));
    }

    // ---- pod 0: per-wave maxima, untouched mask of its list
    PodRec pc = sh.pod[0];
    int4 pcc = sh.pctl[0];
    uint64_t ck = lane < kL ? sh.cand[0][lane] : 0ull;
    // pod p's exact keys on this wave's entries, folded to the wave maximum.  Pruning (exact): the
    // winner is >= the pod's list candidate lbk (the first untouched entry of its list), so an
    // entry whose float upper bound (prune_tmax) puts it below lbk cannot win and is not
    // evaluated; a slot whose 64 entries are all below is skipped by the whole wave.
    auto wave_best = [&](const PodRec& p, uint64_t lbk) -> uint64_t {
        uint64_t bl = 0;
        const float qfc = (float)p.req[0], qfm = (float)p.req[1];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int e = (s * W + wave) * kWave + lane;
            if ((s * W + wave) * kWave < T) {
                bool want = e < T && opf[s].live != 0;
                if (lbk != 0 && want)
                    want = make_key(prune_tmax(a.c, opf[s], qfc, qfm) + 1u, (uint32_t)onode[s]) >= lbk;
                if (__ballot(want)) {
                    const uint64_t k = make_key(eval_t<kMode>(a.c, p, own[s]), (uint32_t)onode[s]);
                    const uint64_t v = (want && k) ? ikey(k, e) : 0ull;
                    bl = v > bl ? v : bl;
                }
            }
        }
        return wave_max_u64(bl);
    };
    uint64_t umask = __ballot(lane < kL && ck != 0 && !is_touched(sh, key_node(ck), exact));
    bool full = __popcll(__ballot(lane < kL && ck != 0)) == kL;
    {
        const uint64_t lbk = umask ? readlane64(ck, __ffsll((unsigned long long)umask) - 1) : 0ull;
        const uint64_t wb = wave_best(pc, lbk);
        if (lane == 0) sh.best[0][wave] = wb;
    }
    __syncthreads();

    int i = 0, stop = 0;
#ifdef KS_R4_STAMPS
    uint64_t acc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t t_bar = r4_stamp();
#endif
    for (; i < nb; ++i) {
        R4_STAMP(s0);
        const bool has_next = i + 1 < nb;
        // every wave: pod i's decision
        uint64_t bw = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint64_t b = sh.best[i & 1][w];
            bw = b > bw ? b : bw;
        }
        const PodRec pn = sh.pod[i + 1];
        const int4 pcn = sh.pctl[i + 1];
        const uint64_t cn = lane < kL ? sh.cand[i + 1][lane] : 0ull;
        const int jpos = umask ? __ffsll((unsigned long long)umask) - 1 : -1;
        if (jpos >= 0) {
            const uint64_t lc = ikey(readlane64(ck, jpos), kEntNone);
            bw = lc > bw ? lc : bw;
        }
        if (!umask && full && i > 0) stop = 1;         // list exhausted: commit, rescan
        else if (bw == 0) stop = 2;                    // NotFound
        else if ((pcc.w >> 16) & (int)(kFlagBadKey | kFlagBadSpec)) stop = 3;  // InvalidArgument
        if (stop) break;
        const int went = (int)(bw & 1023u) == kEntNone ? -1 : (int)(bw & 1023u);
        const int32_t nd = ikey_node(bw);
        const int t = went >= 0 ? went : T;
        if (went < 0) {
            T += 1;
            if (tid == 0) t_insert(sh, nd, exact);
        }
        const int ow = (t >> 6) % W, ol = t & (kWave - 1), os = t / (W * kWave);
        const int64_t j = start + i;
        R4_STAMP(s1);
        R4_ACC(0, s1 - s0);

        // the bind of pod i on entry t (the owner lane)
        bool okb = false;
        if (wave == ow) {
            NS n;
            if (went >= 0) {
                n = own[0];
#pragma unroll
                for (int s = 1; s < S; ++s)
                    if (os == s) n = own[s];
            } else {
                n = rec_from<NS>(&sh.stage[i & 1][jpos * kRecDw]);
            }
            okb = fits_t(pc, n);
            if (okb && pcc.z > 0) {
                n.rc += (decltype(n.rc))pc.req[0];
                n.rm += (decltype(n.rm))pc.req[1];
                n.rg += (decltype(n.rg))pc.req[2];
                n.nr += 1;
            }
            if (lane == ol) {
                const PruneF f = prune_prep(a.c, n);
#pragma unroll
                for (int s = 0; s < S; ++s)
                    if (os == s) { own[s] = n; onode[s] = nd; opf[s] = f; }
                sh.bnode[i] = nd;
                sh.bstat[i] = okb ? 0 : 1;
                const int es = (pcc.w & 0xFFFF) - 1;
                if (es >= 0) { sh.ex_entry[es] = t; sh.ex_ok[es] = okb ? 1 : 0; }
            }
        }
        R4_STAMP(s2);
        R4_ACC(1, s2 - s1);
        if (!has_next) continue;  // last pod of the batch: nothing to evaluate, no barrier needed

        // the expiries due before pod i+1, on the lanes owning their entries
        for (int x = pcn.x; x < pcn.y; ++x) {
            const int32_t q = sh.ex_q[x];
            int tq, okx;
            if (q == j) { tq = t; okx = okb; }  // pod i's own (it runs one tick): okb lives in lane ol
            else { tq = sh.ex_entry[x]; okx = sh.ex_ok[x]; }
            if (tq >= 0 && ((tq >> 6) % W) == wave && lane == (tq & (kWave - 1)) && okx) {
                const int s_ = tq / (W * kWave);
                const int64_t r0 = sh.ex_req[x][0], r1 = sh.ex_req[x][1], r2 = sh.ex_req[x][2];
#pragma unroll
                for (int s = 0; s < S; ++s)
                    if (s_ == s) {
                        own[s].rc -= (decltype(own[s].rc))r0;
                        own[s].rm -= (decltype(own[s].rm))r1;
                        own[s].rg -= (decltype(own[s].rg))r2;
                        own[s].nr -= 1;
                        opf[s] = prune_prep(a.c, own[s]);
                    }
            }
        }

        R4_STAMP(s3);
        R4_ACC(2, s3 - s2);
        // pod i+1's untouched list entries: the filter holds every node inserted up to pod i-1's
        // winner; pod i's is compared directly (its insert above may not be visible yet)
        const int32_t cnd = key_node(cn);
        const bool tch = cn != 0 && (cnd == nd || is_touched(sh, cnd, exact));
        umask = __ballot(lane < kL && cn != 0 && !tch);
        full = __popcll(__ballot(lane < kL && cn != 0)) == kL;
        // pod i+1 on every entry of this wave (nothing to do if its list is exhausted: it stops)
        R4_STAMP(s4);
        R4_ACC(3, s4 - s3);
        uint64_t wb = 0;
        if (umask || !full) {
            const uint64_t lbk = umask ? readlane64(cn, __ffsll((unsigned long long)umask) - 1) : 0ull;
            wb = wave_best(pn, lbk);
        }
        if (lane == 0) sh.best[(i + 1) & 1][wave] = wb;
        ck = cn;
        pc = pn;
        pcc = pcn;
        // staging, off the decision's path: pod i+1's records (loaded during the previous
        // iteration) into LDS for its bind, then the loads of pod i+2's
        if (st_lane) sh.stage[(i + 1) & 1][st_r * kRecDw + st_d] = st_v;
        if (i + 2 < nb && st_lane) {
            const uint64_t key = sh.cand[i + 2][st_r];
            st_v = key ? rec_dword(a.s, st_d, key_node(key)) : 0u;
        }
        R4_STAMP(s5);
        R4_ACC(4, s5 - s4);
        __syncthreads();
#ifdef KS_R4_STAMPS
        t_bar = r4_stamp();
        R4_ACC(5, t_bar - s5);
#endif
    }
    const int committed = i;
    __syncthreads();

    // ---- write-back: the touched nodes' mutable fields, the binds, the expiry marks, counters
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int e = (s * W + wave) * kWave + lane;
        if (e < T) {
            const int64_t n = onode[s];
            gptr(a.s.rc)[n] = (int64_t)own[s].rc;
            gptr(a.s.rm)[n] = (int64_t)own[s].rm;
            gptr(a.s.rg)[n] = (int64_t)own[s].rg;
            gptr(a.s.nr)[n] = (int64_t)own[s].nr;
        }
    }
    for (int k = tid; k < committed; k += kThreads) {
        gptr(a.b_node)[start + k] = sh.bnode[k];
        gptr(a.b_status)[start + k] = sh.bstat[k];
    }
    // expiries applied: those due before pod min(committed, nb - 1) + ... = window prefix
    const int e_done = sh.pctl[committed < nb ? committed : nb - 1].y;
    for (int x = tid; x < e_done; x += kThreads)
        if (sh.ex_ok[x]) gptr(a.expired)[sh.ex_q[x]] = 1;
#ifdef KS_R4_STAMPS
    if (lane == 0 && wave < 4)
        for (int k = 0; k < 6; ++k) atomicAdd((unsigned long long*)a.ctr + 8 + 6 * wave + k, (unsigned long long)acc[k]);
    if (tid == 0) {
        atomicAdd((unsigned long long*)a.ctr + 5, (unsigned long long)committed);
        atomicAdd((unsigned long long*)a.ctr + 6, 1ull);
    }
#endif
    if (tid == 0) {
        a.ctr[kCtrStart] = start + committed;
        if (committed < a.B && stop <= 1 && start + committed < end) a.ctr[kCtrEarly] += 1;
        if (stop >= 2) {
            a.ctr[kCtrErr] = stop == 2 ? kErrNotFound : kErrEinval;
            a.ctr[kCtrErrPod] = start + committed;
        }
    }
}

template <class C>
void launch_t(const EngineArgs* d, int S, int mode, hipStream_t st) {
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL((resolve_kernel<kEvalMicro, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        case kEvalTiny: hipLaunchKernelGGL((resolve_kernel<kEvalTiny, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        case kEvalNarrow: hipLaunchKernelGGL((resolve_kernel<kEvalNarrow, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        default: hipLaunchKernelGGL((resolve_kernel<kEvalWide, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
    }
}

}  // namespace

hipError_t launch_resolve_small(const EngineArgs* d, int S, int mode, hipStream_t st) {
    launch_t<RSmall>(d, S, mode, st);
    return hipGetLastError();
}

int small_resolver_max_batch() { return RSmall::kMaxB; }
int small_resolver_max_nodes() { return RSmall::kFilterBits; }

}  // namespace ks
