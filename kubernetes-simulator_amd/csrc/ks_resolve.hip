// ks_resolve.hip — the speculative resolver (gfx950): one workgroup walks a batch in FIFO order
// with one barrier per pod and no dependent chain of work inside an iteration.
//
// Same exactness argument as resolve_kernel (ks_kernels.hip): a node's key for pod p can differ
// from the batch snapshot only if a bind or an expiry touched it in this batch; touched nodes are
// table entries evaluated exactly, and the best untouched node is the first untouched entry of
// the pod's snapshot top-L list (LC).  What changes is WHEN each piece of work happens.  With
// S_r(p) = entry r's state when pod p is evaluated and t_p = pod p's winner:
//
//     S_r(p+1) = (t_p == r ? S_r(p) + bind(p) : S_r(p)) - expiries due before pod p+1 on r
//     key_p+1(r) = key(pod p+1, S_r(p+1))
//
// so in iteration i (t_i known) the owner of r computes, for pod i+2, BOTH outcomes of pod i+1:
//     K1 = key(pod i+2, S_r(i+1) - exp_{i+2}(r))                  (r does not win pod i+1)
//     K2 = key(pod i+2, S_r(i+1) + bind(i+1) - exp_{i+2}(r))      (r wins pod i+1)
// and in iteration i+1, once t_{i+1} is known, it only selects one of the two and folds it into
// pod i+2's decision word (an LDS atomic max) — the bind of pod i+1 and the evaluation of pod
// i+2 on the bound state are already done.  K2 is needed only when r can win pod i+1 at all
// (its key for pod i+1 reaches the pod's lower bound), so it is almost always skipped.
// Untouched winners come from the pods' lists: the walker walks pod p's list kLA iterations
// early and keeps its first kNC untouched entries (kLA - 1 winners can still join before pod p
// is decided, so kNC = kLA leaves one), issuing their node-record loads; two iterations later the
// records are in LDS, and in iteration p-1 the candidate wave evaluates "candidate c wins pod
// p": its bind status, bound state and its key for pod p+1.  Iteration i then has:
//
//   all      read pod i's decision (winner, stop conditions)
//   owners   (2..)  fold key_{i+1}(r) (the K1 / K2 chosen by t_i), bind pod i if r = t_i, apply
//                   pod i+1's expiries, compute K1 / K2 for pod i+2
//   wave 1   install t_i if it is a new (untouched) node, fold pod i+1's LC and the new entry's
//            key for pod i+1, evaluate pod i+1's candidates
//   wave 0   walk pod i+kLA's list, issue its record loads, stage pod i+2's landed records
//
// None of these depends on another wave's work of the same iteration: the iteration is as long
// as its busiest wave, not as a chain of dependent LDS round trips.
#include "ks_device.h"

namespace ks {

namespace r2 {

constexpr int kL = kTopL;
constexpr int kLA = 4;             // pod p's list is walked in iteration p - kLA
constexpr int kNC = kLA;           // untouched candidates kept per walked list
constexpr int kRing = 8;           // per-pod LDS slots (> kLA + 2)
constexpr int kEntCand = 1016;     // ikey entry field kEntCand + c: candidate c of the pod's list
constexpr int kOwnerWave0 = 2;
constexpr int kFields = 10;        // node record fields (NodeV order)
static_assert(kNC * kFields <= kWave, "candidate records: one field per lane");

// Size classes: kOwn owner waves after the walker and the candidate wave, kE table entries per
// owner lane (entry r = k * kOwn * 64 + owner lane, k < kE: consecutive entries on consecutive
// lanes).  Few waves, several entries per lane: the per-iteration fixed work (decision, reads,
// control) is paid by few waves, and the CU's SIMDs are not shared by many of them.
template <int OWN, int E, int TMAX, int HASH_LOG2, int MAXB, int FBITS_LOG2>
struct Cfg2 {
    static constexpr int kOwn = OWN;
    static constexpr int kE = E;
    static constexpr int kThreads = (kOwnerWave0 + OWN) * kWave;
    static constexpr int kNL = OWN * kWave;  // owner lanes
    static constexpr int kTMax = TMAX;
    static constexpr int kHashLog2 = HASH_LOG2;
    static constexpr int kHash = 1 << HASH_LOG2;
    static constexpr int kMaxBatchR = MAXB;
    static constexpr int kMaxExp = TMAX - MAXB;
    static constexpr int kFilterBits = 1 << FBITS_LOG2;
    static_assert(TMAX <= kNL * E, "every table entry has an owner lane");
    static_assert(MAXB <= kThreads, "one thread per pod in the window search");
    static_assert(TMAX < kEntCand, "entry index below the candidate codes");
};
using RBig2 = Cfg2<3, 4, 768, 11, 256, 16>;
using RSmall2 = Cfg2<2, 2, 256, 10, 128, 13>;

enum : int64_t { kCtrStart = 0, kCtrEnd = 1, kCtrErr = 2, kCtrErrPod = 3, kCtrEarly = 4 };
enum : uint32_t { kFlagBadKey = 1, kFlagBadSpec = 2 };
enum : int64_t { kErrEinval = 1, kErrNotFound = 2 };

struct alignas(16) PodCtl {
    uint32_t flags;
    int32_t ex_lo, ex_hi;  // window range of the expiries due before the pod binds
    int32_t dur;           // ticks the pod runs if bound Ok
    int32_t exp_slot;      // window slot of this pod's own expiry, or -1
    int32_t nxt_own;       // 1: this pod's own expiry is due before the next pod
    int32_t pad[2];
};

template <class C>
struct Shared2 {
    static constexpr int kTMax = C::kTMax, kHash = C::kHash, kMaxBatchR = C::kMaxBatchR, kMaxExp = C::kMaxExp,
                         kFilterBits = C::kFilterBits, kHashLog2 = C::kHashLog2;
    int32_t hkey[kHash];        // node id or -1
    int32_t hval[kHash];        // entry index
    uint32_t tfilt[kFilterBits / 32];
    PodRec pod[kMaxBatchR + 2];  // +2: pods i+1 and i+2 are read unconditionally
    float podf[kMaxBatchR + 2][2];
    PodCtl pctl[kMaxBatchR + 2];
    uint64_t cand[kMaxBatchR][kL];
    int32_t ex_q[kMaxExp];
    int32_t ex_node[kMaxExp];
    int32_t ex_ok[kMaxExp];
    int32_t ex_entry[kMaxExp];
    int64_t ex_req[kMaxExp][3];
    int32_t tnode[kTMax];       // pre-inserted entries' nodes (prologue)
    // per-pod ring (slot p % kRing)
    uint64_t best[kRing];       // pod p's winner (ikey), folded during iteration p - 1
    uint64_t lbk[kRing];        // lower bound of pod p's winner key (walker)
    int32_t kfull[kRing];       // pod p: every candidate taken and the list full -> stop
    int32_t cfull[kRing];       // pod p's list holds L entries
    uint64_t ckey[kRing][kNC];  // pod p's walked candidates (packed keys, 0 = none)
    int64_t crec[kRing][kNC][kFields];  // their snapshot records (walker, iteration p - 2)
    int64_t cpost[kRing][kNC][4];       // bound state rc rm rg nr if candidate c wins pod p
    uint64_t ck2[kRing][kNC];           // ... and its key for pod p + 1
    int32_t cfit[kRing][kNC];           // ... and its bind status (1 = Ok)
    int32_t n_t0, committed, err_code, err_pod, nb, e_cnt, n_final;
};

__device__ __forceinline__ uint64_t ikey(uint64_t key, int ent) {
    const uint32_t node = 0xFFFFFFFFu - (uint32_t)key;
    return ((key >> 32) << 34) | ((uint64_t)(0xFFFFFFu - node) << 10) | (uint64_t)(uint32_t)ent;
}
__device__ __forceinline__ int32_t ikey_node(uint64_t b) { return (int32_t)(0xFFFFFFu - (uint32_t)((b >> 10) & 0xFFFFFFu)); }
__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }
__device__ __forceinline__ void fold(uint64_t* slot, uint64_t k) {
    atomicMax((unsigned long long*)slot, (unsigned long long)k);
}

template <class SH>
__device__ __forceinline__ uint32_t hslot(int32_t node) {
    return ((uint32_t)node * 2654435761u) >> (32 - SH::kHashLog2);
}
template <class SH>
__device__ __forceinline__ int h_find(const SH& sh, int32_t node) {
    uint32_t s = hslot<SH>(node);
    for (int i = 0; i < SH::kHash; ++i) {
        const int32_t k = sh.hkey[s];
        if (k == node) return sh.hval[s];
        if (k == -1) return -1;
        s = (s + 1) & (SH::kHash - 1);
    }
    return -1;
}
template <class SH>
__device__ __forceinline__ void h_insert(SH& sh, int32_t node, int32_t idx) {
    uint32_t s = hslot<SH>(node);
    while (sh.hkey[s] != -1) s = (s + 1) & (SH::kHash - 1);
    sh.hkey[s] = node;
    sh.hval[s] = idx;
}
template <class SH>
__device__ __forceinline__ bool is_touched(const SH& sh, int32_t node, bool exact) {
    const uint32_t f = (uint32_t)node & (SH::kFilterBits - 1);
    if (!((sh.tfilt[f >> 5] >> (f & 31)) & 1u)) return false;
    return exact || h_find(sh, node) >= 0;
}

__device__ __forceinline__ int64_t node_field(const NodeSoA& s, int f, int64_t i) {
    return gptr(s.ac)[(int64_t)f * (s.am - s.ac) + i];
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Pod record from LDS: three 16-byte loads issued together, pinned (see pod_regs in ks_kernels).
__device__ __forceinline__ PodRec pod_lds(const PodRec* src) {
    const uint4* w = reinterpret_cast<const uint4*>(src);
    const uint4 w0 = w[0], w1 = w[1], w2 = w[2];
    asm volatile("" ::"v"(w0.x), "v"(w0.y), "v"(w0.z), "v"(w0.w), "v"(w1.x), "v"(w1.y), "v"(w1.z), "v"(w1.w),
                 "v"(w2.x), "v"(w2.y), "v"(w2.z), "v"(w2.w));
    PodRec p;
    __builtin_memcpy(&p, &w0, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p) + 16, &w1, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p) + 32, &w2, 16);
    return p;
}

__device__ __forceinline__ void add_req(NodeV& n, const PodRec& p, int64_t s) {
    n.rc += s * p.req[0];
    n.rm += s * p.req[1];
    n.rg += s * p.req[2];
    n.nr += s;
}

// Owner-lane state: NodeW (32-bit fields) in the narrow / tiny / micro domains, NodeV otherwise.
template <int kMode>
using StateT = typename std::conditional<kMode == kEvalWide, NodeV, NodeW>::type;

template <class NS>
__device__ __forceinline__ NS state_from(const NodeV& v);
template <>
__device__ __forceinline__ NodeV state_from<NodeV>(const NodeV& v) { return v; }
template <>
__device__ __forceinline__ NodeW state_from<NodeW>(const NodeV& v) {
    NodeW w;
    w.ac = (int32_t)v.ac; w.am = (int32_t)v.am; w.ag = (int32_t)v.ag;
    w.ap = v.ap > 0x7FFFFFFF ? 0x7FFFFFFF : (int32_t)v.ap;  // above any running count
    w.rc = (int32_t)v.rc; w.rm = (int32_t)v.rm; w.rg = (int32_t)v.rg; w.nr = (int32_t)v.nr;
    w.taint = v.taint; w.label = v.label;
    return w;
}

// CreatePod admission (kubesim/node/node.go:44-47) on either state type.  NodeW: requests
// clamped to 2^30 (above every capacity < 2^29 they fail alike), running totals <= capacity.
__device__ __forceinline__ bool fits_s(const PodRec& p, const NodeV& n) { return fits(p, n); }
__device__ __forceinline__ bool fits_s(const PodRec& p, const NodeW& n) {
    bool ok = n.nr < n.ap;
    if (p.keymask & 1) ok &= n.rc + clamp_req(p.req[0]) <= n.ac;
    if (p.keymask & 2) ok &= n.rm + clamp_req(p.req[1]) <= n.am;
    if (p.keymask & 4) ok &= n.rg + clamp_req(p.req[2]) <= n.ag;
    return ok;
}
// add (s = 1) / remove (s = -1) a pod that fits (so its requests are below the capacities)
template <class NS>
__device__ __forceinline__ void add_s(NS& n, const PodRec& p, int s) {
    using F = decltype(n.rc);
    n.rc += (F)s * (F)p.req[0];
    n.rm += (F)s * (F)p.req[1];
    n.rg += (F)s * (F)p.req[2];
    n.nr += (F)s;
}
template <class NS>
__device__ __forceinline__ void sub_req(NS& n, const int64_t* req) {
    using F = decltype(n.rc);
    n.rc -= (F)req[0];
    n.rm -= (F)req[1];
    n.rg -= (F)req[2];
    n.nr -= 1;
}
template <class NS>
__device__ __forceinline__ void acc_req(NS& d, const int64_t* req) {
    using F = decltype(d.rc);
    d.rc += (F)req[0];
    d.rm += (F)req[1];
    d.rg += (F)req[2];
    d.nr += 1;
}

// S minus the expiries of window range [e0, e1) that land on entry r (marking them expired when
// `mark`), skipping slot `skip` (a pod that is not bound yet).  Lane-divergent loop: every lane
// walks the (usually empty or one-slot) range.
template <class SH, class NS>
__device__ __forceinline__ void expire_own(const SH& sh, int e0, int e1, int r, int skip, NS& n,
                                           uint8_t* expired) {
    for (int x = e0; x < e1; ++x) {
        if (x == skip || sh.ex_entry[x] != r || !sh.ex_ok[x]) continue;
        sub_req(n, sh.ex_req[x]);
        if (expired) gptr(expired)[sh.ex_q[x]] = 1;
    }
}

// Upper bound of the total for pod (qc, qm) on a node with capacity reciprocals ic / im
// (ks_device.h prune_tmax), as a packed key with the node's index: below lbk => cannot win.
template <int kMode, class NS>
__device__ __forceinline__ bool may_reach(const Cfg& c, const NS& n, float ic, float im, float qc, float qm,
                                          uint32_t node, uint64_t lbk) {
    if (lbk == 0) return true;
    PruneF f;
    f.ic = ic;
    f.im = im;
    f.bc = n.ac > 0 ? (float)(n.ac - n.rc) * ic : -1.f;
    f.bm = n.am > 0 ? (float)(n.am - n.rm) * im : -1.f;
    f.live = c.has_scorers && !(c.filter_feeds && (c.filters & kFilterFit) && n.nr >= n.ap);
    if (!f.live) return false;
    return make_key(prune_tmax(c, f, qc, qm) + 1u, node) >= lbk;
}

template <int kMode, class C>
__global__ __launch_bounds__(C::kThreads) void resolve2_kernel(const EngineArgs* __restrict__ A) {
    using SH = Shared2<C>;
    constexpr int kHash = C::kHash, kMaxBatchR = C::kMaxBatchR, kMaxExp = C::kMaxExp, kFilterBits = C::kFilterBits,
                  kThreads = C::kThreads;
    __shared__ SH sh;
    const EngineArgs a = A[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const bool exact = a.c.n_nodes <= kFilterBits;
    int nb = (int)min<int64_t>(min<int64_t>(a.B, kMaxBatchR), end - start);
    if (nb <= 0) return;

    // ---- setup: window, pods, lists, expiry slots, pre-insert (as resolve_kernel)
    const int64_t e_base = a.exp_off[start + 1];
    const int64_t off_mid = tid < nb ? a.exp_off[start + tid + 1] : 0;
    const bool fits_win = tid < nb && off_mid - e_base <= kMaxExp;
    if (tid == 0) { sh.err_code = 0; sh.err_pod = -1; sh.n_t0 = 0; }
    if (tid < kRing) {
        sh.best[tid] = 0; sh.lbk[tid] = 0; sh.kfull[tid] = 0; sh.cfull[tid] = 0;
        for (int c = 0; c < kNC; ++c) sh.ckey[tid][c] = 0;
    }
    for (int h = tid; h < kHash; h += kThreads) sh.hkey[h] = -1;
    for (int w = tid; w < kFilterBits / 32; w += kThreads) sh.tfilt[w] = 0;
    nb = __syncthreads_count(fits_win);
    if (tid == nb - 1) { sh.nb = nb; sh.committed = nb; sh.e_cnt = nb > 1 ? (int32_t)(off_mid - e_base) : 0; }
    __syncthreads();
    const int e_cnt = sh.e_cnt;
    for (int i = tid; i < nb + 2; i += kThreads) {
        PodCtl pc{};
        if (i < nb) {
            const PodRec pr = a.pods[start + i];
            sh.pod[i] = pr;
            sh.podf[i][0] = (float)pr.req[0];
            sh.podf[i][1] = (float)pr.req[1];
            const int64_t pos = a.exp_pos[start + i];
            pc.flags = pr.flags;
            pc.ex_lo = i <= 1 ? 0 : (int32_t)(a.exp_off[start + i] - e_base);
            pc.ex_hi = i + 1 <= 1 ? 0 : (int32_t)(a.exp_off[start + i + 1] - e_base);
            pc.dur = a.dur[start + i];
            pc.exp_slot = (pos >= e_base && pos - e_base < e_cnt) ? (int32_t)(pos - e_base) : -1;
            // pod i's own expiry due right before pod i + 1 (it then never counts for pod i+1)
            const int32_t nlo = pc.ex_hi;
            const int32_t nhi = i + 2 <= 1 ? 0 : (i + 1 < nb ? (int32_t)(a.exp_off[start + i + 2] - e_base) : nlo);
            pc.nxt_own = pc.exp_slot >= nlo && pc.exp_slot < nhi;
        } else {
            sh.pod[i] = PodRec{{0, 0, 0}, 0, 0, 0, 0};
            sh.podf[i][0] = sh.podf[i][1] = 0.f;
            pc.exp_slot = -1;
        }
        sh.pctl[i] = pc;
    }
    for (int i = tid; i < nb * kL; i += kThreads) sh.cand[i / kL][i % kL] = a.cand[i];
    for (int e = tid; e < e_cnt; e += kThreads) {
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
    // pre-insert every node an expiry of this batch lands on (q bound before the batch): claim
    // the node's hash slot with a CAS (duplicates find it; the slot parks in ex_entry, bit 30 =
    // claimed), number the claimed slots, then read the entry back
    for (int e = tid; e < e_cnt; e += kThreads) {
        if (!sh.ex_ok[e]) continue;
        const int32_t nd = sh.ex_node[e];
        uint32_t hs = hslot<SH>(nd);
        for (;;) {  // the table holds <= kMaxExp < kHash nodes: terminates
            const int32_t prev = atomicCAS(&sh.hkey[hs], -1, nd);
            if (prev == -1 || prev == nd) { sh.ex_entry[e] = (int32_t)hs | (prev == -1 ? (1 << 30) : 0); break; }
            hs = (hs + 1) & (kHash - 1);
        }
    }
    __syncthreads();
    for (int e = tid; e < e_cnt; e += kThreads) {
        if (!sh.ex_ok[e] || !(sh.ex_entry[e] >> 30)) continue;
        const int32_t nd = sh.ex_node[e];
        const int idx = atomicAdd(&sh.n_t0, 1);
        sh.hval[sh.ex_entry[e] & 0xFFFF] = idx;
        sh.tnode[idx] = nd;
        const uint32_t f = (uint32_t)nd & (kFilterBits - 1);
        atomicOr(&sh.tfilt[f >> 5], 1u << (f & 31));
    }
    __syncthreads();
    for (int e = tid; e < e_cnt; e += kThreads)
        if (sh.ex_ok[e]) sh.ex_entry[e] = sh.hval[sh.ex_entry[e] & 0xFFFF];
    __syncthreads();
    const int n_t0 = sh.n_t0;

    // ---- roles
    constexpr int kE = C::kE, kNL = C::kNL;
    const int oslot = wave - kOwnerWave0;           // owner waves: lane g owns entries k * kNL + g
    const int g = oslot >= 0 ? oslot * kWave + lane : 0;
    // entries grow by at most one per pod: owner waves that can never own one end after setup
    if (oslot >= 0 && oslot * kWave >= n_t0 + nb) return;

    using NT = StateT<kMode>;
    NT S[kE];                 // owner: S_r(i) of entry r = k * kNL + g (state when pod i is evaluated)
    int32_t own_node[kE];
    float ic[kE], im[kE];     // capacity reciprocals (prune bounds)
    uint64_t K1[kE], K2[kE];  // keys for pod i + 1: r does not / does win pod i
#pragma unroll
    for (int k = 0; k < kE; ++k) { S[k] = NT{}; own_node[k] = -1; ic[k] = im[k] = 0.f; K1[k] = K2[k] = 0; }

    // the address a walker lane loads: field lane % 10 of candidate lane / 10 of pod p, or a
    // dummy (node 0's first field) — every lane loads unconditionally, so the loads of one
    // iteration are always one instruction and the wait for them can be counted
    const int64_t* dummy = a.s.ac;
    auto walk = [&](int p, int32_t excl) -> const int64_t* {
        // wave 0: pod p's first kNC untouched list entries (node `excl` counts as touched: it joins
        // the table this iteration), the lower bound of pod p's winner, and their record loads
        const uint64_t c = lane < kL ? sh.cand[p][lane] : 0ull;
        const int32_t cn = key_node(c);
        const bool ok = c != 0 && cn != excl && !is_touched(sh, cn, exact);
        const uint64_t m = __ballot(ok);
        const bool full = __popcll(__ballot(c != 0)) == kL;
        const int rank = __popcll(m & ((1ull << lane) - 1ull));
        const int slot = p % kRing;
        if (ok && rank < kNC) sh.ckey[slot][rank] = c;
        const int nf = __popcll(m) < kNC ? __popcll(m) : kNC;
        if (lane >= nf && lane < kNC) sh.ckey[slot][lane] = 0ull;
        // lbk: the kNC-th candidate survives any kLA - 1 further joins; with fewer, the last one
        // does if the list is full (else the batch stops at an exhausted list), or none
        uint64_t lb = 0;
        const int want = nf == kNC ? kNC - 1 : (full && nf > 0 ? nf - 1 : -1);
        if (want >= 0) {
            uint64_t mm = m;
            for (int k = 0; k < want; ++k) mm &= mm - 1;
            lb = readlane64(c, __ffsll((unsigned long long)mm) - 1);
        }
        if (lane == 0) { sh.lbk[slot] = lb; sh.cfull[slot] = full; }
        // field lane % 10 of candidate lane / 10 (the candidate's node from its rank)
        const int cslot = lane / kFields;
        uint64_t mm = m;
        for (int k = 0; k < cslot && mm; ++k) mm &= mm - 1;
        const int src = mm ? __ffsll((unsigned long long)mm) - 1 : 0;
        const uint64_t ck = __shfl(c, src);
        return (lane < kNC * kFields && cslot < nf)
                   ? a.s.ac + (int64_t)(lane % kFields) * (a.s.am - a.s.ac) + key_node(ck) : dummy;
    };
    auto gload = [](const int64_t* p) -> int64_t { return *gptr(p); };
    auto stage_recs = [&](int p, int64_t v) {
        // wave 0: pod p's landed candidate records into LDS (lane = candidate * 10 + field)
        if (lane < kNC * kFields) sh.crec[p % kRing][lane / kFields][lane % kFields] = v;
    };
    auto eval_cands = [&](int p) {
        // wave 1, lanes < kNC: "candidate c wins pod p": bind status, bound state, key for pod p+1
        const int slot = p % kRing;
        if (lane < kNC) {
            const uint64_t ck = sh.ckey[slot][lane];
            if (ck != 0) {
                const int64_t* f = sh.crec[slot][lane];
                NodeV n;
                n.ac = f[0]; n.am = f[1]; n.ag = f[2]; n.ap = f[3]; n.rc = f[4]; n.rm = f[5]; n.rg = f[6];
                n.nr = f[7]; n.taint = (uint64_t)f[8]; n.label = (uint64_t)f[9];
                const PodRec pp = pod_lds(&sh.pod[p]);
                const PodCtl pc = sh.pctl[p];
                const bool fit = fits(pp, n);
                if (fit && pc.dur > 0) add_req(n, pp, 1);
                sh.cpost[slot][lane][0] = n.rc; sh.cpost[slot][lane][1] = n.rm;
                sh.cpost[slot][lane][2] = n.rg; sh.cpost[slot][lane][3] = n.nr;
                sh.cfit[slot][lane] = fit;
                uint64_t k2 = 0;
                if (p + 1 < nb) {
                    if (fit && pc.dur > 0 && pc.nxt_own) add_req(n, pp, -1);  // expires before pod p+1
                    const PodRec pn = pod_lds(&sh.pod[p + 1]);
                    k2 = make_key(eval_t<kMode>(a.c, pn, n), (uint32_t)key_node(ck));
                }
                sh.ck2[slot][lane] = k2;
            }
        }
    };
    // LC of pod p: its first candidate that none of the recent winners took; `x*` = nodes of the
    // candidate winners since pod p's walk (-1 for touched winners / none)
    auto fold_lc = [&](int p, int32_t x0, int32_t x1, int32_t x2) {
        const int slot = p % kRing;
        const uint64_t ck = lane < kNC ? sh.ckey[slot][lane] : 0ull;
        const int32_t cn = key_node(ck);
        const bool ok = ck != 0 && cn != x0 && cn != x1 && cn != x2;
        const uint64_t m = __ballot(ok);
        if (m) {
            const int l = __ffsll((unsigned long long)m) - 1;
            if (lane == l) fold(&sh.best[slot], ikey(ck, kEntCand + l));
        }
        if (lane == 0) sh.kfull[slot] = (m == 0 && sh.cfull[slot] && p > 0) ? 1 : 0;
    };

    // ---- prologue: walks of pods 0 .. kLA-1 (records staged), owner states, pod 0's contributions
    if (wave == 0) {
        for (int p = 0; p < kLA && p < nb; ++p) stage_recs(p, gload(walk(p, -1)));
    } else if (oslot >= 0) {
#pragma unroll
        for (int k = 0; k < kE; ++k) {
            const int r = k * kNL + g;
            if (r < n_t0) {
                own_node[k] = sh.tnode[r];
                S[k] = state_from<NT>(load_node(a.s, own_node[k]));
                ic[k] = S[k].ac > 0 ? rcp_est((float)S[k].ac) : 0.f;
                im[k] = S[k].am > 0 ? rcp_est((float)S[k].am) : 0.f;
            }
        }
    }
    __syncthreads();
    if (wave == 1) {
        eval_cands(0);
        fold_lc(0, -1, -1, -1);
    } else if (oslot >= 0) {
        // key_0 folded now; K1 / K2 (pod 1, r does not / does win pod 0) into registers
        const PodRec p0 = pod_lds(&sh.pod[0]);
        const PodRec p1 = pod_lds(&sh.pod[1]);
        const PodCtl c0 = sh.pctl[0], c1 = sh.pctl[1];
        const uint64_t lb0 = sh.lbk[0], lb1 = sh.lbk[1 % kRing];
#pragma unroll
        for (int k = 0; k < kE; ++k) {
            const int r = k * kNL + g;
            if (r >= n_t0) continue;
            if (may_reach<kMode>(a.c, S[k], ic[k], im[k], sh.podf[0][0], sh.podf[0][1], own_node[k], lb0)) {
                const uint64_t kk = make_key(eval_t<kMode>(a.c, p0, S[k]), (uint32_t)own_node[k]);
                if (kk != 0 && kk >= lb0) {
                    fold(&sh.best[0], ikey(kk, r));
                    if (nb > 1) {
                        NT T = S[k];
                        if (fits_s(p0, T) && c0.dur > 0 && !c0.nxt_own) add_s(T, p0, 1);
                        expire_own(sh, c1.ex_lo, c1.ex_hi, r, c0.exp_slot, T, nullptr);
                        K2[k] = make_key(eval_t<kMode>(a.c, p1, T), (uint32_t)own_node[k]);
                    }
                }
            }
            if (nb > 1) {
                NT T = S[k];
                expire_own(sh, c1.ex_lo, c1.ex_hi, r, c0.exp_slot, T, nullptr);
                if (may_reach<kMode>(a.c, T, ic[k], im[k], sh.podf[1][0], sh.podf[1][1], own_node[k], lb1))
                    K1[k] = make_key(eval_t<kMode>(a.c, p1, T), (uint32_t)own_node[k]);
            }
        }
    }
    __syncthreads();

    // ---- main loop: one loop per role, one barrier per pod in each (every role reads the same
    // decision words, so all of them stop at the same pod).  Role-local loops keep each role's
    // memory operations out of the others' wait counting: the walker's record loads stay in
    // flight across two barriers.
    int nt = n_t0;  // table size before pod i (uniform)
    int i = 0;
#ifdef KS_STAMPS
    uint64_t acc_work = 0;
#endif
    auto decision = [&](int i, int& ent, int32_t& nd) -> int {
        const uint64_t bw = sh.best[i % kRing];
        const int kf = sh.kfull[i % kRing];
        const uint32_t flags = sh.pctl[i].flags;
        ent = (int)(bw & 1023u);
        nd = ikey_node(bw);
        if (kf) return 1;                                     // list exhausted: rescan
        if (bw == 0) return 2;                                // NotFound
        if (flags & (kFlagBadKey | kFlagBadSpec)) return 3;   // InvalidArgument
        return 0;
    };
    auto barrier = [&]() {
        // LDS only crosses it: the walker's record loads stay in flight (no vmcnt wait)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
#ifdef KS_STAMPS
    // work = from leaving the previous barrier (or the loop entry) to entering the next one,
    // wait = inside the barrier
    uint64_t acc_wait = 0, t_left = __builtin_amdgcn_s_memtime();
#define KS_T0
#define KS_T1 const uint64_t _s1 = __builtin_amdgcn_s_memtime(); acc_work += _s1 - t_left;
#define KS_T2 t_left = __builtin_amdgcn_s_memtime(); acc_wait += t_left - _s1;
#else
#define KS_T0
#define KS_T1
#define KS_T2
#endif

    if (wave == 0) {
        // walker: pod i+kLA's list and its record loads; the loads of iteration i-1 (pod i+3)
        // are staged into LDS first (one iteration in flight)
        int64_t v = 0;
        for (;; ++i) {
            int ent;
            int32_t nd;
            const int stop = i < nb ? decision(i, ent, nd) : 4;
            if (stop) {
                if (lane == 0 && stop < 4) {
                    sh.committed = i;
                    if (stop > 1) { sh.err_code = stop == 2 ? kErrNotFound : kErrEinval; sh.err_pod = (int32_t)(start + i); }
                }
                break;
            }
            KS_T0
            const bool is_cand = ent >= kEntCand;
            if (lane == 0) sh.best[(i + 2) % kRing] = 0;  // pod i+2's word: folded from iteration i+1
            if (i >= 1 && i + kLA - 1 < nb) stage_recs(i + kLA - 1, v);
            v = gload(i + kLA < nb ? walk(i + kLA, is_cand ? nd : -1) : dummy);
            nt += is_cand;
            KS_T1
            barrier();
            KS_T2
        }
    } else if (wave == 1) {
        // candidate wave: folds pod i+1's LC and the new entry's key for pod i+1, evaluates
        // "candidate c wins pod i+1" (lanes < kNC).  All reads of an iteration in one batch.
        int32_t w0 = -1, w1 = -1, w2 = -1;  // nodes of the last three candidate winners
        for (; i < nb; ++i) {
            const int s0 = i % kRing, s1 = (i + 1) % kRing;
            const uint64_t bw = sh.best[s0];
            const int kf = sh.kfull[s0];
            const uint32_t flags = sh.pctl[i].flags;
            const uint64_t k2v = lane < kNC ? sh.ck2[s0][lane] : 0ull;
            const uint64_t ck = lane < kNC ? sh.ckey[s1][lane] : 0ull;
            const int cfl = sh.cfull[s1];
            NodeV n{};
            if (lane < kNC) {
                const int64_t* f = sh.crec[s1][lane];
                n.ac = f[0]; n.am = f[1]; n.ag = f[2]; n.ap = f[3]; n.rc = f[4]; n.rm = f[5]; n.rg = f[6];
                n.nr = f[7]; n.taint = (uint64_t)f[8]; n.label = (uint64_t)f[9];
            }
            const PodRec pp = pod_lds(&sh.pod[i + 1]);
            const PodRec pn = pod_lds(&sh.pod[i + 2]);
            const PodCtl pc = sh.pctl[i + 1];
            if (kf || bw == 0 || (flags & (kFlagBadKey | kFlagBadSpec))) break;
            KS_T0
            const int ent = (int)(bw & 1023u);
            const int32_t nd = ikey_node(bw);
            const bool is_cand = ent >= kEntCand;
            if (is_cand) {
                const uint64_t k2 = readlane64(k2v, ent - kEntCand);
                if (lane == 0 && i + 1 < nb && k2 != 0) fold(&sh.best[s1], ikey(k2, nt));
                w2 = w1; w1 = w0; w0 = nd;
            } else {
                w2 = w1; w1 = w0; w0 = -1;
            }
            if (i + 1 < nb) {
                // pod i+1's LC: its first candidate none of the last three winners took
                const int32_t cn = key_node(ck);
                const bool ok = ck != 0 && cn != w0 && cn != w1 && cn != w2;
                const uint64_t m = __ballot(ok);
                if (m && lane == __ffsll((unsigned long long)m) - 1) fold(&sh.best[s1], ikey(ck, kEntCand + lane));
                if (lane == 0) sh.kfull[s1] = (m == 0 && cfl) ? 1 : 0;
                // "candidate lane wins pod i+1": bind status, bound state, key for pod i+2
                if (lane < kNC && ck != 0) {
                    const bool fit = fits(pp, n);
                    if (fit && pc.dur > 0) add_req(n, pp, 1);
                    sh.cpost[s1][lane][0] = n.rc; sh.cpost[s1][lane][1] = n.rm;
                    sh.cpost[s1][lane][2] = n.rg; sh.cpost[s1][lane][3] = n.nr;
                    sh.cfit[s1][lane] = fit;
                    uint64_t k2 = 0;
                    if (i + 2 < nb) {
                        if (fit && pc.dur > 0 && pc.nxt_own) add_req(n, pp, -1);  // expires before pod i+2
                        k2 = make_key(eval_t<kMode>(a.c, pn, n), (uint32_t)cn);
                    }
                    sh.ck2[s1][lane] = k2;
                }
            }
            nt += is_cand;
            KS_T1
            barrier();
            KS_T2
        }
    } else {
        // owners: the states of lane g's entries in registers.  Everything an iteration reads that
        // does not depend on the decision is read in one batch at its top; the bound states of
        // pod i's candidates are read only by the wave that would own a new entry.
        const int wlo = oslot * kWave;
        int32_t w0 = -1, w1 = -1, w2 = -1;  // nodes of the last three candidate winners
        for (; i < nb; ++i) {
            // ---- batch 1
            const uint64_t bw = sh.best[i % kRing];
            const int kf = sh.kfull[i % kRing];
            const PodCtl cA = sh.pctl[i], cB = sh.pctl[i + 1], cC = sh.pctl[i + 2];
            uint64_t cb[kNC], cc[kNC];  // the walked candidates of pods i+1 and i+2
#pragma unroll
            for (int c = 0; c < kNC; ++c) { cb[c] = sh.ckey[(i + 1) % kRing][c]; cc[c] = sh.ckey[(i + 2) % kRing][c]; }
            const int fullC = sh.cfull[(i + 2) % kRing];
            const float qCc = sh.podf[i + 2][0], qCm = sh.podf[i + 2][1];
            const int gn = nt % kNL;  // owner lane of entry nt (a new entry this pod)
            const bool may_new = gn >= wlo && gn < wlo + kWave;
            int64_t nf[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // lanes < kNC: candidate lane's bound state
            int32_t nfit = 0;
            uint64_t nk2 = 0;
            if (may_new && lane < kNC) {
                const int slot = i % kRing;
                const int64_t* f = sh.crec[slot][lane];
                nf[0] = f[0]; nf[1] = f[1]; nf[2] = f[2]; nf[3] = f[3]; nf[8] = f[8]; nf[9] = f[9];
                nf[4] = sh.cpost[slot][lane][0]; nf[5] = sh.cpost[slot][lane][1];
                nf[6] = sh.cpost[slot][lane][2]; nf[7] = sh.cpost[slot][lane][3];
                nfit = sh.cfit[slot][lane];
                nk2 = sh.ck2[slot][lane];
            }
            if (kf || bw == 0 || (cA.flags & (kFlagBadKey | kFlagBadSpec))) break;
            KS_T0
            const int ent = (int)(bw & 1023u);
            const int32_t nd = ikey_node(bw);
            const int64_t j = start + i;
            const bool is_cand = ent >= kEntCand;
            const int cs = ent - kEntCand;
            const int t = is_cand ? nt : ent;  // the winner's entry (a candidate becomes entry nt)
            const int gt = t % kNL, kt = t / kNL;
            const bool has1 = i + 1 < nb, has2 = i + 2 < nb;
            w2 = w1; w1 = w0; w0 = is_cand ? nd : -1;
            // Thresholds from the candidate lists, with every winner known by now excluded:
            // pod i+1's LC is exact (its remaining joins are t_{i-2}, t_{i-1}, t_i: all known) —
            // no key below it can win; pod i+2's LC is its first remaining candidate unless
            // t_{i+1} takes it, so it is at least the second remaining one (the first when the
            // list is full and only one remains: the batch stops otherwise; else 0).
            uint64_t lbB = 0, lbC = 0;
            {
                int nb_ok = 0, nc_ok = 0;
                uint64_t c0k = 0, c1k = 0;
#pragma unroll
                for (int c = 0; c < kNC; ++c) {
                    const int32_t nb_ = key_node(cb[c]);
                    if (cb[c] != 0 && nb_ != w0 && nb_ != w1 && nb_ != w2 && nb_ok == 0) { lbB = cb[c]; nb_ok = 1; }
                    const int32_t nc_ = key_node(cc[c]);
                    if (cc[c] != 0 && nc_ != w0 && nc_ != w1) {
                        if (nc_ok == 0) c0k = cc[c];
                        else if (nc_ok == 1) c1k = cc[c];
                        ++nc_ok;
                    }
                }
                lbC = nc_ok >= 2 ? c1k : (nc_ok == 1 && fullC ? c0k : 0ull);
            }
            uint64_t kk[kE];                   // key_{i+1} of each entry
#pragma unroll
            for (int k = 0; k < kE; ++k) kk[k] = (k == kt && g == gt) ? K2[k] : K1[k];
            if (gt >= wlo && gt < wlo + kWave) {
                // this wave holds pod i's winner: bind (kubesim/node/node.go:36-58)
                if (is_cand) {  // the candidate wave evaluated the bind; take its bound state
                    NodeV v;
                    v.ac = (int64_t)readlane64((uint64_t)nf[0], cs); v.am = (int64_t)readlane64((uint64_t)nf[1], cs);
                    v.ag = (int64_t)readlane64((uint64_t)nf[2], cs); v.ap = (int64_t)readlane64((uint64_t)nf[3], cs);
                    v.rc = (int64_t)readlane64((uint64_t)nf[4], cs); v.rm = (int64_t)readlane64((uint64_t)nf[5], cs);
                    v.rg = (int64_t)readlane64((uint64_t)nf[6], cs); v.nr = (int64_t)readlane64((uint64_t)nf[7], cs);
                    v.taint = readlane64((uint64_t)nf[8], cs); v.label = readlane64((uint64_t)nf[9], cs);
                    const int32_t f1 = __builtin_amdgcn_readlane(nfit, cs);
                    const uint64_t k2 = readlane64(nk2, cs);
                    if (g == gt) {
#pragma unroll
                        for (int k = 0; k < kE; ++k)
                            if (k == kt) {
                                S[k] = state_from<NT>(v);
                                kk[k] = k2;
                                own_node[k] = nd;
                                ic[k] = v.ac > 0 ? rcp_est((float)v.ac) : 0.f;
                                im[k] = v.am > 0 ? rcp_est((float)v.am) : 0.f;
                            }
                        // install: filter bit (+ hash for inexact filters); the walker of this
                        // iteration excludes nd explicitly
                        const uint32_t fb = (uint32_t)nd & (kFilterBits - 1);
                        atomicOr(&sh.tfilt[fb >> 5], 1u << (fb & 31));
                        if (!exact) h_insert(sh, nd, t);
                        gptr(a.b_node)[j] = nd;
                        gptr(a.b_status)[j] = f1 ? 0 : 1;
                        if (cA.exp_slot >= 0) { sh.ex_entry[cA.exp_slot] = t; sh.ex_ok[cA.exp_slot] = f1 ? 1 : 0; }
                    }
                } else if (g == gt) {
                    const PodRec pA = pod_lds(&sh.pod[i]);
                    bool fit = false;
#pragma unroll
                    for (int k = 0; k < kE; ++k)
                        if (k == kt) {
                            fit = fits_s(pA, S[k]);
                            if (fit && cA.dur > 0) add_s(S[k], pA, 1);
                        }
                    gptr(a.b_node)[j] = nd;
                    gptr(a.b_status)[j] = fit ? 0 : 1;
                    if (cA.exp_slot >= 0) { sh.ex_entry[cA.exp_slot] = t; sh.ex_ok[cA.exp_slot] = fit ? 1 : 0; }
                }
            }
            const int live = nt + (is_cand ? 1 : 0);
            if (has1 && wlo < live) {
                // fold key_{i+1}(r) (the new entry's is folded by the candidate wave)
#pragma unroll
                for (int k = 0; k < kE; ++k) {
                    const int r = k * kNL + g;
                    if (r < live && !(is_cand && r == t) && kk[k] != 0 && kk[k] >= lbB)
                        fold(&sh.best[(i + 1) % kRing], ikey(kk[k], r));
                }
                // ---- batch 2: the expiry slots of pods i+1 and i+2 ([cB.ex_lo, cC.ex_hi),
                // contiguous) that land on this wave's entries, lane-parallel; each hit goes to its
                // entry's lane
                NT D2[kE];  // pod i+2's expiries on each entry (applied to the evaluation state only)
#pragma unroll
                for (int k = 0; k < kE; ++k) D2[k] = NT{};
                const int e0 = cB.ex_lo, e1 = has2 ? cC.ex_hi : cB.ex_hi;
                for (int x0 = e0; x0 < e1; x0 += kWave) {
                    const int x = x0 + lane;
                    int32_t ee = -1, ok = 0;
                    if (x < e1) { ee = sh.ex_entry[x]; ok = sh.ex_ok[x]; }
                    const int ge = ee % kNL;
                    uint64_t hits = __ballot(x < e1 && ok && ee >= 0 && ge >= wlo && ge < wlo + kWave);
                    while (hits) {
                        const int l = __ffsll((unsigned long long)hits) - 1;
                        hits &= hits - 1;
                        const int xe = x0 + l;
                        const int eh = __builtin_amdgcn_readlane(ee, l);
                        if (g == eh % kNL) {
                            const int kh = eh / kNL;
#pragma unroll
                            for (int k = 0; k < kE; ++k)
                                if (k == kh) {
                                    if (xe < cB.ex_hi) {       // due before pod i+1: S_r(i+1)
                                        sub_req(S[k], sh.ex_req[xe]);
                                        gptr(a.expired)[sh.ex_q[xe]] = 1;
                                    } else if (xe != cB.exp_slot) {  // due before pod i+2 (pod i+1 unbound)
                                        acc_req(D2[k], sh.ex_req[xe]);
                                    }
                                }
                        }
                    }
                }
                // ---- K1 / K2 for pod i + 2
                if (has2) {
                    PodRec pC, pB;
                    bool haveC = false, haveB = false;
#pragma unroll
                    for (int k = 0; k < kE; ++k) {
                        K1[k] = 0;
                        K2[k] = 0;
                        const int r = k * kNL + g;
                        const bool mine = r < live;
                        NT T = S[k];
                        T.rc -= D2[k].rc; T.rm -= D2[k].rm; T.rg -= D2[k].rg; T.nr -= D2[k].nr;
                        const bool pass1 = mine && may_reach<kMode>(a.c, T, ic[k], im[k], qCc, qCm, own_node[k], lbC);
                        const bool can_win = mine && kk[k] != 0 && kk[k] >= lbB;  // K2 only if r can win pod i+1
#ifdef KS_STAMPS
                        if (lane == 0) {
                            const uint64_t bp = __ballot(pass1), bc = __ballot(can_win);
                            atomicAdd((unsigned long long*)a.ctr + 9, (unsigned long long)__popcll(bp));
                            atomicAdd((unsigned long long*)a.ctr + 10, (unsigned long long)(bp != 0));
                            atomicAdd((unsigned long long*)a.ctr + 11, (unsigned long long)__popcll(bc));
                            atomicAdd((unsigned long long*)a.ctr + 12, (unsigned long long)(lbC == 0));
                        }
#endif
                        if (__ballot(pass1 || can_win)) {
                            if (!haveC) { pC = pod_lds(&sh.pod[i + 2]); haveC = true; }
                            if (pass1) K1[k] = make_key(eval_t<kMode>(a.c, pC, T), (uint32_t)own_node[k]);
                            if (__ballot(can_win)) {
                                if (!haveB) { pB = pod_lds(&sh.pod[i + 1]); haveB = true; }
                                if (can_win) {
                                    if (fits_s(pB, S[k]) && cB.dur > 0 && !cB.nxt_own) {
                                        add_s(T, pB, 1);
                                        if (may_reach<kMode>(a.c, T, ic[k], im[k], qCc, qCm, own_node[k], lbC))
                                            K2[k] = make_key(eval_t<kMode>(a.c, pC, T), (uint32_t)own_node[k]);
                                    } else {
                                        K2[k] = K1[k];  // the bind leaves the state as it was for pod i+2
                                    }
                                }
                            }
                        }
                    }
                }
            }
            nt += is_cand;
            KS_T1
            barrier();
            KS_T2
        }
    }
#undef KS_T0
#undef KS_T1
#undef KS_T2
    __syncthreads();
#ifdef KS_STAMPS
    if (lane == 0) atomicAdd((unsigned long long*)a.ctr + 16 + wave, (unsigned long long)acc_work);
    if (lane == 0 && wave < 3) atomicAdd((unsigned long long*)a.ctr + 6 + wave, (unsigned long long)acc_wait);
    if (tid == 0) atomicAdd((unsigned long long*)a.ctr + 5, (unsigned long long)sh.committed);
#endif

    // ---- write back the mutable fields of every touched entry
    if (oslot >= 0) {
#pragma unroll
        for (int k = 0; k < kE; ++k)
            if (k * kNL + g < nt) {
                gptr(a.s.rc)[own_node[k]] = S[k].rc;
                gptr(a.s.rm)[own_node[k]] = S[k].rm;
                gptr(a.s.rg)[own_node[k]] = S[k].rg;
                gptr(a.s.nr)[own_node[k]] = S[k].nr;
            }
    }
    if (tid == 0) {
        a.ctr[kCtrStart] = start + sh.committed;
        if (sh.committed < a.B && sh.err_code == 0 && start + sh.committed < end) a.ctr[kCtrEarly] += 1;
        if (sh.err_code) { a.ctr[kCtrErr] = sh.err_code; a.ctr[kCtrErrPod] = sh.err_pod; }
    }
}

}  // namespace r2

template <class C>
static void launch_resolve2_t(const EngineArgs* d, int S, int mode, hipStream_t st) {
    using namespace r2;
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL((resolve2_kernel<kEvalMicro, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        case kEvalTiny: hipLaunchKernelGGL((resolve2_kernel<kEvalTiny, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        case kEvalNarrow: hipLaunchKernelGGL((resolve2_kernel<kEvalNarrow, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
        default: hipLaunchKernelGGL((resolve2_kernel<kEvalWide, C>), dim3(S), dim3(C::kThreads), 0, st, d); break;
    }
}

hipError_t launch_resolve2(const EngineArgs* d, int S, int mode, bool small, hipStream_t st) {
    if (small)
        launch_resolve2_t<r2::RSmall2>(d, S, mode, st);
    else
        launch_resolve2_t<r2::RBig2>(d, S, mode, st);
    return hipGetLastError();
}

}  // namespace ks
