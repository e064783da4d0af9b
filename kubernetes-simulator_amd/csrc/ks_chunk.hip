// ks_chunk.hip — the chunk resolver (gfx950): a batch's binds by chunked Jacobi sweeps in LDS.
//
// The reference binds one pod per tick in FIFO order (kubesim/kubesim.go:105-121, 143-166): pod i
// takes the argmax of its key over every node, on the state that the binds of pods < i (admitted
// per kubesim/node/node.go:36-60) and the expiries due by its tick leave.  Write f_i(w_{<i}) for
// that argmax given the earlier winners.  This resolver splits f_i into
//   S_i(W) = the first entry of pod i's static candidate list cl_i whose node no earlier pod bound
//            (cl_i, built by cand_list, ks_cand.hip: pod i's snapshot top-L list entries that no pre-batch
//            expiry of the window touches — their snapshot key is exact while unbound — and every
//            expiry node E whose exact key at pod i's tick reaches thr_i, the list's last key; any
//            other node scores below thr_i), and
//   D_i(w) = the max over the nodes the earlier pods bound of pod i's key on their replayed state
//            (binds with admission, pre-batch expiries, the bound pods' own expiries),
// f_i = max(S_i, D_i), with the exhausted-list / NotFound / bad-pod stops of the other resolvers.
// The batch is cut into chunks of 64 pods (one lane each).  Pods before a chunk are final; inside
// it w^{t+1}_i = f_i(w^t_{<i}) is iterated until the chunk's winners repeat — after sweep t the
// first t pods are exact (induction), so this is the sequential result — and each sweep recomputes
// only the pods after the previous sweep's first change.  D_i of nodes bound before the chunk is
// computed once per chunk (each pod's top two, a node rebound inside the chunk excluded); only the
// chunk's own binds are replayed every sweep.  One workgroup, every structure in LDS; measured
// design counts on C3 (tests/dev/gv_model.py, exact model): ~18 sweeps per 256-pod batch.
#include <climits>

#include "ks_device.h"
#include "ks_scan.h"
#include "ks_prep.h"

namespace ks {
namespace chk {

constexpr int kThreads = 512;   // 8 waves: 256 VGPRs per lane (no spills)
constexpr int kLanesPerPod = kThreads / 64;  // sweep phases: 64 chunk pods x 8 lanes
constexpr int kB = kWinMaxB;  // pods per batch
constexpr int kC = 64;          // pods per chunk: one lane each
constexpr int kR = kChR;        // static candidates kept per pod
constexpr int kCid = 1024;      // candidate ids per batch (the batch's candidate slots)
constexpr int kMaxPGScan = 32;  // pods per scan group (the host's PG bound, ks_kernels.hip kMaxPG)
constexpr int kCidSlots = kCid - kR;  // claim-order cids: slots that are cids; the rest: pod 0's private cids
constexpr int kSlots = kWinSlots;
constexpr int kSeg = 5;         // stored state segments per replayed node within a chunk
constexpr int kPend = 4;        // pending own expiries per replayed node
constexpr int kWaves = kThreads / kWave;
constexpr int16_t kNoSeg = INT16_MAX;
constexpr int kNoOwn = 0x7FFF;  // (brow: no own expiry in the window)
constexpr int kMOvf = kSeg, kMCid = kSeg + 1;
static_assert(kSeg + 2 <= 8, "slot row");
static_assert(kB <= 256 && kB % kC == 0, "chunks of one wave");
static_assert(kR <= 32, "two entries per lane of a 16-lane pod group");

// Diagnostic build only (-DKS_CHUNK_DIAG, `make chunkdiag`): counters in ctr[5..31]
// (layout: tests/dev/diag_chunk.py); the real kernel executes none of it.
#ifdef KS_CHUNK_DIAG
__device__ __forceinline__ uint64_t dstamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define DG(...) __VA_ARGS__
#else
#undef KS_CHUNK_ABL
#define DG(...)
#endif

#ifndef KS_CHUNK_ABL
#define KS_CHUNK_ABL 0  // diagnostic ablations (timing only, results invalid): 1 no D pairs, 2 no replays
#endif

// A node's state in 32-bit words: capacities and usage as uint32 (scaled capacities < 2^32 - 1;
// 0xFFFFFFFF = an absent capacity, -1), `ap` and `nr` as int32 (`ap` clamped).  Evaluator modes
// >= narrow (capacities < 2^29) read the words as int32 directly; the wide mode (the decimal-SI
// memory class: capacities up to 2^31 after the gcd scaling) widens them (wide_node) and runs the
// wide evaluator.  Usage never exceeds its capacity (admission), so uint32 arithmetic is exact.
struct NS32 {
    int32_t ac, am, ag, ap, rc, rm, rg, nr;
    uint64_t taint, label;
};

__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }
__device__ __forceinline__ int32_t clamp32(int64_t v) { return (int32_t)(v > INT_MAX ? INT_MAX : v); }
__device__ __forceinline__ int64_t cap64(int32_t w) { return w == -1 ? -1 : (int64_t)(uint32_t)w; }
__device__ __forceinline__ int64_t use64(int32_t w) { return (int64_t)(uint32_t)w; }
// a capacity or usage in one word (values in [-1, 2^32 - 1))
__device__ __forceinline__ int32_t word32(int64_t v) { return (int32_t)(uint32_t)v; }

__device__ __forceinline__ NodeV wide_node(const NS32& n) {
    NodeV v;
    v.ac = cap64(n.ac); v.am = cap64(n.am); v.ag = cap64(n.ag); v.ap = n.ap;
    v.rc = use64(n.rc); v.rm = use64(n.rm); v.rg = use64(n.rg); v.nr = n.nr;
    v.taint = n.taint; v.label = n.label;
    return v;
}
template <int kMode>
__device__ __forceinline__ uint32_t eval32(const Cfg& c, const PodRec& p, const NS32& n) {
    if constexpr (kMode == kEvalWide) return eval_t<kEvalWide>(c, p, wide_node(n));
    else return eval_t<kMode>(c, p, n);
}
template <int kMode>
__device__ __forceinline__ PruneF prune32(const Cfg& c, const NS32& n) {
    if constexpr (kMode == kEvalWide) return prune_prep(c, wide_node(n));
    else return prune_prep_t<kMode>(c, n);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

// (k1 > k2 > k3 or zero) with their cids: insert key v of cid c (keys are distinct unless zero)
__device__ __forceinline__ void top3_insert(uint64_t& k1, uint64_t& k2, uint64_t& k3, int& c1, int& c2, int& c3,
                                            uint64_t v, int c) {
    const bool g1 = v > k1, g2 = v > k2, g3 = v > k3;
    k3 = g2 ? k2 : (g3 ? v : k3); c3 = g2 ? c2 : (g3 ? c : c3);
    k2 = g1 ? k1 : (g2 ? v : k2); c2 = g1 ? c1 : (g2 ? c : c2);
    k1 = g1 ? v : k1; c1 = g1 ? c : c1;
}

// ---------------------------------------------------------------------------------------------
enum : uint8_t { kFlRun = 1, kFlTrunc = 2, kFlFull = 4, kFlOvf = 8 };

struct ChShared {
    PodRec pod[kB];
    uint32_t cl[kB][kR];          // (cid << 16) | total + 1, descending
    int32_t cnode[kCid];          // cid -> node (cids 0 .. n_e - 1 are E, in ws order)
    int32_t rs[4][kCid];          // ac am ag ap
    int32_t rd[4][kCid];          // rc rm rg nr at the base: binds < tb, events effective < tb
    uint16_t ecur[kCid];          // first E slot (eslot index) not yet applied; bit 15: pending own expiries
    int16_t fcur[kCid];           // first final bind >= tb (fnext list), -1 none
    uint8_t dirty[kCid];          // chunk binds changed since the node's last replay
    uint64_t rt[kCid], rl[kCid];  // taint label
    uint64_t cmask[kCid];         // this sweep's chunk binds of the cid (bit = pod - c0)
    int16_t fhead[kCid], ftail[kCid];  // final binds of the cid, ascending (fnext links)
    int16_t fnext[kB];
    int16_t wf[kB];               // final winners (cid, -1)
    int16_t w[2][kB];             // sweep winners, double-buffered
    int8_t code[2][kB];
    int8_t adm[kB];               // admission of pod j's bind: 1 ok, 0 over capacity, 2 unknown
    uint8_t clcnt[kB], clfl[kB];
    int16_t win_hi[kB], own[kB];
    int16_t xeff[kSlots];         // slot x is applied from pod xeff[x] on
    int16_t eoff[kSlots + 1];     // slot-E node k's slots: [eoff[k], eoff[k+1]) (E nodes without
                                  // slots — the overlap's touched nodes — are plain nodes here)
    // E-slot u (E node k's slots are [eoff[k], eoff[k+1]), ascending): {xeff of its slot, the
    // expiring pod's requests as words} — a replay's expiry event in one 16-byte read
    int4 erow[kSlots];
    // replayed node (slot = its first binder pod, one 16-byte row): [0, kSeg) segment start pods,
    // [kMOvf] the first pod whose state the slot does not hold, [kMCid] the node's cid (-1: the pod
    // is not a first binder)
    alignas(16) int16_t smeta[kB][8];
    int32_t sst[kB][kSeg][4];     // segment states rc rm rg nr
    uint64_t cd1[kC], cd2[kC], cd3[kC];  // top three keys of pre-chunk nodes per chunk pod
    int16_t cd1c[kC], cd2c[kC], cd3c[kC];
    uint8_t cdbad[kC];
    struct {
        uint64_t k[kWaves][kC][2];  // scratch: slot requests (setup), avail lists (guess), pair totals (sweeps)
    } x;
    uint32_t brow[kC][4];         // chunk pod c0 + r: request words (saturated), key mask | run << 3 |
                                  // own expiry's pod (kNoOwn: none) << 16
    int16_t ceix[kCid];           // cid -> the node's index in E, -1 if not an E node
    int16_t e2c[kSlots];          // slot-E index -> cid, -1: the E node is no candidate of this batch
    int32_t nbc, cut, fc[2], fs[2];
    int64_t t_start, t_end, t_err;  // the counters after this launch (chunk_scan_kernel's window prep)
    uint64_t chg;                 // chunk rows (slots c0 + j) rewritten since the last full sweep
#ifdef KS_CHUNK_DIAG
    int8_t why[kB];  // stop reason of a code-1 decision
#endif
};
static_assert(sizeof(ChShared) <= 160 * 1024, "LDS");

// Replays cid k from its base (state before pod tb: binds < tb, events effective < tb): its final
// binds >= tb (admission known, adm[]), then — `chunk` — the current sweep's chunk binds (admission
// evaluated, written to adm[]), with the pre-batch expiry slots of k (E cids) and each admitted
// running bind's own expiry, in pod order.  Stores the state segments for pods [from, i_end) in
// slot sl (sl < 0: none); returns the state before pod i_end binds (events effective < i_end);
// *ecur_out / *hp_out (optional): the E cursor and whether own expiries remain pending after it.
// A bind whose own expiry cannot be tracked (more than kPend pending) makes the state unknown
// from the next pod on: the slot's ovf, adm 2 for later binds, *lost_at.
struct Replayed {
    NS32 v;
    int ecur;     // E cursor after the replay
    bool hp;      // own expiries still pending
    int lost_at;  // INT_MAX, or the first pod whose state is unknown
};
__device__ __forceinline__ Replayed replay(ChShared& sh, int k, int tb, bool chunk, int c0, int from, int sl, int i_end) {
    // (no lambdas: their by-reference closures kept the state in scratch memory)
    uint32_t vrc = (uint32_t)sh.rd[0][k], vrm = (uint32_t)sh.rd[1][k], vrg = (uint32_t)sh.rd[2][k];
    int32_t vnr = sh.rd[3][k];
    const uint16_t ec = sh.ecur[k];
    int e_u = ec & 0x7FFF;
    const int ex = sh.ceix[k];
    const int e_end = ex >= 0 ? sh.eoff[ex + 1] : 0;
    // pending own expiries: four named slots (eff INT_MAX = empty), updated by value selects only
    static_assert(kPend == 4, "four pending slots");
    int pe0 = INT_MAX, pe1 = INT_MAX, pe2 = INT_MAX, pe3 = INT_MAX, pj0 = 0, pj1 = 0, pj2 = 0, pj3 = 0;
    bool lost = false;
    int ovf = kNoSeg, lost_at = INT_MAX;
#define KS_PUSH(EX, JB)                                                                              \
    do {                                                                                             \
        const int ex_ = (EX), jb_ = (JB);                                                            \
        const bool s0 = pe0 == INT_MAX, s1 = !s0 && pe1 == INT_MAX, s2 = !s0 && !s1 && pe2 == INT_MAX, \
                   s3 = !s0 && !s1 && !s2 && pe3 == INT_MAX;                                          \
        pe0 = s0 ? ex_ : pe0; pj0 = s0 ? jb_ : pj0;                                                  \
        pe1 = s1 ? ex_ : pe1; pj1 = s1 ? jb_ : pj1;                                                  \
        pe2 = s2 ? ex_ : pe2; pj2 = s2 ? jb_ : pj2;                                                  \
        pe3 = s3 ? ex_ : pe3; pj3 = s3 ? jb_ : pj3;                                                  \
        if (!(s0 || s1 || s2 || s3)) { /* untracked: the state is unknown from the next pod on */   \
            lost = true;                                                                             \
            ovf = jb_ + 1 < ovf ? jb_ + 1 : ovf;                                                     \
            lost_at = jb_ + 1 < lost_at ? jb_ + 1 : lost_at;                                         \
        }                                                                                            \
    } while (0)
    if (ec & 0x8000) {  // own expiries of binds before the base that have not fired by it
        for (int j = sh.fhead[k]; j >= 0 && j < tb; j = sh.fnext[j]) {
            const int x = sh.own[j];
            if (sh.adm[j] == 1 && (sh.clfl[j] & kFlRun) && x >= 0 && sh.xeff[x] >= tb) KS_PUSH(sh.xeff[x], j);
        }
    }
    int ns = 0, last_t = -1;
#define KS_STORE(T)                                                                                  \
    do {                                                                                             \
        int t_ = (T);                                                                                \
        t_ = t_ < from ? from : t_;                                                                  \
        if (sl >= 0 && t_ < i_end && t_ < ovf) {                                                     \
            bool ok_ = true;                                                                         \
            if (t_ != last_t) {                                                                      \
                if (ns == kSeg) { ovf = t_; ok_ = false; }                                           \
                else { sh.smeta[sl][ns] = (int16_t)t_; ++ns; last_t = t_; }                          \
            }                                                                                        \
            if (ok_) *reinterpret_cast<int4*>(&sh.sst[sl][ns - 1][0]) = make_int4((int)vrc, (int)vrm, (int)vrg, vnr); \
        }                                                                                            \
    } while (0)
    if (sl >= 0) {
        for (int q = 0; q < kSeg; ++q) sh.smeta[sl][q] = kNoSeg;
        sh.smeta[sl][kMCid] = (int16_t)k;
        KS_STORE(from);
    }
    const int32_t ac = sh.rs[0][k], am = sh.rs[1][k], ag = sh.rs[2][k], ap = sh.rs[3][k];
    const int64_t ac64 = cap64(ac), am64 = cap64(am), ag64 = cap64(ag);
    int j = sh.fcur[k];
    uint64_t m = chunk ? sh.cmask[k] : 0ull;
    // one event loop: the next bind (final list, then the chunk mask) against the next expiry
    for (;;) {
        int jb = j >= 0 ? j : (m ? c0 + __builtin_ctzll(m) : INT_MAX);
        if (jb >= i_end) jb = INT_MAX;
        const int4 er = e_u < e_end ? sh.erow[e_u] : make_int4(INT_MAX, 0, 0, 0);
        const int ne = er.x;
        const int pm01 = pe0 < pe1 ? pe0 : pe1, pm23 = pe2 < pe3 ? pe2 : pe3;
        const int pm = pm01 < pm23 ? pm01 : pm23;
        const int nx = ne < pm ? ne : pm;
        const int lim = jb != INT_MAX ? jb : i_end - 1;
        if (nx <= lim) {  // an expiry effective before the next bind (or before i_end)
            if (ne == nx) {
                ++e_u;
                vrc -= (uint32_t)er.y; vrm -= (uint32_t)er.z; vrg -= (uint32_t)er.w; vnr -= 1;
            } else {
                const bool h0 = pe0 == pm, h1 = !h0 && pe1 == pm, h2 = !h0 && !h1 && pe2 == pm,
                           h3 = !h0 && !h1 && !h2;
                const int jq = h0 ? pj0 : (h1 ? pj1 : (h2 ? pj2 : pj3));
                pe0 = h0 ? INT_MAX : pe0; pe1 = h1 ? INT_MAX : pe1;
                pe2 = h2 ? INT_MAX : pe2; pe3 = h3 ? INT_MAX : pe3;
                const PodRec& p = sh.pod[jq];
                vrc -= (uint32_t)p.req[0]; vrm -= (uint32_t)p.req[1]; vrg -= (uint32_t)p.req[2]; vnr -= 1;
            }
            KS_STORE(nx);
            continue;
        }
        if (jb == INT_MAX) break;
        const bool fin = j >= 0;
        if (fin) j = sh.fnext[j];
        else m &= m - 1;
        // the bind's request words, key mask, run flag and own-expiry pod: a chunk bind's from its
        // 16-byte row (one read), a final bind's from the pod record
        uint32_t q0, q1, q2, meta;
        if (!fin) {
            const uint4 br = *reinterpret_cast<const uint4*>(&sh.brow[jb - c0][0]);
            q0 = br.x; q1 = br.y; q2 = br.z; meta = br.w;
        } else {
            const PodRec& p = sh.pod[jb];
            q0 = (uint32_t)p.req[0]; q1 = (uint32_t)p.req[1]; q2 = (uint32_t)p.req[2];
            const int x = sh.own[jb];
            meta = (uint32_t)p.keymask | ((sh.clfl[jb] & kFlRun) ? 8u : 0u) |
                   ((uint32_t)(x >= 0 ? (int)sh.xeff[x] : kNoOwn) << 16);
        }
        bool ok;
        if (fin) {
            ok = sh.adm[jb] == 1;
        } else {  // CreatePod admission (kubesim/node/node.go:44-47); saturated words: a request
                  // >= 2^32 - 1 exceeds every capacity (< 2^32 - 1) as its int64 value would
            ok = !lost && vnr < ap;
            if (meta & 1) ok &= (int64_t)vrc + q0 <= ac64;
            if (meta & 2) ok &= (int64_t)vrm + q1 <= am64;
            if (meta & 4) ok &= (int64_t)vrg + q2 <= ag64;
            sh.adm[jb] = lost ? 2 : (ok ? 1 : 0);
        }
        if (ok && (meta & 8)) {
            vrc += q0; vrm += q1; vrg += q2; vnr += 1;
            KS_STORE(jb + 1);
            const int oe = (int)(meta >> 16);
            if (oe != kNoOwn) KS_PUSH(oe, jb);
        }
    }
#undef KS_STORE
#undef KS_PUSH
    if (sl >= 0) sh.smeta[sl][kMOvf] = (int16_t)ovf;
    Replayed out;
    out.v.ac = ac; out.v.am = am; out.v.ag = ag; out.v.ap = ap;
    out.v.rc = (int32_t)vrc; out.v.rm = (int32_t)vrm; out.v.rg = (int32_t)vrg; out.v.nr = vnr;
    out.v.taint = 0; out.v.label = 0;
    out.ecur = e_u;
    out.hp = (pe0 & pe1 & pe2 & pe3) != INT_MAX;  // any slot holds a (non-negative) pod index
    out.lost_at = lost_at;
    return out;
}

// a slot's 16-byte row
struct SRow {
    uint4 v;
    __device__ __forceinline__ int m(int q) const {  // q: a compile-time constant after unrolling
        const uint32_t w = q < 2 ? v.x : (q < 4 ? v.y : (q < 6 ? v.z : v.w));
        return (int)(int16_t)(uint16_t)((q & 1) ? (w >> 16) : (w & 0xFFFFu));
    }
    __device__ __forceinline__ void clear_cid() { v.w |= 0xFFFFu; }  // kMCid = 6: low half of v.w
};
static_assert(kMCid == 6, "SRow::clear_cid");
__device__ __forceinline__ SRow srow(const ChShared& sh, int sl) {
    SRow r;
    r.v = *reinterpret_cast<const uint4*>(&sh.smeta[sl][0]);
    return r;
}

// Pod i's key on slot sl's node (cid k) from its row: the segment holding pod i
template <int kMode>
__device__ __forceinline__ uint64_t key_at(const EngineArgs& a, const ChShared& sh, const PodRec& p, int i, int k,
                                           int sl, const SRow& r) {
    int s = 0;
#pragma unroll
    for (int q = 1; q < kSeg; ++q) s += r.m(q) <= i;
    const int4 st = *reinterpret_cast<const int4*>(&sh.sst[sl][s][0]);
    NS32 n;
    n.ac = sh.rs[0][k]; n.am = sh.rs[1][k]; n.ag = sh.rs[2][k]; n.ap = sh.rs[3][k];
    n.rc = st.x; n.rm = st.y; n.rg = st.z; n.nr = st.w;
    n.taint = sh.rt[k]; n.label = sh.rl[k];
    return make_key(eval32<kMode>(a.c, p, n), (uint32_t)sh.cnode[k]);
}

// Pod i's total + 1 (0: infeasible) on slot sl's node from its row
template <int kMode>
__device__ __forceinline__ uint32_t tot_at(const EngineArgs& a, const ChShared& sh, const PodRec& p, int i, int k,
                                           int sl, const SRow& r) {
    int s = 0;
#pragma unroll
    for (int q = 1; q < kSeg; ++q) s += r.m(q) <= i;
    const int4 st = *reinterpret_cast<const int4*>(&sh.sst[sl][s][0]);
    NS32 n;
    n.ac = sh.rs[0][k]; n.am = sh.rs[1][k]; n.ag = sh.rs[2][k]; n.ap = sh.rs[3][k];
    n.rc = st.x; n.rm = st.y; n.rg = st.z; n.nr = st.w;
    n.taint = sh.rt[k]; n.label = sh.rl[k];
    return eval32<kMode>(a.c, p, n);
}

// The same, 0 when the float upper bound of the total (prune_tmax: filters ignored, exact slack)
// says the key stays below lb — most (pod, node) pairs: the full evaluator runs only for the rest.
template <int kMode>
__device__ __forceinline__ uint64_t key_at_lb(const EngineArgs& a, const ChShared& sh, const PodRec& p, int i, int k,
                                              int sl, const SRow& r, uint64_t lb) {
    int s = 0;
#pragma unroll
    for (int q = 1; q < kSeg; ++q) s += r.m(q) <= i;
    const int4 st = *reinterpret_cast<const int4*>(&sh.sst[sl][s][0]);
    NS32 n;
    n.ac = sh.rs[0][k]; n.am = sh.rs[1][k]; n.ag = sh.rs[2][k]; n.ap = sh.rs[3][k];
    n.rc = st.x; n.rm = st.y; n.rg = st.z; n.nr = st.w;
    const uint32_t node = (uint32_t)sh.cnode[k];
    n.taint = 0; n.label = 0;
    const PruneF f = prune32<kMode>(a.c, n);
    if (!f.live || make_key(prune_tmax(a.c, f, (float)p.req[0], (float)p.req[1]) + 1u, node) < lb) return 0;
    n.taint = sh.rt[k]; n.label = sh.rl[k];
    return make_key(eval32<kMode>(a.c, p, n), node);
}

__device__ __forceinline__ uint64_t cl_key(const ChShared& sh, uint32_t e) {
    return ((uint64_t)(e & 0xFFFFu) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)sh.cnode[e >> 16]);
}

// candidate id k's per-batch bookkeeping (its E index set first)
__device__ __forceinline__ void store_book(ChShared& sh, int k) {
    sh.cmask[k] = 0;
    sh.fhead[k] = -1; sh.ftail[k] = -1; sh.fcur[k] = -1;
    sh.ecur[k] = sh.ceix[k] >= 0 ? (uint16_t)sh.eoff[sh.ceix[k]] : 0;
    sh.dirty[k] = 0;
}

// candidate id k's record: int32 state {ac am ag ap} {rc rm rg nr}, {taint label} as u64 pairs —
// the candidate slot's record (ks_cand.hip cand_list, the narrow format)
__device__ __forceinline__ void store_prec(ChShared& sh, int k, const uint4* r) {
    sh.rs[0][k] = (int32_t)r[0].x; sh.rs[1][k] = (int32_t)r[0].y; sh.rs[2][k] = (int32_t)r[0].z; sh.rs[3][k] = (int32_t)r[0].w;
    sh.rd[0][k] = (int32_t)r[1].x; sh.rd[1][k] = (int32_t)r[1].y; sh.rd[2][k] = (int32_t)r[1].z; sh.rd[3][k] = (int32_t)r[1].w;
    sh.rt[k] = r[2].x | ((uint64_t)r[2].y << 32); sh.rl[k] = r[2].z | ((uint64_t)r[2].w << 32);
    store_book(sh, k);
}

template <int kMode>
__device__ __forceinline__ void chunk_body(const EngineArgs* __restrict__ A, ChShared& sh) {
    const EngineArgs& a = A[0];
    const WinWS& ws = *a.sw;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    int nb = ws.nb;
    const int64_t err0 = a.ctr[kCtrErr];
    if (tid == 0) { sh.t_start = start; sh.t_end = end; sh.t_err = err0; }
    if (err0 != 0 || nb <= 0) return;
    const int n_e = ws.n_es, n_eall = ws.n_e, e_cnt = ws.e_cnt;  // (n_e: the slot-E nodes)

    // ---- setup: pods, window, candidate ids, records.  The candidate ids (cids) number the batch's
    // distinct candidate nodes in the order of their first kept entry (pod-major: merge_cl's
    // n_first, ks_cand.hip cand_list) — deterministic, so every rank of a sharded engine cuts a batch
    // at the same pod (round 6: the claim-order slot ids made the cut timing-dependent, and ranks
    // that cut differently issued different numbers of exchanges).  A pod with an entry whose cid is
    // >= kCid cuts the batch before it (never pod 0: its entries are the first cids).  Each cid's
    // record is its candidate slot's, staged by merge_cl (a direct read past the kCid staged slots).
    DG(uint64_t t_setup = dstamp(); uint64_t acc_cd = 0, acc_sw = 0, acc_fin = 0, acc_ph[4] = {0, 0, 0, 0}, acc_cs = 0, acc_rb = 0, acc_cdp = 0, acc_rbase = 0, acc_red = 0, acc_crep = 0; int n_sweeps = 0, n_sonly = 0, n_chunks = 0;)
    const int nslot = ws.nslot < kWinMaxB * kR ? ws.nslot : kWinMaxB * kR;
    // (det: first-appearance cids, every slot < kCid staged; otherwise the claim-order slots are the
    // cids, slots >= kCidSlots cut the batch and pod 0 takes private cids there)
    const bool det = a.det_cids != 0;
    const int ncap = det ? kCid : kCidSlots;
    const int nlo = nslot < ncap ? nslot : ncap;
    // (1) every global read of the setup issued before any is used: one round trip (the lists and
    // records were written by other workgroups, on other XCDs — each dependent read is a fabric
    // round trip)
    static_assert(sizeof(PodRec) == 48, "a pod record is three 16-byte words");
    uint4 prec[3] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    int32_t whi = 0, ownv = -1, info = 0, durv = 0;
    if (tid < nb) {
        const uint4* pr = reinterpret_cast<const uint4*>(a.pods + start + tid);
        prec[0] = pr[0]; prec[1] = pr[1]; prec[2] = pr[2];
        whi = ws.win_hi[tid]; ownv = ws.own[tid]; info = ws.cl_info[tid]; durv = a.dur[start + tid];
    }
    int64_t xr0 = 0, xr1 = 0, xr2 = 0;
    int32_t esl = 0, xq = -1;
    if (tid < e_cnt) {
        xr0 = ws.ex_req[tid][0]; xr1 = ws.ex_req[tid][1]; xr2 = ws.ex_req[tid][2]; esl = ws.e_slot[tid];
        xq = ws.ex_ok[tid] ? ws.ex_q[tid] : -1;  // (for the commit)
    }
    static_assert(kEMax <= 4 * kThreads, "four E nodes per thread");
    int32_t enode[4];  // (for the commit: e_idx reset; [0] the slot-E node tid's expiries)
#pragma unroll
    for (int q = 0; q < 4; ++q) enode[q] = tid + q * kThreads < n_eall ? ws.e_node[tid + q * kThreads] : -1;
    static_assert(kSlots <= kThreads, "one window slot per thread");
    static_assert(kSlots + 1 <= 2 * kThreads, "two E offsets per thread");
    int32_t eo[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) eo[q] = tid + q * kThreads <= n_e ? ws.e_off[tid + q * kThreads] : 0;
    static_assert(kCid <= 2 * kThreads, "two slot records per thread");
    int32_t snd[2], sex[2];
    uint4 srec[2][3];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int k = tid + q * kThreads;
        const bool v = k < nlo;
        snd[q] = v ? ws.slot_node[k] : -1;
        sex[q] = v ? ws.slot_eix[k] : -1;
        if (sex[q] >= n_e) sex[q] = -1;  // an E node without slots: no events here
        const uint4* r = reinterpret_cast<const uint4*>(ws.slot_rec[v ? k : 0]);
#pragma unroll
        for (int w = 0; w < 3; ++w) srec[q][w] = v ? r[w] : make_uint4(0, 0, 0, 0);
    }
    constexpr int kEntPer = (kB * kR + kThreads - 1) / kThreads;
    uint64_t ekey[kEntPer];
    int32_t eslt[kEntPer];
#pragma unroll
    for (int q = 0; q < kEntPer; ++q) {  // every kept position (the counts come with the lists)
        const int idx = tid + q * kThreads, i = idx / kR, r = idx % kR;
        const bool v = i < nb;
        ekey[q] = v ? ws.cl_key[i][r] : 0ull;
        eslt[q] = v ? ws.cl_slot[i][r] : -1;
    }
    // (2) the LDS images
    if (tid == 0) { sh.nbc = nb; sh.cut = INT_MAX; sh.fc[0] = sh.fc[1] = INT_MAX; sh.fs[0] = sh.fs[1] = INT_MAX; }
    if (tid < nb) {
        uint4* pd = reinterpret_cast<uint4*>(&sh.pod[tid]);
        pd[0] = prec[0]; pd[1] = prec[1]; pd[2] = prec[2];
        sh.win_hi[tid] = (int16_t)whi;
        sh.own[tid] = (int16_t)ownv;
        sh.clcnt[tid] = (uint8_t)(info & 0xFF);
        sh.clfl[tid] = (durv > 0 ? kFlRun : 0) | ((info & kClTrunc) ? kFlTrunc : 0) |
                       ((info & kClFull) ? kFlFull : 0) | ((info & kClOvf) ? kFlOvf : 0);
        sh.adm[tid] = 0;
        sh.wf[tid] = -1;
        sh.w[0][tid] = -1; sh.w[1][tid] = -1;
        sh.smeta[tid][kMCid] = -1;
        sh.code[0][tid] = 0; sh.code[1][tid] = 0;
    }
    // cid numbering scratch in the (idle until the sweeps) segment states: per pod the mask of its
    // first-appearance entries and their pod-prefix count; slot -> cid
    uint32_t* omask = reinterpret_cast<uint32_t*>(&sh.sst[0][0][0]);
    int32_t* opre = reinterpret_cast<int32_t*>(omask + kB);
    int16_t* sc = reinterpret_cast<int16_t*>(opre + kB + 4);
    static_assert(sizeof(sh.sst) >= (2 * kB + 4) * 4 + kSlotIds * 2, "cid numbering scratch");
    if (tid < kB) omask[tid] = 0;
    if (det)
        for (int k = tid; k < nlo; k += kThreads) sc[k] = -1;
    // slot x's request words, staged in the cache buffer (idle until the first chunk's cache)
    int32_t (*xtmp)[4] = reinterpret_cast<int32_t (*)[4]>(&sh.x.k[0][0][0]);
    static_assert(sizeof(sh.x.k) >= kSlots * 4 * sizeof(int32_t), "slot request staging");
    if (tid < e_cnt) {
        xtmp[tid][0] = word32(xr0); xtmp[tid][1] = word32(xr1); xtmp[tid][2] = word32(xr2);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int k = tid + q * kThreads;
        if (k <= n_e) sh.eoff[k] = (int16_t)eo[q];
        if (k < n_e) sh.e2c[k] = -1;
    }
    for (int k = tid; k < kCid; k += kThreads) { sh.ceix[k] = -1; sh.cnode[k] = -1; }
    __syncthreads();
    DG(uint64_t ts1 = dstamp();)
    if (det) {
        // (3) each kept entry's node's first entry (a dependent read: the lists' nodes), then the owners
        // (first-appearance entries) per pod
        int32_t fe[kEntPer];
    #pragma unroll
        for (int q = 0; q < kEntPer; ++q) {
            const int idx = tid + q * kThreads, i = idx / kR, r = idx % kR;
            const bool v = i < nb && r < sh.clcnt[i];
            fe[q] = v ? a.n_first[key_node(ekey[q])] : kNoFirst;
        }
        // slot i is applied from the first pod i >= 1 with win_hi[i] > x
        for (int i = tid + 1; i < nb; i += kThreads)
            for (int x = sh.win_hi[i - 1]; x < sh.win_hi[i]; ++x) sh.xeff[x] = (int16_t)i;
    #pragma unroll
        for (int q = 0; q < kEntPer; ++q) {
            const int idx = tid + q * kThreads;
            if (fe[q] == idx) atomicOr(&omask[idx / kR], 1u << (idx % kR));
        }
        __syncthreads();
        if (wave == 0) {  // exclusive prefix of the pods' owner counts (four pods per lane)
            int c[4], sum = 0;
    #pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = lane * 4 + u;
                c[u] = i < nb ? __popc(omask[i]) : 0;
                sum += c[u];
            }
            int incl = sum;
    #pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const int v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            int run = incl - sum;
    #pragma unroll
            for (int u = 0; u < 4; ++u) {
                opre[lane * 4 + u] = run;
                run += c[u];
            }
        }
        static_assert(kB == 4 * kWave, "four pods per lane");
        __syncthreads();
        // (4) every entry's cid: its node's first entry's rank in pod-major order; owners map their slot
        // to it (the slot records below) or, past the staged slots, read the node directly
    #pragma unroll
        for (int q = 0; q < kEntPer; ++q) {
            const int idx = tid + q * kThreads, i = idx / kR, r = idx % kR;
            if (fe[q] == kNoFirst) continue;
            const int f = fe[q], fi = f / kR, fr = f % kR;
            const int cid = opre[fi] + __popc(omask[fi] & ((1u << fr) - 1u));
            if (cid >= kCid) { atomicMin(&sh.nbc, i); continue; }  // (i > 0: pod 0's entries are cids < kR)
            const uint64_t key = ekey[q];
            sh.cl[i][r] = ((uint32_t)cid << 16) | (uint32_t)(key >> 32);
            if (f != idx) continue;
            const int sl = eslt[q];
            if (sl >= 0 && sl < nlo) {
                sc[sl] = (int16_t)cid;
            } else {  // (a slot past the staged records: the node read here)
                const int32_t nd = key_node(key);
                int ex = a.e_idx[nd];
                if (ex >= n_e) ex = -1;  // (an E node without slots)
                sh.cnode[cid] = nd;
                sh.ceix[cid] = (int16_t)ex;
                if (ex >= 0) sh.e2c[ex] = (int16_t)cid;
                const NodeV v = load_node(a.s, nd);
                const uint4 rr[3] = {make_uint4((uint32_t)v.ac, (uint32_t)v.am, (uint32_t)v.ag, (uint32_t)clamp32(v.ap)),
                                     make_uint4((uint32_t)v.rc, (uint32_t)v.rm, (uint32_t)v.rg, (uint32_t)v.nr),
                                     make_uint4((uint32_t)v.taint, (uint32_t)(v.taint >> 32), (uint32_t)v.label, (uint32_t)(v.label >> 32))};
                store_prec(sh, cid, rr);
            }
        }
        __syncthreads();
        const int n_cid = opre[kB - 1] + __popc(omask[kB - 1]) < kCid ? opre[kB - 1] + __popc(omask[kB - 1]) : kCid;
    #pragma unroll
        for (int q = 0; q < 2; ++q) {  // the staged slot records at their cids; the other cids inert
            const int k = tid + q * kThreads;
            if (k < nlo) {
                const int c = sc[k];
                if (c >= 0 && c < kCid) {
                    sh.cnode[c] = snd[q];
                    sh.ceix[c] = (int16_t)sex[q];
                    if (sex[q] >= 0) sh.e2c[sex[q]] = (int16_t)c;
                    store_prec(sh, c, srec[q]);
                }
            }
        }
        for (int k = tid; k < kCid; k += kThreads)
            if (k >= n_cid) store_book(sh, k);
    } else {
        // claim-order cids (one engine: its batching may depend on claim timing — results do not)
        for (int i = tid + 1; i < nb; i += kThreads)
            for (int x = sh.win_hi[i - 1]; x < sh.win_hi[i]; ++x) sh.xeff[x] = (int16_t)i;
#pragma unroll
        for (int q = 0; q < 2; ++q) {  // slot records; the other cids inert
            const int k = tid + q * kThreads;
            if (k < nlo) {
                sh.cnode[k] = snd[q];
                sh.ceix[k] = (int16_t)sex[q];
                if (sex[q] >= 0) sh.e2c[sex[q]] = (int16_t)k;
                store_prec(sh, k, srec[q]);
            }
        }
        for (int k = tid; k < kCid; k += kThreads)
            if (k >= nlo) store_book(sh, k);
#pragma unroll
        for (int q = 0; q < kEntPer; ++q) {
            const int idx = tid + q * kThreads, i = idx / kR, r = idx % kR;
            if (i >= nb || r >= sh.clcnt[i] || eslt[q] < 0) continue;
            const uint64_t key = ekey[q];
            const int sl = eslt[q];
            int cid = sl;
            if (sl >= kCidSlots) {
                if (i > 0) { atomicMin(&sh.nbc, i); continue; }
                cid = kCidSlots + r;  // pod 0's private cid
                const int32_t nd = key_node(key);
                int ex = a.e_idx[nd];
                if (ex >= n_e) ex = -1;  // (an E node without slots)
                sh.cnode[cid] = nd;
                sh.ceix[cid] = (int16_t)ex;
                if (ex >= 0) sh.e2c[ex] = (int16_t)cid;
                const NodeV v = load_node(a.s, nd);
                const uint4 rr[3] = {make_uint4((uint32_t)v.ac, (uint32_t)v.am, (uint32_t)v.ag, (uint32_t)clamp32(v.ap)),
                                     make_uint4((uint32_t)v.rc, (uint32_t)v.rm, (uint32_t)v.rg, (uint32_t)v.nr),
                                     make_uint4((uint32_t)v.taint, (uint32_t)(v.taint >> 32), (uint32_t)v.label, (uint32_t)(v.label >> 32))};
                store_prec(sh, cid, rr);
            }
            sh.cl[i][r] = ((uint32_t)cid << 16) | (uint32_t)(key >> 32);
        }
    }
    __syncthreads();
    nb = sh.nbc < nb ? sh.nbc : nb;
    const int ncid = kCid;  // (inert cids have no events: skipped by every loop)
    if (tid < e_cnt && tid < sh.eoff[n_e]) {  // E-slot tid is window slot esl
        const int32_t* q = xtmp[esl];
        sh.erow[tid] = make_int4(sh.xeff[esl], q[0], q[1], q[2]);
    }
    DG(uint64_t ts2 = dstamp(); uint64_t cs_e = 0, cs_r = 0, cs_x = 0;)
    __syncthreads();

    // ---- chunks
    DG(uint64_t ts3 = dstamp(); (void)ts1; (void)ts2; t_setup = ts3 - t_setup;)
    int committed = nb, stop_code = 0, tb = 0;
    for (int c0 = 0; c0 < nb; c0 += kC) {
        const int c1 = nb < c0 + kC ? nb : c0 + kC;
        DG(uint64_t t0 = dstamp(); ++n_chunks;)
        // (1) pre-chunk nodes: replay each over [c0, c1) into its first final binder's slot, then
        // per chunk pod the top two keys (lane = pod, waves over nodes)
        if (c0 > 0) {
            // rebase every node with events to c0 (binds < c0, events effective < c0)
            for (int k = tid; k < ncid; k += kThreads) {
                if (sh.ceix[k] >= 0 || sh.fhead[k] >= 0) {
                    const Replayed r = replay(sh, k, tb, false, c0, c0, -1, c0);
                    if (r.lost_at != INT_MAX) atomicMin(&sh.cut, c0);
                    sh.rd[0][k] = r.v.rc; sh.rd[1][k] = r.v.rm; sh.rd[2][k] = r.v.rg; sh.rd[3][k] = r.v.nr;
                    sh.ecur[k] = (uint16_t)(r.ecur | (r.hp ? 0x8000 : 0));
                    sh.fcur[k] = -1;
                }
            }
            __syncthreads();
            DG(acc_rbase += dstamp() - t0;)
            tb = c0;
            if (sh.cut <= c0) {  // an own expiry could not be tracked: commit the pods before c0
                committed = c0;
                stop_code = 1;
                break;
            }
            // replays spread over the waves: pod j's thread is 2 j
            if ((tid & 1) == 0 && (tid >> 1) < c0) {
                const int j = tid >> 1;
                const int k = sh.wf[j];
                if (k >= 0 && sh.fhead[k] == j) (void)replay(sh, k, tb, false, c0, c0, j, c1);
                else sh.smeta[j][kMCid] = -1;
            }
            __syncthreads();
            DG(uint64_t tr1 = dstamp(); acc_rb += tr1 - t0;)
            {  // eight lanes per chunk pod (pod c0 + tid / 8), lane s8 takes the rows j = s8 + 8 t
                const int pi = tid >> 3, s8 = tid & 7;
                const int i = c0 + pi;
                const bool li = i < c1;
                const PodRec p = sh.pod[li ? i : c0];
                // a cached key below thr_i never decides pod i: a winner from the static list is
                // >= thr_i, and without one D must beat thr_i (or the last kept entry, >= thr_i)
                const uint64_t lbc = li ? ws.cl_thr[i] : 0ull;
                uint64_t k1 = 0, k2 = 0, k3 = 0;
                int q1 = -1, q2 = -1, q3 = -1;
                bool bad = false;
                // four rows per step (j = s8 + 8 (4 t + q)), their loads issued together
                for (int j0 = s8; j0 < c0; j0 += 4 * kLanesPerPod) {
                    SRow r[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int j = j0 + q * kLanesPerPod;
                        r[q] = srow(sh, j < c0 ? j : 0);
                        if (j >= c0) r[q].clear_cid();
                    }
                    // the exact keys (keys below lbc dropped); the wide evaluator first tries the
                    // float bound — for the 32-bit evaluators the prune saved nothing: in SIMT the
                    // evaluation runs whenever one lane passes, and these nodes, the batch's earlier
                    // winners, are near the top of most pods' lists.  The 32-bit evaluators run the
                    // four rows without branches (an empty row evaluates cid 0 and is masked), so
                    // their four dependent LDS-and-VALU chains interleave.
                    uint64_t key[4];
                    int kc[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int j = j0 + q * kLanesPerPod;
                        const int k = r[q].m(kMCid);
                        const bool on = k >= 0 && li;
                        const bool ok = on && r[q].m(kMOvf) > i;
                        bad |= on && !ok;
                        kc[q] = k;
                        if constexpr (kMode == kEvalWide) {
                            key[q] = ok ? key_at_lb<kMode>(a, sh, p, i, k, j, r[q], lbc) : 0ull;
                        } else {
                            const uint64_t kq = key_at<kMode>(a, sh, p, i, k >= 0 ? k : 0, j, r[q]);
                            key[q] = ok ? kq : 0ull;
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) top3_insert(k1, k2, k3, q1, q2, q3, key[q] < lbc ? 0ull : key[q], kc[q]);
                }
                // the pod's top three over its eight lanes (distinct keys: one node per row)
#pragma unroll
                for (int o = 1; o < kLanesPerPod; o <<= 1) {
                    const uint64_t o1 = shfl_xor64(k1, o), o2 = shfl_xor64(k2, o), o3 = shfl_xor64(k3, o);
                    const int c1_ = __shfl_xor(q1, o), c2_ = __shfl_xor(q2, o), c3_ = __shfl_xor(q3, o);
                    top3_insert(k1, k2, k3, q1, q2, q3, o1, c1_);
                    top3_insert(k1, k2, k3, q1, q2, q3, o2, c2_);
                    top3_insert(k1, k2, k3, q1, q2, q3, o3, c3_);
                }
                bad = ((__ballot(bad) >> (lane & ~7)) & 0xFFull) != 0;
                if (s8 == 0) {
                    sh.cd1[pi] = k1; sh.cd2[pi] = k2; sh.cd3[pi] = k3;
                    sh.cd1c[pi] = (int16_t)q1; sh.cd2c[pi] = (int16_t)q2; sh.cd3c[pi] = (int16_t)q3;
                    sh.cdbad[pi] = bad;
                }
            }
            DG(__syncthreads(); acc_cdp += dstamp() - tr1;)
        } else if (tid < kC) {
            sh.cd1[tid] = 0; sh.cd2[tid] = 0; sh.cd3[tid] = 0;
            sh.cd1c[tid] = -1; sh.cd2c[tid] = -1; sh.cd3c[tid] = -1; sh.cdbad[tid] = 0;
        }
        __syncthreads();

        // (2) sweeps
        DG(uint64_t t1 = dstamp(); acc_cd += t1 - t0;)
        if (wave == 1 && c0 + lane < c1) {  // the chunk's bind rows (beside the guess in wave 0)
            const int i = c0 + lane;
            const PodRec& p = sh.pod[i];
            const int x = sh.own[i];
            auto word = [](int64_t q) { return (uint32_t)(q < 0xFFFFFFFFll ? q : 0xFFFFFFFFll); };
            *reinterpret_cast<uint4*>(&sh.brow[lane][0]) =
                make_uint4(word(p.req[0]), word(p.req[1]), word(p.req[2]),
                           (uint32_t)p.keymask | ((sh.clfl[i] & kFlRun) ? 8u : 0u) |
                               ((uint32_t)(x >= 0 ? (int)sh.xeff[x] : kNoOwn) << 16));
        }
        // (2a) The guess: exclusion-only rounds (w_i = the first static candidate no earlier pod
        // takes; no evaluation, no replay) to their fixed point — the sequential greedy over the
        // lists, without the piles a cold start makes (every pod on its own best node).  One wave,
        // lane = pod, no barrier: a round reads every lane's entries, then moves the changed
        // lanes' mask bits; the pods before the first change are final.
        if (wave == 0) {
            const int i = c0 + lane;
            const int nc = i < c1 ? sh.clcnt[i] : 0;
            const uint64_t below = (1ull << lane) - 1ull;
            // the lane's entries no pre-chunk bind took, in list order (static in the chunk): the
            // list in the cache phase's (idle) buffer, its first eight in registers
            uint32_t* al = reinterpret_cast<uint32_t*>(&sh.x.k[0][0][0]) + lane * kR;
            static_assert(sizeof(sh.x.k) >= kC * kR * sizeof(uint32_t), "avail lists");
            int na = 0;
            {
                uint32_t e[kR];
#pragma unroll
                for (int q = 0; q < kR / 4; ++q) {
                    const uint4 v = *reinterpret_cast<const uint4*>(&sh.cl[i < c1 ? i : c0][4 * q]);
                    e[4 * q] = v.x; e[4 * q + 1] = v.y; e[4 * q + 2] = v.z; e[4 * q + 3] = v.w;
                }
                int16_t fh[kR];
#pragma unroll
                for (int r = 0; r < kR; ++r) fh[r] = sh.fhead[r < nc ? (e[r] >> 16) : 0];
#pragma unroll
                for (int r = 0; r < kR; ++r) {  // compacted without branches
                    al[na] = e[r];
                    na += (r < nc && fh[r] < 0) ? 1 : 0;
                }
            }
            static_assert(kR % 4 == 0 && kR > 8, "entry rows in 16-byte reads; two probe stages");
            int rg[kR];
            uint32_t rt[kR];  // (cid, total) words
#pragma unroll
            for (int q = 0; q < kR; ++q) {
                rt[q] = q < na ? al[q] : 0u;
                rg[q] = (int)(rt[q] >> 16);
            }
            // the guess also takes the pod's cached pre-chunk D (the best node bound before the
            // chunk, on its replayed state) when it beats the static pick — fewer full sweeps
            // correct it (the guess only seeds the sweeps: any guess gives the sequential result)
            const bool dok = c0 > 0 && i < c1 && !sh.cdbad[lane];
            const uint64_t d1 = dok ? sh.cd1[lane] : 0ull, d2 = dok ? sh.cd2[lane] : 0ull, d3 = dok ? sh.cd3[lane] : 0ull;
            const int dc1 = d1 ? sh.cd1c[lane] : 0, dc2 = d2 ? sh.cd2c[lane] : 0, dc3 = d3 ? sh.cd3c[lane] : 0;
            int cur = -1, lo_l = 0;
            for (;;) {
                DG(++n_sonly;)
                const bool act = lane >= lo_l && nc > 0;
                int nw = act ? -1 : cur;
                uint32_t nwt = 0;
                uint64_t m1, m2, m3;
                {  // probe the first eight (every lane, unconditional loads), then the rest if needed
                    uint64_t cm[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) cm[q] = sh.cmask[rg[q]];
                    m1 = sh.cmask[dc1]; m2 = sh.cmask[dc2]; m3 = sh.cmask[dc3];
#pragma unroll
                    for (int q = 7; q >= 0; --q)  // the lowest free entry wins
                        if (act && q < na && (cm[q] & below) == 0) { nw = rg[q]; nwt = rt[q]; }
                }
                if (__ballot(act && nw < 0 && na > 8)) {
                    uint64_t cm[kR - 8];
#pragma unroll
                    for (int q = 8; q < kR; ++q) cm[q - 8] = sh.cmask[rg[q]];
                    int nw2 = -1;
                    uint32_t nwt2 = 0;
#pragma unroll
                    for (int q = kR - 1; q >= 8; --q)
                        if (q < na && (cm[q - 8] & below) == 0) { nw2 = rg[q]; nwt2 = rt[q]; }
                    if (act && nw < 0) { nw = nw2; nwt = nwt2; }
                }
                if (act && d1) {
                    const bool f1 = !(m1 & below), f2 = d2 && !(m2 & below), f3 = d3 && !(m3 & below);
                    const uint64_t dk = f1 ? d1 : (f2 ? d2 : (f3 ? d3 : 0ull));
                    const int dc = f1 ? dc1 : (f2 ? dc2 : dc3);
                    const uint64_t sk = nw >= 0 ? cl_key(sh, nwt) : 0ull;
                    if (dk > sk) nw = dc;
                }
                const bool ch = nw != cur;
                const uint64_t chm = __ballot(ch);
                if (chm == 0ull) break;
                if (ch) {
                    if (cur >= 0) atomicAnd((unsigned long long*)&sh.cmask[cur], ~(1ull << lane));
                    if (nw >= 0) atomicOr((unsigned long long*)&sh.cmask[nw], 1ull << lane);
                    cur = nw;
                }
                lo_l = __builtin_ctzll(chm) + 1;
            }
            if (i < c1) {
                sh.w[0][i] = (int16_t)cur; sh.w[1][i] = (int16_t)cur;
                sh.code[0][i] = 0; sh.code[1][i] = 0;
            }
        }
        __syncthreads();
        DG(uint64_t tx = dstamp(); acc_cs += tx - t1;)
        // (2b) full sweeps from the guess.  The first evaluates every (pod, chunk row) pair and
        // keeps the totals (tt, in the idle cache buffer: 16-bit totals, 8 KB); later sweeps
        // re-evaluate only the rows phase B rewrote (chg), one wave-uniform row per step, and read
        // the rest
        uint16_t (*tt)[kC] = reinterpret_cast<uint16_t (*)[kC]>(&sh.x.k[0][0][0]);
        static_assert(sizeof(sh.x.k) >= kC * kC * sizeof(uint16_t), "per-pair totals");
        int par = 0, lo = c0, fsv = INT_MAX;
        bool fresh = true;
        if (tid == 0) sh.chg = 0ull;
        for (;;) {
            DG(++n_sweeps; uint64_t q0 = dstamp();)
            // A: the guesses' chunk binds (pod c0 + jr on thread 8 jr: spread over the waves)
            // incrementally: a pod whose guess changed moves its bit and marks both nodes dirty
            int wcur = -1;
            const int jr = tid / kLanesPerPod;
            const bool jlead = tid % kLanesPerPod == 0;
            if (jlead && c0 + jr < c1) {
                wcur = sh.w[par][c0 + jr];
                const int wprv = sh.w[par ^ 1][c0 + jr];
                if (wcur != wprv) {
                    if (wprv >= 0) { atomicAnd((unsigned long long*)&sh.cmask[wprv], ~(1ull << jr)); sh.dirty[wprv] = 1; }
                    if (wcur >= 0) { atomicOr((unsigned long long*)&sh.cmask[wcur], 1ull << jr); sh.dirty[wcur] = 1; }
                }
            }
            __syncthreads();
            DG(uint64_t q1 = dstamp(); acc_ph[0] += q1 - q0;)
            // B: replay each changed chunk node (or one whose first binder moved) into its first
            // chunk binder's slot
            if (jlead && c0 + jr < c1) {
                const int j = c0 + jr;
                if (wcur >= 0 && __builtin_ctzll(sh.cmask[wcur]) == jr) {
                    if (!(KS_CHUNK_ABL & 2) && (sh.dirty[wcur] || sh.smeta[j][kMCid] != wcur)) {
                        sh.dirty[wcur] = 0;
                        (void)replay(sh, wcur, tb, true, c0, c0, j, c1);
                        if (!fresh) atomicOr((unsigned long long*)&sh.chg, 1ull << jr);
                    }
                } else {
                    if (!fresh && sh.smeta[j][kMCid] >= 0) atomicOr((unsigned long long*)&sh.chg, 1ull << jr);
                    sh.smeta[j][kMCid] = -1;
                }
            }
            __syncthreads();
            DG(uint64_t q2 = dstamp(); acc_ph[1] += q2 - q1;)
            if (!fresh) {  // C1: the rewritten rows, wave-uniform (row = the wave's k-th changed row, lane = pod)
                const uint64_t chg = sh.chg;
                if (chg) {
                    const int i = c0 + lane;
                    const bool li = i < c1 && i >= lo;
                    const PodRec p = sh.pod[li ? i : c0];
                    int kx = 0;
                    for (uint64_t m = chg; m; m &= m - 1, ++kx) {
                        if ((kx & (kWaves - 1)) != wave) continue;
                        const int jr = __builtin_ctzll(m);
                        const SRow r = srow(sh, c0 + jr);
                        const int k = r.m(kMCid);
                        const bool v = li && jr < lane;
                        uint32_t t = 0;
                        if (v && k >= 0 && r.m(kMOvf) > i) t = tot_at<kMode>(a, sh, p, i, k, c0 + jr, r);
                        if (v) tt[lane][jr] = (uint16_t)t;
                    }
                }
                __syncthreads();
            }
            // C: the pods c0 + g and c0 + 63 - g on the 16 lanes of group g — together 63 rows
            // (chunk binders before them), four per lane, so every wave evaluates the same
            {
                constexpr int G = 16;
                static_assert(kThreads / G == kC / 2, "two pods per 16-lane group");
                static_assert(kR <= 3 * (G / 2), "three entries per lane of a pod's 8-lane half");
                const int g = tid / G, sub = tid % G, half = sub >> 3, s8 = sub & 7;
                const int iA = c0 + g, iB = c0 + kC - 1 - g;
                const bool actA = iA < c1 && iA >= lo, actB = iB < c1 && iB >= lo;
                const int ih = half ? iB : iA;
                const bool acth = half ? actB : actA;
                // the static list of this half's pod: the lowest free entry
                bool f[3] = {false, false, false};
                uint32_t e[3] = {0u, 0u, 0u};
                if (acth) {
                    const int nc = sh.clcnt[ih];
                    const uint64_t belowh = (1ull << (ih - c0)) - 1ull;
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        if (s8 + 8 * q < nc) e[q] = sh.cl[ih][s8 + 8 * q];
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        if (s8 + 8 * q < nc) {
                            const int c = e[q] >> 16;
                            f[q] = sh.fhead[c] < 0 && (sh.cmask[c] & belowh) == 0;
                        }
                }
                const int rowsh = lane & ~7;
                DG(uint64_t c_a = dstamp(); cs_e += c_a - q2;)
                int rfree = kR;
                uint32_t efree = 0u;
#pragma unroll
                for (int q = 2; q >= 0; --q) {
                    const uint32_t rq = (uint32_t)(__ballot(f[q]) >> rowsh) & 0xFFu;
                    const uint32_t eq = (uint32_t)__shfl((int)e[q], rowsh + (rq ? __builtin_ctz(rq) : 0));
                    if (rq) { rfree = 8 * q + __builtin_ctz(rq); efree = eq; }
                }
                // D over the chunk's first binders: row index rr < g is pod A's row c0 + rr, the
                // rest pod B's row c0 + rr - g (no float-bound pruning: in SIMT the exact evaluation
                // runs whenever one lane of the wave passes the bound)
                uint64_t dkA = 0, dkB = 0;
                int dcA = -1, dcB = -1;
                bool badA = false, badB = false;
                DG(int dwhy = 0;)  // (diagnostic, pod A bits 0-2 / pod B bits 3-5: row state unknown, cached state unknown, both cached rebound)
                if (actA || actB) {
                    const PodRec pA = sh.pod[actA ? iA : iB], pB = sh.pod[actB ? iB : iA];
                    SRow r[4];
                    bool isA[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int rr = sub + G * q;
                        isA[q] = rr < g;
                        const int j = isA[q] ? rr : rr - g;
                        const bool v = isA[q] ? actA : (rr < kC - 1 && actB);
                        r[q] = srow(sh, c0 + (v ? j : 0));
                        if (!v) r[q].clear_cid();
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int k = r[q].m(kMCid);
                        if (k < 0) continue;
                        const int rr = sub + G * q;
                        const int i = isA[q] ? iA : iB;
                        if (r[q].m(kMOvf) <= i) {
                            if (isA[q]) badA = true; else badB = true;
                            DG(dwhy |= isA[q] ? 1 : 8;)
                            continue;
                        }
                        if (KS_CHUNK_ABL & 1) continue;
                        const int jr = isA[q] ? rr : rr - g;
                        uint32_t t;
                        if (fresh) {
                            t = tot_at<kMode>(a, sh, isA[q] ? pA : pB, i, k, c0 + jr, r[q]);
                            tt[i - c0][jr] = (uint16_t)t;
                        } else {
                            t = tt[i - c0][jr];
                        }
                        const uint64_t key = make_key(t, (uint32_t)sh.cnode[k]);
                        if (isA[q]) { if (key > dkA) { dkA = key; dcA = k; } }
                        else if (key > dkB) { dkB = key; dcB = k; }
                    }
                }
                DG(uint64_t c_b = dstamp(); cs_r += c_b - c_a;)
                if ((sub & 7) == 0 && acth) {  // pre-chunk nodes: the best one not rebound before the pod
                    const int pi = ih - c0;
                    const uint64_t below = (1ull << pi) - 1ull;
                    uint64_t& dk = half ? dkB : dkA;
                    int& dc = half ? dcB : dcA;
                    bool& bad = half ? badB : badA;
                    if (sh.cdbad[pi]) {
                        bad = true;
                        DG(dwhy |= half ? 16 : 2;)
                    } else {
                        uint64_t ck = sh.cd1[pi];
                        int cc = sh.cd1c[pi];
                        if (ck != 0 && (sh.cmask[cc] & below)) {
                            ck = sh.cd2[pi];
                            cc = sh.cd2c[pi];
                            if (ck != 0 && (sh.cmask[cc] & below)) {
                                ck = sh.cd3[pi];
                                cc = sh.cd3c[pi];
                                if (ck != 0 && (sh.cmask[cc] & below)) { bad = true; DG(dwhy |= half ? 32 : 4;) }
                            }
                        }
                        if (ck > dk) { dk = ck; dc = cc; }
                    }
                }
#pragma unroll
                for (int o = 1; o < G; o <<= 1) {
                    const uint64_t okA = shfl_xor64(dkA, o), okB = shfl_xor64(dkB, o);
                    const int ocA = __shfl_xor(dcA, o), ocB = __shfl_xor(dcB, o);
                    if (okA > dkA) { dkA = okA; dcA = ocA; }
                    if (okB > dkB) { dkB = okB; dcB = ocB; }
                }
                DG(cs_x += dstamp() - c_b;)
                const int gsh = lane & ~(G - 1);
                // Both ballots with every lane active: each pod's rows are spread over all 16 lanes
                // of the group (pod B's row j on lane (j + g) % 16, either half).  (Until round 6 the
                // ballots sat in the two arms of `half ? ... : ...` — a divergent branch, so each
                // ballot saw only its own half's lanes: a row whose state overflowed its segments on
                // the other half's lane was dropped from D instead of stopping the batch, and the pod
                // could bind a lower node — tests/test_resolvers_gpu.py segment-overflow test.)
#ifdef KS_BALLOT_LEGACY  // (diagnostic build only: the pre-round-6 form, for the regression test's A/B)
                const bool bad = half ? ((__ballot(badB) >> gsh) & 0xFFFFu) != 0 : ((__ballot(badA) >> gsh) & 0xFFFFu) != 0;
#else
                const uint64_t bmA = __ballot(badA), bmB = __ballot(badB);
                const bool bad = (((half ? bmB : bmA) >> gsh) & 0xFFFFull) != 0;
#endif
                DG(int wa = 0; for (int o = 0; o < G; ++o) wa |= __shfl(dwhy, gsh + o);)  // (the group's stop reasons)
                const uint64_t dk = half ? dkB : dkA;
                const int dc = half ? dcB : dcA;
                if (s8 == 0 && ih < c1) {
                    const int i = ih;
                    int code;
                    int nw;
                    if (acth) {
                        const uint8_t fl = sh.clfl[i];
                        uint64_t win = 0;
                        int wc = -1;
                        code = 0;
                        if (bad || (fl & kFlOvf)) {
                            code = 1;
                            DG({
                                const int mine = half ? (wa >> 3) & 7 : wa & 7;
                                sh.why[i] = !bad ? 1 : (mine & 4) ? 6 : (mine & 2) ? 5 : 0;
                            })
                        } else if (rfree < kR) {
                            const uint64_t sk = cl_key(sh, efree);
                            if (sk > dk) { win = sk; wc = (int)(efree >> 16); }
                            else { win = dk; wc = dc; }
                        } else if (fl & kFlTrunc) {  // kept entries all bound: D must beat the last kept
                            if (dk > cl_key(sh, sh.cl[i][kR - 1])) { win = dk; wc = dc; }
                            else { code = 1; DG(sh.why[i] = 2;) }
                        } else if (fl & kFlFull) {   // exhausted list: D must beat the list's last key
                            if (dk > ws.cl_thr[i]) { win = dk; wc = dc; }
                            else { code = 1; DG(sh.why[i] = 3;) }
                        } else {
                            win = dk; wc = dc;
                        }
                        if (code == 0) {
                            if (win == 0) code = 2;                                                  // NotFound
                            else if (sh.pod[i].flags & (kFlagBadKey | kFlagBadSpec)) code = 3;   // InvalidArgument
                        }
                        nw = code == 0 ? wc : -1;
                        if (nw != sh.w[par][i] || code != sh.code[par][i]) atomicMin(&sh.fc[par], i);
                    } else {
                        nw = sh.w[par][i];
                        code = sh.code[par][i];
                    }
#ifdef KS_BATCH_LOG
                    if (start + i == a.sw->watch_pod && !a.sw->watch_done) {
                        WinWS& wl = *a.sw;
                        const int k = wl.w_nsw;
                        if (k < 64) {
                            wl.w_dec[k][0] = fresh; wl.w_dec[k][1] = lo; wl.w_dec[k][2] = bad; wl.w_dec[k][3] = code;
                            wl.w_dec[k][4] = nw; wl.w_dec[k][5] = dc; wl.w_dec[k][6] = (int)(dk >> 32); wl.w_dec[k][7] = c0;
                        }
                        wl.w_nsw = k + 1;
                    }
#endif
                    sh.w[par ^ 1][i] = (int16_t)nw;
                    sh.code[par ^ 1][i] = (int8_t)code;
                    if (code != 0) atomicMin(&sh.fs[par], i);
                }
            }
            __syncthreads();
            DG(uint64_t q3 = dstamp(); acc_ph[2] += q3 - q2;)
            // D: convergence; clear this sweep's masks and the next sweep's accumulators
            const int fcv = sh.fc[par];
            fsv = sh.fs[par];
            // No barrier here: the next round's accumulators (par ^ 1) are only written after its
            // phase-A barrier, which tid 0 reaches after this reset; this round's (par) are reset
            // two rounds on, after every thread has passed the next phase-A barrier.
            if (tid == 0) { sh.fc[par ^ 1] = INT_MAX; sh.fs[par ^ 1] = INT_MAX; sh.chg = 0ull; }
            DG(acc_ph[3] += dstamp() - q3;)
            par ^= 1;
            fresh = false;
            if (fcv == INT_MAX || fcv >= fsv) break;
            lo = fcv + 1;
        }
        DG(uint64_t t2 = dstamp(); acc_sw += t2 - t1;)

#ifdef KS_BATCH_LOG
        {
            WinWS& wl = *a.sw;
            const int64_t wi = (int64_t)wl.watch_pod - start;
            if (!wl.watch_done && wi >= c0 && wi < c1 && tid < kC) {
                for (int q = 0; q < 8; ++q) wl.w_smeta[tid][q] = sh.smeta[c0 + tid][q];
                wl.w_rowcid[tid] = sh.w[par][c0 + tid];
            }
        }
#endif
        // (3) finalize the chunk's prefix [c0, cend): admissions known, final bind lists
        int cend = fsv < c1 ? fsv : c1;
        if (tid < kC) {
            const int i = c0 + tid;
            if (i < cend && sh.adm[i] == 2) atomicMin(&sh.cut, i);
        }
        __syncthreads();
        // every thread has read this chunk's last accumulators (before the barrier above)
        if (tid == 0) { sh.fc[0] = sh.fc[1] = INT_MAX; sh.fs[0] = sh.fs[1] = INT_MAX; }
        const bool cut = sh.cut < cend;
        if (cut) cend = sh.cut;
        // the masks hold the last sweep's guesses (= the final winners before cend)
        const uint64_t keep = cend - c0 >= 64 ? ~0ull : ((1ull << (cend - c0)) - 1ull);
        int wk = -1;
        if (tid < kC) {
            const int i = c0 + tid;
            if (i < c1) wk = sh.w[par ^ 1][i];
            if (i < cend) sh.wf[i] = (int16_t)sh.w[par][i];
        }
        if (wk >= 0 && __builtin_ctzll(sh.cmask[wk]) == tid) {
            uint64_t m = sh.cmask[wk] & keep;
            int tail = sh.ftail[wk];
            if (m && sh.fcur[wk] < 0) sh.fcur[wk] = (int16_t)(c0 + __builtin_ctzll(m));
            while (m) {
                const int j = c0 + __builtin_ctzll(m);
                m &= m - 1;
                if (tail >= 0) sh.fnext[tail] = (int16_t)j;
                else sh.fhead[wk] = (int16_t)j;
                sh.fnext[j] = -1;
                tail = j;
            }
            sh.ftail[wk] = (int16_t)tail;
        }
        __syncthreads();
        if (wk >= 0) { sh.cmask[wk] = 0; sh.dirty[wk] = 0; }
        if (tid < kC && c0 + tid < c1) { sh.w[0][c0 + tid] = -1; sh.w[1][c0 + tid] = -1; }
        __syncthreads();
        DG(acc_fin += dstamp() - t2;)
        if (cend < c1) {
            committed = cend;
            stop_code = cut ? 1 : sh.code[par][cend];
#ifdef KS_CHUNK_DIAG
            if (tid == 0) {
                unsigned long long* d = (unsigned long long*)a.ctr;
                const int r = cut ? 4 : (stop_code == 1 ? sh.why[cend] : 4);  // (4: adm unknown or NotFound/bad)
                atomicAdd(&d[r == 5 ? 14 : r == 6 ? 22 : 9 + r], 1ull);
            }
#endif
            break;
        }
    }
    DG(uint64_t t3 = dstamp();)

    // ---- commit pods [0, c): outputs, expiry marks, node state write-back
    const int c = committed;
#ifdef KS_BATCH_LOG  // (diagnostic builds only)
    {
        WinWS& wl = *a.sw;
        if (tid == 0) {
            const int k = wl.blog_n;
            if (k < 16384) {
                wl.blog[k][0] = (int32_t)(start & 0x7FFFFFFF); wl.blog[k][1] = c; wl.blog[k][2] = stop_code; wl.blog[k][3] = nb;
            }
            wl.blog_n = k + 1;
        }
        const int64_t wp = wl.watch_pod;
        if (!wl.watch_done && wp >= start && wp < start + c) {
            for (int q = tid; q < nb * kR; q += kThreads) wl.w_cl_key[q / kR][q % kR] = ws.cl_key[q / kR][q % kR];
            if (tid < nb) { wl.w_cl_info[tid] = ws.cl_info[tid]; wl.w_cl_thr[tid] = ws.cl_thr[tid]; }
            for (int q = tid; q < n_eall; q += kThreads) wl.w_e_node[q] = ws.e_node[q];
            if (tid < c) { wl.w_bind[tid] = sh.cnode[sh.wf[tid]]; wl.w_adm[tid] = sh.adm[tid]; }
            __syncthreads();
            if (tid == 0) { wl.w_start = (int32_t)start; wl.w_nb = nb; wl.w_c = c; wl.w_n_e = n_eall; wl.w_n_es = n_e; wl.watch_done = 1; }
        }
    }
#endif
    const int h_end = c >= 1 ? sh.win_hi[c - 1] : 0;  // slots applied: < win_hi[c - 1]
    if (tid < c) {
        const int64_t j = start + tid;
        const int k = sh.wf[tid];
        gptr(a.b_node)[j] = sh.cnode[k];
        const bool ok = sh.adm[tid] == 1;
        gptr(a.b_status)[j] = ok ? 0 : 1;
        const int x = sh.own[tid];
        if (ok && (sh.clfl[tid] & kFlRun) && x >= 0 && x < h_end) gptr(a.expired)[j] = 1;
    }
    if (tid < h_end && xq >= 0) gptr(a.expired)[xq] = 1;  // (h_end <= e_cnt <= kSlots <= kThreads)
    for (int k = tid; k < ncid; k += kThreads) {
        if (sh.ceix[k] >= 0 || sh.fhead[k] >= 0) {
            const NS32 v = replay(sh, k, tb, false, 0, 0, -1, c).v;
            const int32_t n = sh.cnode[k];
            a.s.rc[n] = use64(v.rc); a.s.rm[n] = use64(v.rm); a.s.rg[n] = use64(v.rg); a.s.nr[n] = v.nr;
        }
    }
    DG(__syncthreads(); acc_crep = dstamp() - t3;)
    // slot-E nodes that are no candidate of this batch: their expiries before pod c - 1's bind
    // here (requests from the LDS words: exact, an admitted request is below its capacity < 2^32)
    static_assert(kSlots <= kThreads, "one slot-E node per thread");
    if (tid < n_e && sh.e2c[tid] < 0) {
        const int32_t n = enode[0];
        int64_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
        for (int u = sh.eoff[tid]; u < sh.eoff[tid + 1]; ++u) {
            const int4 r = sh.erow[u];
            if (r.x >= c) break;  // ascending; slot < win_hi[c - 1] <=> applied from a pod < c
            d0 += use64(r.y); d1 += use64(r.z); d2 += use64(r.w); d3 += 1;
        }
        if (d3) {  // (no other thread touches the node: fire-and-forget atomics, no read back)
            atomicAdd((unsigned long long*)&a.s.rc[n], (unsigned long long)-d0);
            atomicAdd((unsigned long long*)&a.s.rm[n], (unsigned long long)-d1);
            atomicAdd((unsigned long long*)&a.s.rg[n], (unsigned long long)-d2);
            atomicAdd((unsigned long long*)&a.s.nr[n], (unsigned long long)-d3);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)  // every E node's index mark
        if (tid + q * kThreads < n_eall) a.e_idx[enode[q]] = -1;
#pragma unroll
    for (int q = 0; q < 2; ++q)
        if (tid + q * kThreads < nlo) {
            a.n_slot[snd[q]] = -1;
            if (det) a.n_first[snd[q]] = kNoFirst;
        }
    for (int k = nlo + tid; k < nslot; k += kThreads) {
        const int32_t nd = ws.slot_node[k];
        a.n_slot[nd] = -1;
        if (det) a.n_first[nd] = kNoFirst;
    }
    // the nodes this batch changed — its binds' nodes (every cid with a final bind) and its window's
    // expiry nodes — for the next batch's overlapped scan (ks_cand.hip window_prep_kernel)
    {
        WinWS& wo = *a.sw;
        if (tid == 0) sh.nbc = 0;
        __syncthreads();
        for (int k = tid; k < ncid; k += kThreads)
            if (sh.fhead[k] >= 0) wo.touched[atomicAdd(&sh.nbc, 1)] = sh.cnode[k];
        if (tid < n_e) wo.touched[atomicAdd(&sh.nbc, 1)] = enode[0];  // (every slot-E node has slots)
        __syncthreads();
        if (tid == 0) {
            wo.n_touched = sh.nbc;
            if (ws.nslot > wo.nslot_hw) wo.nslot_hw = ws.nslot;  // (diagnostics: ks_debug_invariants)
        }
    }
    if (tid == 0) {
        a.ctr[kCtrStart] = start + c;
        const bool err = stop_code == 2 || stop_code == 3;
        if (err) {
            a.ctr[kCtrErr] = stop_code == 2 ? kErrNotFound : kErrEinval;
            a.ctr[kCtrErrPod] = start + c;
        }
        sh.t_start = start + c;
        sh.t_err = err ? 1 : 0;
        if (c < a.B && !err && start + c < end) a.ctr[kCtrEarly] += 1;
    }
#ifdef KS_CHUNK_DIAG
    __syncthreads();
    if (tid == 0) {
        unsigned long long* d = (unsigned long long*)a.ctr;
        atomicAdd(&d[5], 1ull);
        atomicAdd(&d[6], (unsigned long long)c);
        atomicAdd(&d[7], (unsigned long long)n_sweeps);
        atomicAdd(&d[8], (unsigned long long)n_chunks);
        atomicAdd(&d[16], t_setup);
        atomicAdd(&d[17], acc_cd);
        atomicAdd(&d[18], acc_sw);
        atomicAdd(&d[19], acc_fin);
        atomicAdd(&d[20], dstamp() - t3);
        atomicAdd(&d[21], (unsigned long long)ncid);
        (void)acc_cdp; (void)acc_rb;  // (d[14], d[22]: stop reasons 5, 6)
        atomicAdd(&d[23], (unsigned long long)nb);
#if KS_CHUNK_DIAG == 2  // finer split (tests/dev/diag_chunk.py --d2): cache parts, commit replays, setup loads
        atomicAdd(&d[24], acc_rbase); atomicAdd(&d[25], acc_rb - acc_rbase); atomicAdd(&d[26], acc_cdp);
        atomicAdd(&d[27], acc_red); atomicAdd(&d[28], acc_crep); atomicAdd(&d[31], ts1 - (ts3 - t_setup));
        (void)acc_ph; (void)n_sonly; (void)cs_e; (void)cs_r; (void)cs_x;
#else
        (void)acc_rbase; (void)acc_red; (void)acc_crep;
        for (int q = 0; q < 4; ++q) atomicAdd(&d[24 + q], acc_ph[q]);
        atomicAdd(&d[28], (unsigned long long)n_sonly);
        atomicAdd(&d[29], cs_e); atomicAdd(&d[30], cs_r); atomicAdd(&d[31], cs_x);
#endif
        atomicAdd(&d[15], acc_cs);
    }
#endif
}

template <int kMode>
__global__ __launch_bounds__(kThreads) void resolve_chunk_kernel(const EngineArgs* __restrict__ A) {
    __shared__ ChShared sh;
    chunk_body<kMode>(A, sh);
}

// The chunk kernel with the next batch's scan fused in (the overlap on one stream): workgroup 0
// resolves the batch; the others — one per CU, the resolver's LDS footprint fixes that — scan the
// speculative pods (As: counters window prep wrote) in the resolver's LDS image, two (node block,
// pod group) items at a time, one per 256-thread half, from its XCD's share of the batch's
// block-major item list.  The scan reads node records the resolver may be committing: only
// nodes the batch touches, which the next batch re-evaluates (ks_cand.hip window_prep_kernel).
// (Leaving the batch's candidate slots out of these lists, so that the next batch's top-L holds no
// node the batch could bind, was measured worse: those nodes then all join the next batch's E,
// enough of them reach its lists' thresholds to overflow the candidate slots, and the batches
// commit ~104 pods instead of ~181.)
// After its commit the resolver workgroup also computes the next batch's window (ks_prep.h, with the
// head expiries and the touched nodes; `slot`: that batch's speculative-counter parity) in its LDS:
// the standalone window-prep launch and its kernel boundary leave the critical path.
template <int kMode, bool kPrune, int kLL>
__global__ __launch_bounds__(kThreads) void chunk_scan_kernel(const EngineArgs* __restrict__ A,
                                                              const EngineArgs* __restrict__ As, int slot) {
    __shared__ ChShared sh;
    if (blockIdx.x == 0) {
        chunk_body<kMode>(A, sh);
        __syncthreads();
        const int64_t st = sh.t_start, en = sh.t_end, er = sh.t_err;
        __syncthreads();  // (the window's scratch overlays the resolver's LDS)
#if defined(KS_CHUNK_DIAG) && KS_CHUNK_DIAG == 2
        const uint64_t tp0 = dstamp();
#endif
        static_assert(sizeof(prep::PrepLDS) <= sizeof(ChShared), "window scratch");
        prep::prep_body<kThreads>(A[0], st, en, er, 1, 1, slot, *reinterpret_cast<prep::PrepLDS*>(&sh));
#if defined(KS_CHUNK_DIAG) && KS_CHUNK_DIAG == 2
        __syncthreads();
        if (threadIdx.x == 0) atomicAdd((unsigned long long*)&A[0].ctr[30], dstamp() - tp0);
#endif
        return;
    }
    static_assert(kThreads == 2 * scn::kNodes, "two scan groups per workgroup");
    const EngineArgs& a = As[0];
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    const int64_t nb = min<int64_t>(a.B, end - start);
    if (a.ctr[kCtrErr] != 0 || nb <= 0) return;
    const int groups = (int)((nb + a.PG - 1) / a.PG);
    const int64_t tot = (int64_t)a.blk_n * groups;
    const int half = threadIdx.x / scn::kNodes, lt = threadIdx.x % scn::kNodes;
    uint16_t* kv = reinterpret_cast<uint16_t*>(&sh) + (size_t)half * a.PG * scn::kNodes;
    // XCD-aware deal (blocks b and b + 8 share an XCD): XCD x = b % 8 takes the contiguous item
    // range [x per, (x + 1) per) — whole node blocks with their pod groups — shared by its
    // workgroups, so a node block's records come from HBM once and from that XCD's L2 after
    const int x = (int)(blockIdx.x % 8), j = (int)(blockIdx.x / 8) - (x == 0 ? 1 : 0);  // (block 0: the resolver)
    const int nx = (int)((gridDim.x - x + 7) / 8) - (x == 0 ? 1 : 0);                  // workgroups of XCD x
    const int64_t per = (tot + 7) / 8, lo = x * per, hi = min<int64_t>(tot, lo + per);
    for (int64_t r = lo + 2 * (int64_t)j; r < hi; r += 2 * (int64_t)nx) {  // (uniform per workgroup)
        if (r != lo + 2 * (int64_t)j) __syncthreads();  // the previous round's extraction has read kv
        const int64_t it = r + half;
        scn::scan_item<kMode, uint16_t, kPrune, kLL>(a, kv, start, nb, groups, it, it < hi, lt, x);
    }
}
static_assert(sizeof(ChShared) >= 2 * kMaxPGScan * scn::kNodes * sizeof(uint16_t), "two 16-bit key tables");

}  // namespace chk

// the chunk resolver proper (its window and candidate lists: launch_window_prep(head) and
// launch_merge_cl, ks_cand.hip)
template <bool kPrune, int kLL>
static void launch_chunk_scan_t(const EngineArgs* d, const EngineArgs* ds, const dim3& g, int sl, int mode, hipStream_t st) {
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL((chk::chunk_scan_kernel<kEvalMicro, kPrune, kLL>), g, dim3(chk::kThreads), 0, st, d, ds, sl); break;
        case kEvalTiny: hipLaunchKernelGGL((chk::chunk_scan_kernel<kEvalTiny, kPrune, kLL>), g, dim3(chk::kThreads), 0, st, d, ds, sl); break;
        case kEvalNarrow: hipLaunchKernelGGL((chk::chunk_scan_kernel<kEvalNarrow, kPrune, kLL>), g, dim3(chk::kThreads), 0, st, d, ds, sl); break;
        default: hipLaunchKernelGGL((chk::chunk_scan_kernel<kEvalWide, kPrune, kLL>), g, dim3(chk::kThreads), 0, st, d, ds, sl); break;
    }
}

hipError_t launch_chunk_scan(const EngineArgs* d, const EngineArgs* ds, int workers, int next_slot, int mode,
                             bool prune, int L, hipStream_t st) {
    const dim3 g(1 + workers);
    if (L != kTopL) {
        if (prune || L != kTopLOverlap) return hipErrorInvalidValue;
        launch_chunk_scan_t<false, kTopLOverlap>(d, ds, g, next_slot & 1, mode, st);
    } else if (prune) {
        launch_chunk_scan_t<true, kTopL>(d, ds, g, next_slot & 1, mode, st);
    } else {
        launch_chunk_scan_t<false, kTopL>(d, ds, g, next_slot & 1, mode, st);
    }
    return hipGetLastError();
}

hipError_t launch_chunk_only(const EngineArgs* d, int mode, hipStream_t st) {
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL(chk::resolve_chunk_kernel<kEvalMicro>, dim3(1), dim3(chk::kThreads), 0, st, d); break;
        case kEvalTiny: hipLaunchKernelGGL(chk::resolve_chunk_kernel<kEvalTiny>, dim3(1), dim3(chk::kThreads), 0, st, d); break;
        case kEvalNarrow: hipLaunchKernelGGL(chk::resolve_chunk_kernel<kEvalNarrow>, dim3(1), dim3(chk::kThreads), 0, st, d); break;
        default: hipLaunchKernelGGL(chk::resolve_chunk_kernel<kEvalWide>, dim3(1), dim3(chk::kThreads), 0, st, d); break;
    }
    return hipGetLastError();
}

}  // namespace ks
