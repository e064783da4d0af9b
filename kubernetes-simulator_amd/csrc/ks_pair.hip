// ks_pair.hip — the pair resolver (gfx950): one 1024-thread workgroup walks a batch in FIFO
// order deciding TWO pods per barrier.
//
// Same exactness argument as resolve_kernel (ks_kernels.hip): a node's key for pod p can differ
// from the batch snapshot only if a bind or an expiry of this batch touched it; touched nodes
// are table entries evaluated exactly, the best untouched node is the first untouched entry of
// the pod's snapshot top-L list, and a full list with every entry touched stops the batch.
// The reference binds one pod per tick in FIFO order (kubesim/kubesim.go:105-121, 143-166) with
// admission per kubesim/node/node.go:36-60; that order is kept exactly.
//
// What changes is the shape of an iteration.  Iteration k decides pods a = 2k and b = 2k+1,
// binds both and prepares the next pair (c, d) = (a+2, a+3).  Pod b's decision depends on pod
// a's winner w_a, so everything it needs is computed one iteration early for both outcomes:
//
//   K1_b(e)   e's key for pod b if e does NOT win pod a
//   K2_b(e)   e's key for pod b if e wins pod a (admission, bound state, the expiries due
//             between a and b) — only for the candidates of pod a (key_a(e) >= lbk_a, a lower
//             bound of pod a's winner known before the iteration): ~1-3 entries per pair
//
// and folded with LDS atomics into four words of the pair's control record Pc:
//
//   best  max over pod a's candidates of (key_a | K2_b in the low bits)   -> w_a, K2_b(w_a)
//   m2    max over the non-candidates of K1_b  (they cannot be w_a)
//   mc    max over the candidates of K1_b      (valid unless it belongs to w_a)
//   vb1/2 pod b's first two untouched list entries (minus the table and the known winners)
//
// so that after the barrier every wave computes, with a few selects,
//   w_b = max(m2, K2_b(w_a), mc unless it is w_a's, vb1 unless it is w_a else vb2).
// If mc belongs to w_a and beats the rest, the candidates other than w_a refold their K1_b in
// one extra barrier round (rare: the exact CPU model, tests/dev/pair_pipeline_model.py, checks
// the whole scheme bind-for-bind against the oracle).
//
// Waves:
//   0        walker: K2 of pod c's kept list candidates (records prefetched the iteration
//            before), picks pod c's untouched candidate (the first kept one that is neither w_a
//            nor w_b) and folds it, narrows pod d's to two, stages their records for the bind,
//            walks the lists of the pair after next — keeping 3 and 4 untouched entries, since
//            2 and 3 winners before them are still unknown — and issues those records' loads.
//   1        bind wave, lanes 0-5: lane = (variant << 1) | node.  Every lane fetches its node's
//            state (w_a or w_b), binds pod a / pod b on it with the expiries due between them,
//            then evaluates its variant (key_c, K1_d, K2_d) in ONE evaluator pass; lanes 0/1 fold.
//   2..15    owners: lane r keeps touched entry r in registers, applies the expiries of the
//            windows b and c that land on it, evaluates key_c / K1_d / K2_d when the float bound
//            reaches the lower bounds, folds.
//
// Windows: pod i's window is the expiries due before pod i binds (a contiguous slot range; the
// windows of consecutive pods are adjacent).  Window b is applied whenever pod a binds, window c
// only when pod b binds too (a batch that stops at b must not apply expiries due after b: the
// next launch rescans from b), window d only speculatively (K1_d, K2_d).
#include "ks_device.h"

namespace ks {
namespace pr {

constexpr int kL = kTopL;
constexpr int kThreads = 1024;
constexpr int kTMax = 768;               // touched entries
constexpr int kHashLog2 = 11, kHash = 1 << kHashLog2;
constexpr int kMaxB = 256;               // pods per launch
constexpr int kMaxExp = kTMax - kMaxB;   // expiries pre-inserted per batch
constexpr int kFilterBits = 1 << 16;
constexpr int kOwner0 = 2;               // waves 2..15 own the entries
constexpr int kUnt = 1023;               // entry field of an untouched node
constexpr int kKeep = 7;                 // walker lanes: 3 candidates of pod c, 4 of pod d
constexpr int kPodPad = 4;
static_assert(kTMax <= (kThreads / kWave - kOwner0) * kWave, "one entry per owner lane");  // slots 0..13
static_assert(kMaxExp <= kThreads, "one thread per pre-inserted expiry");
static_assert(kTMax < kUnt, "entry index fits 10 bits");

// Decision word: (total+1) << 49 | (2^24-1-node) << 25 | entry << 15 | K2 total+1 (15 bits).
// Orders like the packed key (highest total, ties to the lowest node) for any two distinct
// nodes; the host uses this kernel only when every total + 1 < 2^15 (nodes < 2^24 always).
__device__ __forceinline__ uint64_t dword(uint32_t t1, uint32_t node, uint32_t ent, uint32_t k2) {
    return t1 ? ((uint64_t)t1 << 49) | ((uint64_t)(0xFFFFFFu - node) << 25) | ((uint64_t)ent << 15) | (uint64_t)k2
              : 0ull;
}
// from the packed key form (total+1) << 32 | (0xFFFFFFFF - node)
__device__ __forceinline__ uint64_t dword_key(uint64_t key, uint32_t ent, uint32_t k2) {
    return key ? dword((uint32_t)(key >> 32), 0xFFFFFFFFu - (uint32_t)key, ent, k2) : 0ull;
}
__device__ __forceinline__ int32_t dw_node(uint64_t w) { return (int32_t)(0xFFFFFFu - (uint32_t)((w >> 25) & 0xFFFFFFu)); }
__device__ __forceinline__ int32_t dw_ent(uint64_t w) { return (int32_t)((w >> 15) & 1023u); }
__device__ __forceinline__ uint32_t dw_k2(uint64_t w) { return (uint32_t)(w & 0x7FFFu); }
__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }
__device__ __forceinline__ void fold(uint64_t* slot, uint64_t v) {
    atomicMax((unsigned long long*)slot, (unsigned long long)v);
}
__device__ __forceinline__ uint64_t umax64(uint64_t x, uint64_t y) { return x > y ? x : y; }

// Control record of pair k (ring of three): folds made in iteration k-1, the walker's list
// candidates of pod b (iteration k-1) and lower bounds of both pods (iteration k-2).  The first
// 48 bytes are what every wave's decision reads.
struct alignas(16) Pc {
    uint64_t best, m2, mc;       // folds (zeroed two iterations ahead)
    uint64_t vb1, vb2;           // pod b's untouched list candidates, decision words (entry kUnt), 0 = none
    uint32_t fl;                 // kfull_a | full_b << 1 | (sa + 1) << 4 | (sb1 + 1) << 8 | (sb2 + 1) << 12
    uint32_t pad0;
    uint64_t lbk_a, lbk_b;       // lower bounds of the pair's winners (packed-key form)
    uint64_t mcx, pad1;          // extra fold round
};
static_assert(sizeof(Pc) == 80, "Pc: five 16-byte words");
__device__ __forceinline__ bool pc_kfull_a(const Pc& p) { return p.fl & 1u; }
__device__ __forceinline__ bool pc_full_b(const Pc& p) { return (p.fl >> 1) & 1u; }
__device__ __forceinline__ int32_t pc_slot(const Pc& p, int which) { return (int32_t)((p.fl >> (4 + 4 * which)) & 15u) - 1; }

// Per-pod control: flags | (own expiry slot + 1) << 2, run ticks, the pod's window [lo, hi).
struct alignas(16) PodW {
    uint32_t w0;
    int32_t dur, lo, hi;
};

struct Shared {
    int64_t ts[8][kTMax];  // touched-node state: ac am ag ap rc rm rg nr
    uint64_t tu[2][kTMax];  // taint label
    int32_t tnode[kTMax];
    int32_t dirty[kTMax];  // iteration at which the owner must reload the mutable fields
    int32_t hkey[kHash];   // node id or -1
    int32_t hval[kHash];   // entry index
    uint32_t tfilt[kFilterBits / 32];
    PodRec pod[kMaxB + kPodPad];
    float podf[kMaxB + kPodPad][2];
    PodW pwx[kMaxB + kPodPad + 2];  // pod i at pwx[i + 2] (the prologue reads pods -2, -1)
    uint64_t cand[kMaxB][kL];
    int32_t ex_q[kMaxExp];
    int32_t ex_node[kMaxExp];
    int32_t ex_ok[kMaxExp];     // the expiring pod was bound Ok and has not expired yet
    int32_t ex_entry[kMaxExp];  // table entry of its node (set at the bind for in-batch pods)
    int64_t ex_req[kMaxExp][3];
    Pc pc[3];
    int64_t stage[2][kKeep][10];  // snapshot records of a pair's kept list candidates
    uint64_t dec_word;  // the bind wave's published decision: (2k + final) << 32 | dec_pack()
    int32_t n_t, nb, e_cnt, pad_;
};

// Diagnostic build only (-DKS_STAMPS, `make stamps`): per-role cycle sums accumulated in
// ctr[16..31] (layout: tests/dev/diag_pair.py); the real kernel executes no stamp.
#ifdef KS_STAMPS
__device__ __forceinline__ uint64_t pstamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define PR_STAMP(var) const uint64_t var = pstamp()
#define PR_ACC(i, v) acc[i] += (v)
#else
#define PR_STAMP(var)
#define PR_ACC(i, v)
#endif

__device__ __forceinline__ uint32_t hslot(int32_t node) { return ((uint32_t)node * 2654435761u) >> (32 - kHashLog2); }

__device__ __forceinline__ int h_find(const Shared& sh, int32_t node) {
    uint32_t s = hslot(node);
    for (int i = 0; i < kHash; ++i) {
        const int32_t k = sh.hkey[s];
        if (k == node) return sh.hval[s];
        if (k == -1) return -1;
        s = (s + 1) & (kHash - 1);
    }
    return -1;
}

// touched?  The filter is exact (node & 0xFFFF injective) for clusters of <= kFilterBits nodes,
// otherwise a set bit is confirmed in the hash.
__device__ __forceinline__ bool is_touched(const Shared& sh, int32_t node, bool exact) {
    const uint32_t f = (uint32_t)node & (kFilterBits - 1);
    if (!((sh.tfilt[f >> 5] >> (f & 31)) & 1u)) return false;
    return exact || h_find(sh, node) >= 0;
}

// table insert of an in-loop winner (two lanes may insert at once: CAS on the hash slot)
__device__ __forceinline__ void t_insert(Shared& sh, int32_t node, int32_t idx, bool exact) {
    if (!exact) {
        uint32_t s = hslot(node);
        for (int i = 0; i < kHash; ++i) {  // the table holds < kHash nodes: terminates
            if (atomicCAS(&sh.hkey[s], -1, node) == -1) {
                sh.hval[s] = idx;
                break;
            }
            s = (s + 1) & (kHash - 1);
        }
    }
    const uint32_t f = (uint32_t)node & (kFilterBits - 1);
    atomicOr(&sh.tfilt[f >> 5], 1u << (f & 31));
}

__device__ __forceinline__ NodeV t_node(const Shared& sh, int e) {
    NodeV v;
    v.ac = sh.ts[0][e]; v.am = sh.ts[1][e]; v.ag = sh.ts[2][e]; v.ap = sh.ts[3][e];
    v.rc = sh.ts[4][e]; v.rm = sh.ts[5][e]; v.rg = sh.ts[6][e]; v.nr = sh.ts[7][e];
    v.taint = sh.tu[0][e]; v.label = sh.tu[1][e];
    return v;
}
__device__ __forceinline__ NodeV stage_node(const Shared& sh, int par, int s) {
    const int64_t* r = sh.stage[par][s];
    NodeV v;
    v.ac = r[0]; v.am = r[1]; v.ag = r[2]; v.ap = r[3]; v.rc = r[4]; v.rm = r[5]; v.rg = r[6]; v.nr = r[7];
    v.taint = (uint64_t)r[8]; v.label = (uint64_t)r[9];
    return v;
}
__device__ __forceinline__ int64_t node_field(const NodeSoA& s, int f, int64_t i) {
    return gptr(s.ac)[(int64_t)f * (s.am - s.ac) + i];
}
__device__ __forceinline__ void add_req(NodeV& n, const PodRec& p, int64_t sgn) {
    n.rc += sgn * p.req[0]; n.rm += sgn * p.req[1]; n.rg += sgn * p.req[2]; n.nr += sgn;
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
// a 48-byte pod record read from LDS as three 16-byte loads issued together, pinned in registers
__device__ __forceinline__ PodRec pod_regs(const PodRec* src) {
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
// The decision's 48 bytes of a control record.  Every wave reads the same bytes: as a
// full-wave ds_read each 16-byte load costs the LDS 64 lanes x 16 B; KS_PR_UNI reads them with
// lane 0 alone and broadcasts through SGPRs (readfirstlane).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
#ifndef KS_PR_UNI
#define KS_PR_UNI 0
#endif
__device__ __forceinline__ Pc pc_regs(const Pc* src) {
    u32x4 w0, w1, w2;
#if KS_PR_UNI
    uint64_t sv;
    asm volatile(
        "s_mov_b64 %[sv], exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "ds_read_b128 %[a], %[ad]\n\t"
        "ds_read_b128 %[b], %[ad] offset:16\n\t"
        "ds_read_b128 %[c], %[ad] offset:32\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_mov_b64 exec, %[sv]"
        : [a] "=&v"(w0), [b] "=&v"(w1), [c] "=&v"(w2), [sv] "=&s"(sv)
        : [ad] "v"(lds_addr(src))
        : "memory");
    w0 = u32x4{rfl(w0.x), rfl(w0.y), rfl(w0.z), rfl(w0.w)};
    w1 = u32x4{rfl(w1.x), rfl(w1.y), rfl(w1.z), rfl(w1.w)};
    w2 = u32x4{rfl(w2.x), rfl(w2.y), rfl(w2.z), rfl(w2.w)};
#else
    const u32x4* w = reinterpret_cast<const u32x4*>(src);
    w0 = w[0]; w1 = w[1]; w2 = w[2];
    asm volatile("" ::"v"(w0), "v"(w1), "v"(w2));
#endif
    Pc p;
    __builtin_memcpy(&p, &w0, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p) + 16, &w1, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&p) + 32, &w2, 16);
    return p;
}

// Everything uniform an iteration starts from: the pair's control record, the four pods' PodW
// (a, b, c, d: contiguous), the next pair's lower bounds.  One round of LDS reads.
struct Head {
    Pc p;
    PodW w[4];
    uint64_t lbk_c, lbk_d;
};
__device__ __forceinline__ PodW podw_of(u32x4 v) { return PodW{v.x, (int32_t)v.y, (int32_t)v.z, (int32_t)v.w}; }
__device__ __forceinline__ Head head_regs(const Pc* pcur, const PodW* pw4, const Pc* pnxt) {
    u32x4 w0, w1, w2, q0, q1, q2, q3, l;
#if KS_PR_UNI
    uint64_t sv;
    asm volatile(
        "s_mov_b64 %[sv], exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "ds_read_b128 %[w0], %[ap]\n\t"
        "ds_read_b128 %[w1], %[ap] offset:16\n\t"
        "ds_read_b128 %[w2], %[ap] offset:32\n\t"
        "ds_read_b128 %[q0], %[aw]\n\t"
        "ds_read_b128 %[q1], %[aw] offset:16\n\t"
        "ds_read_b128 %[q2], %[aw] offset:32\n\t"
        "ds_read_b128 %[q3], %[aw] offset:48\n\t"
        "ds_read_b128 %[l], %[al] offset:48\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_mov_b64 exec, %[sv]"
        : [w0] "=&v"(w0), [w1] "=&v"(w1), [w2] "=&v"(w2), [q0] "=&v"(q0), [q1] "=&v"(q1), [q2] "=&v"(q2),
          [q3] "=&v"(q3), [l] "=&v"(l), [sv] "=&s"(sv)
        : [ap] "v"(lds_addr(pcur)), [aw] "v"(lds_addr(pw4)), [al] "v"(lds_addr(pnxt))
        : "memory");
#define PR_RFL(v) v = u32x4{rfl(v.x), rfl(v.y), rfl(v.z), rfl(v.w)}
    PR_RFL(w0); PR_RFL(w1); PR_RFL(w2); PR_RFL(q0); PR_RFL(q1); PR_RFL(q2); PR_RFL(q3); PR_RFL(l);
#undef PR_RFL
#else
    const u32x4* a = reinterpret_cast<const u32x4*>(pcur);
    const u32x4* b = reinterpret_cast<const u32x4*>(pw4);
    w0 = a[0]; w1 = a[1]; w2 = a[2];
    q0 = b[0]; q1 = b[1]; q2 = b[2]; q3 = b[3];
    l = reinterpret_cast<const u32x4*>(pnxt)[3];
    asm volatile("" ::"v"(w0), "v"(w1), "v"(w2), "v"(q0), "v"(q1), "v"(q2), "v"(q3), "v"(l));
#endif
    Head h;
    __builtin_memcpy(&h.p, &w0, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&h.p) + 16, &w1, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&h.p) + 32, &w2, 16);
    h.w[0] = podw_of(q0); h.w[1] = podw_of(q1); h.w[2] = podw_of(q2); h.w[3] = podw_of(q3);
    h.lbk_c = (uint64_t)l.x | (uint64_t)l.y << 32;
    h.lbk_d = (uint64_t)l.z | (uint64_t)l.w << 32;
    return h;
}

// The pair's decision, computed identically by every wave from Pc[k] (uniform values).
struct Dec {
    int32_t wa, ea, wb, eb;      // winners and their entries (-1: none)
    int32_t na, nbw;             // 1: the node joins the table this iteration
    int32_t sa, sb;              // stage slots of untouched winners
    int32_t stop_a;              // 0 go; 1 exhausted list (commit before a); 2 NotFound; 3 InvalidArgument
    int32_t stop_b;              // the same for pod b (after pod a binds); 4: pod b is past the batch
};

// Pod a's winner and pod b's maximum without the extra round, straight-line (selects only: a
// struct filled through references on early-return paths became a scratch-memory alloca on the
// per-pair chain).  Returns pod b's decision word (before the extra round) in *wbw, its
// candidates-excluded part in *rest, and whether the extra fold round is needed.
__device__ __forceinline__ Dec decide(const Pc& p, uint32_t fa, uint32_t fb, bool b_in, int nt,
                                      uint64_t* wbw_out, uint64_t* rest_out, bool* extra_out, int32_t* su_out) {
    // Every wave makes this decision from the same words, and the compiler runs it on the scalar
    // unit: it is the per-pair burst that fills each SIMD's scalar issue after the barrier, so it
    // is written for the fewest scalar instructions — node identity by masked XOR, the K2 word
    // by one shift and mask, b's list candidates pre-packed as decision words by the walker.
    constexpr uint32_t kBad = kFlagBadKey | kFlagBadSpec;
    constexpr uint64_t kNodeBits = 0xFFFFFFull << 25;
    constexpr uint64_t kNodeEntBits = ((1ull << 34) - 1) << 15;
    const uint64_t best = p.best;
    const int32_t stop_a = (p.fl & 1u) ? 1 : (best == 0 ? 2 : ((fa & kBad) ? 3 : 0));
    const int e = dw_ent(best);
    const int32_t na = e == kUnt ? 1 : 0;
    const int32_t ea = na ? nt : e;
    const uint64_t k2 = best & 0x7FFFull;
    const uint64_t k2w = k2 ? (k2 << 49) | (best & kNodeEntBits) : 0ull;
    const bool v1_is_a = p.vb1 != 0 && ((p.vb1 ^ best) & kNodeBits) == 0;
    const uint64_t uw = v1_is_a ? p.vb2 : p.vb1;
    const int32_t su = pc_slot(p, v1_is_a ? 2 : 1);
    const bool exhausted_b = uw == 0 && (p.fl & 2u);
    const uint64_t rest = umax64(umax64(p.m2, k2w), uw);
    const bool mc_a = p.mc != 0 && ((p.mc ^ best) & kNodeBits) == 0;
    const uint64_t wbw = mc_a ? rest : umax64(rest, p.mc);
    // pod b's stop before its word is final (NotFound / bad pod: finish_b, after the extra round)
    const int32_t stop_b = stop_a ? 4 : (!b_in ? 4 : (exhausted_b ? 1 : 0));
    *extra_out = stop_b == 0 && mc_a && p.mc > rest;
    *wbw_out = wbw;
    *rest_out = rest;
    *su_out = su;
    Dec d;
    d.stop_a = stop_a;
    d.stop_b = stop_b;
    d.wa = dw_node(best);
    d.ea = ea;
    d.na = na;
    d.sa = na ? pc_slot(p, 0) : -1;
    d.wb = d.eb = -1;
    d.nbw = 0;
    d.sb = -1;
    return d;
}

// pod b's winner from its decision word (after the extra round when there was one); only
// meaningful while stop_a == 0 (the loop ends otherwise)
__device__ __forceinline__ Dec finish_b(Dec d, uint64_t wbw, uint64_t best, uint32_t fb, int nt, int32_t su) {
    constexpr uint32_t kBad = kFlagBadKey | kFlagBadSpec;
    constexpr uint64_t kNodeBits = 0xFFFFFFull << 25;
    if (d.stop_b == 0) d.stop_b = wbw == 0 ? 2 : ((fb & kBad) ? 3 : 0);
    const int e = dw_ent(wbw);
    const bool same = ((wbw ^ best) & kNodeBits) == 0;
    const bool bnew = !same && e >= nt;  // b's untouched list candidate: its word carries kUnt
    const bool ok = d.stop_b == 0;
    d.wb = ok ? dw_node(wbw) : -1;
    d.eb = ok ? (same ? d.ea : (bnew ? nt + d.na : e)) : -1;
    d.nbw = ok && bnew ? 1 : 0;
    d.sb = ok && bnew ? su : -1;
    return d;
}

// The owners' part of a decision, as the bind wave publishes it (KS_PR_PUB): entries of the two
// winners, the table growth, the stops and the extra-round flag in 29 bits.
#ifndef KS_PR_PUB
#define KS_PR_PUB 1
#endif
#ifndef KS_PR_PRE
#define KS_PR_PRE 0
#endif
// KS_PR_LATE: owners do their decision-independent work (window deltas, prune, evaluations,
// assuming both pods bind) before they wait for the bind wave's decision word, then commit
#ifndef KS_PR_LATE
#define KS_PR_LATE 0
#endif
__device__ __forceinline__ uint32_t dec_pack(const Dec& d, bool extra) {
    return (uint32_t)(d.ea + 1) | (uint32_t)(d.eb + 1) << 10 | (uint32_t)(d.na + d.nbw) << 20 |
           (uint32_t)d.stop_a << 22 | (uint32_t)d.stop_b << 25 | (extra ? 1u << 28 : 0u);
}
__device__ __forceinline__ Dec dec_unpack(uint32_t w) {
    Dec d;
    d.ea = (int32_t)(w & 1023u) - 1;
    d.eb = (int32_t)((w >> 10) & 1023u) - 1;
    d.na = (int32_t)((w >> 20) & 3u);  // na + nbw: only the table growth matters to an owner
    d.nbw = 0;
    d.stop_a = (int32_t)((w >> 22) & 7u);
    d.stop_b = (int32_t)((w >> 25) & 7u);
    d.wa = d.wb = -1;
    d.sa = d.sb = -1;
    return d;
}
// an owner waits for the bind wave's word of iteration k, phase ph (0: pre-extra, 1: final)
__device__ __forceinline__ uint32_t dec_wait(const uint64_t* word, int k, int ph) {
    const uint32_t want = (uint32_t)(2 * k + ph);
    for (;;) {
        const uint64_t w = *reinterpret_cast<const volatile uint64_t*>(word);
        const uint32_t hi = (uint32_t)(w >> 32);
        if (hi == want || (ph == 0 && hi == want + 1)) return (uint32_t)w | (hi & 1u) << 31;
        __builtin_amdgcn_s_sleep(1);
    }
}

// Entry state in registers: 32-bit fields for the narrow evaluators (every capacity < 2^29 and
// every requested total <= capacity; the pods capacity clamped, nr < 2^31 either way), NodeV for
// the wide one.  The LDS table and the staged records stay int64.
struct S32 {
    int32_t ac, am, ag, ap, rc, rm, rg, nr;
    uint64_t taint, label;
};
template <int kMode> struct StSel { using T = S32; };
template <> struct StSel<kEvalWide> { using T = NodeV; };
template <int kMode> struct DlSel { using T = int32_t; };
template <> struct DlSel<kEvalWide> { using T = int64_t; };

__device__ __forceinline__ void conv(const NodeV& v, NodeV& o) { o = v; }
__device__ __forceinline__ void conv(const NodeV& v, S32& o) {
    o.ac = (int32_t)v.ac; o.am = (int32_t)v.am; o.ag = (int32_t)v.ag;
    o.ap = (int32_t)(v.ap < 0x7FFFFFFF ? v.ap : 0x7FFFFFFF);
    o.rc = (int32_t)v.rc; o.rm = (int32_t)v.rm; o.rg = (int32_t)v.rg; o.nr = (int32_t)v.nr;
    o.taint = v.taint; o.label = v.label;
}
template <class T>
__device__ __forceinline__ T st_entry(const Shared& sh, int e) {
    T o;
    conv(t_node(sh, e), o);
    return o;
}
template <class T>
__device__ __forceinline__ T st_stage(const Shared& sh, int par, int s) {
    T o;
    conv(stage_node(sh, par, s), o);
    return o;
}
template <class T>
__device__ __forceinline__ void st_reload(const Shared& sh, int e, T& o) {
    o.rc = (decltype(o.rc))sh.ts[4][e]; o.rm = (decltype(o.rm))sh.ts[5][e];
    o.rg = (decltype(o.rg))sh.ts[6][e]; o.nr = (decltype(o.nr))sh.ts[7][e];
}
template <class T>
__device__ __forceinline__ void st_store(Shared& sh, int e, const T& s) {
    sh.ts[4][e] = s.rc; sh.ts[5][e] = s.rm; sh.ts[6][e] = s.rg; sh.ts[7][e] = s.nr;
}
// CreatePod admission (kubesim/node/node.go:44-47) in 64-bit sums
template <class T>
__device__ __forceinline__ bool fits_t(const PodRec& p, const T& n) {
    bool ok = (int64_t)n.nr < (int64_t)n.ap;
    if (p.keymask & 1) ok &= (int64_t)n.rc + p.req[0] <= (int64_t)n.ac;
    if (p.keymask & 2) ok &= (int64_t)n.rm + p.req[1] <= (int64_t)n.am;
    if (p.keymask & 4) ok &= (int64_t)n.rg + p.req[2] <= (int64_t)n.ag;
    return ok;
}
// add (sgn 1) or remove (sgn -1) a pod's requests: only ever for a pod that passed admission on
// this node, so every sum stays within the node's capacity
template <class T>
__device__ __forceinline__ void add_t(T& n, const PodRec& p, int sgn) {
    using F = decltype(n.rc);
    n.rc += (F)sgn * (F)p.req[0]; n.rm += (F)sgn * (F)p.req[1]; n.rg += (F)sgn * (F)p.req[2]; n.nr += (F)sgn;
}
// summed requests of expiries landing on one node
template <class F>
struct Dl {
    F c, m, g, n;
};
template <class T, class F>
__device__ __forceinline__ void sub_dl(T& s, const Dl<F>& d) {
    s.rc -= d.c; s.rm -= d.m; s.rg -= d.g; s.nr -= d.n;
}
template <class T, class F>
__device__ __forceinline__ void add_dl(T& s, const Dl<F>& d) {
    s.rc += d.c; s.rm += d.m; s.rg += d.g; s.nr += d.n;
}
// the pod's own expiry slot within the batch window, or -1
__device__ __forceinline__ int own_slot(const PodW& w) { return (int)(w.w0 >> 2) - 1; }

// One role's whole loop (kRole 0 walker, 1 bind wave, 2 owners): each role carries only its own
// state around its loop, so the register allocator sees three disjoint loops instead of one
// loop whose every branch keeps every role's loop-carried values live.  All roles execute the
// same barriers (one per pair, one more per extra fold round).
struct LoopOut {
    int nt, committed, err_code, err_pod;
};
template <int kMode, int kRole>
__device__ __forceinline__ LoopOut pair_loop(const EngineArgs& a, Shared& sh, const int tid, const int lane,
                                             const int wave, const int nb, const int n_pre, const bool exact,
                                             const int64_t start, const int oslot) {
    using St = typename StSel<kMode>::T;
    using DF = typename DlSel<kMode>::T;
    const int r = oslot >= 0 ? oslot * kWave + lane : kTMax;
    bool loaded = false, pf_stale = true, full_c = false, full_d = false;
    St st{};
    int32_t st_node = 0;
    PruneF pf{};
    uint64_t xk = 0;
    uint64_t mc_keep = 0;                        // this lane's K1 folded into the next pair's mc

    // walker: walk pods pe, pe+1 (the pair after next) excluding the table and the nodes x0, x1;
    // keep 3 (pod pe) and 4 (pod pe+1) untouched entries, publish their lower bounds, issue the
    // records' loads (they land while the next iteration runs)
    auto walk = [&](int pe, int slot_pc, int32_t x0, int32_t x1) {
        const int pf1 = pe + 1;
        uint64_t x = 0;
        if (lane < kL && pe < nb) x = sh.cand[pe][lane];
        else if (lane >= kL && lane < 2 * kL && pf1 < nb) x = sh.cand[pf1][lane - kL];
        const int32_t xn = key_node(x);
        const bool unt = x != 0 && xn != x0 && xn != x1 && !is_touched(sh, xn, exact);
        const uint64_t bx = __ballot(x != 0), bu = __ballot(unt);
        full_c = __popcll(bx & 0xFFull) == kL;
        full_d = __popcll((bx >> kL) & 0xFFull) == kL;
        const uint64_t me = bu & 0xFFull, mf = (bu >> kL) & 0xFFull;
        uint64_t m = lane < 3 ? me : mf;
        const int skip = lane < 3 ? lane : lane - 3;
        for (int s = 0; s < 3; ++s)
            if (s < skip) m &= m - 1;
        const int src = (lane < kKeep && m) ? (__ffsll((unsigned long long)m) - 1 + (lane < 3 ? 0 : kL)) : -1;
        const uint64_t v = shfl64(x, src < 0 ? 0 : src);
        xk = src < 0 ? 0ull : v;
        const int ce = __popcll(me), cf = __popcll(mf);
        const uint64_t lbe = ce >= 3 ? rl64(xk, 2) : (full_c && ce ? rl64(xk, ce - 1) : 0ull);
        const uint64_t lbf = cf >= 4 ? rl64(xk, 6) : (full_d && cf ? rl64(xk, 3 + cf - 1) : 0ull);
        if (lane == 0) {
            sh.pc[slot_pc].lbk_a = lbe;
            sh.pc[slot_pc].lbk_b = lbf;
        }
        if (xk != 0) {
            const int32_t nd = key_node(xk);
            NodeV v;
            v.ac = node_field(a.s, 0, nd); v.am = node_field(a.s, 1, nd); v.ag = node_field(a.s, 2, nd);
            v.ap = node_field(a.s, 3, nd); v.rc = node_field(a.s, 4, nd); v.rm = node_field(a.s, 5, nd);
            v.rg = node_field(a.s, 6, nd); v.nr = node_field(a.s, 7, nd);
            v.taint = (uint64_t)node_field(a.s, 8, nd); v.label = (uint64_t)node_field(a.s, 9, nd);
            conv(v, st);
        }
    };

    // pre-prologue: pair 0's lists (no winner known yet)
    if constexpr (kRole == 0) walk(0, 0, -1, -1);
    __syncthreads();

    int nt = n_pre;
    int committed = nb, err_code = 0, err_pod = -1;
#ifdef KS_STAMPS
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // work, wait, decision, role segments 1-4, extra rounds
#endif
    int s_cur = 2, s_nxt = 0, s_nn = 1;  // control-record ring slots of pairs k, k+1, k+2 (k = -1 first)
    for (int k = -1;; ++k) {
        PR_STAMP(s0);
        const int pa = 2 * k, pb = pa + 1, pcn = pa + 2, pd = pa + 3;
        Dec dc;
        dc.wa = dc.ea = dc.wb = dc.eb = -1;
        dc.na = dc.nbw = 0;
        dc.sa = dc.sb = -1;
        dc.stop_a = 0;
        dc.stop_b = 4;
        const Head hd = head_regs(&sh.pc[s_cur], &sh.pwx[pa + 2], &sh.pc[s_nxt]);
        // bind wave (KS_PR_PRE): what its bind reads that does not depend on the decision, loaded before it
        // (the loads' latency hides under the decision's scalar work): the expiry slots of
        // windows b..d (first 64) and the staged record of pod a's (even lanes) / pod b's first
        // (odd lanes) list candidate
        int32_t pq = -1, pte = -1, pok = 0, pslot = -1;
        DF pr0 = 0, pr1 = 0, pr2 = 0;
        St spre{};
        if constexpr (kRole == 1 && KS_PR_PRE) {
            if (k >= 0) {
                const int x = hd.w[1].lo + lane;
                if (x < hd.w[3].hi) {
                    pq = sh.ex_q[x]; pte = sh.ex_entry[x]; pok = sh.ex_ok[x];
                    pr0 = (DF)sh.ex_req[x][0]; pr1 = (DF)sh.ex_req[x][1]; pr2 = (DF)sh.ex_req[x][2];
                }
                pslot = pc_slot(hd.p, lane & 1);
                if (lane < 6 && pslot >= 0) spre = st_stage<St>(sh, k & 1, pslot);
            }
        }
        if (k >= 0 && (!KS_PR_PUB || kRole <= 1)) {
            // the walker and the bind wave decide for themselves; the bind wave publishes the
            // owners' part (KS_PR_PUB) so that the other waves do not repeat the decision — it
            // runs on the scalar unit, and 10-16 waves repeating it filled each SIMD's scalar
            // issue for ~1,200 cycles after every barrier
            const Pc& p = hd.p;
            const uint32_t fa = hd.w[0].w0, fb = hd.w[1].w0;
            uint64_t wbw, rest;
            bool extra;
            int32_t su;
            dc = decide(p, fa, fb, pb < nb, nt, &wbw, &rest, &extra, &su);
            if (extra) {
                // the candidates of pod a other than w_a refold their K1_b (kept from the last
                // iteration) into mcx; one more barrier
                if (KS_PR_PUB && kRole == 1 && lane == 0)
                    *reinterpret_cast<volatile uint64_t*>(&sh.dec_word) = (uint64_t)(2 * k) << 32 | dec_pack(dc, true);
                if (mc_keep != 0 && dw_ent(mc_keep) != dc.ea) fold(&sh.pc[s_cur].mcx, mc_keep);
                PR_ACC(7, 1);
                __syncthreads();
                wbw = umax64(rest, sh.pc[s_cur].mcx);
            }
            dc = finish_b(dc, wbw, p.best, fb, nt, su);
            if (KS_PR_PUB && kRole == 1 && lane == 0)
                *reinterpret_cast<volatile uint64_t*>(&sh.dec_word) = (uint64_t)(2 * k + 1) << 32 | dec_pack(dc, false);
        } else if (k >= 0 && !(kRole == 2 && KS_PR_LATE)) {
            uint32_t w = dec_wait(&sh.dec_word, k, 0);
            if (!(w >> 31)) {  // the extra fold round (phase 0 word): refold, barrier, final word
                const Dec d0 = dec_unpack(w);
                if (mc_keep != 0 && dw_ent(mc_keep) != d0.ea) fold(&sh.pc[s_cur].mcx, mc_keep);
                __syncthreads();
                w = dec_wait(&sh.dec_word, k, 1);
            }
            dc = dec_unpack(w);
        }
        if (k >= 0 && dc.stop_a) {
            committed = pa;
            if (dc.stop_a > 1) { err_code = dc.stop_a == 2 ? kErrNotFound : kErrEinval; err_pod = (int32_t)(start + pa); }
            break;
        }
        PR_STAMP(sd);
        PR_ACC(2, sd - s0);
        bool have_b = k >= 0 && dc.stop_b == 0;
        bool prep = pcn < nb && (k < 0 || have_b);  // the next pair will be decided
        // window ranges: b = [lo_b, hi_b), c = [hi_b, hi_c), d = [lo_d, hi_d) — adjacent; for the
        // prologue (k = -1) only window d (pod 1's) exists
        const PodW wpc = hd.w[2], wpd = hd.w[3];
        const PodW wpb = k >= 0 ? hd.w[1] : hd.w[3];
        const int lo_b = k >= 0 ? wpb.lo : wpd.lo, hi_b = k >= 0 ? wpb.hi : wpd.lo;
        const int hi_c = k >= 0 ? (have_b ? wpc.hi : hi_b) : wpd.lo;
        const int lo_d = k >= 0 ? wpc.hi : wpd.lo;
        const int hi_d = prep && pd < nb ? wpd.hi : (have_b ? hi_c : hi_b);
        const uint64_t lbk_c = hd.lbk_c, lbk_d = hd.lbk_d;

        if constexpr (kRole == 0) {
            // ================= walker =================
            // K2 of pod c's kept candidates (lanes 0..2): admission of c, bind, c's own expiry
            // when it is due before d, then d's key
            uint32_t k2 = 0;
            if (prep && pd < nb) {
                const PodRec p_c = pod_regs(&sh.pod[pcn]);
                St s2 = st;
                const bool okc = fits_t(p_c, s2);
                const int oc = own_slot(wpc);
                if (okc && wpc.dur > 0) add_t(s2, p_c, 1);
                if (okc && oc >= lo_d && oc < hi_d) add_t(s2, p_c, -1);
                const PodRec p_d = pod_regs(&sh.pod[pd]);
                k2 = eval_t<kMode>(a.c, p_d, s2);
                if (!(lane < 3 && xk != 0)) k2 = 0;
            }
            PR_STAMP(w1);
            PR_ACC(3, w1 - sd);
            // stage the pair's kept records for the bind (next iteration)
            if (prep && lane < kKeep && xk != 0) {
                int64_t* d = sh.stage[(k + 1) & 1][lane];
                d[0] = st.ac; d[1] = st.am; d[2] = st.ag; d[3] = st.ap; d[4] = st.rc;
                d[5] = st.rm; d[6] = st.rg; d[7] = st.nr; d[8] = (int64_t)st.taint; d[9] = (int64_t)st.label;
            }
            const int32_t xa = dc.wa, xb = have_b ? dc.wb : -1;
            if (prep) {
                const int32_t kn = key_node(xk);
                const bool okc = lane < 3 && xk != 0 && kn != xa && kn != xb;
                const bool okd = lane >= 3 && lane < kKeep && xk != 0 && kn != xa && kn != xb;
                const uint64_t mcb = __ballot(okc), mdb = __ballot(okd);
                const int lc = mcb ? __ffsll((unsigned long long)mcb) - 1 : -1;
                const uint64_t uc = lc >= 0 ? rl64(xk, lc) : 0ull;
                const uint32_t k2u = lc >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)k2, lc) : 0u;
                const int l1 = mdb ? __ffsll((unsigned long long)mdb) - 1 : -1;
                const uint64_t mdb2 = mdb & (mdb - 1);
                const int l2 = mdb2 ? __ffsll((unsigned long long)mdb2) - 1 : -1;
                const uint64_t v1 = l1 >= 0 ? rl64(xk, l1) : 0ull, v2 = l2 >= 0 ? rl64(xk, l2) : 0ull;
                if (lane == 0) {
                    Pc& q = sh.pc[s_nxt];
                    if (uc) fold(&q.best, dword_key(uc, kUnt, k2u));
                    q.fl = ((uc == 0 && full_c && pcn > 0) ? 1u : 0u) | (full_d ? 2u : 0u) | (uint32_t)(lc + 1) << 4 |
                           (uint32_t)(l1 + 1) << 8 | (uint32_t)(l2 + 1) << 12;
                    q.vb1 = dword_key(v1, kUnt, 0);  // decision words; entry kUnt = untouched
                    q.vb2 = dword_key(v2, kUnt, 0);
                }
            }
            // zero the folds of the pair after next (its slot was last read in iteration k-1)
            if (lane == 0) {
                Pc& q = sh.pc[s_nn];
                q.best = 0; q.m2 = 0; q.mc = 0; q.mcx = 0;
            }
            PR_STAMP(w2);
            PR_ACC(4, w2 - w1);
            if (prep && pcn + 2 < nb) walk(pcn + 2, s_nn, xa, xb);
            else xk = 0;
            PR_STAMP(w3);
            PR_ACC(5, w3 - w2);
        } else if constexpr (kRole == 1) {
            // ================= bind wave =================
            if (k >= 0) {
                const bool same = have_b && dc.wb == dc.wa;
                const int sel = lane & 1, var = lane >> 1;
                const bool act = lane < 6 && (sel == 0 || have_b);
                const bool on_b = sel && have_b;  // this lane's node is w_b
                const int32_t n = on_b ? dc.wb : dc.wa;
                const int32_t ent = on_b ? dc.eb : dc.ea;
                const bool isnew = on_b && !same ? dc.nbw : dc.na;
                const int slot = on_b && !same ? dc.sb : dc.sa;
                const int64_t ja = start + pa, jb = start + pb;
                const PodW wpa = hd.w[0];
                // expiries of earlier-bound pods in windows b..d landing on this lane's node
                // (own expiries of pods a, b: below), summed per window; applied ones marked
                Dl<DF> d0{}, d1{}, d2{};
                for (int x0 = lo_b; x0 < hi_d; x0 += kWave) {
                    const int x = x0 + lane;
                    bool hit = false;
                    int32_t te = -1;
                    DF q0 = 0, q1 = 0, q2 = 0;
                    if (x < hi_d) {
                        int32_t q, ok;
                        if (KS_PR_PRE && x0 == lo_b) {
                            q = pq; te = pte; ok = pok; q0 = pr0; q1 = pr1; q2 = pr2;
                        } else {
                            q = sh.ex_q[x]; te = sh.ex_entry[x]; ok = sh.ex_ok[x];
                            q0 = (DF)sh.ex_req[x][0]; q1 = (DF)sh.ex_req[x][1]; q2 = (DF)sh.ex_req[x][2];
                        }
                        hit = ok != 0 && q != ja && q != jb && (te == dc.ea || (have_b && te == dc.eb));
                        if (hit && x < hi_c) gptr(a.expired)[q] = 1;
                    }
                    uint64_t m = __ballot(hit);
                    while (m) {
                        const int l = __ffsll((unsigned long long)m) - 1;
                        m &= m - 1;
                        const int xl = x0 + l;
                        const int el = __builtin_amdgcn_readlane(te, l);
                        const DF c0 = (DF)rl64((uint64_t)(int64_t)q0, l), c1 = (DF)rl64((uint64_t)(int64_t)q1, l),
                                 c2 = (DF)rl64((uint64_t)(int64_t)q2, l);
                        if (el == ent) {
                            Dl<DF>& dd = xl < hi_b ? d0 : (xl < hi_c ? d1 : d2);
                            dd.c += c0; dd.m += c1; dd.g += c2; dd.n += 1;
                        }
                    }
                }
                PR_STAMP(b1);
                PR_ACC(3, b1 - sd);
                const int own_a = own_slot(wpa), own_b = own_slot(wpb);
                St s = isnew ? ((KS_PR_PRE && slot == pslot) ? spre : st_stage<St>(sh, k & 1, slot < 0 ? 0 : slot))
                             : st_entry<St>(sh, ent < 0 ? 0 : ent);
                bool ok_a = false, ok_b = false;
                {
                    const PodRec p_a = pod_regs(&sh.pod[pa]);
                    if (n == dc.wa) {
                        ok_a = fits_t(p_a, s);
                        if (ok_a && wpa.dur > 0) add_t(s, p_a, 1);
                        sub_dl(s, d0);
                        if (ok_a && own_a >= lo_b && own_a < hi_b) add_t(s, p_a, -1);
                    }
                    if (have_b && n == dc.wb) {
                        const PodRec p_b = pod_regs(&sh.pod[pb]);
                        if (!same) sub_dl(s, d0);
                        ok_b = fits_t(p_b, s);
                        if (ok_b && wpb.dur > 0) add_t(s, p_b, 1);
                        sub_dl(s, d1);
                        if (same && ok_a && own_a >= hi_b && own_a < hi_c) add_t(s, p_a, -1);
                        if (ok_b && own_b >= hi_b && own_b < hi_c) add_t(s, p_b, -1);
                    } else if (have_b && n == dc.wa) {
                        sub_dl(s, d1);
                        if (ok_a && own_a >= hi_b && own_a < hi_c) add_t(s, p_a, -1);
                    }
                }
                PR_STAMP(b2);
                PR_ACC(4, b2 - b1);
                // s: the node's state before pod c.  One evaluator pass over the six lanes:
                // var 0 key_c, var 1 K1_d (window d applied), var 2 K2_d (c bound, window d)
                uint32_t t = 0;
                if (prep) {
                    St se = s;
                    if (var >= 1) {
                        sub_dl(se, d2);
                        if (n == dc.wa && ok_a && own_a >= lo_d && own_a < hi_d) add_t(se, sh.pod[pa], -1);
                        if (have_b && n == dc.wb && ok_b && own_b >= lo_d && own_b < hi_d) add_t(se, sh.pod[pb], -1);
                    }
                    if (var == 2) {
                        const PodRec p_c = pod_regs(&sh.pod[pcn]);
                        const int oc = own_slot(wpc);
                        const bool okc = fits_t(p_c, s);
                        if (okc && wpc.dur > 0) add_t(se, p_c, 1);
                        if (okc && oc >= lo_d && oc < hi_d) add_t(se, p_c, -1);
                    }
                    const PodRec pe = pod_regs(&sh.pod[var == 0 ? pcn : pd]);
                    t = eval_t<kMode>(a.c, pe, se);
                    if (var >= 1 && pd >= nb) t = 0;
                }
                const uint32_t t_k1a = (uint32_t)__builtin_amdgcn_readlane((int)t, 2);
                const uint32_t t_k1b = (uint32_t)__builtin_amdgcn_readlane((int)t, 3);
                const uint32_t t_k2a = (uint32_t)__builtin_amdgcn_readlane((int)t, 4);
                const uint32_t t_k2b = (uint32_t)__builtin_amdgcn_readlane((int)t, 5);
                mc_keep = 0;
                const bool writer = act && lane < 2 && !(same && sel);
                if (prep && writer) {
                    const uint64_t kc = make_key(t, (uint32_t)n);
                    const uint64_t k1 = make_key(sel ? t_k1b : t_k1a, (uint32_t)n);
                    const bool cand = kc != 0 && kc >= lbk_c;
                    if (cand) fold(&sh.pc[s_nxt].best, dword_key(kc, (uint32_t)ent, sel ? t_k2b : t_k2a));
                    if (k1 != 0 && k1 >= lbk_d) {
                        const uint64_t w1 = dword_key(k1, (uint32_t)ent, 0);
                        if (cand) { fold(&sh.pc[s_nxt].mc, w1); mc_keep = w1; }
                        else fold(&sh.pc[s_nxt].m2, w1);
                    }
                }
                PR_STAMP(b3);
                PR_ACC(5, b3 - b2);
                // state, table and outputs (lane 0: w_a; lane 1: w_b when distinct)
                if (writer) {
                    if (isnew) {
                        sh.ts[0][ent] = s.ac; sh.ts[1][ent] = s.am; sh.ts[2][ent] = s.ag; sh.ts[3][ent] = s.ap;
                        sh.tu[0][ent] = s.taint; sh.tu[1][ent] = s.label;
                        sh.tnode[ent] = n;
                        t_insert(sh, n, ent, exact);
                    }
                    st_store(sh, ent, s);
                    sh.dirty[ent] = k + 1;
                }
                if (lane == 0) {
                    gptr(a.b_node)[ja] = dc.wa;
                    gptr(a.b_status)[ja] = ok_a ? 0 : 1;
                    if (own_a >= 0) { sh.ex_entry[own_a] = dc.ea; sh.ex_ok[own_a] = ok_a ? 1 : 0; }
                    if (ok_a && own_a >= lo_b && own_a < hi_c) gptr(a.expired)[ja] = 1;
                }
                if (lane == 1 && have_b) {
                    gptr(a.b_node)[jb] = dc.wb;
                    gptr(a.b_status)[jb] = ok_b ? 0 : 1;
                    if (own_b >= 0) { sh.ex_entry[own_b] = dc.eb; sh.ex_ok[own_b] = ok_b ? 1 : 0; }
                    if (ok_b && own_b >= hi_b && own_b < hi_c) gptr(a.expired)[jb] = 1;
                }
            }
        } else {
            // ================= owners =================
#if KS_PR_LATE
            // ---- speculative part (pods a and b both bind; otherwise the loop ends at this
            // iteration and nothing of it is kept but what the commit below writes)
            const int base = oslot * kWave;
            if (r < nt) {
                if (!loaded) {
                    st = st_entry<St>(sh, r);
                    st_node = sh.tnode[r];
                    loaded = true;
                    pf_stale = true;
                } else if (sh.dirty[r] == k) {
                    st_reload(sh, r, st);
                    pf_stale = true;
                }
            }
            const bool s_prep = pcn < nb;
            const int s_hi_b = k >= 0 ? wpb.hi : wpd.lo;
            const int s_hi_c = k >= 0 ? wpc.hi : wpd.lo;
            const int s_hi_d = s_prep && pd < nb ? wpd.hi : s_hi_c;
            Dl<DF> dwb{}, dwc{}, dd{};
            bool has_b = false, has_c = false, has_dd = false, any_hit = false;
            for (int x0 = lo_b; x0 < s_hi_d; x0 += kWave) {
                const int x = x0 + lane;
                int32_t te = -1;
                bool hit = false;
                if (x < s_hi_d) {
                    te = sh.ex_entry[x];
                    hit = sh.ex_ok[x] != 0 && te >= base && te < base + kWave;
                }
                uint64_t m = __ballot(hit);
                any_hit |= m != 0;
                while (m) {
                    const int l = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    const int xl = x0 + l;
                    const int el = __builtin_amdgcn_readlane(te, l);
                    if (r == el) {
                        const DF q0 = (DF)sh.ex_req[xl][0], q1 = (DF)sh.ex_req[xl][1], q2 = (DF)sh.ex_req[xl][2];
                        const int wsel = xl < s_hi_b ? 0 : (xl < s_hi_c ? 1 : 2);
                        dwb.c += wsel == 0 ? q0 : 0; dwb.m += wsel == 0 ? q1 : 0; dwb.g += wsel == 0 ? q2 : 0; dwb.n += wsel == 0;
                        dwc.c += wsel == 1 ? q0 : 0; dwc.m += wsel == 1 ? q1 : 0; dwc.g += wsel == 1 ? q2 : 0; dwc.n += wsel == 1;
                        dd.c += wsel == 2 ? q0 : 0; dd.m += wsel == 2 ? q1 : 0; dd.g += wsel == 2 ? q2 : 0; dd.n += wsel == 2;
                        has_b |= wsel == 0; has_c |= wsel == 1; has_dd |= wsel == 2;
                    }
                }
            }
            St sbc = st;  // the entry's state before pod c (windows b and c applied)
            sub_dl(sbc, dwb);
            sub_dl(sbc, dwc);
            PR_STAMP(o1);
            PR_ACC(3, o1 - sd);
            bool pass_c = false, pass_d = false;
            if (s_prep && r < nt) {
                if (pf_stale || has_b || has_c) { pf = prune_prep_t<kMode>(a.c, sbc); pf_stale = has_b || has_c; }
                const float qc0 = sh.podf[pcn][0], qc1 = sh.podf[pcn][1];
                pass_c = pf.live && make_key(prune_tmax(a.c, pf, qc0, qc1) + 1u, (uint32_t)st_node) >= lbk_c;
                if (pd < nb) {
                    const float qd0 = sh.podf[pd][0], qd1 = sh.podf[pd][1];
                    pass_d = has_dd ||
                             (pf.live && make_key(prune_tmax(a.c, pf, qd0, qd1) + 1u, (uint32_t)st_node) >= lbk_d);
                }
            }
            PR_STAMP(o2);
            PR_ACC(4, o2 - o1);
            uint64_t kc = 0, k1 = 0;
            uint32_t t2 = 0;
            if (__ballot(pass_c || pass_d)) {
                St s1 = sbc;
                sub_dl(s1, dd);
                const PodRec p_c = pod_regs(&sh.pod[pcn]);
                const PodRec p_d = pod_regs(&sh.pod[pd]);
                const uint32_t tc = eval_t<kMode>(a.c, p_c, sbc);
                const uint32_t t1 = eval_t<kMode>(a.c, p_d, s1);
                kc = pass_c ? make_key(tc, (uint32_t)st_node) : 0ull;
                k1 = pass_d ? make_key(t1, (uint32_t)st_node) : 0ull;
                if (__ballot(kc != 0 && kc >= lbk_c) && pd < nb) {
                    St s2 = s1;
                    const int oc = own_slot(wpc);
                    const bool okc = fits_t(p_c, sbc);
                    if (okc && wpc.dur > 0) add_t(s2, p_c, 1);
                    if (okc && oc >= s_hi_c && oc < s_hi_d) add_t(s2, p_c, -1);
                    t2 = eval_t<kMode>(a.c, p_d, s2);
                }
            }
            PR_STAMP(o3);
            PR_ACC(5, o3 - o2);
            // ---- the decision (the bind wave's word), then the commit
            if (k >= 0) {
                uint32_t w = dec_wait(&sh.dec_word, k, 0);
                if (!(w >> 31)) {
                    const Dec d0 = dec_unpack(w);
                    if (mc_keep != 0 && dw_ent(mc_keep) != d0.ea) fold(&sh.pc[s_cur].mcx, mc_keep);
                    __syncthreads();
                    w = dec_wait(&sh.dec_word, k, 1);
                }
                dc = dec_unpack(w);
                if (dc.stop_a) break;  // the walker holds committed / err for the launch
                have_b = dc.stop_b == 0;
                prep = pcn < nb && have_b;
            }
            const bool valid = r < nt && r != dc.ea && r != dc.eb;
            // applied windows: b when pod a binds, c when pod b binds too
            if (valid && (has_b || (have_b && has_c))) {
                st = sbc;
                if (!have_b) add_dl(st, dwc);
                st_store(sh, r, st);
                pf_stale = true;
            }
            if (any_hit) {  // mark the applied expiries (windows b, c) of this wave's valid entries
                const int hc = have_b ? s_hi_c : s_hi_b;
                for (int x0 = lo_b; x0 < hc; x0 += kWave) {
                    const int x = x0 + lane;
                    if (x < hc && sh.ex_ok[x] != 0) {
                        const int32_t te = sh.ex_entry[x];
                        if (te >= base && te < base + kWave && te < nt && te != dc.ea && te != dc.eb)
                            gptr(a.expired)[sh.ex_q[x]] = 1;
                    }
                }
            }
            mc_keep = 0;
            if (prep && valid) {
                const bool cand = kc != 0 && kc >= lbk_c;
                if (cand) fold(&sh.pc[s_nxt].best, dword_key(kc, (uint32_t)r, t2));
                if (k1 != 0 && k1 >= lbk_d) {
                    const uint64_t w1 = dword_key(k1, (uint32_t)r, 0);
                    if (cand) { fold(&sh.pc[s_nxt].mc, w1); mc_keep = w1; }
                    else fold(&sh.pc[s_nxt].m2, w1);
                }
            }
#else
            const int base = oslot * kWave;
            const bool valid = r < nt && r != dc.ea && r != dc.eb;
            if (r < nt) {
                if (!loaded) {
                    st = st_entry<St>(sh, r);
                    st_node = sh.tnode[r];
                    loaded = true;
                    pf_stale = true;
                } else if (sh.dirty[r] == k) {
                    st_reload(sh, r, st);
                    pf_stale = true;
                }
            }
            // windows b, c (applied) and d (speculative) landing on this wave's entries
            Dl<DF> dd{};
            bool has_dd = false, changed = false;
            for (int x0 = lo_b; x0 < hi_d; x0 += kWave) {
                const int x = x0 + lane;
                int32_t te = -1;
                bool hit = false;
                if (x < hi_d) {
                    te = sh.ex_entry[x];
                    hit = sh.ex_ok[x] != 0 && te >= base && te < base + kWave && te != dc.ea && te != dc.eb;
                }
                uint64_t m = __ballot(hit);
                while (m) {
                    const int l = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    const int xl = x0 + l;
                    const int el = __builtin_amdgcn_readlane(te, l);
                    if (r == el) {
                        const DF q0 = (DF)sh.ex_req[xl][0], q1 = (DF)sh.ex_req[xl][1], q2 = (DF)sh.ex_req[xl][2];
                        if (xl < hi_c) {
                            st.rc -= q0; st.rm -= q1; st.rg -= q2; st.nr -= 1;
                            gptr(a.expired)[sh.ex_q[xl]] = 1;
                            changed = true;
                        } else {
                            dd.c += q0; dd.m += q1; dd.g += q2; dd.n += 1;
                            has_dd = true;
                        }
                    }
                }
            }
            if (changed) {
                st_store(sh, r, st);
                pf_stale = true;
            }
            PR_STAMP(o1);
            PR_ACC(3, o1 - sd);
            mc_keep = 0;
            bool pass_c = false, pass_d = false;
            if (prep && valid) {
                if (pf_stale) { pf = prune_prep_t<kMode>(a.c, st); pf_stale = false; }
                const float qc0 = sh.podf[pcn][0], qc1 = sh.podf[pcn][1];
                pass_c = pf.live && make_key(prune_tmax(a.c, pf, qc0, qc1) + 1u, (uint32_t)st_node) >= lbk_c;
                if (pd < nb) {
                    const float qd0 = sh.podf[pd][0], qd1 = sh.podf[pd][1];
                    pass_d = has_dd ||
                             (pf.live && make_key(prune_tmax(a.c, pf, qd0, qd1) + 1u, (uint32_t)st_node) >= lbk_d);
                }
            }
            PR_STAMP(o2);
            PR_ACC(4, o2 - o1);
            if (__ballot(pass_c || pass_d)) {
                // key_c on the entry's state, K1_d with window d applied
                St s1 = st;
                sub_dl(s1, dd);
                const PodRec p_c = pod_regs(&sh.pod[pcn]);
                const PodRec p_d = pod_regs(&sh.pod[pd]);
                const uint32_t tc = eval_t<kMode>(a.c, p_c, st);
                const uint32_t t1 = eval_t<kMode>(a.c, p_d, s1);
                const uint64_t kc = pass_c ? make_key(tc, (uint32_t)st_node) : 0ull;
                const uint64_t k1 = pass_d ? make_key(t1, (uint32_t)st_node) : 0ull;
                const bool cand = kc != 0 && kc >= lbk_c;
                uint32_t t2 = 0;
                if (__ballot(cand) && pd < nb) {
                    // K2_d: pod c bound on this entry (its own expiry when due before d)
                    St s2 = s1;
                    const int oc = own_slot(wpc);
                    const bool okc = fits_t(p_c, st);
                    if (okc && wpc.dur > 0) add_t(s2, p_c, 1);
                    if (okc && oc >= lo_d && oc < hi_d) add_t(s2, p_c, -1);
                    t2 = eval_t<kMode>(a.c, p_d, s2);
                }
                if (cand) fold(&sh.pc[s_nxt].best, dword_key(kc, (uint32_t)r, t2));
                if (k1 != 0 && k1 >= lbk_d) {
                    const uint64_t w1 = dword_key(k1, (uint32_t)r, 0);
                    if (cand) { fold(&sh.pc[s_nxt].mc, w1); mc_keep = w1; }
                    else fold(&sh.pc[s_nxt].m2, w1);
                }
            }
            PR_STAMP(o3);
            PR_ACC(5, o3 - o2);
#endif
        }
        PR_STAMP(s1);
        __syncthreads();
        PR_STAMP(s2);
        PR_ACC(0, s1 - s0);
        PR_ACC(1, s2 - s1);
        nt += dc.na + dc.nbw;
        if (k >= 0) {
            if (!have_b) {
                committed = pa + 1;
                if (dc.stop_b == 2 || dc.stop_b == 3) {
                    err_code = dc.stop_b == 2 ? kErrNotFound : kErrEinval;
                    err_pod = (int32_t)(start + pb);
                }
                break;
            }
            if (pb + 1 >= nb) { committed = nb; break; }
        }
        const int s_old = s_cur;
        s_cur = s_nxt;
        s_nxt = s_nn;
        s_nn = s_old;
    }
#ifdef KS_STAMPS
    {   // ctr[8 + 6 * role + i] for role 0 walker, 1 bind wave (i: 0 work, 1 barrier wait, 2
        // decision, 3-5 role segments); ctr[20 + w - 2]: work of owner wave w (2..13); ctr[5]
        // launches, ctr[6] pods, ctr[7] extra fold rounds
        unsigned long long* d = (unsigned long long*)a.ctr;
        if (lane == 0 && kRole <= 1)
            for (int q = 0; q < 6; ++q) atomicAdd(&d[8 + 6 * kRole + q], acc[q]);
        if (lane == 0 && kRole == 2 && wave <= 13) atomicAdd(&d[20 + wave - 2], acc[0]);
        if (tid == 0) {
            atomicAdd(&d[5], 1ull);
            atomicAdd(&d[6], (unsigned long long)committed);
            atomicAdd(&d[7], acc[7]);
        }
    }
#endif
    return LoopOut{nt, committed, err_code, err_pod};
}

// ---------------------------------------------------------------------------------------------
template <int kMode>
__global__ __launch_bounds__(kThreads) void resolve_pair_kernel(const EngineArgs* __restrict__ A) {
    __shared__ Shared sh;
    const EngineArgs& a = A[blockIdx.x];  // fields read where used (scalar loads): fewer live SGPRs
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    if (a.ctr[kCtrErr] != 0) return;
    const bool exact = a.c.n_nodes <= kFilterBits;
    int nb = (int)min<int64_t>(min<int64_t>(a.B, kMaxB), end - start);
    if (nb <= 0) return;

    // ---- setup (as resolve_kernel): the largest batch whose expiry window fits the pre-insert
    // budget, pods / lists / window slots into LDS, pre-insert the nodes the window's expiries
    // land on, their records
    const int64_t e_base = a.exp_off[start + 1];
    const int64_t off_mid = tid < nb ? a.exp_off[start + tid + 1] : 0;
    const bool fits_win = tid < nb && off_mid - e_base <= kMaxExp;
    if (tid == 0) { sh.n_t = 0; sh.dec_word = ~0ull; }
    if (tid < 3) {
        uint4* w = reinterpret_cast<uint4*>(&sh.pc[tid]);
        for (int q = 0; q < (int)(sizeof(Pc) / 16); ++q) w[q] = make_uint4(0, 0, 0, 0);
    }
    for (int h = tid; h < kHash; h += kThreads) sh.hkey[h] = -1;
    for (int w = tid; w < kFilterBits / 32; w += kThreads) sh.tfilt[w] = 0;
    nb = __syncthreads_count(fits_win);
    if (tid == nb - 1) { sh.nb = nb; sh.e_cnt = nb > 1 ? (int32_t)(off_mid - e_base) : 0; }
    __syncthreads();
    const int e_cnt = sh.e_cnt;
    for (int i = tid; i < kMaxB + kPodPad; i += kThreads) {
        PodRec p{};
        PodW w{0, 0, e_cnt, e_cnt};
        if (i < nb) {
            p = a.pods[start + i];
            const int64_t pos = a.exp_pos[start + i];
            const int32_t own = (pos >= e_base && pos - e_base < e_cnt) ? (int32_t)(pos - e_base) : -1;
            w.w0 = p.flags | (uint32_t)(own + 1) << 2;
            w.dur = a.dur[start + i];
            w.lo = i >= 1 ? (int32_t)(a.exp_off[start + i] - e_base) : 0;
            w.hi = i >= 1 ? (int32_t)(a.exp_off[start + i + 1] - e_base) : 0;
        }
        sh.pod[i] = p;
        sh.podf[i][0] = (float)p.req[0];
        sh.podf[i][1] = (float)p.req[1];
        sh.pwx[i + 2] = w;
    }
    if (tid < 2) sh.pwx[tid] = PodW{0, 0, 0, 0};
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
    const bool pre_want = tid < e_cnt && sh.ex_ok[tid];
    int pre_slot = -1;
    bool pre_claim = false;
    if (pre_want) {
        const int32_t nd = sh.ex_node[tid];
        uint32_t hs = hslot(nd);
        for (;;) {  // the table holds <= kMaxExp < kHash nodes: terminates
            const int32_t prev = atomicCAS(&sh.hkey[hs], -1, nd);
            if (prev == -1 || prev == nd) { pre_slot = (int)hs; pre_claim = prev == -1; break; }
            hs = (hs + 1) & (kHash - 1);
        }
    }
    __syncthreads();
    if (pre_claim) {
        const int32_t nd = sh.ex_node[tid];
        const int idx = atomicAdd(&sh.n_t, 1);
        sh.hval[pre_slot] = idx;
        sh.tnode[idx] = nd;
        const uint32_t f = (uint32_t)nd & (kFilterBits - 1);
        atomicOr(&sh.tfilt[f >> 5], 1u << (f & 31));
    }
    __syncthreads();
    if (pre_want) sh.ex_entry[tid] = sh.hval[pre_slot];
    const int n_pre = sh.n_t;
    for (int e = tid; e < kTMax; e += kThreads) sh.dirty[e] = -1;
    for (int e = tid; e < n_pre; e += kThreads) {
        const NodeV v = load_node(a.s, sh.tnode[e]);
        sh.ts[0][e] = v.ac; sh.ts[1][e] = v.am; sh.ts[2][e] = v.ag; sh.ts[3][e] = v.ap;
        sh.ts[4][e] = v.rc; sh.ts[5][e] = v.rm; sh.ts[6][e] = v.rg; sh.ts[7][e] = v.nr;
        sh.tu[0][e] = v.taint; sh.tu[1][e] = v.label;
    }

    // ---- per-thread state, shared by the roles (a wave has one role for the whole launch):
    // st = an owner's entry state / the walker's kept record; xk = the walker's kept key
    // owner slot of this wave (-1: walker / bind wave).  KS_PR_SIMD fills the SIMDs the walker
    // (wave 0, SIMD 0) and the bind wave (wave 1, SIMD 1) do not run on first: waves 2, 3, 6, 7,
    // 10, 11, 14, 15 own slots 0-7 (512 entries), waves 4, 5, 8, 9, 12, 13 slots 8-13 — with a
    // typical table the critical waves then have their SIMDs to themselves.
#ifndef KS_PR_SIMD
#define KS_PR_SIMD 0
#endif
    const int oslot = wave < kOwner0 ? -1
                    : !KS_PR_SIMD ? wave - kOwner0
                    : (wave & 3) >= 2 ? (wave >> 2) * 2 + (wave & 3) - 2 : 8 + ((wave >> 2) - 1) * 2 + (wave & 3);
    __syncthreads();
    // owner waves that can never own an entry end here (the table grows by <= nb entries);
    // s_barrier waits only for the surviving waves
    if (oslot >= 0 && oslot * kWave >= n_pre + nb) return;
    LoopOut lo;
    if (wave == 0) lo = pair_loop<kMode, 0>(a, sh, tid, lane, wave, nb, n_pre, exact, start, oslot);
    else if (wave == 1) lo = pair_loop<kMode, 1>(a, sh, tid, lane, wave, nb, n_pre, exact, start, oslot);
    else lo = pair_loop<kMode, 2>(a, sh, tid, lane, wave, nb, n_pre, exact, start, oslot);
    const int nt = lo.nt, committed = lo.committed, err_code = lo.err_code, err_pod = lo.err_pod;
    __syncthreads();
    // ---- write back the mutable fields of every touched node (by each entry's owner lane: with
    // KS_PR_SIMD the waves that ended early may hold low thread ids)
    const int r_own = oslot >= 0 ? oslot * kWave + lane : kTMax;
    for (int e = KS_PR_SIMD ? r_own : tid; e < nt; e += KS_PR_SIMD ? kTMax : kThreads) {
        const int64_t ndx = sh.tnode[e];
        a.s.rc[ndx] = sh.ts[4][e];
        a.s.rm[ndx] = sh.ts[5][e];
        a.s.rg[ndx] = sh.ts[6][e];
        a.s.nr[ndx] = sh.ts[7][e];
    }
    if (tid == 0) {
        a.ctr[kCtrStart] = start + committed;
        if (committed < a.B && err_code == 0 && start + committed < end) a.ctr[kCtrEarly] += 1;
        if (err_code) { a.ctr[kCtrErr] = err_code; a.ctr[kCtrErrPod] = err_pod; }
    }
}

}  // namespace pr

hipError_t launch_resolve_pair(const EngineArgs* d, int S, int mode, hipStream_t st) {
    switch (mode) {
        case kEvalMicro: hipLaunchKernelGGL(pr::resolve_pair_kernel<kEvalMicro>, dim3(S), dim3(pr::kThreads), 0, st, d); break;
        case kEvalTiny: hipLaunchKernelGGL(pr::resolve_pair_kernel<kEvalTiny>, dim3(S), dim3(pr::kThreads), 0, st, d); break;
        case kEvalNarrow: hipLaunchKernelGGL(pr::resolve_pair_kernel<kEvalNarrow>, dim3(S), dim3(pr::kThreads), 0, st, d); break;
        default: hipLaunchKernelGGL(pr::resolve_pair_kernel<kEvalWide>, dim3(S), dim3(pr::kThreads), 0, st, d); break;
    }
    return hipGetLastError();
}
int pair_resolver_max_batch() { return pr::kMaxB; }

}  // namespace ks
