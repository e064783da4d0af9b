// ks_device.h — device-side records and the fused Filter + Score evaluator (gfx950).
//
// One (pod, node) evaluation = the reference's Filter loop (kubesim/kubesim.go:168-188) and
// score aggregation (:190-206) collapsed into one integer expression:
//   * resource fit   == Node.CreatePod's admission test (kubesim/node/node.go:44-47)
//   * taint          == every NoSchedule/NoExecute taint tolerated (toleration.go:37-56),
//                       pre-reduced on the host to (node_taint & ~pod_tol) == 0
//   * node selector  == (node_label & pod_sel) == pod_sel
//   * scores         == const / LeastRequested / BalancedAllocation, integer-exact
// and returns total+1 (0 = not a candidate), so the argmax key
//   key = (total+1) << 32 | (0xFFFFFFFF - node)
// is maximal for the highest total and, among ties, the lowest node index.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ks {

constexpr int kWave = 64;
constexpr int kTopL = 8;  // exact top-L snapshot candidates kept per pod
// the overlap's single-shard engines scan longer lists: their candidate lists keep the first kTopL
// entries no node of the previous batch touched (ks_cand.hip cand_list), so a list whose top
// entries the previous batch bound (stale) still holds kTopL exact ones (fewer exhausted-list stops).
// 12 measured best on C3 (EXPERIMENTS.md: 8 -> 12 cuts exhausted stops 21 -> 3 per step for ~1.5 us
// more merge per batch; 16 costs more merge than it saves)
#ifndef KS_OVERLAP_LIST
#define KS_OVERLAP_LIST 12
#endif
constexpr int kTopLOverlap = KS_OVERLAP_LIST;
static_assert(kTopLOverlap >= kTopL && kTopLOverlap <= 16 && kTopLOverlap % 2 == 0, "overlap list length");

enum : uint32_t { kFilterFit = 1, kFilterTaint = 2, kFilterSelector = 4 };

// Launch-uniform configuration (kernel argument, lives in SGPRs).
struct Cfg {
    int32_t n_nodes;       // real nodes; indices >= n_nodes are padding
    int32_t nwb;           // wave-blocks of 64 nodes (padded node count / 64)
    int32_t filter_feeds;  // 1: filters gate the candidate set
    uint32_t filters;      // kFilter* bits (only used when filter_feeds)
    int32_t has_scorers;   // 0: nodeScore stays empty ⇒ NotFound
    int32_t w_lr;          // summed weight of LeastRequested scorers
    int32_t w_ba;          // summed weight of BalancedAllocation scorers
    int32_t const_total;   // Σ weight*value over constant scorers
    int32_t tick_seconds;
    int32_t pad_;
};

// Pod record, 48 B, read with scalar loads (uniform per pod).
struct alignas(16) PodRec {
    int64_t req[3];    // milli cpu, milli memory, milli gpu (absent ⇒ 0)
    uint64_t tol;      // dictionary taints this pod tolerates
    uint64_t sel;      // dictionary labels this pod requires
    uint32_t keymask;  // request keys present: 1 cpu, 2 memory, 4 gpu
    uint32_t flags;    // KS_PODFLAG_*
};
static_assert(sizeof(PodRec) == 48, "PodRec layout");

// Node state: 80 B per node, stored struct-of-arrays in HBM.
// One allocation, field k at ac + k * stride (ks_load_nodes), so a field index is an offset.
struct NodeSoA {
    int64_t* ac;   // alloc cpu (milli; -1 absent)
    int64_t* am;   // alloc memory
    int64_t* ag;   // alloc gpu
    int64_t* ap;   // Capacity.Pods().Value()
    int64_t* rc;   // requested cpu of running pods
    int64_t* rm;
    int64_t* rg;
    int64_t* nr;   // running pods
    uint64_t* taint;
    uint64_t* label;
};

struct NodeV {
    int64_t ac, am, ag, ap, rc, rm, rg, nr;
    uint64_t taint, label;
};

__device__ __forceinline__ NodeV load_node(const NodeSoA& s, int64_t i) {
    NodeV v;
    v.ac = s.ac[i]; v.am = s.am[i]; v.ag = s.ag[i]; v.ap = s.ap[i];
    v.rc = s.rc[i]; v.rm = s.rm[i]; v.rg = s.rg[i]; v.nr = s.nr[i];
    v.taint = s.taint[i]; v.label = s.label[i];
    return v;
}

// A node's record in 12 words — the chunk resolver's format (ks_chunk.hip NS32): capacities and usage
// as uint32 (-1 = an absent capacity; the engine routes an engine there only when its scaled
// capacities are < 2^32 - 1), ap clamped to INT_MAX, taint, label — three 16-byte words.
__device__ __forceinline__ void put_rec12(uint32_t* o, const NodeV& v) {
    uint4* w = reinterpret_cast<uint4*>(o);
    w[0] = make_uint4((uint32_t)v.ac, (uint32_t)v.am, (uint32_t)v.ag, (uint32_t)(v.ap > 0x7FFFFFFF ? 0x7FFFFFFF : v.ap));
    w[1] = make_uint4((uint32_t)v.rc, (uint32_t)v.rm, (uint32_t)v.rg, (uint32_t)v.nr);
    w[2] = make_uint4((uint32_t)v.taint, (uint32_t)(v.taint >> 32), (uint32_t)v.label, (uint32_t)(v.label >> 32));
}
__device__ __forceinline__ NodeV get_rec12(const uint4 (&w)[3]) {
    auto cap = [](uint32_t x) { return x == 0xFFFFFFFFu ? (int64_t)-1 : (int64_t)x; };
    NodeV v;
    v.ac = cap(w[0].x); v.am = cap(w[0].y); v.ag = cap(w[0].z); v.ap = (int32_t)w[0].w;
    v.rc = (int64_t)w[1].x; v.rm = (int64_t)w[1].y; v.rg = (int64_t)w[1].z; v.nr = (int32_t)w[1].w;
    v.taint = w[2].x | ((uint64_t)w[2].y << 32); v.label = w[2].z | ((uint64_t)w[2].w << 32);
    return v;
}
// Admission / resource-fit (kubesim/node/node.go:44-47).  Keys requested only by running
// pods cannot fail: they passed admission against the same static capacity and requests are
// non-negative.  An absent capacity key is -1, so any request of that
// key — including 0 — fails, as resourceListGE does (kubesim/node/resource.go:54-55).
__host__ __device__ __forceinline__ bool fits(const PodRec& p, const NodeV& n) {
    bool ok = n.nr < n.ap;
    if (p.keymask & 1) ok &= n.rc + p.req[0] <= n.ac;
    if (p.keymask & 2) ok &= n.rm + p.req[1] <= n.am;
    if (p.keymask & 4) ok &= n.rg + p.req[2] <= n.ag;
    return ok;
}

// floor(y / a) for 0 <= y <= 10*a (restoring division, 4 steps, no hardware divide).
template <typename T>
__host__ __device__ __forceinline__ int32_t div_upto10(T y, T a) {
    int32_t q = 0;
    if (y >= (a << 3)) { q = 8; y -= (a << 3); }
    if (y >= (a << 2)) { q += 4; y -= (a << 2); }
    if (y >= (a << 1)) { q += 2; y -= (a << 1); }
    if (y >= a) q += 1;
    return q;
}

// LeastRequested per resource: (A - u) * 10 / A, 0 if A <= 0 or u > A.
__host__ __device__ __forceinline__ int32_t lr_one(int64_t A, int64_t u) {
    if (A <= 0 || u > A) return 0;
    return div_upto10<int64_t>((A - u) * 10, A);
}

__host__ __device__ __forceinline__ int bitlen(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return x ? 64 - __clzll((long long)x) : 0;
#else
    return x ? 64 - __builtin_clzll(x) : 0;
#endif
}

// BalancedAllocation, exact: floor(10 * (1 - |uc/Ac - um/Am|)), 0 if a fraction >= 1.
// With D = Ac*Am and X = |uc*Am - um*Ac| the score is floor(10 (D - X) / D).  When Ac*Am
// < 2^59 every intermediate fits 64 bits (the common case once memory is held in bytes, see
// ks_engine.cpp's memory scale); otherwise the same formula runs in 128 bits.
__host__ __device__ __forceinline__ int32_t ba_score(int64_t Ac, int64_t Am, int64_t uc, int64_t um) {
    if (Ac <= 0 || Am <= 0 || uc >= Ac || um >= Am) return 0;
    if (bitlen((uint64_t)Ac) + bitlen((uint64_t)Am) <= 59) {
        const uint64_t D = (uint64_t)Ac * (uint64_t)Am;
        const uint64_t a = (uint64_t)uc * (uint64_t)Am, b = (uint64_t)um * (uint64_t)Ac;
        const uint64_t X = a > b ? a - b : b - a;
        return div_upto10<uint64_t>((D - X) * 10, D);
    }
    typedef unsigned __int128 u128;
    const u128 D = (u128)(uint64_t)Ac * (uint64_t)Am;
    const u128 a = (u128)(uint64_t)uc * (uint64_t)Am;
    const u128 b = (u128)(uint64_t)um * (uint64_t)Ac;
    const u128 X = a > b ? a - b : b - a;
    return div_upto10<u128>((D - X) * 10, D);
}

// Fused Filter + Score.  Returns weighted total + 1, or 0 when the node is not a candidate.
__host__ __device__ __forceinline__ uint32_t eval_total1(const Cfg& c, const PodRec& p, const NodeV& n) {
    if (!c.has_scorers) return 0;
    if (c.filter_feeds) {
        bool ok = true;
        if (c.filters & kFilterFit) ok &= fits(p, n);
        if (c.filters & kFilterTaint) ok &= (n.taint & ~p.tol) == 0;
        if (c.filters & kFilterSelector) ok &= (n.label & p.sel) == p.sel;
        if (!ok) return 0;
    }
    int64_t uc = n.rc + p.req[0];
    int64_t um = n.rm + p.req[1];
    int32_t total = c.const_total;
    if (c.w_lr) total += c.w_lr * ((lr_one(n.ac, uc) + lr_one(n.am, um)) >> 1);
    if (c.w_ba) total += c.w_ba * ba_score(n.ac, n.am, uc, um);
    return (uint32_t)total + 1u;
}

// ---------------------------------------------------------------------------------------------
// Narrow evaluator.  The host holds every resource in units of the gcd of all its quantities
// (exact: every fit / LeastRequested / BalancedAllocation result is unit-free) and selects this
// variant when every scaled capacity is below 2^29 (ks_engine.cpp, resource scale).  Requests
// are clamped to 2^30 — any request above every capacity behaves identically — so sums stay in
// int32, the 32x32 products in 64 bits, and each integer floor is a float estimate (error far
// below 1) corrected exactly by one 64-bit compare on each side.
// ---------------------------------------------------------------------------------------------
constexpr int64_t kNarrowCap = 1LL << 29;
constexpr int64_t kNarrowReq = 1LL << 30;

__host__ __device__ __forceinline__ int32_t clamp_req(int64_t q) { return (int32_t)(q < kNarrowReq ? q : kNarrowReq); }

// reciprocal estimates: hardware v_rcp on the device (~1 ulp), exact division on the host
__host__ __device__ __forceinline__ float rcp_est(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
__host__ __device__ __forceinline__ double rcp_est(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcp(x);
#else
    return 1.0 / x;
#endif
}

// floor(10 x / A) for 0 <= x <= A < 2^29: float estimate (error << 1), one exact step either way
__host__ __device__ __forceinline__ int32_t lr_frac10(uint32_t x, uint32_t A) {
    int32_t q = (int32_t)((10.0f * (float)x) * rcp_est((float)A));
    q = q < 0 ? 0 : (q > 10 ? 10 : q);
    const uint64_t y = (uint64_t)x * 10u, t = (uint64_t)(uint32_t)q * A;
    q += (y >= t + A) ? 1 : 0;
    q -= (y < t) ? 1 : 0;
    return q;
}

__host__ __device__ __forceinline__ int32_t lr_one_n(int32_t A, int32_t u) {
    if (A <= 0 || u > A) return 0;
    return lr_frac10((uint32_t)(A - u), (uint32_t)A);
}

// floor(10 (D - X) / D), D = Ac Am < 2^58, X = |uc Am - um Ac| < D: double estimate, exact step
__host__ __device__ __forceinline__ int32_t ba_score_n(int32_t Ac, int32_t Am, int32_t uc, int32_t um) {
    if (Ac <= 0 || Am <= 0 || uc >= Ac || um >= Am) return 0;
    const uint64_t D = (uint64_t)(uint32_t)Ac * (uint32_t)Am;
    const uint64_t a = (uint64_t)(uint32_t)uc * (uint32_t)Am, b = (uint64_t)(uint32_t)um * (uint32_t)Ac;
    const uint64_t X = a > b ? a - b : b - a;
    int32_t q = (int32_t)(10.0 - 10.0 * ((double)X * rcp_est((double)D)));
    q = q < 0 ? 0 : (q > 10 ? 10 : q);
    const uint64_t y = (D - X) * 10u, t = (uint64_t)(uint32_t)q * D;
    q += (y >= t + D) ? 1 : 0;
    q -= (y < t) ? 1 : 0;
    return q;
}

template <class NS>
__host__ __device__ __forceinline__ uint32_t eval_total1_narrow(const Cfg& c, const PodRec& p, const NS& n) {
    if (!c.has_scorers) return 0;
    const int32_t ac = (int32_t)n.ac, am = (int32_t)n.am, ag = (int32_t)n.ag;
    const int32_t rc = (int32_t)n.rc, rm = (int32_t)n.rm, rg = (int32_t)n.rg;
    const int32_t qc = clamp_req(p.req[0]), qm = clamp_req(p.req[1]), qg = clamp_req(p.req[2]);
    if (c.filter_feeds) {
        bool ok = true;
        if (c.filters & kFilterFit) {
            ok &= n.nr < n.ap;
            if (p.keymask & 1) ok &= rc + qc <= ac;
            if (p.keymask & 2) ok &= rm + qm <= am;
            if (p.keymask & 4) ok &= rg + qg <= ag;
        }
        if (c.filters & kFilterTaint) ok &= (n.taint & ~p.tol) == 0;
        if (c.filters & kFilterSelector) ok &= (n.label & p.sel) == p.sel;
        if (!ok) return 0;
    }
    const int32_t uc = rc + qc, um = rm + qm;
    int32_t total = c.const_total;
    if (c.w_lr) total += c.w_lr * ((lr_one_n(ac, uc) + lr_one_n(am, um)) >> 1);
    if (c.w_ba) total += c.w_ba * ba_score_n(ac, am, uc, um);
    return (uint32_t)total + 1u;
}

// ---------------------------------------------------------------------------------------------
// Tiny evaluator: every scaled capacity below 2^26 and Ac * Am below 2^26 (C2 / C3 after the gcd
// scaling: cpu <= 1280 units, memory <= 2048).  Requests are clamped to 2^27 (any request above
// every capacity behaves the same), so every product and sum — 10 (A - u), q A, Ac Am,
// uc Am, 10 (D - X), q D — fits int32; each floor is a float estimate (error < 1e-5) corrected
// exactly by one int32 compare on each side.  No 64-bit multiply and no double on the path.
// ---------------------------------------------------------------------------------------------
constexpr int64_t kTinyCap = 1LL << 26;
constexpr int64_t kTinyReq = 1LL << 27;

__host__ __device__ __forceinline__ int32_t clamp_tiny(int64_t q) { return (int32_t)(q < kTinyReq ? q : kTinyReq); }

// floor(y / A) for 0 <= y <= 10 A, A < 2^26, given iA ~ 1/A
__host__ __device__ __forceinline__ int32_t div10_tiny(int32_t y, int32_t A, float iA) {
    int32_t q = (int32_t)((float)y * iA);
    q = q < 0 ? 0 : (q > 10 ? 10 : q);
    const int32_t t = q * A;
    q += (y >= t + A) ? 1 : 0;
    q -= (y < t) ? 1 : 0;
    return q;
}

template <class NS>
__host__ __device__ __forceinline__ uint32_t eval_total1_tiny(const Cfg& c, const PodRec& p, const NS& n) {
    // Branch-free: every floor is computed on safe inputs and selected, so the LR / LR / BA
    // chains interleave even when a single lane evaluates (the resolver's bind wave).
    const int32_t ac = (int32_t)n.ac, am = (int32_t)n.am, ag = (int32_t)n.ag;
    const int32_t rc = (int32_t)n.rc, rm = (int32_t)n.rm, rg = (int32_t)n.rg;
    const int32_t qc = clamp_tiny(p.req[0]), qm = clamp_tiny(p.req[1]), qg = clamp_tiny(p.req[2]);
    const int32_t uc = rc + qc, um = rm + qm;
    const bool fit_on = c.filter_feeds && (c.filters & kFilterFit);
    const bool taint_on = c.filter_feeds && (c.filters & kFilterTaint);
    const bool sel_on = c.filter_feeds && (c.filters & kFilterSelector);
    // bitwise, not short-circuit: no branch, so the pod record stays in SGPRs (scan_kernel)
    const uint32_t km = p.keymask;
    bool ok = c.has_scorers != 0;
    ok &= !fit_on | ((n.nr < n.ap) & (!(km & 1) | (uc <= ac)) & (!(km & 2) | (um <= am)) &
                     (!(km & 4) | (rg + qg <= ag)));
    ok &= !taint_on | ((n.taint & ~p.tol) == 0);
    ok &= !sel_on | ((n.label & p.sel) == p.sel);
    const bool lc_on = ac > 0 && uc <= ac, lm_on = am > 0 && um <= am;
    const int32_t acs = ac > 0 ? ac : 1, ams = am > 0 ? am : 1;
    const float iac = rcp_est((float)acs), iam = rcp_est((float)ams);  // node-invariant: hoisted
    const int32_t lc = div10_tiny(lc_on ? 10 * (ac - uc) : 0, acs, iac);
    const int32_t lm = div10_tiny(lm_on ? 10 * (am - um) : 0, ams, iam);
    const bool ba_on = ac > 0 && am > 0 && uc < ac && um < am;
    const int32_t ucs = ba_on ? uc : 0, ums = ba_on ? um : 0;
    const int32_t D = acs * ams, a = ucs * ams, b = ums * acs;
    const int32_t X = a > b ? a - b : b - a;
    const int32_t N = 10 * (D - X);
    int32_t q = (int32_t)(10.f - 10.f * fabsf((float)ucs * iac - (float)ums * iam));
    q = q < 0 ? 0 : (q > 10 ? 10 : q);
    const int32_t t = q * D;
    q += (N >= t + D) ? 1 : 0;
    q -= (N < t) ? 1 : 0;
    const int32_t total = c.const_total + c.w_lr * (((lc_on ? lc : 0) + (lm_on ? lm : 0)) >> 1) +
                          c.w_ba * (ba_on ? q : 0);
    return ok ? (uint32_t)total + 1u : 0u;
}

// ---------------------------------------------------------------------------------------------
// Micro evaluator: every scaled capacity below 2^16 and Ac * Am below 2^24 (C2-C5 after the gcd
// scaling).  Requests are clamped to 2^17.  Every product has both factors below 2^24, so each
// is one full-rate 24-bit multiply (v_mul_u32_u24) instead of a 32-bit one.  LeastRequested
// needs no correction step: for integers 0 <= x <= A < 2^16, floor(10 x / A) =
// trunc(fma(x, r, 2^-17)) with r = 10 * rcp(A).  The fma's value is within 2.3e-6 of 10x/A + 2^-17
// (v_rcp 1 ulp, two roundings, 10x/A <= 10).  At an integer k = 10x/A the bias (7.6e-6) keeps it
// >= k; otherwise 10x/A <= k + 1 - 1/A and bias + error (9.9e-6) < 1/A (> 1.5e-5) keeps it < k + 1.
// Checked on the device for every (x, A) pair (ks_selftest).  BalancedAllocation keeps the exact
// correction step of the tiny evaluator.
// ---------------------------------------------------------------------------------------------
constexpr int64_t kMicroCap = 1LL << 16;
constexpr int64_t kMicroProd = 1LL << 24;
constexpr int64_t kMicroReq = 1LL << 17;
constexpr float kMicroBias = 1.0f / 131072.0f;  // 2^-17

// requests are >= 0: q < 2^17 tested on the two 32-bit halves, which the scalar unit can do for a
// uniform pod (it has no 64-bit less-than, so a 64-bit compare would go to the VALU)
__host__ __device__ __forceinline__ int32_t clamp_micro(int64_t q) {
    const uint32_t lo = (uint32_t)q, hi = (uint32_t)((uint64_t)q >> 32);
    return (int32_t)((hi | (lo >> 17)) ? (uint32_t)kMicroReq : lo);
}

// a * b for 0 <= a, b < 2^24 (full-rate 24-bit multiply on the device)
__host__ __device__ __forceinline__ int32_t mul24(int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (int32_t)__umul24((unsigned)a, (unsigned)b);
#else
    return a * b;
#endif
}
// a * b + c for 0 <= a, b < 2^24 (v_mad_u32_u24); only the low 32 bits are kept.  Inline asm:
// with a uniform operand the compiler would otherwise emit a quarter-rate v_mul_lo_u32.
__host__ __device__ __forceinline__ uint32_t umad24(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return (uint32_t)((uint64_t)a * b) + c;
#endif
}
// |a - b| in one v_sad_u32 (__usad compiles to max / min / sub: three instructions)
__host__ __device__ __forceinline__ uint32_t usad(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_sad_u32 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return a > b ? a - b : b - a;
#endif
}
// max(trunc(x), 0) for |x| < 2^31 in one v_cvt_u32_f32 (it saturates negatives to 0); a C cast
// of a negative float to unsigned is undefined, hence the instruction
__host__ __device__ __forceinline__ uint32_t f2u_sat(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
#else
    return x < 1.f ? 0u : (uint32_t)x;
#endif
}
// largest weight the micro evaluator multiplies with a 24-bit multiply (the host's mode choice)
constexpr int64_t kMicroWeight = 1LL << 24;

// floor(10 x / A) for 0 <= x <= A < 2^16 given r = 10 * rcp_est(A) (exactness: above)
__host__ __device__ __forceinline__ int32_t lr10_micro(int32_t x, float r) {
    return (int32_t)fmaf((float)x, r, kMicroBias);
}

// Per-node invariants of the micro evaluator — 1/Ac, 1/Am (v_rcp) and Ac*Am — computed per call,
// unless the state type carries them (the resolver's register entries: found by overload, same
// values, so the results are bit-identical).
template <class NS>
__host__ __device__ __forceinline__ float micro_ic(const NS&, int32_t acs) { return rcp_est((float)acs); }
template <class NS>
__host__ __device__ __forceinline__ float micro_im(const NS&, int32_t ams) { return rcp_est((float)ams); }
template <class NS>
__host__ __device__ __forceinline__ int32_t micro_d(const NS&, int32_t acs, int32_t ams) { return mul24(acs, ams); }

// Written for a short dependent chain (the resolver evaluates a just-bound node on its critical
// path): every term is computed unconditionally from the free amounts f = A - u and selected at
// the end, so LeastRequested, both BalancedAllocation paths and the filters run side by side.
//   * LeastRequested: max(trunc(fma(f, r, 2^-17)), 0) — the exact floor for 0 <= f <= A; for
//     f < 0 (does not fit) or A <= 0 (then f <= 0) the fma is < 1, so the clamp gives the
//     reference's 0.
//   * BalancedAllocation is non-zero only when both free amounts are > 0 (which implies A > 0);
//     otherwise its products are computed on out-of-domain values (unsigned, no overflow trap)
//     and discarded.
//   * weights < kMicroWeight (the host's mode choice): the weighted sum is two 24-bit mads.
template <class NS>
__host__ __device__ __forceinline__ uint32_t eval_total1_micro(const Cfg& c, const PodRec& p, const NS& n) {
    const int32_t ac = (int32_t)n.ac, am = (int32_t)n.am, ag = (int32_t)n.ag;
    const int32_t qc = clamp_micro(p.req[0]), qm = clamp_micro(p.req[1]), qg = clamp_micro(p.req[2]);
    // free after placing: (A - r) is per node (hoisted out of the scan's pod loop)
    const int32_t fc = (ac - (int32_t)n.rc) - qc, fm = (am - (int32_t)n.rm) - qm, fg = (ag - (int32_t)n.rg) - qg;
    const bool fit_on = c.filter_feeds && (c.filters & kFilterFit);
    const bool taint_on = c.filter_feeds && (c.filters & kFilterTaint);
    const bool sel_on = c.filter_feeds && (c.filters & kFilterSelector);
    const uint32_t km = p.keymask;
    bool ok = c.has_scorers != 0;
    ok &= !fit_on | ((n.nr < n.ap) & (!(km & 1) | (fc >= 0)) & (!(km & 2) | (fm >= 0)) & (!(km & 4) | (fg >= 0)));
    ok &= !taint_on | ((n.taint & ~p.tol) == 0);
    ok &= !sel_on | ((n.label & p.sel) == p.sel);
    const int32_t acs = ac > 0 ? ac : 1, ams = am > 0 ? am : 1;
    const float iac = micro_ic(n, acs), iam = micro_im(n, ams);  // node-invariant: hoisted
    const float rc10 = 10.f * iac, rm10 = 10.f * iam;
    const float fcf = (float)fc, fmf = (float)fm;  // exact: |f| < 2^24
    // LeastRequested: max(trunc(fma), 0) per key in one saturating conversion
    const uint32_t lrs = (f2u_sat(fmaf(fcf, rc10, kMicroBias)) + f2u_sat(fmaf(fmf, rm10, kMicroBias))) >> 1;
    const bool ba_on = (fc < fm ? fc : fm) > 0;
    const uint32_t D = (uint32_t)micro_d(n, acs, ams);
    // X = |uc Am - um Ac| = |fm Ac - fc Am| (u = A - f)
    const uint32_t a = umad24((uint32_t)fm, (uint32_t)acs, 0u), b = umad24((uint32_t)fc, (uint32_t)ams, 0u);
    const uint32_t X = usad(a, b);
    const uint32_t N = umad24(D - X, 10u, 0u);
    // estimate of 10 (D - X) / D = 10 - 10 |fm/Am - fc/Ac| (within 1e-5; the step below is exact)
    uint32_t q = f2u_sat(10.f - fabsf(fmaf(fmf, rm10, -fcf * rc10)));  // clamp below: the conversion
    q = q > 10u ? 10u : q;
    const uint32_t t = umad24(q, D, 0u);
    q += (N >= t + D) ? 1u : 0u;
    q -= (N < t) ? 1u : 0u;
    const uint32_t base = umad24((uint32_t)c.w_lr, lrs, (uint32_t)c.const_total + 1u);
    const uint32_t total1 = umad24((uint32_t)c.w_ba, ba_on ? (uint32_t)q : 0u, base);
    return ok ? total1 : 0u;
}

// ---------------------------------------------------------------------------------------------
// The scan's form of the micro evaluator.  A scan workgroup evaluates every pod of its group on
// its node, so whatever depends on the pod only is computed once per pod on the host instead of
// in every wave: the requests clamped to the micro range, the Filter's per-key tests folded into
// biased requests, the tolerations complemented, the disabled filters neutralised.  The scalar
// work per (pod, wave) drops from ~38 to a handful of instructions (the scan issues on one scalar
// unit per CU beside four SIMDs: C5 scan 0.31 -> 0.26 ms for the clamp and key tests alone), and
// the filters combine as integers in VALU instead of as lane masks.  Results are those of
// eval_total1_micro bit for bit (tests/test_evaluator_host.py):
//   fit (node.go:44-47): every requested key k satisfies f_k = (A_k - r_k) - q_k >= 0 and
//     nr < ap  <=>  min(f_c', f_m', f_g', npen) >= 0 with f_k' = (A_k - r_k) - qf_k, qf_k = q_k
//     for a requested key and -2^30 otherwise (f_k' > 0: A_k - r_k >= -1 - 2^16), npen = -1 when
//     nr >= ap (or no scorer, or every node fails), else 0; fit filter off: qf_k = -2^30, npen 0;
//   taint / selector: (taint & ~tol) | (sel & ~label) == 0, ntol = ~tol (0: taint filter off),
//     sel (0: selector filter off).
struct alignas(8) ScanRec {
    int32_t qc, qm;          // clamp_micro(req) (0 for an absent key, as PodRec)
    int32_t qfc, qfm, qfg;   // the fit test's requests (above)
    int32_t pad_;
    uint64_t ntol, sel;
};
static_assert(sizeof(ScanRec) == 40, "ScanRec layout");
constexpr int32_t kFitPass = -(1 << 30);

__host__ __device__ __forceinline__ ScanRec scan_rec_micro(const Cfg& c, const PodRec& p) {
    const bool fit_on = c.filter_feeds && (c.filters & kFilterFit);
    const bool taint_on = c.filter_feeds && (c.filters & kFilterTaint);
    const bool sel_on = c.filter_feeds && (c.filters & kFilterSelector);
    ScanRec r{};
    r.qc = clamp_micro(p.req[0]);
    r.qm = clamp_micro(p.req[1]);
    const int32_t qg = clamp_micro(p.req[2]);
    r.qfc = fit_on && (p.keymask & 1) ? r.qc : kFitPass;
    r.qfm = fit_on && (p.keymask & 2) ? r.qm : kFitPass;
    r.qfg = fit_on && (p.keymask & 4) ? qg : kFitPass;
    r.ntol = taint_on ? ~p.tol : 0ull;
    r.sel = sel_on ? p.sel : 0ull;
    return r;
}

// npen: -1 when no pod can make the node a candidate (no scorer, or the fit filter on and nr >= ap)
template <class NS>
__host__ __device__ __forceinline__ int32_t scan_npen(const Cfg& c, const NS& n) {
    const bool fit_on = c.filter_feeds && (c.filters & kFilterFit);
    return (!c.has_scorers || (fit_on && !(n.nr < n.ap))) ? -1 : 0;
}

template <class NS>
__host__ __device__ __forceinline__ uint32_t eval_scan_micro(const Cfg& c, const ScanRec& p, const NS& n, int32_t npen) {
    const int32_t ac = (int32_t)n.ac, am = (int32_t)n.am, ag = (int32_t)n.ag;
    const int32_t bc = ac - (int32_t)n.rc, bm = am - (int32_t)n.rm, bg = ag - (int32_t)n.rg;  // per node
    const int32_t fc = bc - p.qc, fm = bm - p.qm;
    const int32_t f1 = bc - p.qfc, f2 = bm - p.qfm, f3 = bg - p.qfg;
    int32_t fmin = f1 < f2 ? f1 : f2;
    fmin = fmin < f3 ? fmin : f3;
    fmin = fmin < npen ? fmin : npen;
    const uint32_t nt_lo = (uint32_t)n.taint, nt_hi = (uint32_t)(n.taint >> 32);
    const uint32_t nl_lo = ~(uint32_t)n.label, nl_hi = ~(uint32_t)(n.label >> 32);
    uint32_t bad = (nt_lo & (uint32_t)p.ntol) | (nt_hi & (uint32_t)(p.ntol >> 32));
    bad |= (nl_lo & (uint32_t)p.sel) | (nl_hi & (uint32_t)(p.sel >> 32));
    bad |= (uint32_t)(fmin >> 31);
    const int32_t acs = ac > 0 ? ac : 1, ams = am > 0 ? am : 1;
    const float iac = micro_ic(n, acs), iam = micro_im(n, ams);  // node-invariant: hoisted
    const float rc10 = 10.f * iac, rm10 = 10.f * iam;
    const float fcf = (float)fc, fmf = (float)fm;  // exact: |f| < 2^24
    // LeastRequested: max(trunc(fma), 0) per key in one saturating conversion
    const uint32_t lrs = (f2u_sat(fmaf(fcf, rc10, kMicroBias)) + f2u_sat(fmaf(fmf, rm10, kMicroBias))) >> 1;
    const bool ba_on = (fc < fm ? fc : fm) > 0;
    const uint32_t D = (uint32_t)micro_d(n, acs, ams);
    const uint32_t a = umad24((uint32_t)fm, (uint32_t)acs, 0u), b = umad24((uint32_t)fc, (uint32_t)ams, 0u);
    const uint32_t X = usad(a, b);
    const uint32_t N = umad24(D - X, 10u, 0u);
    uint32_t q = f2u_sat(10.f - fabsf(fmaf(fmf, rm10, -fcf * rc10)));  // clamp below: the conversion
    q = q > 10u ? 10u : q;
    const uint32_t t = umad24(q, D, 0u);
    q += (N >= t + D) ? 1u : 0u;
    q -= (N < t) ? 1u : 0u;
    const uint32_t base = umad24((uint32_t)c.w_lr, lrs, (uint32_t)c.const_total + 1u);
    const uint32_t total1 = umad24((uint32_t)c.w_ba, ba_on ? (uint32_t)q : 0u, base);
    return bad == 0 ? total1 : 0u;
}

// Evaluator variants: 0 wide (64/128-bit), 1 narrow (capacities < 2^29), 2 tiny, 3 micro (above).
// A larger value is a narrower domain; each evaluator is exact on every narrower domain.
enum : int { kEvalWide = 0, kEvalNarrow = 1, kEvalTiny = 2, kEvalMicro = 3 };

template <int kMode, class NS>
__host__ __device__ __forceinline__ uint32_t eval_t(const Cfg& c, const PodRec& p, const NS& n) {
    if constexpr (kMode == kEvalMicro) return eval_total1_micro(c, p, n);
    else if constexpr (kMode == kEvalTiny) return eval_total1_tiny(c, p, n);
    else if constexpr (kMode == kEvalNarrow) return eval_total1_narrow(c, p, n);
    else return eval_total1(c, p, n);
}

// Pod-dependent upper bound of the total, used by the resolver's owner waves to pass the decider
// only the touched entries that can reach a pod's lower bound.  Per entry the resolver keeps b = (A - r) / A and 1/A in
// float; for a pod with requests q, f = b - q/A = (A - u) / A and
//   LeastRequested  floor(10 f)              <= floor(10 f~ + kBoundLR)
//   Balanced        floor(10 (1 - |fc - fm|)) <= floor(10 (1 - |fc~ - fm~|) + kBoundBA)
// where f~ is the float value: |f~ - f| < 6e-7 (rounding 2^-24 per op, v_rcp 1 ulp), so the
// slacks below cover every rounding and each bounded floor is the exact one except within the
// slack of an integer.  LR is 0 once u > A, Balanced once uc >= Ac or um >= Am (only claimed when
// f~ is clearly negative).  Filters are not applied (a bound).
constexpr float kBoundLR = 1.5e-5f;
constexpr float kBoundBA = 3.0e-5f;
struct PruneF {
    float bc, ic, bm, im;
    int32_t live;  // 0: no pod can make this node a candidate
};
template <class NS>
__host__ __device__ __forceinline__ PruneF prune_prep(const Cfg& c, const NS& n) {
    PruneF f;
    f.ic = n.ac > 0 ? rcp_est((float)n.ac) : 0.f;
    f.bc = n.ac > 0 ? (float)(int64_t)(n.ac - n.rc) * f.ic : -1.f;
    f.im = n.am > 0 ? rcp_est((float)n.am) : 0.f;
    f.bm = n.am > 0 ? (float)(int64_t)(n.am - n.rm) * f.im : -1.f;
    f.live = c.has_scorers && !(c.filter_feeds && (c.filters & kFilterFit) && n.nr >= n.ap);
    return f;
}
// The same for capacities < 2^29 (every evaluator but the wide one): A - r fits int32, so each
// conversion is one v_cvt instead of an int64-to-float sequence (identical values).
template <int kMode, class NS>
__host__ __device__ __forceinline__ PruneF prune_prep_t(const Cfg& c, const NS& n) {
    if constexpr (kMode >= kEvalNarrow) {
        const int32_t ac = (int32_t)n.ac, am = (int32_t)n.am;
        PruneF f;
        f.ic = ac > 0 ? rcp_est((float)ac) : 0.f;
        f.bc = ac > 0 ? (float)(ac - (int32_t)n.rc) * f.ic : -1.f;
        f.im = am > 0 ? rcp_est((float)am) : 0.f;
        f.bm = am > 0 ? (float)(am - (int32_t)n.rm) * f.im : -1.f;
        f.live = c.has_scorers && !(c.filter_feeds && (c.filters & kFilterFit) && n.nr >= n.ap);
        return f;
    } else {
        return prune_prep(c, n);
    }
}
__host__ __device__ __forceinline__ uint32_t prune_tmax(const Cfg& c, const PruneF& f, float qc, float qm) {
    const float fc = fmaf(-qc, f.ic, f.bc), fm = fmaf(-qm, f.im, f.bm);
    int32_t total = c.const_total;
    const int32_t lc = fc > -kBoundLR ? (int32_t)(10.f * fc + kBoundLR) : 0;
    const int32_t lm = fm > -kBoundLR ? (int32_t)(10.f * fm + kBoundLR) : 0;
    total += c.w_lr * ((lc + lm) >> 1);
    if (fc > -kBoundLR && fm > -kBoundLR)
        total += c.w_ba * (int32_t)(10.f - 10.f * fabsf(fc - fm) + kBoundBA);
    return (uint32_t)total;
}

// Wave-uniform load through the constant address space: the compiler emits s_load (scalar cache,
// SGPR result) instead of a flat vector load per lane.  Only for data no kernel in flight writes
// (pod records, the batch counters written by an earlier kernel of the stream).
// (Copied dword by dword: a struct copy would go through a generic memcpy and lose the space.)
template <typename T>
__device__ __forceinline__ T sload(const T* p) {
    static_assert(sizeof(T) % 4 == 0, "sload: dword-sized types only");
    typedef const __attribute__((address_space(4))) uint32_t* cp;
    const cp q = (cp)p;
    T v;
    uint32_t* d = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) d[i] = q[i];
    return v;
}

// The same pointer in the global address space: global_load / global_store instead of flat_.
// A flat access is counted in lgkmcnt as well as vmcnt, so the s_waitcnt lgkmcnt(0) that every
// LDS wait and every __syncthreads() carries would also wait for it — an HBM round trip on the
// resolver's per-pod barrier.  A global access is counted in vmcnt only.
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

__host__ __device__ __forceinline__ uint64_t make_key(uint32_t total1, uint32_t node) {
    return total1 ? (((uint64_t)total1 << 32) | (uint64_t)(0xFFFFFFFFu - node)) : 0ull;
}

// Insert one sorted (descending, 0-padded) list of L keys into a sorted top-L: the per-thread step
// of the merge kernel, also the host's ks_merge_candidates.  Keys are distinct (node in the low
// bits), so the result is the exact top-L of the union.
template <int L = kTopL>
__host__ __device__ __forceinline__ void topl_insert(uint64_t (&top)[L], const uint64_t (&lv)[L]) {
#pragma unroll
    for (int k = 0; k < L; ++k) {
        uint64_t v = lv[k];
        if (v <= top[L - 1]) break;  // lists are sorted: nothing further can enter
#pragma unroll
        for (int s = 0; s < L; ++s) {
            const uint64_t t = top[s];
            const bool gt = v > t;
            top[s] = gt ? v : t;
            v = gt ? t : v;
        }
    }
}

// Wave-wide unsigned max in VALU DPP moves (no LDS crossbar): Hillis-Steele row_shr 1/2/4/8
// leaves each 16-lane row's max in its lane 15, row_bcast 15/31 folds the rows into lane 63.
__device__ __forceinline__ uint32_t dpp_max_step(uint32_t v, uint32_t w) { return v > w ? v : w; }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = dpp_max_step(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = dpp_max_step(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = dpp_max_step(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = dpp_max_step(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = dpp_max_step(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = dpp_max_step(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// 64-bit max as two 32-bit maxes: the high words, then the low words of the lanes at it.
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    const uint32_t mh = wave_max_u32(hi);
    const uint32_t ml = wave_max_u32(hi == mh ? lo : 0u);
    return ((uint64_t)mh << 32) | ml;
}

// ctr[] slots of a batch (EngineArgs::ctr), pod flags the resolvers stop on, error codes
// (5, 6: cumulative counts of the window prep's rescans and list reuses — diagnostic builds use
// ctr[5..31] for their own counters)
enum : int64_t { kCtrStart = 0, kCtrEnd = 1, kCtrErr = 2, kCtrErrPod = 3, kCtrEarly = 4, kCtrRescan = 5, kCtrReuse = 6 };
enum : uint32_t { kFlagBadKey = 1, kFlagBadSpec = 2 };
enum : int64_t { kErrEinval = 1, kErrNotFound = 2 };

// Batch window workspace, one per engine, in HBM: the expiry window and the static candidate lists
// of a batch (window_prep_kernel and the candidate-list kernels, ks_cand.hip), read by the chunk and
// sequential resolvers.  Batches of up to kWinMaxB pods whose expiry window holds up to kWinSlots
// slots.
constexpr int kWinMaxB = 256;
constexpr int kWinSlots = 512;
#ifndef KS_CHR
#define KS_CHR 20  // (A/B: make variant DEFS=-DKS_CHR=24; 20: C3 +1.5 %, C3q -3.4 % against 24)
#endif
constexpr int kChR = KS_CHR;  // static candidates kept per pod
constexpr int kRecDw = 20;  // a candidate node's record, dwords (the widest format: ten int64, ks_cand.hip)
constexpr int kSlotMax = 1536;  // candidate slots whose record / E index merge_cl stages
// claims a batch can make: every kept entry of every pod (slot_node holds each one, so the commit
// can reset node_slot for every claimed node — the slots past kSlotMax included)
constexpr int kSlotIds = kWinMaxB * kChR;
constexpr int32_t kNoFirst = 0x7F7F7F7F;  // (a byte-filled memset value above every entry index)
constexpr int kEMax = 2048;     // E nodes per batch: the window's expiry nodes + the overlap's touched nodes
constexpr int kTouchMax = kWinMaxB + kWinSlots;
constexpr int kSpecStride = 8;  // int64 counters per speculative set
constexpr int kSpecPrev = 3;    // (in a set: the start of the batch that wrote it)
enum : int32_t { kClTrunc = 1 << 8, kClFull = 1 << 9, kClOvf = 1 << 10 };
struct WinWS {
    int32_t nb, e_cnt, n_e, n_es;         // E nodes; the first n_es have window slots (<= kWinSlots)
    int32_t win_hi[kWinMaxB];             // pod i: expiry slots < win_hi[i] are applied before it binds
    int32_t own[kWinMaxB];                // pod i's own expiry slot in the window, or -1
    int32_t ex_q[kWinSlots];              // slot -> expiring pod
    int32_t ex_ok[kWinSlots];             // pre-batch pod bound Ok and not expired yet
    int64_t ex_req[kWinSlots][3];
    // E: the distinct nodes of the pre-batch expiries, then (overlapped scan) the nodes changed since
    // the scan read the node table, with no slots
    int32_t e_node[kEMax];
    int32_t e_off[kWinSlots + 1];         // E node k < n_es: its slots e_slot[e_off[k] .. e_off[k+1]) ascending
    int32_t e_slot[kWinSlots];
    // E node k's record after the window's head (put_rec12), staged by the first workgroups of the
    // scan launch before merge_cl (ks_kernels.hip scan_kernel): each merge_cl workgroup reads three
    // contiguous 16-byte words per E node instead of gathering ten scattered fields
    uint32_t e_rec[kEMax][12];
    // pod i's static candidates, sorted descending
    uint64_t cl_key[kWinMaxB][kChR];
    int32_t cl_info[kWinMaxB];            // kept count | kClTrunc | kClFull | kClOvf
    uint64_t cl_thr[kWinMaxB];            // the list's last key when full, else 1
    // each distinct candidate node of the batch has one slot (ks_cand.hip):
    // entry r of pod i is slot cl_slot[i][r] (-2: claimed by another workgroup of the same launch,
    // read node_slot; -3: no slot left)
    int32_t cl_slot[kWinMaxB][kChR];
    int32_t nslot;                        // slots handed out (may exceed kSlotMax: overflow)
    int32_t nslot_hw;                     // the largest nslot any batch reached (ks_debug_invariants)
    // slot -> node for every claim.  (Until round 6 this array had kSlotMax entries: a batch with more
    // than kSlotMax distinct candidates wrote slot_node[kSlotMax + s] over slot_eix[s] — racing the
    // claimer of slot s, so a candidate's E index could come out as a node id — and the commit's
    // reset missed the claims past kSlotMax.)
#ifdef KS_SLOT_IDS_LEGACY  // (diagnostic build only: the round-3..5 layout, for the regression test's A/B)
    int32_t slot_node[kSlotMax];
#else
    int32_t slot_node[kSlotIds];
#endif
    int32_t slot_eix[kSlotMax];           // the node's index in E, -1 if not an E node
    uint32_t slot_rec[kSlotMax][kRecDw];  // the node's record at the batch start (narrow: 12 dwords)
    // overlap (scan of batch k+1 beside the resolve of batch k): the nodes batch k changed (its
    // binds, its window's expiry nodes), written by its commit; and whether batch k+1's lists must
    // be rescanned (the speculative scan covered other pods, or the touched nodes overflow E)
    int32_t touched[kTouchMax];
    int32_t n_touched, rescan;
    int32_t lset, pad_;                   // pruned lists: the set holding this batch's lists (EngineArgs)
    // Early stop without a rescan (round 6): when the previous batch k stopped early, this batch's
    // first `split` pods are batch k's pods [moff, moff + split) and take the merged top-L lists
    // merge_cl kept for them (mrg[mpar ^ 1]); the others take the speculative scan's lists at slot
    // b - split.  merge_cl keeps every batch's merged lists in mrg[mpar] (mpar = the batch parity).
    int32_t split, moff, mpar, pad2_;
    uint64_t mrg[2][kWinMaxB][kTopLOverlap];
#ifdef KS_BATCH_LOG  // (diagnostic builds only: per-batch log and one watched pod's batch, ks_debug_window)
    int32_t blog_n, watch_pod, watch_done, wpad_;
    int32_t blog[16384][4];               // per chunk-resolver batch: start (low 31 bits), committed, stop code, nb
    int32_t w_start, w_nb, w_c, w_n_e, w_n_es, w_pad[3];
    uint64_t w_cl_key[kWinMaxB][kChR];
    int32_t w_cl_info[kWinMaxB];
    uint64_t w_cl_thr[kWinMaxB];
    int32_t w_e_node[kEMax];
    int32_t w_bind[kWinMaxB];             // the batch's committed binds (node)
    int32_t w_adm[kWinMaxB];
    int32_t w_nsw, w_pad2;
    int32_t w_dec[64][8];                 // watched pod, per sweep: fresh, lo, bad, code, nw cid, dc cid, dk total, c0
    int16_t w_smeta[64][8];               // its chunk's rows at the chunk's end
    int32_t w_rowcid[64];
#endif
};

// Arguments of the batch kernels (expire_head / scan / resolve).
struct EngineArgs {
    Cfg c;
    NodeSoA s;
    const PodRec* pods;
    const int32_t* dur;      // ticks a bound-Ok pod runs (0: never counted)
    const int64_t* exp_off;  // [P+1]: expiries due before pod j binds
    const int32_t* exp_pod;
    const int64_t* exp_pos;  // [P]: index in exp_pod of pod q's own expiry, -1 if none yet
    int32_t* b_node;
    int32_t* b_status;
    uint8_t* expired;
    uint64_t* lists;         // [B][nblk][kTopL] per-block top-L keys (scan -> merge)
    uint64_t* cand;          // [B][kTopL] per-pod global top-L keys (merge -> resolve)
    int64_t* ctr;            // start, end, error code, error pod, early stops
    int32_t B;
    int32_t PG;              // pods per scan workgroup
    int32_t nblk;            // 256-node scan blocks (whole cluster; the lists' stride)
    int32_t blk_lo;          // this rank's scan range [blk_lo, blk_lo + blk_n) (node sharding)
    int32_t blk_n;
    WinWS* sw;               // batch window workspace (nullptr unless allocated)
    int32_t* e_idx;          // [n_pad] node -> index in the window's E, -1 otherwise
    int32_t* n_slot;         // [n_pad] node -> its candidate slot in this batch, -1 otherwise
    int32_t* n_first;        // [n_pad] node -> its first kept entry (pod * kChR + rank) in this batch,
                             // kNoFirst otherwise (ks_cand.hip cand_list, ks_chunk.hip setup)
    int64_t* spec_ctr;       // the speculative scan's counters, two sets of kSpecStride (window prep
                             // writes: the next batch if this one commits all its pods)
    // pruned block lists (ks_scan.h; nullptr: every block writes its whole list): per pod a bitmap of
    // the blocks that wrote one and a running threshold key, in two sets — [2][B][nwl] u64 and
    // [2][B]: set 0 written by the overlap's speculative scan (which may still run while the next
    // batch's window prep decides on a rescan), set 1 by the engine's own scans (plain chain, a
    // pass's first batch, the rescan).  merge_cl reads the set window prep names (WinWS::lset) and
    // clears both for the next batch
    uint64_t* lbit;
    uint64_t* lthr;
    int32_t nwl;             // bitmap words per pod: ceil(nblk / 64)
    int32_t lset;            // the set this argument record's scans write
    int32_t det_cids;        // chunk resolver: number the candidates by first appearance (sharded engines:
                             // every rank must cut its batches at the same pods), not by claim order
    int32_t pad3_;
    const ScanRec* srec;     // [P] the pods' scan records (the micro evaluator's scan form)
};
// pruned lists: pod b's bitmap / threshold in set `set`
__host__ __device__ __forceinline__ uint64_t* lbit_of(const EngineArgs& a, int set, int b) {
    return a.lbit + ((int64_t)set * a.B + b) * a.nwl;
}
// thresholds: [2][kThrCopies][B], one copy per XCD-sized group of workgroups (any copy is a valid
// threshold; plain loads and stores, no contended atomics)
constexpr int kThrCopies = 8;
__host__ __device__ __forceinline__ uint64_t* lthr_of(const EngineArgs& a, int set, int copy, int b) {
    return a.lthr + ((int64_t)set * kThrCopies + copy) * a.B + b;
}

// Launchers and limits (defined in ks_kernels.hip).  The batch launchers take a device array of
// S engines' arguments (S = 1 for ks_step, the group's scenarios for ks_group_step).
int max_batch_pods();
int max_pods_per_scan_wg();
int block_nodes();
// expiries due before each scenario's batch head
hipError_t launch_expire_head(const EngineArgs* d, int S, hipStream_t st);
// scan of each scenario's blocks [blk_lo, blk_lo + blk_n); grid x = the largest blk_n
// key16: every total + 1 < 2^16 (scan_kernel's 16-bit key table)
// cond: only when the window workspace's rescan flag is set (the overlap's fallback)
// prune: the pruned-list form (the engine's lbit / lthr set, ks_scan.h)
// L: the block lists' length (kTopL; kTopLOverlap for the overlap's single-shard engines: key16, not
// pruned)
// pw > 0 (one engine): a grid of at most pw workgroups, each looping over its XCD's items (the
// pipelined engines' conditional rescan: cheap to launch when nothing is flagged)
hipError_t launch_scan(const EngineArgs* d, int S, int blk_n, int B, int PG, int mode, bool key16, hipStream_t st,
                       bool cond = false, bool prune = false, int L = kTopL, bool stage = false, int pw = 0);
// per scenario and pod b < batch size: exact top-L over nl sorted lists
// lists[b*pod_stride + k*list_stride] into out (lists == nullptr: the scenario's own block lists
// into its candidate lists)
// nl_max: the largest nl of the launch (<= 64 / L candidates per pod: one wave per pod)
// bits (pruned lists, ks_scan.h; nullptr: read every list): the pods' bitmaps ([B][nwl]); list k of
// the range is block blk0 + k
// lset_fixed >= 0: read that list set's bitmaps (not the window's WinWS::lset)
// L: the lists' length (kTopL, or kTopLOverlap for the pipelined sharded engines' part merges)
hipError_t launch_merge(const EngineArgs* d, int S, int B, const uint64_t* lists, int64_t pod_stride, int32_t nl,
                        int64_t list_stride, uint64_t* out, int nl_max, hipStream_t st, const uint64_t* bits = nullptr,
                        int32_t nwl = 0, int32_t blk0 = 0, int32_t lset_fixed = -1, int L = kTopL);
// the role-split resolver (ks_kernels.hip): batches of up to max_batch_pods() pods, any cluster
hipError_t launch_resolve(const EngineArgs* d, int S, int mode, hipStream_t st);
// the register-table resolver (ks_resolve.hip): batches of <= small_resolver_max_batch() pods of
// clusters of <= small_resolver_max_nodes() nodes, four per CU
hipError_t launch_resolve_small(const EngineArgs* d, int S, int mode, hipStream_t st);
int small_resolver_max_batch();
int small_resolver_max_nodes();
// the chunk resolver (ks_chunk.hip): one engine (S = 1), batches of <= kWinMaxB pods, node state in
// 32-bit words (scaled capacities < 2^32 - 1) and every total + 1 < 2^16; its batch is
// launch_window_prep(head) -> scan -> launch_merge_cl -> launch_chunk_only, or with the overlap
// launch_window_prep(head, spec) -> conditional scan -> merge_cl -> chunk, the next batch's scan
// on a second stream beside the chunk kernel (its commit writes the touched nodes)
hipError_t launch_chunk_only(const EngineArgs* d, int mode, hipStream_t st);
// the same with the next batch's speculative scan fused in (ds: its arguments; `workers` scan
// workgroups beside the resolver's; 16-bit key tables, so key16 engines only); after its commit the
// resolver workgroup runs the next batch's window prep (head, spec; next_slot: that batch's parity)
hipError_t launch_chunk_scan(const EngineArgs* d, const EngineArgs* ds, int workers, int next_slot, int mode,
                             bool prune, int L, hipStream_t st);
// the batch window (expiries of the batch's pods, the node set E): the resolvers' first kernel;
// head: also apply the expiries due before the batch's first pod (expire_head's work); spec: the
// batch's lists come from the speculative scan (the touched nodes join E, or a rescan is flagged)
// slot: the speculative counters' buffer this batch writes (batch parity; the previous batch's is
// slot ^ 1)
hipError_t launch_window_prep(const EngineArgs* d, bool head, bool spec, int slot, hipStream_t st);
// merge + candidate lists (ks_cand.hip): per pod the merge kernel's exact top-L over its lists, then
// its static candidates and their slots
// L: the lists' length (the engine's block lists, or kTopL for the sharded second merge)
#ifdef KS_MCL_BYVAL
extern thread_local const EngineArgs* ks_mcl_host_args;
#endif
// own_fallback: when the window prep flagged a rescan, read the engine's own block lists over the
// whole cluster instead of `lists` (the pipelined engines' rescan scans every block locally)
hipError_t launch_merge_cl(const EngineArgs* d, int mode, int B, const uint64_t* lists, int64_t pod_stride,
                           int32_t nl, int64_t list_stride, int nl_max, hipStream_t st, int L = kTopL,
                           bool own_fallback = false);
struct BindSeg {
    const int32_t* node;
    const int32_t* status;
    int64_t lo, n, off;  // copy [lo, lo + n) to [off, off + n)
};
hipError_t launch_gather_binds(const BindSeg* segs, int S, int64_t max_n, int32_t* node, int32_t* status,
                               hipStream_t st);
hipError_t launch_rescale(const NodeSoA& s, int64_t n_pad, PodRec* pods, int64_t P, const int64_t f[3], hipStream_t st);

// Host-staged submits (ks_engine.cpp): copy `bytes` from device-visible pinned host memory to dst.
struct CopySeg {
    uint8_t* dst;
    const uint8_t* src;
    int64_t bytes;
};
hipError_t launch_scatter(const CopySeg* segs, int n, hipStream_t st);

// The per-tick path (ks_tick.hip): one pod, one launch.
constexpr int kTickMaxExp = 16;  // expiries due before the pod, passed by value
struct TickExp {
    int32_t node, q;    // the expiring pod q and its node
    int64_t req[3];
};
struct TickScratch {    // device, zero between launches (the last workgroup resets it)
    uint64_t best;
    uint32_t count, pad_;
};
struct TickOut {        // host-mapped
    int32_t node, status, code, pad_;
};
constexpr int kTickInl = 1024;   // inline staged bytes per per-tick launch
constexpr int kTickInlSeg = 32;  // inline staged segments per per-tick launch
struct TickSeg {
    uint8_t* dst;
    int32_t off, bytes;
};
struct TickArgs {
    Cfg c;
    NodeSoA s;
    PodRec pod;
    int64_t j;          // the pod's FIFO index
    int32_t run;        // bound Ok, it counts toward the node's totals (dur > 0)
    int32_t n_exp;
    TickExp exp[kTickMaxExp];
    int32_t* b_node;
    int32_t* b_status;
    uint8_t* expired;
    TickScratch* scr;
    TickOut* out;
    // this call's host-staged submits, inline in the kernel arguments (no device read of pinned
    // host memory): segment k copies bytes [off, off + bytes) of inl to dst
    int32_t n_iseg, pad_;
    TickSeg iseg[kTickInlSeg];
    alignas(16) uint8_t inl[kTickInl];
};
hipError_t launch_tick(const TickArgs& a, int mode, hipStream_t st);
struct ExpList {
    int32_t n, pad_;
    TickExp x[kTickMaxExp];
};
// apply the listed expiries to the node state and mark them expired (ks_filter / ks_score's flush)
hipError_t launch_apply_exp(const NodeSoA& s, uint8_t* expired, const ExpList& l, hipStream_t st);
hipError_t launch_eval_pod(const Cfg& c, const NodeSoA& s, const PodRec* pod, uint32_t filters, uint8_t* mask,
                           int64_t* score, int mode, hipStream_t st);
hipError_t launch_flush(const NodeSoA& s, const PodRec* pods, const int64_t* fin, int64_t t, int64_t n_done,
                        const int32_t* b_node, const int32_t* b_status, uint8_t* expired, hipStream_t st);
hipError_t launch_selftest_lr_micro(unsigned long long* bad, hipStream_t st);
// usage queries: grids of candidate pod blocks of usage_block_pods() pods each (pods < q_hi)
int usage_block_pods();
hipError_t launch_usage(const int32_t* blocks, int64_t nblocks, int64_t q_hi, int64_t t, int32_t tick_s,
                        const int32_t* b_node, const int32_t* b_status, const int64_t* t0, const int32_t* dur,
                        const int32_t* phase_off, const int32_t* cum_sec, const int64_t* use,
                        unsigned long long* usage, hipStream_t st);
// diff: [6][t_hi - t_lo + 1] zeroed; out: [t_hi - t_lo][6]
hipError_t launch_usage_digest(const int32_t* blocks, int64_t nblocks, int64_t q_hi, int64_t t_lo, int64_t t_hi,
                               int32_t tick_s, const int32_t* b_node, const int32_t* b_status, const int64_t* t0,
                               const int32_t* dur, const uint8_t* preg, const int32_t* phase_off,
                               const int32_t* cum_sec, const int64_t* use, unsigned long long* diff,
                               unsigned long long* out, hipStream_t st);

}  // namespace ks
