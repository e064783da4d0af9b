// ks_chunk.hip — the chunk resolver (gfx950): a batch's binds by chunked Jacobi sweeps in LDS.
//
// The reference binds one pod per tick in FIFO order (kubesim/kubesim.go:105-121, 143-166): pod i
// takes the argmax of its key over every node, on the state that the binds of pods < i (admitted
// per kubesim/node/node.go:36-60) and the expiries due by its tick leave.  Write f_i(w_{<i}) for
// that argmax given the earlier winners.  This resolver splits f_i into
//   S_i(W) = the first entry of pod i's static candidate list cl_i whose node no earlier pod bound
//            (cl_i, built by chunk_cl_kernel: pod i's snapshot top-L list entries that no pre-batch
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

namespace ks {
namespace chk {

constexpr int kThreads = 1024;
constexpr int kB = kSweepMaxB;  // pods per batch
constexpr int kC = 64;          // pods per chunk: one lane each
constexpr int kR = kChR;        // static candidates kept per pod
constexpr int kCid = 1024;      // distinct candidate nodes per batch (E nodes first)
constexpr int kSlots = kChSlots;
constexpr int kSeg = 5;         // stored state segments per replayed node within a chunk
constexpr int kPend = 4;        // pending own expiries per replayed node
constexpr int kHashLog2 = 11, kHash = 1 << kHashLog2;
constexpr int kL = kTopL;
constexpr int kClBuf = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int16_t kNoSeg = INT16_MAX;
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
#define DG(...)
#endif

// A node's state in int32 (evaluator modes >= narrow: capacities < 2^29; `ap` clamped)
struct NS32 {
    int32_t ac, am, ag, ap, rc, rm, rg, nr;
    uint64_t taint, label;
};

__device__ __forceinline__ int32_t key_node(uint64_t key) { return (int32_t)(0xFFFFFFFFu - (uint32_t)key); }
__device__ __forceinline__ uint32_t hslot(int32_t n) { return ((uint32_t)n * 2654435761u) >> (32 - kHashLog2); }
__device__ __forceinline__ int32_t clamp32(int64_t v) { return (int32_t)(v > INT_MAX ? INT_MAX : v); }

// CreatePod admission (kubesim/node/node.go:44-47), requests in int64
__device__ __forceinline__ bool fits32(const PodRec& p, const NS32& n) {
    bool ok = n.nr < n.ap;
    if (p.keymask & 1) ok &= (int64_t)n.rc + p.req[0] <= n.ac;
    if (p.keymask & 2) ok &= (int64_t)n.rm + p.req[1] <= n.am;
    if (p.keymask & 4) ok &= (int64_t)n.rg + p.req[2] <= n.ag;
    return ok;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------------------------------------
// Static candidates of pod i (one workgroup per pod): its top-L entries outside E and the E nodes
// whose key at pod i's tick (the pre-batch expiries of slots < win_hi[i] applied) reaches thr.
template <int kMode>
__global__ __launch_bounds__(256) void chunk_cl_kernel(const EngineArgs* __restrict__ A) {
    const EngineArgs& a = A[0];
    SweepWS& ws = *a.sw;
    const int i = blockIdx.x, tid = threadIdx.x;
    if (i >= ws.nb) return;
    const int64_t start = a.ctr[kCtrStart];
    __shared__ uint64_t buf[kClBuf];
    __shared__ int cnt;
    if (tid == 0) cnt = 0;
    __syncthreads();
    const PodRec p = a.pods[start + i];
    const uint64_t last = a.cand[(int64_t)i * kL + kL - 1];
    const bool full = last != 0;
    const uint64_t thr = full ? last : 1ull;
    const int hi = ws.win_hi[i], n_e = ws.n_e;
    for (int k = tid; k < n_e; k += 256) {
        const int32_t n = ws.e_node[k];
        NodeV v = load_node(a.s, n);
        for (int u = ws.e_off[k], ue = ws.e_off[k + 1]; u < ue; ++u) {
            const int x = ws.e_slot[u];
            if (x >= hi) break;  // ascending
            v.rc -= ws.ex_req[x][0]; v.rm -= ws.ex_req[x][1]; v.rg -= ws.ex_req[x][2]; v.nr -= 1;
        }
        const uint64_t key = make_key(eval_t<kMode>(a.c, p, v), (uint32_t)n);
        if (key >= thr) {
            const int pos = atomicAdd(&cnt, 1);
            if (pos < kClBuf) buf[pos] = key;
        }
    }
    if (tid < kL) {
        const uint64_t x = a.cand[(int64_t)i * kL + tid];
        if (x != 0 && a.e_idx[key_node(x)] < 0) {
            const int pos = atomicAdd(&cnt, 1);
            if (pos < kClBuf) buf[pos] = x;
        }
    }
    __syncthreads();
    const int c = cnt, n = c < kClBuf ? c : kClBuf;
    if (tid < n) {  // rank by counting (keys are distinct: the node is in the low bits)
        const uint64_t me = buf[tid];
        int r = 0;
        for (int u = 0; u < n; ++u) r += buf[u] > me;
        if (r < kR) ws.cl_key[i][r] = me;
    }
    if (tid == 0) {
        ws.cl_info[i] = (c < kR ? c : kR) | (c > kR ? kClTrunc : 0) | (full ? kClFull : 0) | (c > kClBuf ? kClOvf : 0);
        ws.cl_thr[i] = thr;
    }
}

// ---------------------------------------------------------------------------------------------
enum : uint8_t { kFlRun = 1, kFlTrunc = 2, kFlFull = 4, kFlOvf = 8 };

struct ChShared {
    PodRec pod[kB];
    uint32_t cl[kB][kR];          // (cid << 16) | total + 1, descending
    uint64_t thr[kB];
    int32_t cnode[kCid];          // cid -> node (cids 0 .. n_e - 1 are E, in ws order)
    int32_t rs[4][kCid];          // ac am ag ap
    int32_t rd[4][kCid];          // rc rm rg nr at the batch start
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
    int32_t xreq[3][kSlots];
    int16_t xeff[kSlots];         // slot x is applied from pod xeff[x] on
    int16_t eoff[kSlots + 1], eslot[kSlots];
    int16_t seff[kB][kSeg];       // replayed node (slot = its first binder pod): segment start pods
    int32_t sst[kB][kSeg][4];     // and states rc rm rg nr
    int16_t sovf[kB];             // first pod whose state the slot does not hold
    uint64_t cd1[kC], cd2[kC];    // top two keys of pre-chunk nodes per chunk pod
    int16_t cd1c[kC], cd2c[kC];
    uint8_t cdbad[kC];
    union {
        struct {
            int32_t hk[kHash], hv[kHash];
        } h;
        struct {
            uint64_t k[kWaves][kC][2];
            int16_t c[kWaves][kC][2];  // k[.][.][1] == ~0: the lane met an unknown state
        } x;
    } u;
    int32_t ncid, nbc, cut, fc[2], fs[2];
#ifdef KS_CHUNK_DIAG
    int8_t why[kB];  // stop reason of a code-1 decision
#endif
};
static_assert(sizeof(ChShared) <= 160 * 1024, "LDS");

// Replays cid k: its final binds (pods < c0), then — `chunk` — the current sweep's chunk binds,
// with the pre-batch expiry slots of k (E cids) and each admitted running bind's own expiry, in
// pod order.  Stores the state segments for pods [from, i_end) in slot sl (sl < 0: none), writes
// adm[] of every bind (`wadm`), returns the state before pod i_end binds.
__device__ NS32 replay(ChShared& sh, int k, int n_e, bool chunk, int c0, int from, int sl, int i_end, bool wadm) {
    NS32 v;
    v.ac = sh.rs[0][k]; v.am = sh.rs[1][k]; v.ag = sh.rs[2][k]; v.ap = sh.rs[3][k];
    v.rc = sh.rd[0][k]; v.rm = sh.rd[1][k]; v.rg = sh.rd[2][k]; v.nr = sh.rd[3][k];
    v.taint = 0; v.label = 0;
    int e_u = 0, e_end = 0;
    if (k < n_e) { e_u = sh.eoff[k]; e_end = sh.eoff[k + 1]; }
    // pending own expiries: fixed register slots (eff INT_MAX = empty), no dynamic indexing
    int pe[kPend], pj[kPend];
#pragma unroll
    for (int q = 0; q < kPend; ++q) { pe[q] = INT_MAX; pj[q] = 0; }
    bool lost = false;
    int ns = 0, last_t = -1, ovf = kNoSeg;
    auto store = [&](int t) {
        if (sl < 0) return;
        t = t < from ? from : t;
        if (t >= i_end || t >= ovf) return;
        if (t != last_t) {
            if (ns == kSeg) { ovf = t; return; }
            sh.seff[sl][ns] = (int16_t)t;
            ++ns;
            last_t = t;
        }
        int32_t* d = sh.sst[sl][ns - 1];
        d[0] = v.rc; d[1] = v.rm; d[2] = v.rg; d[3] = v.nr;
    };
    if (sl >= 0) {
        for (int q = 0; q < kSeg; ++q) sh.seff[sl][q] = kNoSeg;
        store(from);
    }
    auto advance = [&](int t) {  // apply every event effective at pods <= t
        for (;;) {
            const int ne = e_u < e_end ? sh.xeff[sh.eslot[e_u]] : INT_MAX;
            int pq = 0, pm = INT_MAX;
#pragma unroll
            for (int q = 0; q < kPend; ++q)
                if (pe[q] < pm) { pm = pe[q]; pq = q; }
            const int nx = ne < pm ? ne : pm;
            if (nx > t) break;
            if (ne == nx) {
                const int x = sh.eslot[e_u++];
                v.rc -= sh.xreq[0][x]; v.rm -= sh.xreq[1][x]; v.rg -= sh.xreq[2][x]; v.nr -= 1;
            } else {
                int jq = 0;
#pragma unroll
                for (int q = 0; q < kPend; ++q)
                    if (q == pq) { jq = pj[q]; pe[q] = INT_MAX; }
                const PodRec& p = sh.pod[jq];
                v.rc -= (int32_t)p.req[0]; v.rm -= (int32_t)p.req[1]; v.rg -= (int32_t)p.req[2]; v.nr -= 1;
            }
            store(nx);
        }
    };
    int j = sh.fhead[k];
    uint64_t m = chunk ? sh.cmask[k] : 0ull;
    for (;;) {
        int jb;
        if (j >= 0) { jb = j; j = sh.fnext[j]; }
        else if (m) { jb = c0 + __builtin_ctzll(m); m &= m - 1; }
        else break;
        if (jb >= i_end) break;
        advance(jb);
        const PodRec& p = sh.pod[jb];
        const bool ok = !lost && fits32(p, v);
        if (wadm) sh.adm[jb] = lost ? 2 : (ok ? 1 : 0);
        if (ok && (sh.clfl[jb] & kFlRun)) {
            v.rc += (int32_t)p.req[0]; v.rm += (int32_t)p.req[1]; v.rg += (int32_t)p.req[2]; v.nr += 1;
            store(jb + 1);
            const int x = sh.own[jb];
            if (x >= 0) {
                const int ex = sh.xeff[x];
                bool placed = false;
#pragma unroll
                for (int q = 0; q < kPend; ++q)
                    if (!placed && pe[q] == INT_MAX) { pe[q] = ex; pj[q] = jb; placed = true; }
                if (!placed) {  // untracked: the state is unknown from the next pod on
                    lost = true;
                    if (jb + 1 < ovf) ovf = jb + 1;
                }
            }
        }
    }
    advance(i_end - 1);
    if (sl >= 0) sh.sovf[sl] = (int16_t)ovf;
    return v;
}

// state of slot sl's node at pod i (i >= the slot's first segment)
__device__ __forceinline__ int seg_of(const ChShared& sh, int sl, int i) {
    int s = 0;
#pragma unroll
    for (int q = 1; q < kSeg; ++q) s += sh.seff[sl][q] <= i;
    return s;
}

template <int kMode>
__device__ __forceinline__ uint64_t key_on(const EngineArgs& a, const ChShared& sh, int i, int k, int sl) {
    const int s = seg_of(sh, sl, i);
    NS32 n;
    n.ac = sh.rs[0][k]; n.am = sh.rs[1][k]; n.ag = sh.rs[2][k]; n.ap = sh.rs[3][k];
    n.rc = sh.sst[sl][s][0]; n.rm = sh.sst[sl][s][1]; n.rg = sh.sst[sl][s][2]; n.nr = sh.sst[sl][s][3];
    n.taint = sh.rt[k]; n.label = sh.rl[k];
    return make_key(eval_t<kMode>(a.c, sh.pod[i], n), (uint32_t)sh.cnode[k]);
}

__device__ __forceinline__ uint64_t cl_key(const ChShared& sh, uint32_t e) {
    return ((uint64_t)(e & 0xFFFFu) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)sh.cnode[e >> 16]);
}

template <int kMode>
__global__ __launch_bounds__(kThreads) void resolve_chunk_kernel(const EngineArgs* __restrict__ A) {
    __shared__ ChShared sh;
    const EngineArgs& a = A[0];
    const SweepWS& ws = *a.sw;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
    const int64_t start = a.ctr[kCtrStart], end = a.ctr[kCtrEnd];
    int nb = ws.nb;
    if (a.ctr[kCtrErr] != 0 || nb <= 0) return;
    const int n_e = ws.n_e, e_cnt = ws.e_cnt;

    // ---- setup: pods, window, candidate ids, records
    DG(uint64_t t_setup = dstamp(); uint64_t acc_cd = 0, acc_sw = 0, acc_fin = 0, acc_ph[4] = {0, 0, 0, 0}; int n_sweeps = 0, n_chunks = 0;)
    if (tid == 0) { sh.ncid = n_e; sh.nbc = nb; sh.cut = INT_MAX; sh.fc[0] = sh.fc[1] = INT_MAX; sh.fs[0] = sh.fs[1] = INT_MAX; }
    for (int h = tid; h < kHash; h += kThreads) sh.u.h.hk[h] = -1;
    if (tid < nb) {
        sh.pod[tid] = a.pods[start + tid];
        sh.win_hi[tid] = (int16_t)ws.win_hi[tid];
        sh.own[tid] = (int16_t)ws.own[tid];
        const int info = ws.cl_info[tid];
        sh.clcnt[tid] = (uint8_t)(info & 0xFF);
        sh.clfl[tid] = (a.dur[start + tid] > 0 ? kFlRun : 0) | ((info & kClTrunc) ? kFlTrunc : 0) |
                       ((info & kClFull) ? kFlFull : 0) | ((info & kClOvf) ? kFlOvf : 0);
        sh.thr[tid] = ws.cl_thr[tid];
        sh.adm[tid] = 0;
        sh.wf[tid] = -1;
        sh.w[0][tid] = -1; sh.w[1][tid] = -1;
        sh.code[0][tid] = 0; sh.code[1][tid] = 0;
    }
    for (int x = tid; x < e_cnt; x += kThreads) {
        sh.xreq[0][x] = clamp32(ws.ex_req[x][0]);
        sh.xreq[1][x] = clamp32(ws.ex_req[x][1]);
        sh.xreq[2][x] = clamp32(ws.ex_req[x][2]);
        sh.eslot[x] = (int16_t)ws.e_slot[x];
    }
    for (int k = tid; k <= n_e; k += kThreads) sh.eoff[k] = (int16_t)ws.e_off[k];
    __syncthreads();
    // slot x is applied from the first pod i >= 1 with win_hi[i] > x
    for (int i = tid + 1; i < nb; i += kThreads)
        for (int x = sh.win_hi[i - 1]; x < sh.win_hi[i]; ++x) sh.xeff[x] = (int16_t)i;
    // candidate ids: E nodes are cids 0 .. n_e - 1; then every list node, claimed by CAS
    auto insert = [&](int32_t node, int32_t val, int32_t* slot_out) -> bool {
        uint32_t h = hslot(node);
        for (int t = 0; t < kHash; ++t) {
            const int32_t prev = atomicCAS(&sh.u.h.hk[h], -1, node);
            if (prev == -1) { if (val >= 0) sh.u.h.hv[h] = val; *slot_out = (int)h; return true; }
            if (prev == node) { *slot_out = (int)h; return false; }
            h = (h + 1) & (kHash - 1);
        }
        *slot_out = -1;
        return false;
    };
    if (tid < n_e) {
        int32_t s;
        insert(ws.e_node[tid], tid, &s);
        sh.cnode[tid] = ws.e_node[tid];
    }
    __syncthreads();
    // each thread: pod i = tid / 4, entries (tid % 4) + 4 r
    int32_t eslot_of[kR / 4 + 1];
    bool claim[kR / 4 + 1];
    {
        const int i = tid >> 2;
        const int nc = i < nb ? sh.clcnt[i] : 0;
#pragma unroll
        for (int q = 0; q < kR / 4; ++q) {
            const int r = (tid & 3) + 4 * q;
            eslot_of[q] = -1;
            claim[q] = false;
            if (r < nc) {
                const int32_t node = key_node(ws.cl_key[i][r]);
                int32_t s;
                claim[q] = insert(node, -1, &s);
                eslot_of[q] = s;
                if (s < 0) atomicMin(&sh.nbc, i);  // hash full: cut the batch before this pod
            }
        }
    }
    __syncthreads();
    {
        const int i = tid >> 2;
#pragma unroll
        for (int q = 0; q < kR / 4; ++q)
            if (claim[q]) {
                const int c = atomicAdd(&sh.ncid, 1);
                sh.u.h.hv[eslot_of[q]] = c;
                if (c < kCid) sh.cnode[c] = sh.u.h.hk[eslot_of[q]];
                else atomicMin(&sh.nbc, i);
            }
    }
    __syncthreads();
    {
        const int i = tid >> 2;
        const int nc = i < nb ? sh.clcnt[i] : 0;
#pragma unroll
        for (int q = 0; q < kR / 4; ++q) {
            const int r = (tid & 3) + 4 * q;
            if (r < nc && eslot_of[q] >= 0) {
                const int c = sh.u.h.hv[eslot_of[q]];
                if (c >= kCid) atomicMin(&sh.nbc, i);
                else sh.cl[i][r] = ((uint32_t)c << 16) | (uint32_t)(ws.cl_key[i][r] >> 32);
            }
        }
    }
    __syncthreads();
    nb = sh.nbc < nb ? sh.nbc : nb;
    const int ncid = sh.ncid < kCid ? sh.ncid : kCid;
    for (int k = tid; k < ncid; k += kThreads) {
        const int32_t n = sh.cnode[k];
        const NodeV v = load_node(a.s, n);
        sh.rs[0][k] = (int32_t)v.ac; sh.rs[1][k] = (int32_t)v.am; sh.rs[2][k] = (int32_t)v.ag; sh.rs[3][k] = clamp32(v.ap);
        sh.rd[0][k] = (int32_t)v.rc; sh.rd[1][k] = (int32_t)v.rm; sh.rd[2][k] = (int32_t)v.rg; sh.rd[3][k] = (int32_t)v.nr;
        sh.rt[k] = v.taint; sh.rl[k] = v.label;
        sh.cmask[k] = 0;
        sh.fhead[k] = -1; sh.ftail[k] = -1;
    }
    __syncthreads();

    // ---- chunks
    DG(t_setup = dstamp() - t_setup;)
    int committed = nb, stop_code = 0;
    for (int c0 = 0; c0 < nb; c0 += kC) {
        const int c1 = nb < c0 + kC ? nb : c0 + kC;
        DG(uint64_t t0 = dstamp(); ++n_chunks;)
        // (1) pre-chunk nodes: replay each over [c0, c1) into its first final binder's slot, then
        // per chunk pod the top two keys (lane = pod, waves over nodes)
        if (c0 > 0) {
            if (tid < c0) {
                const int k = sh.wf[tid];
                if (k >= 0 && sh.fhead[k] == tid) (void)replay(sh, k, n_e, false, c0, c0, tid, c1, false);
            }
            __syncthreads();
            {
                const int i = c0 + lane;
                uint64_t k1 = 0, k2 = 0;
                int16_t q1 = -1, q2 = -1;
                bool bad = false;
                for (int j = wave; j < c0; j += kWaves) {
                    const int k = sh.wf[j];
                    if (k < 0 || sh.fhead[k] != j) continue;
                    if (i < c1) {
                        if (sh.sovf[j] <= i) {
                            bad = true;
                        } else {
                            const uint64_t key = key_on<kMode>(a, sh, i, k, j);
                            if (key > k1) { k2 = k1; q2 = q1; k1 = key; q1 = (int16_t)k; }
                            else if (key > k2) { k2 = key; q2 = (int16_t)k; }
                        }
                    }
                }
                sh.u.x.k[wave][lane][0] = k1; sh.u.x.k[wave][lane][1] = bad ? ~0ull : k2;
                sh.u.x.c[wave][lane][0] = q1; sh.u.x.c[wave][lane][1] = q2;
            }
            __syncthreads();
            if (wave == 0) {
                uint64_t k1 = 0, k2 = 0;
                int16_t q1 = -1, q2 = -1;
                bool bad = false;
                for (int g = 0; g < kWaves; ++g) {
                    if (sh.u.x.k[g][lane][1] == ~0ull) { bad = true; continue; }
#pragma unroll
                    for (int z = 0; z < 2; ++z) {
                        const uint64_t key = sh.u.x.k[g][lane][z];
                        const int16_t q = sh.u.x.c[g][lane][z];
                        if (key > k1) { k2 = k1; q2 = q1; k1 = key; q1 = q; }
                        else if (key > k2) { k2 = key; q2 = q; }
                    }
                }
                sh.cd1[lane] = k1; sh.cd2[lane] = k2; sh.cd1c[lane] = q1; sh.cd2c[lane] = q2; sh.cdbad[lane] = bad;
            }
        } else if (tid < kC) {
            sh.cd1[tid] = 0; sh.cd2[tid] = 0; sh.cd1c[tid] = -1; sh.cd2c[tid] = -1; sh.cdbad[tid] = 0;
        }
        __syncthreads();

        // (2) sweeps
        DG(uint64_t t1 = dstamp(); acc_cd += t1 - t0;)
        int par = 0, lo = c0, fsv = INT_MAX;
        for (;;) {
            DG(++n_sweeps; uint64_t q0 = dstamp();)
            // A: the guesses' chunk binds
            int wold = -1;
            if (tid < kC) {
                const int i = c0 + tid;
                if (i < c1) {
                    wold = sh.w[par][i];
                    if (wold >= 0) atomicOr((unsigned long long*)&sh.cmask[wold], 1ull << tid);
                }
            }
            __syncthreads();
            DG(uint64_t q1 = dstamp(); acc_ph[0] += q1 - q0;)
            // B: replay each chunk node (its first chunk binder's thread) into that pod's slot
            if (wold >= 0 && __builtin_ctzll(sh.cmask[wold]) == tid)
                (void)replay(sh, wold, n_e, true, c0, c0, c0 + tid, c1, true);
            __syncthreads();
            DG(uint64_t q2 = dstamp(); acc_ph[1] += q2 - q1;)
            // C: pod i = c0 + tid / 16, 16 lanes each
            {
                const int pi = tid >> 4, sub = tid & 15, rowsh = lane & ~15;
                const int i = c0 + pi;
                const bool act = i < c1 && i >= lo;
                const uint64_t below = (1ull << pi) - 1ull;
                bool f0 = false, f1 = false;
                uint32_t e0 = 0, e1 = 0;
                if (act) {
                    const int nc = sh.clcnt[i];
                    if (sub < nc) {
                        e0 = sh.cl[i][sub];
                        const int c = e0 >> 16;
                        f0 = sh.fhead[c] < 0 && (sh.cmask[c] & below) == 0;
                    }
                    if (sub + 16 < nc) {
                        e1 = sh.cl[i][sub + 16];
                        const int c = e1 >> 16;
                        f1 = sh.fhead[c] < 0 && (sh.cmask[c] & below) == 0;
                    }
                }
                const uint32_t r0 = (uint32_t)(__ballot(f0) >> rowsh) & 0xFFFFu;
                const uint32_t r1 = (uint32_t)(__ballot(f1) >> rowsh) & 0xFFFFu;
                const int rfree = r0 ? __builtin_ctz(r0) : (r1 ? 16 + __builtin_ctz(r1) : kR);
                const uint32_t efree = r0 ? (uint32_t)__shfl((int)e0, rowsh + rfree)
                                          : (r1 ? (uint32_t)__shfl((int)e1, rowsh + rfree - 16) : 0u);
                uint64_t dk = 0;
                int dc = -1;
                bool bad = false;
                if (act) {
                    for (int jj = sub; jj < pi; jj += 16) {
                        const int j = c0 + jj;
                        const int k = sh.w[par][j];
                        if (k < 0 || __builtin_ctzll(sh.cmask[k]) != jj) continue;
                        if (sh.sovf[j] <= i) { bad = true; continue; }
                        const uint64_t key = key_on<kMode>(a, sh, i, k, j);
                        if (key > dk) { dk = key; dc = k; }
                    }
                    if (sub == 0) {  // pre-chunk nodes: the best one not rebound before pod i
                        if (sh.cdbad[pi]) {
                            bad = true;
                        } else {
                            uint64_t ck = sh.cd1[pi];
                            int cc = sh.cd1c[pi];
                            if (ck != 0 && (sh.cmask[cc] & below)) {
                                ck = sh.cd2[pi];
                                cc = sh.cd2c[pi];
                                if (ck != 0 && (sh.cmask[cc] & below)) bad = true;
                            }
                            if (ck > dk) { dk = ck; dc = cc; }
                        }
                    }
                }
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const uint64_t ok = shfl_xor64(dk, o);
                    const int oc = __shfl_xor(dc, o);
                    if (ok > dk) { dk = ok; dc = oc; }
                }
                bad = ((__ballot(bad) >> rowsh) & 0xFFFFu) != 0;
                if (sub == 0 && i < c1) {
                    int code;
                    int nw;
                    if (act) {
                        const uint8_t fl = sh.clfl[i];
                        uint64_t win = 0;
                        int wc = -1;
                        code = 0;
                        if (bad || (fl & kFlOvf)) {
                            code = 1;
                            DG(sh.why[i] = bad ? 0 : 1;)
                        } else if (rfree < kR) {
                            const uint64_t sk = cl_key(sh, efree);
                            if (sk > dk) { win = sk; wc = (int)(efree >> 16); }
                            else { win = dk; wc = dc; }
                        } else if (fl & kFlTrunc) {  // kept entries all bound: D must beat the last kept
                            if (dk > cl_key(sh, sh.cl[i][kR - 1])) { win = dk; wc = dc; }
                            else { code = 1; DG(sh.why[i] = 2;) }
                        } else if (fl & kFlFull) {   // exhausted list: D must beat the list's last key
                            if (dk > sh.thr[i]) { win = dk; wc = dc; }
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
            if (wold >= 0) sh.cmask[wold] = 0;
            if (tid == 0) { sh.fc[par ^ 1] = INT_MAX; sh.fs[par ^ 1] = INT_MAX; }
            __syncthreads();
            DG(acc_ph[3] += dstamp() - q3;)
            par ^= 1;
            if (fcv == INT_MAX || fcv >= fsv) break;
            lo = fcv + 1;
        }
        if (tid == 0) { sh.fc[0] = sh.fc[1] = INT_MAX; sh.fs[0] = sh.fs[1] = INT_MAX; }
        DG(uint64_t t2 = dstamp(); acc_sw += t2 - t1;)

        // (3) finalize the chunk's prefix [c0, cend): admissions known, final bind lists
        int cend = fsv < c1 ? fsv : c1;
        if (tid < kC) {
            const int i = c0 + tid;
            if (i < cend && sh.adm[i] == 2) atomicMin(&sh.cut, i);
        }
        __syncthreads();
        const bool cut = sh.cut < cend;
        if (cut) cend = sh.cut;
        int wk = -1;
        if (tid < kC) {
            const int i = c0 + tid;
            if (i < cend) {
                wk = sh.w[par][i];
                sh.wf[i] = (int16_t)wk;
                if (wk >= 0) atomicOr((unsigned long long*)&sh.cmask[wk], 1ull << tid);
            }
        }
        __syncthreads();
        if (wk >= 0 && __builtin_ctzll(sh.cmask[wk]) == tid) {
            uint64_t m = sh.cmask[wk];
            int tail = sh.ftail[wk];
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
        if (wk >= 0) sh.cmask[wk] = 0;
        __syncthreads();
        DG(acc_fin += dstamp() - t2;)
        if (cend < c1) {
            committed = cend;
            stop_code = cut ? 1 : sh.code[par][cend];
#ifdef KS_CHUNK_DIAG
            if (tid == 0) {
                unsigned long long* d = (unsigned long long*)a.ctr;
                const int r = cut ? 4 : (stop_code == 1 ? sh.why[cend] : 5);
                atomicAdd(&d[9 + r], 1ull);
            }
#endif
            break;
        }
    }
    DG(uint64_t t3 = dstamp();)

    // ---- commit pods [0, c): outputs, expiry marks, node state write-back
    const int c = committed;
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
    for (int x = tid; x < h_end; x += kThreads)
        if (ws.ex_ok[x]) gptr(a.expired)[ws.ex_q[x]] = 1;
    for (int k = tid; k < ncid; k += kThreads) {
        if (k < n_e || sh.fhead[k] >= 0) {
            const NS32 v = replay(sh, k, n_e, false, 0, 0, -1, c, false);
            const int32_t n = sh.cnode[k];
            a.s.rc[n] = v.rc; a.s.rm[n] = v.rm; a.s.rg[n] = v.rg; a.s.nr[n] = v.nr;
        }
        if (k < n_e) a.e_idx[sh.cnode[k]] = -1;
    }
    if (tid == 0) {
        a.ctr[kCtrStart] = start + c;
        const bool err = stop_code == 2 || stop_code == 3;
        if (err) {
            a.ctr[kCtrErr] = stop_code == 2 ? kErrNotFound : kErrEinval;
            a.ctr[kCtrErrPod] = start + c;
        }
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
        atomicAdd(&d[22], (unsigned long long)n_e);
        atomicAdd(&d[23], (unsigned long long)nb);
        for (int q = 0; q < 4; ++q) atomicAdd(&d[24 + q], acc_ph[q]);
    }
#endif
}

}  // namespace chk

hipError_t launch_sweep_prep(const EngineArgs* d, int max_slots, hipStream_t st);

hipError_t launch_resolve_chunk(const EngineArgs* d, int mode, hipStream_t st) {
    hipError_t r = launch_sweep_prep(d, kChSlots, st);
    if (r != hipSuccess) return r;
    switch (mode) {
        case kEvalMicro:
            hipLaunchKernelGGL(chk::chunk_cl_kernel<kEvalMicro>, dim3(kSweepMaxB), dim3(256), 0, st, d);
            hipLaunchKernelGGL(chk::resolve_chunk_kernel<kEvalMicro>, dim3(1), dim3(chk::kThreads), 0, st, d);
            break;
        case kEvalTiny:
            hipLaunchKernelGGL(chk::chunk_cl_kernel<kEvalTiny>, dim3(kSweepMaxB), dim3(256), 0, st, d);
            hipLaunchKernelGGL(chk::resolve_chunk_kernel<kEvalTiny>, dim3(1), dim3(chk::kThreads), 0, st, d);
            break;
        default:
            hipLaunchKernelGGL(chk::chunk_cl_kernel<kEvalNarrow>, dim3(kSweepMaxB), dim3(256), 0, st, d);
            hipLaunchKernelGGL(chk::resolve_chunk_kernel<kEvalNarrow>, dim3(1), dim3(chk::kThreads), 0, st, d);
            break;
    }
    return hipGetLastError();
}

}  // namespace ks
