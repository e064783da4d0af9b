// Host build of the engine's fused Filter+Score evaluator (ks_device.h), for CPU tests
// only: the same source the kernels inline, compiled for the host so its integer math can be
// checked against the oracle without a GPU.  Not part of the product.
#include "../../kubernetes-simulator_amd/csrc/ks_device.h"

extern "C" int ks_host_eval(const ks::Cfg* c, int64_t n, const int64_t* alloc /*[n][4]*/,
                            const int64_t* reqtot /*[n][3]*/, const int64_t* nrun, const uint64_t* taint,
                            const uint64_t* label, const ks::PodRec* pod, int64_t* score_out) {
    for (int64_t i = 0; i < n; i++) {
        ks::NodeV v;
        v.ac = alloc[i * 4 + 0]; v.am = alloc[i * 4 + 1]; v.ag = alloc[i * 4 + 2]; v.ap = alloc[i * 4 + 3];
        v.rc = reqtot[i * 3 + 0]; v.rm = reqtot[i * 3 + 1]; v.rg = reqtot[i * 3 + 2]; v.nr = nrun[i];
        v.taint = taint[i]; v.label = label[i];
        uint32_t t1 = ks::eval_total1(*c, *pod, v);
        score_out[i] = t1 ? (int64_t)t1 - 1 : -1;
    }
    return 0;
}
extern "C" int ks_host_lr(int64_t A, int64_t u) { return ks::lr_one(A, u); }
extern "C" int ks_host_ba(int64_t Ac, int64_t Am, int64_t uc, int64_t um) { return ks::ba_score(Ac, Am, uc, um); }
extern "C" int ks_host_lr_n(int32_t A, int32_t u) { return ks::lr_one_n(A, u); }
extern "C" int ks_host_ba_n(int32_t Ac, int32_t Am, int32_t uc, int32_t um) { return ks::ba_score_n(Ac, Am, uc, um); }

// batched forms for the CPU tests (tests/test_evaluator_host.py)
extern "C" void ks_host_lr_n_batch(int64_t n, const int32_t* A, const int32_t* u, int32_t* out) {
    for (int64_t i = 0; i < n; i++) out[i] = ks::lr_one_n(A[i], u[i]);
}
extern "C" void ks_host_ba_n_batch(int64_t n, const int32_t* Ac, const int32_t* Am, const int32_t* uc,
                                   const int32_t* um, int32_t* out) {
    for (int64_t i = 0; i < n; i++) out[i] = ks::ba_score_n(Ac[i], Am[i], uc[i], um[i]);
}
extern "C" void ks_host_ba_batch(int64_t n, const int64_t* Ac, const int64_t* Am, const int64_t* uc,
                                 const int64_t* um, int32_t* out) {
    for (int64_t i = 0; i < n; i++) out[i] = ks::ba_score(Ac[i], Am[i], uc[i], um[i]);
}
// per case: exact eval_total1 (wide and narrow) of pod req[i] on node i, and prune_tmax
extern "C" void ks_host_prune_batch(const ks::Cfg* c, int64_t n, const int64_t* alloc /*[n][4]*/,
                                    const int64_t* run /*[n][3]*/, const int64_t* req /*[n][3]*/,
                                    uint32_t* total1, uint32_t* total1_n, uint32_t* tmax, uint32_t* total1_t) {
    for (int64_t i = 0; i < n; i++) {
        ks::NodeV v{};
        v.ac = alloc[i * 4 + 0]; v.am = alloc[i * 4 + 1]; v.ag = alloc[i * 4 + 2]; v.ap = alloc[i * 4 + 3];
        v.rc = run[i * 3 + 0]; v.rm = run[i * 3 + 1]; v.rg = run[i * 3 + 2]; v.nr = 0;
        ks::PodRec p{};
        p.req[0] = req[i * 3 + 0]; p.req[1] = req[i * 3 + 1]; p.req[2] = req[i * 3 + 2];
        p.keymask = 0xFF;
        total1[i] = ks::eval_total1(*c, p, v);
        total1_n[i] = ks::eval_total1_narrow(*c, p, v);
        total1_t[i] = ks::eval_total1_tiny(*c, p, v);
        tmax[i] = ks::prune_tmax(*c, ks::prune_prep(*c, v), (float)p.req[0], (float)p.req[1]);
    }
}
// per case: the micro evaluator (capacities < 2^16, Ac*Am < 2^24) of pod req[i] on node i;
// tol/sel/taint/label exercise the filter masks
extern "C" void ks_host_micro_batch(const ks::Cfg* c, int64_t n, const int64_t* alloc /*[n][4]*/,
                                    const int64_t* run /*[n][4]: rc rm rg nr*/, const int64_t* req /*[n][3]*/,
                                    const uint32_t* keymask, const uint64_t* masks /*[n][4]: taint label tol sel*/,
                                    uint32_t* total1, uint32_t* total1_m) {
    for (int64_t i = 0; i < n; i++) {
        ks::NodeV v{};
        v.ac = alloc[i * 4 + 0]; v.am = alloc[i * 4 + 1]; v.ag = alloc[i * 4 + 2]; v.ap = alloc[i * 4 + 3];
        v.rc = run[i * 4 + 0]; v.rm = run[i * 4 + 1]; v.rg = run[i * 4 + 2]; v.nr = run[i * 4 + 3];
        v.taint = masks[i * 4 + 0]; v.label = masks[i * 4 + 1];
        ks::PodRec p{};
        p.req[0] = req[i * 3 + 0]; p.req[1] = req[i * 3 + 1]; p.req[2] = req[i * 3 + 2];
        p.keymask = keymask[i];
        p.tol = masks[i * 4 + 2]; p.sel = masks[i * 4 + 3];
        total1[i] = ks::eval_total1(*c, p, v);
        total1_m[i] = ks::eval_total1_micro(*c, p, v);
    }
}
// the same with the scan's form of the micro evaluator (per-pod ScanRec, per-node npen)
extern "C" void ks_host_scan_micro_batch(const ks::Cfg* c, int64_t n, const int64_t* alloc, const int64_t* run,
                                         const int64_t* req, const uint32_t* keymask, const uint64_t* masks,
                                         uint32_t* total1_s) {
    for (int64_t i = 0; i < n; i++) {
        ks::NodeV v{};
        v.ac = alloc[i * 4 + 0]; v.am = alloc[i * 4 + 1]; v.ag = alloc[i * 4 + 2]; v.ap = alloc[i * 4 + 3];
        v.rc = run[i * 4 + 0]; v.rm = run[i * 4 + 1]; v.rg = run[i * 4 + 2]; v.nr = run[i * 4 + 3];
        v.taint = masks[i * 4 + 0]; v.label = masks[i * 4 + 1];
        ks::PodRec p{};
        p.req[0] = req[i * 3 + 0]; p.req[1] = req[i * 3 + 1]; p.req[2] = req[i * 3 + 2];
        p.keymask = keymask[i];
        p.tol = masks[i * 4 + 2]; p.sel = masks[i * 4 + 3];
        total1_s[i] = ks::eval_scan_micro(*c, ks::scan_rec_micro(*c, p), v, ks::scan_npen(*c, v));
    }
}
