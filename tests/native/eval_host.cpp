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
