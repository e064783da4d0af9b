/*
 * ks_ingest.h — host ingest of the reference's wire formats into the engine's int64 / bitmask
 * records.  Plain C, no device needed; part of libks_engine.so.
 *
 * What each entry point replaces in the reference (wangchen615/kubernetes-simulator):
 *   ks_parse_quantity ........ resource.ParseQuantity (vendor/k8s.io/apimachinery/pkg/api/
 *                              resource/quantity.go:146-377) + Quantity.MilliValue
 *   ks_parse_simspec ......... parseSpecYAML + util.BuildResourceList (kubesim/pod/spec.go:35-63,
 *                              kubesim/util/util.go:11-23)
 *   ks_cluster_parse ......... the cluster config viper reads (kubesim/config/config.go:15-41,
 *                              kubesim/kubesim.go:228-251) and BuildNode / buildTaint
 *                              (kubesim/config/config.go:44-110)
 *   ks_cluster_tolerations ... Toleration.ToleratesTaint over the cluster's taint dictionary
 *                              (vendor/k8s.io/api/core/v1/toleration.go:37-56)
 *   ks_cluster_selector ...... nodeSelector pairs over the cluster's label dictionary
 *
 * Status codes: KS_EINVAL = what the reference rejects (ErrFormatWrong / ErrNumeric / ErrSuffix,
 * errInvalidResourceUsageField, an unsupported taint effect, malformed YAML); KS_ERANGE = a valid
 * input outside the engine's exact domain (a quantity that is negative, not a whole number of
 * milli-units or >= 2^63 milli-units; a simSpec resource other than cpu / memory / nvidia.com/gpu;
 * more than 64 NoSchedule/NoExecute taints or 63 label pairs — or, sealed with the pods noted,
 * more than 64 toleration classes or 63 referenced pairs; a pod the seal did not see that splits a
 * class or names an unreferenced node pair).
 */
#ifndef KS_INGEST_H
#define KS_INGEST_H
#include <stdint.h>

#include "ks_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Quantity string -> exact milli-units (>= 0). */
ks_status ks_parse_quantity(const char* s, int64_t* milli_out);

/* simSpec annotation (a YAML list of {seconds: int32, resourceUsage: {name: quantity}}) ->
 * n phases: seconds[i], usage[i][3] (milli cpu, memory, nvidia.com/gpu; 0 when absent),
 * usage_mask[i] (1 cpu, 2 memory, 4 gpu).  At most max_phases are written; *n_phases is the
 * total.  err (may be NULL) receives a message. */
ks_status ks_parse_simspec(const char* yaml, int32_t max_phases, int32_t* n_phases, int32_t* seconds,
                           int64_t* usage, uint8_t* usage_mask, char* err, int32_t err_len);

/* Cluster config YAML (config/sample.yml schema).  The parsed cluster holds, in config order
 * (node index = config order, the engine's tie-break order): alloc[n][4] = {milli cpu, milli
 * memory, milli nvidia.com/gpu (-1 absent), Capacity.Pods().Value() (0 absent)}, the dictionary
 * masks of each node's NoSchedule/NoExecute taints and of its labels, and "namespace/name". */
typedef struct ks_cluster ks_cluster;
ks_status ks_cluster_parse(const char* yaml, ks_cluster** out, char* err, int32_t err_len);

/* The two-phase form for clusters past one 64-bit mask (a unique kubernetes.io/hostname label per
 * node, hundreds of taints): parse with KS_CLUSTER_DEFER_MASKS, note every pod's tolerations and
 * nodeSelector (ks_cluster_note_pod, the same strings ks_cluster_tolerations / _selector take),
 * then ks_cluster_seal.  The seal gives bits only to label pairs some noted selector references and
 * one bit per class of taints the same noted toleration lists tolerate — exact for every noted pod
 * (toleration.go:37-56 decides identically on interchangeable taints; an unreferenced label cannot
 * change a placement).  A cluster that fits one mask seals to the plain one-bit-per-entry encoding
 * ks_cluster_parse gives.  Until sealed, ks_cluster_arrays / _tolerations / _selector return
 * KS_EINVAL.  Replaces nothing in the reference (its maps hold any number of entries): it is how
 * the masks reach the reference's domain. */
#define KS_CLUSTER_DEFER_MASKS 1
ks_status ks_cluster_parse_ex(const char* yaml, int32_t flags, ks_cluster** out, char* err, int32_t err_len);
ks_status ks_cluster_note_pod(ks_cluster* c, int32_t n_tol, const char* const* key, const char* const* op,
                              const char* const* value, const char* const* effect, int32_t n_sel,
                              const char* const* sel_key, const char* const* sel_value);
ks_status ks_cluster_seal(ks_cluster* c, char* err, int32_t err_len);
void ks_cluster_free(ks_cluster* c);
int64_t ks_cluster_nodes(const ks_cluster* c);
int32_t ks_cluster_tick(const ks_cluster* c);          /* `tick`, default 10 (kubesim.go:239) */
const char* ks_cluster_start_clock(const ks_cluster* c); /* `startClock` as written, "" if absent */
ks_status ks_cluster_arrays(const ks_cluster* c, int64_t* alloc, uint64_t* taint, uint64_t* label);
const char* ks_cluster_node_name(const ks_cluster* c, int64_t i);

/* Pod tolerations -> the mask of dictionary taints they tolerate (ks_submit_pods `tol`).
 * Toleration i: key[i], op[i] ("" / "Equal" / "Exists"; anything else tolerates nothing),
 * value[i], effect[i] ("" = every effect).  NULL strings are "". */
ks_status ks_cluster_tolerations(const ks_cluster* c, int32_t n, const char* const* key, const char* const* op,
                                 const char* const* value, const char* const* effect, uint64_t* tol_out);
/* nodeSelector pairs -> `sel` mask; a pair no node carries sets bit 63 (infeasible everywhere). */
ks_status ks_cluster_selector(const ks_cluster* c, int32_t n, const char* const* key, const char* const* value,
                              uint64_t* sel_out);

#ifdef __cplusplus
}
#endif
#endif
