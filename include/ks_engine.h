/*
 * ks_engine.h — C-ABI of the MI355X-native kubesim scheduling engine.
 *
 * This is the boundary a kubesim host binds (cgo / ctypes / JNI).
 * Plain C types only: caller-owned host buffers are copied in, outputs go to
 * caller-allocated buffers with explicit lengths, device state is owned by the opaque
 * handle.  A handle is single-threaded (not re-entrant), like the reference's
 * single-goroutine Run loop (kubesim/kubesim.go:101-122).
 *
 * What each entry point replaces in the reference (wangchen615/kubernetes-simulator):
 *   ks_create / ks_load_nodes ... NewKubeSim node construction (kubesim/kubesim.go:32-61,
 *                                 kubesim/config/config.go:44-90, kubesim/node/node.go:22-27)
 *   ks_submit_pods .............. submit + podQueue.append (kubesim/kubesim.go:126-139,
 *                                 kubesim/podqueue.go:18-23); api.Submitter output
 *                                 (api/submitter.go:15) with its arrival tick
 *   ks_step ..................... Run's tick loop + scheduleOne (kubesim/kubesim.go:90-166):
 *                                 Filter (:168-188), Score + argmax (:190-225),
 *                                 Node.CreatePod (kubesim/node/node.go:36-60)
 *   ks_filter ................... api.Filter.Filter for every node (api/scheduler.go:19)
 *   ks_score .................... api.Scorer.Score aggregated over the registered scorers
 *                                 (api/scheduler.go:36, kubesim/kubesim.go:193-206)
 *   ks_usage / ks_usage_at ...... Σ Pod.ResourceUsage(clock) per node (kubesim/pod/pod.go:47-63)
 *   ks_usage_digest ............. the same for every tick of a window, as a fingerprint
 *   ks_pod_status ............... Pod.BuildStatus phase / times (kubesim/pod/pod.go:78-167)
 *   ks_pod_lookup / ks_node_pods  Node.GetPod / GetPodStatus / GetPodList (kubesim/node/node.go:62-93)
 *   ks_group_* .................. one KubeSim.Run per what-if scenario, stepped together
 *   ks_last_error ............... the error text Run would return
 *
 * Status codes map 1:1 onto the reference's error kinds (strongerrors):
 *   KS_EINVAL    InvalidArgument (bad names, bad simSpec, bad quantities, bad config)
 *   KS_ENOTFOUND NotFound — no node selected; the run stops exactly as kubesim.go:217-220
 *   KS_EDEVICE   HIP / RCCL failure (no reference counterpart)
 * After KS_ENOTFOUND or a bind-time KS_EINVAL the run is aborted: later ks_step calls return
 * the same code, as Run would have returned.  A KS_EDEVICE from ks_step / ks_group_step is
 * sticky too (the engine's tick and binds stay at the last completed step).
 *
 * Units: cpu, memory and nvidia.com/gpu quantities are int64 milli-units (exact for every
 * resource.Quantity that is a whole number of milli-units); the pods capacity is
 * Capacity.Pods().Value() (a count; absent ⇒ 0).  An absent cpu / memory / gpu capacity key
 * is -1.  All inputs must be non-negative and below 2^59.
 */
#ifndef KS_ENGINE_H
#define KS_ENGINE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KS_ABI_VERSION 2  /* 2: ks_submit_pods takes key_id */

typedef enum {
    KS_OK = 0,
    KS_EINVAL = 1,
    KS_ENOTFOUND = 2,
    KS_EDEVICE = 3,
    KS_ENOMEM = 4,
    KS_ERANGE = 5,  /* valid input outside the engine's exact domain (ks_ingest.h) */
} ks_status;

/* filter_mode: the reference discards the Filter result (kubesim/kubesim.go:182) —
 * REFERENCE_LITERAL reproduces that; FEEDS_SCORE lets the filters gate the candidates. */
enum { KS_FILTER_REFERENCE_LITERAL = 0, KS_FILTER_FEEDS_SCORE = 1 };
/* filters (bitmask) */
enum { KS_FILTER_FIT = 1, KS_FILTER_TAINT = 2, KS_FILTER_SELECTOR = 4 };
/* scorers: CONST returns `value` for every node (examples/main.go:147-155 with value 1);
 * LEAST_REQUESTED / BALANCED are the integer forms of SURVEY.md §8(a14). */
enum { KS_SCORER_CONST = 0, KS_SCORER_LEAST_REQUESTED = 1, KS_SCORER_BALANCED = 2 };
/* bind status (kubesim/pod/pod.go:20-27) */
enum { KS_POD_OK = 0, KS_POD_OVER_CAPACITY = 1 };
/* per-pod flags: the pod will fail at bind with InvalidArgument
 * (empty namespace/name: kubesim/node/node.go:133-143; bad simSpec: kubesim/pod/pod.go:31-39) */
enum { KS_PODFLAG_BAD_KEY = 1, KS_PODFLAG_BAD_SPEC = 2 };

typedef struct {
    int32_t kind;   /* KS_SCORER_* */
    int32_t weight; /* >= 0 */
    int32_t value;  /* CONST only, >= 0 */
} ks_scorer;
/* ks_create rejects (KS_EINVAL) a scorer set whose maximum total
 * sum(weight*value) + 10*sum(weight of LR/BA) is >= 2^30 - 2. */

typedef struct {
    int32_t abi_version;  /* KS_ABI_VERSION */
    int32_t tick_seconds; /* config `tick` (kubesim/kubesim.go:239), >= 1 */
    int32_t filter_mode;  /* KS_FILTER_REFERENCE_LITERAL / KS_FILTER_FEEDS_SCORE */
    uint32_t filters;     /* KS_FILTER_* bits */
    int32_t n_scorers;    /* 0..8; registration order */
    ks_scorer scorers[8];
    int32_t device;       /* HIP device ordinal */
    int32_t batch_pods;   /* pods resolved per scan (0 = default) */
    uint32_t engine_flags; /* KS_ENGINE_* */
    int32_t reserved[7];
} ks_config;

/* engine_flags: the engine picks the narrowest exact evaluator the scaled capacities allow
 * (micro 24-bit / tiny int32 / narrow 32x32->64 / wide 64/128-bit).  FORCE_WIDE keeps the wide
 * one, NO_TINY skips tiny and micro, NO_MICRO skips micro; all are exact, the flags exist to test
 * them against each other. */
enum { KS_ENGINE_FORCE_WIDE = 1, KS_ENGINE_NO_TINY = 2, KS_ENGINE_NO_MICRO = 4,
       /* resolvers for batches of clusters above the small class (both give the same binds; the
        * flags exist to test them against each other): ONE_POD = the role-split one-pod-per-
        * barrier resolver; CHUNK = chunked Jacobi sweeps in one workgroup's LDS (ks_step only,
        * evaluator modes >= narrow, totals < 2^16).  Bits 16, 32 and 128 (the retired pair, sweep
        * and sequential resolvers) are rejected.
        * NO_OVERLAP: the chunk resolver's batches run the plain chain (each batch's scan before its
        * resolve) instead of fusing the next batch's speculative scan into the resolve launch — the
        * same binds; for A/B timing and to test the two chains against each other. */
       KS_ENGINE_ONE_POD_RESOLVER = 8, KS_ENGINE_CHUNK_RESOLVER = 64, KS_ENGINE_NO_OVERLAP = 256,
       /* PRUNED_LISTS: the scan writes a block's top-L list only when it can reach the pod's global
        * top-L (a running per-pod threshold) and the merge reads only those — the default for chunk-
        * resolver clusters of >= 1,024 scan blocks (262,144 nodes); the flag forces it at every size
        * (same binds; to test the two list forms against each other). */
       KS_ENGINE_PRUNED_LISTS = 512 };

typedef struct {
    int64_t pod;    /* FIFO index (submission order) */
    int32_t node;   /* node index (ks_load_nodes order) */
    int32_t status; /* KS_POD_* */
    int64_t tick;   /* bind tick (clock = start + tick * tick_seconds) */
} ks_bind;

typedef struct ks_engine ks_engine;

ks_status ks_create(const ks_config* cfg, ks_engine** out);
void ks_destroy(ks_engine* eng);

/* Scenario groups (BASELINE.json configs[3]: independent what-if clusters × pod traces).  A
 * group owns a stream and up to max_scenarios engines created with ks_group_add (same device and
 * batch size; ks_load_nodes / ks_submit_pods / ks_usage / ks_filter / ks_score / ks_step work on
 * them as on any engine).  ks_group_step advances every member by `ticks` ticks with one launch
 * per kernel for all of them (scenario = a grid dimension, one resolve workgroup each) — the
 * reference would run one KubeSim.Run per scenario (kubesim/kubesim.go:90-123).  Per member i:
 * binds into out[i * cap ...] (out may be NULL), their count in n_out[i] and the member's status
 * in status_out[i] (an aborting error stops only that scenario).  Members are destroyed with the
 * group (ks_destroy on a member is a no-op).  stats (may be NULL): device ms of the whole step,
 * batch rounds, pods bound. */
typedef struct ks_group ks_group;
ks_status ks_group_create(int32_t device, int32_t max_scenarios, ks_group** out);
void ks_group_destroy(ks_group* g);
ks_status ks_group_add(ks_group* g, const ks_config* cfg, ks_engine** out);
int32_t ks_group_size(const ks_group* g);

/* Node sharding across ranks (the reference's argmax over all nodes,
 * kubesim/kubesim.go:208-222, becomes an exact merge of per-shard candidate lists).  One
 * process per GPU; every rank loads the whole cluster and submits the same pods, scans only its
 * contiguous node range, and all-gathers the per-pod top-L candidates once per batch over RCCL.
 * Binds are identical on every rank.  Call on every rank before ks_load_nodes; rank 0 creates
 * the communicator id with ks_comm_unique_id and the host broadcasts it (any channel).
 * vshards > 1 splits each rank's range further (same merge path; lets one GPU test it).
 * id may be NULL when world == 1 (no communicator). */
/* The layout ks_load_nodes and ks_step use for n_nodes over world ranks x vshards parts:
 * part_lo_out[world * vshards + 1] = first 256-node scan block of each part (the last entry = the
 * block count); rank r scans parts [r * vshards, (r + 1) * vshards).  Exchange: part p's per-pod
 * top-L keys fill cand_all[p][B][L]; rank r's parts are one contiguous all-gather slice; the
 * second merge reads cand_all[p][b][*] for every part p.  Pure host function (no device). */
ks_status ks_shard_layout(int64_t n_nodes, int32_t world, int32_t vshards, int32_t* part_lo_out);
/* The second merge on the host: out[B][L] = exact top-L over parts of cand_all[parts][B][L]
 * (each list sorted descending, 0-padded) — the device merge's per-list step (topl_insert,
 * ks_device.h), for checking an exchange without a GPU.  Pure host function. */
ks_status ks_merge_candidates(const uint64_t* cand_all, int32_t parts, int32_t B, uint64_t* out);
#define KS_COMM_ID_BYTES 128
ks_status ks_comm_unique_id(uint8_t* id_out /* [KS_COMM_ID_BYTES] */);
ks_status ks_shard(ks_engine* eng, int32_t world, int32_t rank, const uint8_t* id, int32_t vshards);
/* The same sharding with a host exchange instead of RCCL (no communicator): at every batch the
 * engine copies this rank's parts of cand_all[G][B][L] to host memory and calls fn with a buffer of
 * world x bytes_per_rank bytes (rank-major, this rank's slice filled); fn must fill the other
 * ranks' slices (an all-gather) and return KS_OK, after which the whole array goes back to the
 * device.  For ranks that share no RCCL communicator: threads of one process on one or several
 * GPUs (ks_local_allgather, ks_kubesim.h), or any host transport.  Before ks_load_nodes. */
typedef ks_status (*ks_allgather_fn)(void* user, int32_t rank, int32_t world, void* buf, int64_t bytes_per_rank);
ks_status ks_shard_host(ks_engine* eng, int32_t world, int32_t rank, int32_t vshards, ks_allgather_fn fn,
                        void* user);

/* Load the cluster (once).  alloc[n][4] = {cpu, memory, nvidia.com/gpu, pods};
 * taint[n] = OR of dictionary bits of the node's NoSchedule/NoExecute taints;
 * label[n] = OR of dictionary bits of its (key,value) labels (W = 1). */
ks_status ks_load_nodes(ks_engine* eng, int64_t n, const int64_t* alloc, const uint64_t* taint,
                        const uint64_t* label);

/* Append m pods to the FIFO.  arrival_tick = the tick whose Submit call returned the pod
 * (non-decreasing; <= the current tick means "next tick").  req[m][3] container-summed
 * requests with keymask (1 cpu, 2 memory, 4 gpu); tol = dictionary taints tolerated; sel =
 * dictionary labels required (bit 63 = impossible); simSpec as CSR: phase_off[m+1],
 * phase_sec[Φ] (int32), phase_use[Φ][3]; flags = KS_PODFLAG_* (may be NULL).
 *
 * key_id[m] (>= 0; may be NULL: every pod its own key, key id = -(FIFO index) - 1, a namespace
 * no explicit key shares): the caller's interned
 * "namespace-name" pod key (kubesim/node/node.go:146-160).  Node.CreatePod stores the pod under
 * its key, replacing a same-key pod already stored on that node (node.go:58,
 * kubesim/pod/podmap.go:27-29); a replaced pod that is still running stops counting toward the
 * node's totals at that moment.  The engine keeps placements exact by refusing, with KS_ERANGE
 * and nothing appended, a pod whose key was used by an earlier pod that may still be running at
 * the new pod's bind tick (the only case in which the replacement can change a placement or a
 * usage; which node each lands on is not known at submit).  Reused keys of finished pods are
 * accepted and resolved exactly by ks_pod_lookup / ks_node_pods. */
ks_status ks_submit_pods(ks_engine* eng, int64_t m, const int64_t* arrival_tick,
                         const int64_t* req, const uint8_t* keymask, const uint64_t* tol,
                         const uint64_t* sel, const int32_t* phase_off, const int32_t* phase_sec,
                         const int64_t* phase_use, const uint8_t* flags, const int64_t* key_id);

/* Advance `ticks` ticks.  Writes up to `cap` binds to out (one per tick that had a queued
 * pod) and the number of binds made to *n_out.
 *
 * Domain: Pod.passedSeconds is int32(seconds since the pod's start) (kubesim/pod/pod.go:148-153);
 * past 2^31 s Go's conversion is implementation-defined and IsRunning (pod.go:67-69) may revive
 * finished pods.  A step that would take the clock 2^31 s or more past the run's first bind, and
 * a ks_submit_pods whose pods would bind there, are refused with KS_ERANGE (nothing changes). */
ks_status ks_step(ks_engine* eng, int64_t ticks, ks_bind* out, int64_t cap, int64_t* n_out);

/* Filter mask (all enabled filters) / aggregated score (-1 = no entry) of queued pod `pod`
 * against the cluster state at the current tick.  mask_out[n], score_out[n]. */
ks_status ks_filter(ks_engine* eng, int64_t pod, uint8_t* mask_out);
ks_status ks_score(ks_engine* eng, int64_t pod, int64_t* score_out);

/* usage_out[n][3]: Σ over pods on each node of ResourceUsage at the current tick. */
ks_status ks_usage(ks_engine* eng, int64_t* usage_out);

/* usage_out[n][3] at any past tick 0 <= t <= the current tick (Pod.ResourceUsage,
 * kubesim/pod/pod.go:47-63, sampled after tick t's bind): placements of every pod bound by t are
 * final, so any tick of a batched ks_step can be read back.  Cost: the pods that may run at t
 * (an index over run intervals skips finished pods), not the run's length. */
ks_status ks_usage_at(ks_engine* eng, int64_t t, int64_t* usage_out);

/* Per-tick usage digest for ticks t_lo <= t < t_hi (t_hi - 1 <= the current tick, t_hi - t_lo
 * <= 2^20): out[(t - t_lo) * 6 + k] for k = 0..2 is Σ over nodes of usage[node][k] at tick t, and
 * for k = 3..5 Σ over nodes of ks_node_mix(node) * usage[node][k - 3] (mod 2^64) — a per-tick
 * fingerprint of the whole [n][3] usage matrix, computed from the pods' phase segments
 * (difference arrays + a prefix sum) instead of one [n][3] reduction per tick. */
ks_status ks_usage_digest(ks_engine* eng, int64_t t_lo, int64_t t_hi, uint64_t* out);
/* the digest's node weight: z = (node + 1) * 0x9E3779B97F4A7C15, then the splitmix64 finaliser
 * (z ^= z >> 30; z *= 0xBF58476D1CE4E5B9; z ^= z >> 27; z *= 0x94D049BB133111EB; z ^= z >> 31) */
uint64_t ks_node_mix(int64_t node);

/* Name-keyed queries over the binds made so far (Node.GetPod / GetPodStatus / GetPodList,
 * kubesim/node/node.go:62-93).  ks_pod_lookup: the FIFO index of the pod stored on `node` under
 * key_id (the last one bound there), KS_ENOTFOUND if none ("pod %q not found").  ks_node_pods:
 * the FIFO indices of every pod stored on `node` (one per key, any bind status), in FIFO order;
 * writes min(count, cap) and the count to *n_out.  Phases/times: ks_pod_status. */
ks_status ks_pod_lookup(ks_engine* eng, int32_t node, int64_t key_id, int64_t* pod_out);
ks_status ks_node_pods(ks_engine* eng, int32_t node, int64_t* pods_out, int64_t cap, int64_t* n_out);

/* Pod status (Pod.BuildStatus, kubesim/pod/pod.go:78-145) at the current tick, for pods
 * [pod_lo, pod_lo + n) of the FIFO: PENDING = not bound (queued, or the pod an aborted run stopped
 * at — the reference never stores it); FAILED = bound OverCapacity (PodFailed / CapacityExceeded);
 * RUNNING / SUCCEEDED = bound Ok and IsRunning (pod.go:67-69) or not.  start_tick = the bind tick
 * (StartTime = start clock + start_tick * tick), total_seconds = Σ phase seconds as the reference's
 * int32 sum (FinishedAt = StartTime + total_seconds, pod.go:165-167). */
enum { KS_PHASE_PENDING = 0, KS_PHASE_RUNNING = 1, KS_PHASE_SUCCEEDED = 2, KS_PHASE_FAILED = 3 };
typedef struct {
    int32_t phase;
    int32_t node;           /* -1 when not bound */
    int64_t start_tick;     /* -1 when not bound */
    int32_t total_seconds;
    int32_t pad;
} ks_pod_info;
ks_status ks_pod_status(ks_engine* eng, int64_t pod_lo, int64_t n, ks_pod_info* out);

int64_t ks_current_tick(const ks_engine* eng);
/* the configured tick in seconds (ks_config.tick_seconds); -1 for NULL */
int32_t ks_tick_seconds(const ks_engine* eng);
int64_t ks_queued_pods(const ks_engine* eng);
const char* ks_last_error(const ks_engine* eng);

/* Timing of the last ks_step on the engine's stream (HIP events, recorded only while
 * ks_set_profiling is on): total device ms; the summed ms of the scan kernel alone, of the
 * resolve kernel alone and of everything else (expire_head, merge, RCCL exchange); the number of
 * batches (one launch of each kernel per batch) and of pods bound. */
typedef struct {
    double step_ms;
    double scan_ms;
    double resolve_ms;
    int64_t launches;
    int64_t pods;
    double other_ms;
} ks_step_stats;
ks_status ks_last_step_stats(const ks_engine* eng, ks_step_stats* out);
/* The same per kernel of the batch chain (profiling on): summed HIP-event ms and launch counts of
 * the window prep (launched for a pass's first batch and on the plain chain; an overlapped batch's
 * window is computed inside the previous chunk kernel), the scan (the overlap's conditional rescan
 * included, mostly an empty launch), the list merge (with the candidate lists, a sharded engine's
 * per-part merges and exchange), and the resolve launch — the chunk kernel alone, or fused with the
 * next batch's speculative scan and window prep.  Sharded engines: part_ms = the per-part merges
 * and xchg_ms = the exchange (RCCL all-gather, or the host exchange's copies, callback and wait),
 * both inside merge_ms, xchg_n batches. */
typedef struct {
    double prep_ms, scan_ms, merge_ms, resolve_ms, fused_ms, part_ms, xchg_ms;
    int64_t prep_n, scan_n, merge_n, resolve_n, fused_n, xchg_n;
    /* the pipelined sharded chain (engines the fused overlap does not take): the next batch's
     * speculative scan, part merges and exchange on the second stream beside the resolve (side_n
     * batches), and the main stream's wait for that exchange (inside merge_ms's batches) */
    double side_scan_ms, side_part_ms, side_xchg_ms, wait_ms;
    int64_t side_n;
    /* ks_usage_at calls made while profiling is on (summed since the last ks_step): the usage kernel's
     * HIP-event ms, its launches, and the pods of the candidate blocks it read */
    double usage_ms;
    int64_t usage_n, usage_pods;
} ks_kernel_stats;
ks_status ks_last_step_kernels(const ks_engine* eng, ks_kernel_stats* out);
ks_status ks_group_step(ks_group* g, int64_t ticks, ks_bind* out, int64_t cap, int64_t* n_out,
                        int32_t* status_out, ks_step_stats* stats);
/* Device counters (diagnostics): [0] next pod, [1] step end, [2] error, [3] error pod,
 * [4] batches that committed early (top-L list exhausted), [5] / [6] batches whose lists were
 * rescanned / reused from the previous batch (cumulative, chunk resolver), [16..31] resolver phase cycle
 * sums in a -DKS_STAMPS diagnostic build (tests/dev/diag_resolve.py). */
ks_status ks_debug_counters(ks_engine* eng, int64_t* out32);
/* Between-step invariants of a chunk-resolver engine (diagnostics / regression tests): out4[0] =
 * nodes whose candidate-slot or first-entry mark is set (must be 0: every batch's commit resets the
 * marks of every node its merge claimed), out4[1] = nodes whose E-index mark is set (must be 0), out4[2] = the most
 * candidate slots any batch claimed so far, out4[3] = the slots whose records are staged (beyond
 * them a batch is cut before the first pod that needs one).  All 0 before the first batch. */
ks_status ks_debug_invariants(ks_engine* eng, int64_t* out4);
/* Diagnostics: the raw batch window workspace (ks_device.h WinWS; *size_out = its size, up to cap
 * bytes copied to out), and — in a -DKS_BATCH_LOG diagnostic build only (KS_EINVAL otherwise) — the
 * pod whose batch the chunk resolver records in it (tests/dev/byval_diag.py). */
ks_status ks_debug_window(ks_engine* eng, void* out, int64_t cap, int64_t* size_out);
ks_status ks_debug_watch(ks_engine* eng, int64_t pod);
/* Device self-test of an evaluator identity the exactness argument rests on (no engine needed).
 * test 0: the micro evaluator's correction-free LeastRequested floor for every (x, A) with
 * 0 <= x <= A < 2^16 (ks_device.h).  *failures = mismatching cases (0 = pass). */
enum { KS_SELFTEST_LR_MICRO = 0 };
ks_status ks_selftest(int32_t device, int32_t test, int64_t* failures);
void ks_set_profiling(ks_engine* eng, int enable);
/* Provenance: the first 16 hex digits of the SHA-256 of the sources the library was built from
 * (kubernetes-simulator_amd/csrc/Makefile HASHED, in that order); the Python binding refuses a
 * library whose id differs from the hash of the sources beside it. */
const char* ks_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
