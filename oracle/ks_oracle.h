/*
 * ks_oracle.h — CPU restatement of the kubesim scheduling loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (kubernetes-simulator_amd/, include/)
 * links, loads or calls this.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * Parity pinning: the resource-list arithmetic, Quantity parsing and simSpec decoding the
 * oracle relies on are pinned against the reference's own unit-test vectors
 * (tests/golden/reference_kats.json, tests/test_oracle_kats.py).  The scheduling loop itself
 * (placements, bind order, per-tick usage) is NOT covered by any reference test
 * (SURVEY.md §4, §8(c)); it is pinned by a hand-derived KAT of config/sample.yml +
 * examples/main.go (tests/golden/c1_kat.json) and by agreement with an independent
 * pure-Python restatement (oracle/pysim.py) on seeded traces.  The Go reference cannot be
 * built here (no Go toolchain), so scheduling parity is "partially pinned".
 *
 * Deterministic tie-break: the reference takes argmax over a Go map (random iteration,
 * kubesim/kubesim.go:208-215); the oracle returns the lowest node index among the maxima,
 * which is always a member of the reference's possible outcome set.
 */
#ifndef KS_ORACLE_H
#define KS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* KO_ERANGE (= KS_ERANGE): a tick 2^31 s or more after the first bind — outside the int32
 * passed-seconds domain (kubesim/pod/pod.go:148-153); the step stops before it, not sticky. */
enum { KO_OK = 0, KO_EINVAL = 1, KO_ENOTFOUND = 2, KO_ERANGE = 5 };
enum { KO_FILTER_REFERENCE_LITERAL = 0, KO_FILTER_FEEDS_SCORE = 1 };
enum { KO_FILTER_FIT = 1, KO_FILTER_TAINT = 2, KO_FILTER_SELECTOR = 4 };
enum { KO_SCORER_CONST = 0, KO_SCORER_LEAST_REQUESTED = 1, KO_SCORER_BALANCED = 2 };
enum { KO_STATUS_OK = 0, KO_STATUS_OVER_CAPACITY = 1 };
enum { KO_FLAG_BAD_KEY = 1, KO_FLAG_BAD_SPEC = 2 };

typedef struct {
    int32_t tick_seconds;
    int32_t filter_mode;
    uint32_t filters;
    int32_t n_scorers;
    int32_t scorer_kind[8];
    int32_t scorer_weight[8];
    int32_t scorer_value[8];
} ko_config;

typedef struct ko_sim ko_sim;

/* Nodes: alloc[n][4] (milli cpu, milli memory, milli gpu, pods count) with presence bits
 * alloc_has (1 cpu, 2 mem, 4 gpu, 8 pods); taints CSR rows (key, value, effect 1..3);
 * labels CSR rows (key, value).  String ids: 0 = "". */
ko_sim* ko_create(const ko_config* cfg, int64_t n, const int64_t* alloc, const uint8_t* alloc_has,
                  const int32_t* taint_off, const int32_t* taint, const int32_t* label_off,
                  const int32_t* label);
void ko_destroy(ko_sim* s);

/* Pods appended in FIFO order; arrival ticks must be non-decreasing.  req[m][3] with
 * presence req_has; tolerations CSR rows (key, op, value, effect 0..3); selector CSR rows
 * (key, value); simSpec CSR (seconds, usage[3], usage presence); key_id = interned
 * "namespace-name"; flags = KO_FLAG_*. */
int ko_submit(ko_sim* s, int64_t m, const int64_t* arrival, const int64_t* req,
              const uint8_t* req_has, const int32_t* tol_off, const int32_t* tol,
              const int32_t* sel_off, const int32_t* sel, const int32_t* phase_off,
              const int32_t* phase_sec, const int64_t* phase_use, const uint8_t* phase_has,
              const int64_t* key_id, const uint8_t* flags);

/* Advance `ticks` ticks (kubesim.go:90-123).  Binds are appended to the out arrays (at most
 * cap); returns KO_OK or the error that aborted the run (the run stays aborted). */
int ko_step(ko_sim* s, int64_t ticks, int64_t* out_pod, int32_t* out_node, int64_t* out_tick,
            int32_t* out_status, int64_t cap, int64_t* n_out);

/* Per-node usage at the current tick: sum over pods stored on the node of
 * Pod.ResourceUsage(clock) (kubesim/pod/pod.go:47-63).  out[n][3]. */
void ko_usage(ko_sim* s, int64_t* out);

/* Filter mask / weighted score of queued-or-future pod `pod` against the cluster state at
 * the current tick (what api.Filter / api.Scorer would see).  score = -1 for no entry. */
int ko_eval(ko_sim* s, int64_t pod, uint8_t* feasible, int64_t* score);

int64_t ko_tick(const ko_sim* s);
/* Per-node loops on `threads` OpenMP threads (default 1); results are identical. */
void ko_set_threads(ko_sim* s, int threads);
const char* ko_last_error(const ko_sim* s);

#ifdef __cplusplus
}
#endif
#endif
