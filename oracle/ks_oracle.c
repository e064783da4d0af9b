/*
 * ks_oracle.c — CPU restatement of kubesim's scheduling loop.  TEST INFRASTRUCTURE ONLY
 * (see ks_oracle.h for what pins it and who may use it).
 *
 * Follows, rule by rule:
 *   KubeSim.Run tick loop ........................ kubesim/kubesim.go:90-123
 *   submit + FIFO podQueue ....................... kubesim/kubesim.go:126-139, podqueue.go:18-42
 *   scheduleOne / Filter (result discarded) ...... kubesim/kubesim.go:143-188
 *   Score aggregation + argmax + NotFound ........ kubesim/kubesim.go:190-225
 *   Node.CreatePod admission + Store ............. kubesim/node/node.go:36-60, 97-118
 *   resourceListSum / resourceListGE ............. kubesim/node/resource.go:10-21, 52-61
 *   Pod.IsRunning / ResourceUsage / passedSeconds  kubesim/pod/pod.go:47-69, 148-162
 *   Capacity.Pods() default 0 .................... vendor/k8s.io/api/core/v1/resource.go:44-49
 *   Toleration.ToleratesTaint .................... vendor/k8s.io/api/core/v1/toleration.go:37-56
 *   buildKey error (InvalidArgument) ............. kubesim/node/node.go:133-148
 *   simSpec parse error at bind .................. kubesim/pod/pod.go:31-39
 * It is deliberately literal: node totals are recomputed from the pods stored on the node
 * with IsRunning(clock) at every evaluation, exactly as totalResourceRequest does; pods
 * that have terminated (they can never run again) are pruned from the scan list, which
 * changes no result.  Build-defined plugins: resource fit,
 * taint/toleration and node-selector filters; constant, LeastRequested and
 * BalancedAllocation scorers in exact integer arithmetic.
 *
 * ko_set_threads(s, T > 1) runs the per-node loops (node totals, filters, scores, argmax) on T
 * OpenMP threads — the multi-core CPU baseline of SURVEY.md §8(d).  Every node's work is
 * independent and the argmax combines per-thread winners in node order, so results are the
 * same as with one thread.
 */
#include "ks_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

typedef struct {
    int32_t* v;
    int32_t n, cap;
} ivec;

static void ivec_push(ivec* a, int32_t x) {
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 4;
        a->v = (int32_t*)realloc(a->v, sizeof(int32_t) * (size_t)a->cap);
    }
    a->v[a->n++] = x;
}

struct ko_sim {
    ko_config cfg;
    int64_t n;
    int64_t* alloc;
    uint8_t* alloc_has;
    int32_t *taint_off, *taint, *label_off, *label;
    ivec* live; /* per node: pods stored with status Ok that may still be running */

    int64_t m, mcap;
    int64_t *arrival, *req, *key_id;
    uint8_t *req_has, *flags;
    int32_t *tol_off, *sel_off, *phase_off;
    int32_t *tol, *sel, *phase_sec;
    int64_t* phase_use;
    uint8_t* phase_has;
    int64_t ntol, nsel, nphase;
    /* runtime per pod */
    int32_t* p_node;
    int32_t* p_status;
    int64_t* p_t0;
    int32_t* p_total; /* int32 (wrapping) sum of phase seconds, pod.go:155-162 */

    int64_t tick, qhead, arrived;
    int64_t first_bind; /* tick of the run's first bind, -1 before */
    int err;
    char errmsg[256];
    /* scratch */
    int64_t* tot;     /* [n][3] */
    uint8_t* tot_has; /* [n] */
    int64_t* nrun;    /* [n] */
    uint8_t* cand;
    int64_t* score;
    int threads; /* OpenMP threads for the per-node loops (1 = serial) */
};

#define GROW(ptr, type, count)                                                  \
    do {                                                                        \
        (ptr) = (type*)realloc((ptr), sizeof(type) * (size_t)((count) > 0 ? (count) : 1)); \
    } while (0)

static void* dupmem(const void* p, size_t bytes) {
    void* q = malloc(bytes ? bytes : 1);
    if (bytes) memcpy(q, p, bytes);
    return q;
}

ko_sim* ko_create(const ko_config* cfg, int64_t n, const int64_t* alloc, const uint8_t* alloc_has,
                  const int32_t* taint_off, const int32_t* taint, const int32_t* label_off,
                  const int32_t* label) {
    if (!cfg || cfg->tick_seconds < 1) return NULL;  /* the engine's ks_create refuses the same */
    ko_sim* s = (ko_sim*)calloc(1, sizeof(ko_sim));
    s->cfg = *cfg;
    s->n = n;
    s->threads = 1;
    s->first_bind = -1;
    s->alloc = (int64_t*)dupmem(alloc, sizeof(int64_t) * 4 * (size_t)n);
    s->alloc_has = (uint8_t*)dupmem(alloc_has, (size_t)n);
    s->taint_off = (int32_t*)dupmem(taint_off, sizeof(int32_t) * (size_t)(n + 1));
    s->taint = (int32_t*)dupmem(taint, sizeof(int32_t) * 3 * (size_t)taint_off[n]);
    s->label_off = (int32_t*)dupmem(label_off, sizeof(int32_t) * (size_t)(n + 1));
    s->label = (int32_t*)dupmem(label, sizeof(int32_t) * 2 * (size_t)label_off[n]);
    s->live = (ivec*)calloc((size_t)(n ? n : 1), sizeof(ivec));
    s->tot = (int64_t*)calloc((size_t)(n ? n : 1) * 3, sizeof(int64_t));
    s->tot_has = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
    s->nrun = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
    s->cand = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
    s->score = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
    s->tol_off = (int32_t*)calloc(1, sizeof(int32_t));
    s->sel_off = (int32_t*)calloc(1, sizeof(int32_t));
    s->phase_off = (int32_t*)calloc(1, sizeof(int32_t));
    return s;
}

void ko_destroy(ko_sim* s) {
    if (!s) return;
    for (int64_t i = 0; i < s->n; i++) free(s->live[i].v);
    free(s->live);
    free(s->alloc); free(s->alloc_has); free(s->taint_off); free(s->taint);
    free(s->label_off); free(s->label);
    free(s->arrival); free(s->req); free(s->key_id); free(s->req_has); free(s->flags);
    free(s->tol_off); free(s->sel_off); free(s->phase_off); free(s->tol); free(s->sel);
    free(s->phase_sec); free(s->phase_use); free(s->phase_has);
    free(s->p_node); free(s->p_status); free(s->p_t0); free(s->p_total);
    free(s->tot); free(s->tot_has); free(s->nrun); free(s->cand); free(s->score);
    free(s);
}

int64_t ko_tick(const ko_sim* s) { return s->tick; }
void ko_set_threads(ko_sim* s, int threads) { s->threads = threads > 1 ? threads : 1; }
const char* ko_last_error(const ko_sim* s) { return s->errmsg; }

int ko_submit(ko_sim* s, int64_t m, const int64_t* arrival, const int64_t* req,
              const uint8_t* req_has, const int32_t* tol_off, const int32_t* tol,
              const int32_t* sel_off, const int32_t* sel, const int32_t* phase_off,
              const int32_t* phase_sec, const int64_t* phase_use, const uint8_t* phase_has,
              const int64_t* key_id, const uint8_t* flags) {
    int64_t last = s->m ? s->arrival[s->m - 1] : 0;
    for (int64_t i = 0; i < m; i++) {
        if (arrival[i] < last) {
            snprintf(s->errmsg, sizeof s->errmsg, "arrival ticks must be non-decreasing");
            return KO_EINVAL;
        }
        last = arrival[i];
    }
    int64_t nm = s->m + m;
    GROW(s->arrival, int64_t, nm);
    GROW(s->req, int64_t, nm * 3);
    GROW(s->key_id, int64_t, nm);
    GROW(s->req_has, uint8_t, nm);
    GROW(s->flags, uint8_t, nm);
    GROW(s->tol_off, int32_t, nm + 1);
    GROW(s->sel_off, int32_t, nm + 1);
    GROW(s->phase_off, int32_t, nm + 1);
    GROW(s->p_node, int32_t, nm);
    GROW(s->p_status, int32_t, nm);
    GROW(s->p_t0, int64_t, nm);
    GROW(s->p_total, int32_t, nm);
    int64_t nt = s->ntol + tol_off[m], ns = s->nsel + sel_off[m], nf = s->nphase + phase_off[m];
    GROW(s->tol, int32_t, nt * 4);
    GROW(s->sel, int32_t, ns * 2);
    GROW(s->phase_sec, int32_t, nf);
    GROW(s->phase_use, int64_t, nf * 3);
    GROW(s->phase_has, uint8_t, nf);
    memcpy(s->tol + s->ntol * 4, tol, sizeof(int32_t) * 4 * (size_t)tol_off[m]);
    memcpy(s->sel + s->nsel * 2, sel, sizeof(int32_t) * 2 * (size_t)sel_off[m]);
    memcpy(s->phase_sec + s->nphase, phase_sec, sizeof(int32_t) * (size_t)phase_off[m]);
    memcpy(s->phase_use + s->nphase * 3, phase_use, sizeof(int64_t) * 3 * (size_t)phase_off[m]);
    memcpy(s->phase_has + s->nphase, phase_has, (size_t)phase_off[m]);
    for (int64_t i = 0; i < m; i++) {
        int64_t j = s->m + i;
        s->arrival[j] = arrival[i];
        for (int k = 0; k < 3; k++) s->req[j * 3 + k] = req[i * 3 + k];
        s->key_id[j] = key_id[i];
        s->req_has[j] = req_has[i];
        s->flags[j] = flags[i];
        s->tol_off[j + 1] = (int32_t)(s->ntol + tol_off[i + 1]);
        s->sel_off[j + 1] = (int32_t)(s->nsel + sel_off[i + 1]);
        s->phase_off[j + 1] = (int32_t)(s->nphase + phase_off[i + 1]);
        /* totalSeconds: int32 accumulation (pod.go:155-162) */
        uint32_t acc = 0;
        for (int32_t f = phase_off[i]; f < phase_off[i + 1]; f++) acc += (uint32_t)phase_sec[f];
        s->p_total[j] = (int32_t)acc;
        s->p_node[j] = -1;
        s->p_status[j] = -1;
        s->p_t0[j] = 0;
    }
    s->ntol = nt;
    s->nsel = ns;
    s->nphase = nf;
    s->m = nm;
    return KO_OK;
}

/* passedSeconds (pod.go:148-153): int32 of whole seconds since the pod's start clock.  Go's
 * float64 -> int32 conversion is implementation-defined past 2^31, so the oracle (like the
 * engine) stays inside the domain: ko_step never evaluates a tick 2^31 s or more after the first
 * bind (KO_ERANGE).  There secs < 2^31 and the conversion is exact. */
static int32_t passed_seconds(const ko_sim* s, int64_t p, int64_t t) {
    if (s->p_status[p] != KO_STATUS_OK) return 0;
    int64_t secs = (t - s->p_t0[p]) * (int64_t)s->cfg.tick_seconds;
    return (int32_t)secs;
}

/* IsRunning (pod.go:67-69). */
static int is_running(const ko_sim* s, int64_t p, int64_t t) {
    return s->p_status[p] == KO_STATUS_OK && passed_seconds(s, p, t) < s->p_total[p];
}

/* totalResourceRequest + runningPodsNum (node.go:97-118) for every node at tick t. */
static void node_views(ko_sim* s, int64_t t) {
#pragma omp parallel for schedule(static) num_threads(s->threads) if (s->threads > 1)
    for (int64_t nd = 0; nd < s->n; nd++) {
        ivec* L = &s->live[nd];
        int64_t tot[3] = {0, 0, 0};
        uint8_t has = 0;
        int64_t nrun = 0;
        int32_t w = 0;
        for (int32_t i = 0; i < L->n; i++) {
            int32_t p = L->v[i];
            if (!is_running(s, p, t)) {
                /* terminated (Ok and passed >= total): inside the domain passed only grows with
                 * t (no int32 wrap, see passed_seconds), so it can never run again — prune */
                continue;
            }
            L->v[w++] = p;
            for (int k = 0; k < 3; k++)
                if (s->req_has[p] & (1u << k)) tot[k] += s->req[p * 3 + k];
            has |= s->req_has[p] & 7;
            nrun++;
        }
        L->n = w;
        for (int k = 0; k < 3; k++) s->tot[nd * 3 + k] = tot[k];
        s->tot_has[nd] = has;
        s->nrun[nd] = nrun;
    }
}

static int64_t pods_value(const ko_sim* s, int64_t nd) {
    return (s->alloc_has[nd] & 8) ? s->alloc[nd * 4 + 3] : 0;
}

/* CreatePod admission test (node.go:44-47) == the build's resource-fit predicate. */
static int fits(const ko_sim* s, int64_t nd, int64_t p) {
    uint8_t keys = s->tot_has[nd] | (s->req_has[p] & 7);
    for (int k = 0; k < 3; k++) {
        if (!(keys & (1u << k))) continue;
        int64_t total = s->tot[nd * 3 + k] + ((s->req_has[p] & (1u << k)) ? s->req[p * 3 + k] : 0);
        if (!(s->alloc_has[nd] & (1u << k))) return 0; /* resource.go:54-55 */
        if (s->alloc[nd * 4 + k] < total) return 0;    /* Cmp < 0 */
    }
    return !(s->nrun[nd] >= pods_value(s, nd));
}

/* ToleratesTaint (toleration.go:37-56); string id 0 is "". */
static int tolerates(const int32_t* tl, const int32_t* tt) {
    if (tl[3] != 0 && tl[3] != tt[2]) return 0;
    if (tl[0] != 0 && tl[0] != tt[0]) return 0;
    switch (tl[1]) {
        case 0: return tl[2] == tt[1];
        case 1: return 1;
        default: return 0;
    }
}

static int taint_ok(const ko_sim* s, int64_t nd, int64_t p) {
    for (int32_t i = s->taint_off[nd]; i < s->taint_off[nd + 1]; i++) {
        const int32_t* tt = s->taint + 3 * (int64_t)i;
        if (tt[2] != 1 && tt[2] != 3) continue; /* only NoSchedule / NoExecute filter */
        int ok = 0;
        for (int32_t j = s->tol_off[p]; j < s->tol_off[p + 1] && !ok; j++)
            ok = tolerates(s->tol + 4 * (int64_t)j, tt);
        if (!ok) return 0;
    }
    return 1;
}

static int selector_ok(const ko_sim* s, int64_t nd, int64_t p) {
    for (int32_t j = s->sel_off[p]; j < s->sel_off[p + 1]; j++) {
        const int32_t* kv = s->sel + 2 * (int64_t)j;
        int found = 0;
        for (int32_t i = s->label_off[nd]; i < s->label_off[nd + 1]; i++) {
            const int32_t* lb = s->label + 2 * (int64_t)i;
            if (lb[0] == kv[0]) {
                found = lb[1] == kv[1];
                break;
            }
        }
        if (!found) return 0;
    }
    return 1;
}

static int64_t cap_of(const ko_sim* s, int64_t nd, int k) {
    return (s->alloc_has[nd] & (1u << k)) ? s->alloc[nd * 4 + k] : 0;
}
static int64_t used_of(const ko_sim* s, int64_t nd, int64_t p, int k) {
    return s->tot[nd * 3 + k] + ((s->req_has[p] & (1u << k)) ? s->req[p * 3 + k] : 0);
}

/* LeastRequested, integer form. */
static int64_t score_lr(const ko_sim* s, int64_t nd, int64_t p) {
    int64_t sum = 0;
    for (int k = 0; k < 2; k++) {
        int64_t A = cap_of(s, nd, k), u = used_of(s, nd, p, k);
        if (A <= 0 || u > A) continue;
        sum += (A - u) * 10 / A;
    }
    return sum / 2;
}

/* BalancedAllocation, exact rational form. */
static int64_t score_ba(const ko_sim* s, int64_t nd, int64_t p) {
    int64_t Ac = cap_of(s, nd, 0), Am = cap_of(s, nd, 1);
    int64_t uc = used_of(s, nd, p, 0), um = used_of(s, nd, p, 1);
    if (Ac <= 0 || Am <= 0 || uc >= Ac || um >= Am) return 0;
    u128 D = (u128)Ac * (u128)Am;
    u128 a = (u128)uc * (u128)Am, b = (u128)um * (u128)Ac;
    u128 X = a > b ? a - b : b - a;
    return (int64_t)((u128)10 * (D - X) / D);
}

static int filter_pass(const ko_sim* s, int64_t nd, int64_t p, uint32_t which) {
    if ((which & KO_FILTER_FIT) && !fits(s, nd, p)) return 0;
    if ((which & KO_FILTER_TAINT) && !taint_ok(s, nd, p)) return 0;
    if ((which & KO_FILTER_SELECTOR) && !selector_ok(s, nd, p)) return 0;
    return 1;
}

/* scheduleOneFilter (kubesim.go:168-188) + the score map of scheduleOneScore (:190-206).
 * cand[n] = node has an entry in nodeScore. */
static void filter_and_score(ko_sim* s, int64_t p) {
    static const uint32_t order[3] = {KO_FILTER_FIT, KO_FILTER_TAINT, KO_FILTER_SELECTOR};
#pragma omp parallel num_threads(s->threads) if (s->threads > 1)
    {
        /* Filter loop: filter-major, each filter sees the survivors of the previous one. */
#pragma omp for schedule(static)
        for (int64_t nd = 0; nd < s->n; nd++) s->cand[nd] = 1;
        for (int f = 0; f < 3; f++) {
            if (!(s->cfg.filters & order[f])) continue;
#pragma omp for schedule(static)
            for (int64_t nd = 0; nd < s->n; nd++)
                if (s->cand[nd]) s->cand[nd] = (uint8_t)filter_pass(s, nd, p, order[f]);
        }
#pragma omp for schedule(static)
        for (int64_t nd = 0; nd < s->n; nd++) {
            /* kubesim.go:182 reassigns a local only: in the literal mode scoring sees the
             * unfiltered node list.  With no scorers nodeScore stays empty. */
            if (s->cfg.filter_mode == KO_FILTER_REFERENCE_LITERAL) s->cand[nd] = 1;
            if (s->cfg.n_scorers == 0) s->cand[nd] = 0;
            s->score[nd] = 0;
        }
        for (int i = 0; i < s->cfg.n_scorers; i++) {
            int64_t w = s->cfg.scorer_weight[i];
#pragma omp for schedule(static)
            for (int64_t nd = 0; nd < s->n; nd++) {
                if (!s->cand[nd]) continue;
                int64_t sc;
                switch (s->cfg.scorer_kind[i]) {
                    case KO_SCORER_CONST: sc = s->cfg.scorer_value[i]; break;
                    case KO_SCORER_LEAST_REQUESTED: sc = score_lr(s, nd, p); break;
                    default: sc = score_ba(s, nd, p); break;
                }
                s->score[nd] += sc * w;
            }
        }
    }
}

/* argmax over nodeScore, scoreMax = -1, strict '>' (kubesim.go:208-215); deterministic order =
 * node index, so ties go to the lowest index.  Threaded: thread k scans the k-th contiguous
 * index range and the ranges' winners are combined in index order. */
#define KO_MAX_THREADS 256
static int64_t argmax_node(const ko_sim* s) {
    int64_t best = -1, bn = -1;
    if (s->threads <= 1) {
        for (int64_t nd = 0; nd < s->n; nd++)
            if (s->cand[nd] && s->score[nd] > best) {
                best = s->score[nd];
                bn = nd;
            }
        return bn;
    }
    int64_t tb[KO_MAX_THREADS], tn[KO_MAX_THREADS];
    const int nt = s->threads < KO_MAX_THREADS ? s->threads : KO_MAX_THREADS;
    for (int k = 0; k < nt; k++) tb[k] = tn[k] = -1;
#pragma omp parallel for schedule(static, 1) num_threads(nt)
    for (int k = 0; k < nt; k++) {
        const int64_t lo = s->n * k / nt, hi = s->n * (k + 1) / nt;
        int64_t b = -1, n = -1;
        for (int64_t nd = lo; nd < hi; nd++)
            if (s->cand[nd] && s->score[nd] > b) {
                b = s->score[nd];
                n = nd;
            }
        tb[k] = b;
        tn[k] = n;
    }
    for (int k = 0; k < nt; k++)
        if (tn[k] >= 0 && tb[k] > best) {
            best = tb[k];
            bn = tn[k];
        }
    return bn;
}

static int schedule_one(ko_sim* s, int64_t p, int64_t t, int64_t* out_node, int32_t* out_status) {
    node_views(s, t);
    filter_and_score(s, p);
    const int64_t bn = argmax_node(s);
    if (bn < 0) {
        snprintf(s->errmsg, sizeof s->errmsg, "node \"\" not found (pod %lld)", (long long)p);
        return KO_ENOTFOUND; /* kubesim.go:217-220 */
    }
    /* CreatePod (node.go:36-60) */
    if (s->flags[p] & KO_FLAG_BAD_KEY) {
        snprintf(s->errmsg, sizeof s->errmsg, "Empty pod namespace or name (pod %lld)", (long long)p);
        return KO_EINVAL;
    }
    int32_t status = fits(s, bn, p) ? KO_STATUS_OK : KO_STATUS_OVER_CAPACITY;
    if (s->flags[p] & KO_FLAG_BAD_SPEC) {
        snprintf(s->errmsg, sizeof s->errmsg, "invalid simSpec (pod %lld)", (long long)p);
        return KO_EINVAL;
    }
    /* node.pods.Store(key, pod): a stored pod with the same key is replaced. */
    ivec* L = &s->live[bn];
    int32_t w = 0;
    for (int32_t i = 0; i < L->n; i++)
        if (s->key_id[L->v[i]] != s->key_id[p]) L->v[w++] = L->v[i];
    L->n = w;
    s->p_node[p] = (int32_t)bn;
    s->p_status[p] = status;
    s->p_t0[p] = t;
    if (s->first_bind < 0) s->first_bind = t;
    if (status == KO_STATUS_OK) ivec_push(L, (int32_t)p);
    *out_node = bn;
    *out_status = status;
    return KO_OK;
}

int ko_step(ko_sim* s, int64_t ticks, int64_t* out_pod, int32_t* out_node, int64_t* out_tick,
            int32_t* out_status, int64_t cap, int64_t* n_out) {
    *n_out = 0;
    if (s->err) return s->err;
    /* The int32 passed-seconds domain, checked for the whole step before any tick runs (as the
     * engine's ks_step does): the run's first bind is first_bind, or — none yet — the next queued
     * pod's bind tick (it binds at the first tick >= its arrival) when that falls in this step. */
    {
        int64_t fb = s->first_bind;
        if (fb < 0 && s->qhead < s->m) {
            fb = s->arrival[s->qhead] > s->tick + 1 ? s->arrival[s->qhead] : s->tick + 1;
            if (fb > s->tick + ticks) fb = -1;
        }
        if (fb >= 0 && s->tick + ticks - fb > (int64_t)INT32_MAX / s->cfg.tick_seconds) {
            snprintf(s->errmsg, sizeof s->errmsg, "step to tick %lld: 2^31 s after the first bind (tick %lld)",
                     (long long)(s->tick + ticks), (long long)fb);
            return KO_ERANGE;
        }
    }
    for (int64_t i = 0; i < ticks; i++) {
        int64_t t = s->tick + 1;
        while (s->arrived < s->m && s->arrival[s->arrived] <= t) s->arrived++;
        if (s->qhead < s->arrived) {
            int64_t p = s->qhead;
            int64_t nd;
            int32_t st;
            int rc = schedule_one(s, p, t, &nd, &st);
            if (rc != KO_OK) {
                s->err = rc;
                s->tick = t;
                s->qhead++;
                return rc;
            }
            s->qhead++;
            if (*n_out < cap) {
                out_pod[*n_out] = p;
                out_node[*n_out] = (int32_t)nd;
                out_tick[*n_out] = t;
                out_status[*n_out] = st;
            }
            (*n_out)++;
        }
        s->tick = t;
    }
    return KO_OK;
}

void ko_usage(ko_sim* s, int64_t* out) {
    int64_t t = s->tick;
    for (int64_t nd = 0; nd < s->n; nd++) {
        int64_t u[3] = {0, 0, 0};
        ivec* L = &s->live[nd];
        for (int32_t i = 0; i < L->n; i++) {
            int32_t p = L->v[i];
            if (!is_running(s, p, t)) continue; /* ResourceUsage of a non-running pod = {} */
            int32_t passed = passed_seconds(s, p, t);
            uint32_t acc = 0;
            for (int32_t f = s->phase_off[p]; f < s->phase_off[p + 1]; f++) {
                acc += (uint32_t)s->phase_sec[f];
                if (passed < (int32_t)acc) {
                    for (int k = 0; k < 3; k++)
                        if (s->phase_has[f] & (1u << k)) u[k] += s->phase_use[(int64_t)f * 3 + k];
                    break;
                }
            }
        }
        for (int k = 0; k < 3; k++) out[nd * 3 + k] = u[k];
    }
}

int ko_eval(ko_sim* s, int64_t pod, uint8_t* feasible, int64_t* score) {
    if (pod < 0 || pod >= s->m) return KO_EINVAL;
    node_views(s, s->tick);
    /* feasibility under every enabled filter, independent of filter_mode */
    for (int64_t nd = 0; nd < s->n; nd++) feasible[nd] = (uint8_t)filter_pass(s, nd, pod, s->cfg.filters);
    filter_and_score(s, pod);
    for (int64_t nd = 0; nd < s->n; nd++) score[nd] = s->cand[nd] ? s->score[nd] : -1;
    return KO_OK;
}
