/*
 * ks_kubesim.h — KubeSim.Run over the engine's C-ABI, in C++ (libks_kubesim.so).
 *
 * The reference's Run loop (kubesim/kubesim.go:90-123) calls every registered api.Submitter
 * (api/submitter.go:10-16) at each tick, appends the returned pods to the FIFO (submit,
 * kubesim.go:126-139) and schedules one queued pod (scheduleOne, :143-166).  Its host is compiled
 * Go; neither this image nor the GPU box has a Go toolchain, so this is the same loop as a C++ host
 * of ks_engine.h — the call sequence the cgo shim (go/kubesim/engine/kubesim.go) makes, with
 * native submitters:
 *
 *   ks_run            per tick: each submitter callback returns the pods arriving at that tick
 *                     (encoded as ks_submit_pods takes them) — then ks_step(1) (window = 1, Run
 *                     itself), or one ks_step(window) after `window` ticks of submits (RunWindowed:
 *                     valid for submitters whose output never depends on placements, like the
 *                     reference example's, examples/main.go:96-128).
 *   ks_trace_submit   a built-in submitter that replays an encoded trace by arrival tick.
 *
 * Errors are Run's: the first non-OK status of ks_submit_pods / ks_step stops the loop and is
 * returned; the binds made before it are in out[0 .. *n_out).  A submitter or submit error at tick
 * t with window > 1 first steps the ticks before t (Run had scheduled them before it called the
 * submitters at t).  Submitters get clock_seconds = tick * tick_seconds (the start clock is the
 * caller's: kubesim.go:94-97 adds it).
 */
#ifndef KS_KUBESIM_H
#define KS_KUBESIM_H
#include <stdint.h>

#include "ks_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Pods as ks_submit_pods takes them (phase CSR rebased to 0; key_id / flags may be NULL). */
typedef struct {
    int64_t m;
    const int64_t* arrival;
    const int64_t* req;        /* [m][3] */
    const uint8_t* keymask;
    const uint64_t* tol;
    const uint64_t* sel;
    const int32_t* phase_off;  /* [m + 1] */
    const int32_t* phase_sec;
    const int64_t* phase_use;  /* [phases][3] */
    const uint8_t* flags;
    const int64_t* key_id;
} ks_pods;

/* api.Submitter.Submit (api/submitter.go:15): the pods returned at `tick` (clock = start +
 * tick * tick_seconds) into *out (pointers valid until the next call; out->m = 0 for none);
 * returns KS_OK or an error that stops the run. */
typedef ks_status (*ks_submit_fn)(void* user, int64_t tick, int64_t clock_seconds, ks_pods* out);

/* Run for `ticks` ticks from the engine's current tick with the submitters in registration
 * order.  window >= 1 (1 = Run; > 1 = RunWindowed).  *seconds_out (may be NULL): wall time. */
ks_status ks_run(ks_engine* eng, int64_t ticks, int64_t window, int32_t n_submitters, const ks_submit_fn* fns,
                 void* const* users, ks_bind* out, int64_t cap, int64_t* n_out, double* seconds_out);

/* A trace submitter: the pods of `trace` whose arrival tick is t, in order (arrival
 * non-decreasing); `next` is its cursor (start at 0). */
typedef struct {
    ks_pods trace;
    int64_t next;
    int64_t tick_seconds;
} ks_trace_submitter;
ks_status ks_trace_submit(void* user /* ks_trace_submitter* */, int64_t tick, int64_t clock_seconds, ks_pods* out);

/* In-process all-gather for ks_shard_host: `world` engines driven by threads of one process
 * (one per rank, on one GPU or several) exchange their candidate parts through host memory.
 * Pass ks_local_allgather as the fn and the exchange as the user pointer of every rank. */
typedef struct ks_local_exchange ks_local_exchange;
ks_local_exchange* ks_local_exchange_create(int32_t world);
void ks_local_exchange_destroy(ks_local_exchange* x);
ks_status ks_local_allgather(void* user /* ks_local_exchange* */, int32_t rank, int32_t world, void* buf,
                             int64_t bytes_per_rank);
/* A rank whose step failed before it reached the exchange would leave the others waiting: its
 * driver calls this, and every current and later ks_local_allgather on x returns KS_EDEVICE. */
void ks_local_exchange_abort(ks_local_exchange* x);
/* Provenance of libks_kubesim.so: the same source hash as ks_build_id (ks_engine.h). */
const char* ks_run_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
