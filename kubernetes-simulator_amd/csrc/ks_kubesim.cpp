// ks_kubesim.cpp — KubeSim.Run (kubesim/kubesim.go:90-123) as a C++ host of the engine's C-ABI
// (include/ks_kubesim.h): the loop the Go shim runs (go/kubesim/engine/kubesim.go), native.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/ks_kubesim.h"

extern "C" {

ks_status ks_trace_submit(void* user, int64_t tick, int64_t /*clock_seconds*/, ks_pods* out) {
    ks_trace_submitter* s = static_cast<ks_trace_submitter*>(user);
    const ks_pods& t = s->trace;
    int64_t lo = s->next, hi = lo;
    while (hi < t.m && t.arrival[hi] <= tick) hi++;
    s->next = hi;
    *out = ks_pods{};
    if (hi == lo) return KS_OK;
    const int64_t f0 = t.phase_off[lo];
    out->m = hi - lo;
    out->arrival = t.arrival + lo;
    out->req = t.req + 3 * lo;
    out->keymask = t.keymask + lo;
    out->tol = t.tol + lo;
    out->sel = t.sel + lo;
    out->phase_off = t.phase_off + lo;  // rebased by ks_run (the engine wants phase_off[0] == 0)
    out->phase_sec = t.phase_sec + f0;
    out->phase_use = t.phase_use + 3 * f0;
    out->flags = t.flags ? t.flags + lo : nullptr;
    out->key_id = t.key_id ? t.key_id + lo : nullptr;
    return KS_OK;
}

ks_status ks_run(ks_engine* eng, int64_t ticks, int64_t window, int32_t n_submitters, const ks_submit_fn* fns,
                 void* const* users, ks_bind* out, int64_t cap, int64_t* n_out, double* seconds_out) {
    if (!eng || ticks < 0 || window < 1 || n_submitters < 0 || (n_submitters && (!fns || !users)) || !n_out ||
        cap < 0 || (cap && !out))
        return KS_EINVAL;
    *n_out = 0;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<int64_t> arr;
    std::vector<int32_t> off;
    const int64_t start = ks_current_tick(eng);
    const int64_t tick_s = ks_tick_seconds(eng);
    int64_t tick = start, stepped = start;
    ks_status rc = KS_OK;
    auto step = [&](int64_t k) -> ks_status {
        if (k <= 0) return KS_OK;
        int64_t nb = 0;
        const ks_status r = ks_step(eng, k, out ? out + *n_out : nullptr, cap - *n_out, &nb);
        *n_out += nb < cap - *n_out ? nb : cap - *n_out;
        stepped += k;
        return r;
    };
    while (tick < start + ticks && rc == KS_OK) {
        tick++;
        for (int32_t s = 0; s < n_submitters && rc == KS_OK; s++) {  // kubesim.go:126-139, registration order
            ks_pods p{};
            rc = fns[s](users[s], tick, tick * tick_s, &p);  // clock = start + tick * tick (kubesim.go:94-97)
            if (rc != KS_OK || p.m == 0) continue;
            // the pods arrive at this tick; phase CSR rebased to 0
            arr.assign(p.m, tick);
            off.resize(p.m + 1);
            for (int64_t i = 0; i <= p.m; i++) off[i] = p.phase_off[i] - p.phase_off[0];
            rc = ks_submit_pods(eng, p.m, arr.data(), p.req, p.keymask, p.tol, p.sel, off.data(), p.phase_sec,
                                p.phase_use, p.flags, p.key_id);
        }
        if (rc != KS_OK) {
            // Run would have scheduled every tick before this one before calling the submitters at
            // it: the window's ticks (stepped, tick) are stepped first; the submit error is returned
            // (a step error before it wins, as it would have stopped Run sooner)
            const ks_status r = step(tick - 1 - stepped);
            if (r != KS_OK) rc = r;
            break;
        }
        if (tick - stepped >= window) rc = step(tick - stepped);  // window 1: scheduleOne every tick
    }
    if (rc == KS_OK) rc = step(tick - stepped);
    if (seconds_out)
        *seconds_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

}  // extern "C"

// ---- in-process all-gather (ks_shard_host between threads) ----------------------------------
struct ks_local_exchange {
    int32_t world = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint8_t> buf;
    int32_t arrived = 0, left = 0;
    uint64_t gen = 0;
    bool aborted = false;  // ks_local_exchange_abort: every wait ends with KS_EDEVICE
};

extern "C" {

ks_local_exchange* ks_local_exchange_create(int32_t world) {
    if (world < 1) return nullptr;
    ks_local_exchange* x = new ks_local_exchange();
    x->world = world;
    return x;
}

void ks_local_exchange_destroy(ks_local_exchange* x) { delete x; }

void ks_local_exchange_abort(ks_local_exchange* x) {
    if (!x) return;
    std::lock_guard<std::mutex> lk(x->mu);
    x->aborted = true;
    x->cv.notify_all();
}

// Two phases per exchange: every rank deposits its slice, the last depositor releases them all;
// every rank copies the whole array out, the last to leave opens the next exchange.  A rank that
// fails before its deposit would leave the others waiting: its driver aborts the exchange, which
// ends every current and later wait with KS_EDEVICE (the engines' steps then fail, sticky).
ks_status ks_local_allgather(void* user, int32_t rank, int32_t world, void* buf, int64_t bytes_per_rank) {
    ks_local_exchange* x = static_cast<ks_local_exchange*>(user);
    if (!x || world != x->world || rank < 0 || rank >= world || bytes_per_rank < 0) return KS_EINVAL;
    uint8_t* b = static_cast<uint8_t*>(buf);
    std::unique_lock<std::mutex> lk(x->mu);
    x->cv.wait(lk, [&] { return x->left == 0 || x->aborted; });  // the previous exchange has been read by everyone
    if (x->aborted) return KS_EDEVICE;
    const uint64_t g = x->gen;
    if ((int64_t)x->buf.size() < bytes_per_rank * world) x->buf.resize(bytes_per_rank * world);
    std::memcpy(x->buf.data() + rank * bytes_per_rank, b + rank * bytes_per_rank, bytes_per_rank);
    if (++x->arrived == world) {
        x->arrived = 0;
        x->left = world;
        x->gen++;
        x->cv.notify_all();
    } else {
        x->cv.wait(lk, [&] { return x->gen != g || x->aborted; });
        if (x->gen == g) return KS_EDEVICE;  // aborted before every rank deposited
    }
    std::memcpy(b, x->buf.data(), bytes_per_rank * world);
    if (--x->left == 0) x->cv.notify_all();
    return KS_OK;
}

#ifndef KS_SRC_HASH
#define KS_SRC_HASH "unhashed"
#endif
const char* ks_run_build_id(void) { return KS_SRC_HASH; }

}  // extern "C"
