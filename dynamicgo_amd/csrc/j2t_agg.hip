/*
 * j2t_agg.hip — the batching aggregator behind BinaryConv.Do (SURVEY.md
 * §8(f) row 1).
 *
 * The reference's callers convert ONE message per call, from many goroutines
 * at once (conv/j2t/conv_timing_test.go:76-99, b.RunParallel over
 * BinaryConv.Do, conv/j2t/conv.go:53-77). A GPU needs batches. The
 * aggregator turns concurrent single-message calls into device batches: a
 * caller thread enqueues its message and blocks; one flusher thread per
 * aggregator takes up to max_batch queued messages as soon as max_batch are
 * waiting or the oldest has waited max_wait_us, converts them with one
 * dg_j2t_batch_host call (H2D, kernels, exact-size reruns, D2H) and hands
 * every caller its bytes and the reference's packed status word. A cgo shim
 * calls dg_agg_do from BinaryConv.Do; the Go side keeps its
 * signature.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/dgj2t.h"

namespace {

struct Req {
    const uint8_t *json;
    size_t len;
    uint8_t *out;
    size_t cap;
    size_t out_len = 0;
    uint64_t ret = 0;
    int rc = DG_OK;
    bool done = false;
};

}  // namespace

struct dg_agg {
    dg_ctx *ctx;
    const dg_desc *desc;
    uint32_t root;
    uint64_t flags;
    uint32_t max_batch;
    std::chrono::microseconds max_wait;
    std::mutex mu;
    std::condition_variable cv_in;   /* flusher: work arrived / shutdown */
    std::condition_variable cv_out;  /* callers: their batch is done */
    std::deque<std::pair<Req *, std::chrono::steady_clock::time_point>> q;
    bool stop = false;
    uint64_t batches = 0, msgs = 0;
    std::thread th;
    /* flusher-owned staging, reused across batches */
    std::vector<uint8_t> arena, out;
    std::vector<uint64_t> in_off, out_off, ret;

    void run();
    void flush(std::vector<Req *> &b);
};

void dg_agg::flush(std::vector<Req *> &b)
{
    const size_t n = b.size();
    size_t bytes = 0;
    for (Req *r : b) bytes += r->len;
    arena.resize(bytes + 64);
    in_off.resize(n + 1);
    out_off.resize(n + 1);
    ret.resize(n);
    in_off[0] = 0;
    for (size_t i = 0; i < n; i++) {
        if (b[i]->len) memcpy(arena.data() + in_off[i], b[i]->json, b[i]->len);
        in_off[i + 1] = in_off[i] + b[i]->len;
    }
    memset(arena.data() + bytes, 0, 64);
    uint64_t need = 0;
    if (out.size() < 4 * bytes + 64 * n + 64) out.resize(4 * bytes + 64 * n + 64);
    int rc = dg_j2t_batch_host(ctx, desc, root, arena.data(), in_off.data(), n, flags, out.data(), out.size(),
                               out_off.data(), ret.data(), &need);
    if (rc == DG_E_NOMEM && need > out.size()) {
        out.resize(need + 64);
        rc = dg_j2t_batch_host(ctx, desc, root, arena.data(), in_off.data(), n, flags, out.data(), out.size(),
                               out_off.data(), ret.data(), &need);
    }
    for (size_t i = 0; i < n; i++) {
        Req *r = b[i];
        r->rc = rc;
        if (rc != DG_OK) continue;
        r->ret = ret[i];
        r->out_len = out_off[i + 1] - out_off[i];
        if (r->out_len > r->cap) r->rc = DG_E_NOMEM; /* the caller retries with out_len bytes */
        else if (r->out_len) memcpy(r->out, out.data() + out_off[i], r->out_len);
    }
}

void dg_agg::run()
{
    std::vector<Req *> b;
    for (;;) {
        {
            std::unique_lock<std::mutex> g(mu);
            cv_in.wait(g, [&] { return stop || !q.empty(); });
            if (q.empty() && stop) return;
            /* a full batch, or the oldest request's deadline */
            const auto deadline = q.front().second + max_wait;
            cv_in.wait_until(g, deadline, [&] { return stop || q.size() >= max_batch; });
            b.clear();
            while (!q.empty() && b.size() < max_batch) {
                b.push_back(q.front().first);
                q.pop_front();
            }
        }
        flush(b);
        {
            std::lock_guard<std::mutex> g(mu);
            batches++;
            msgs += b.size();
            for (Req *r : b) r->done = true;
        }
        cv_out.notify_all();
    }
}

extern "C" {

int dg_agg_create(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, uint64_t flags, uint32_t max_batch,
                  uint32_t max_wait_us, dg_agg **out)
{
    if (!ctx || !desc || !out || max_batch == 0) return DG_E_INVALID;
    dg_agg *a = new dg_agg();
    a->ctx = ctx;
    a->desc = desc;
    a->root = root_type;
    a->flags = flags;
    a->max_batch = max_batch;
    a->max_wait = std::chrono::microseconds(max_wait_us);
    a->th = std::thread([a] { a->run(); });
    *out = a;
    return DG_OK;
}

int dg_agg_do(dg_agg *a, const uint8_t *json, size_t len, uint8_t *out, size_t out_cap, size_t *out_len,
              uint64_t *ret)
{
    if (!a || (!json && len) || (!out && out_cap) || !out_len || !ret) return DG_E_INVALID;
    static const uint8_t empty = 0;
    Req r;
    r.json = len ? json : &empty;
    r.len = len;
    r.out = out;
    r.cap = out_cap;
    {
        std::unique_lock<std::mutex> g(a->mu);
        if (a->stop) return DG_E_INVALID;
        a->q.emplace_back(&r, std::chrono::steady_clock::now());
        if (a->q.size() == 1 || a->q.size() >= a->max_batch) a->cv_in.notify_one();
        a->cv_out.wait(g, [&] { return r.done; });
    }
    *out_len = r.out_len;
    *ret = r.ret;
    return r.rc;
}

int dg_agg_stats(dg_agg *a, uint64_t *batches, uint64_t *msgs)
{
    if (!a) return DG_E_INVALID;
    std::lock_guard<std::mutex> g(a->mu);
    if (batches) *batches = a->batches;
    if (msgs) *msgs = a->msgs;
    return DG_OK;
}

void dg_agg_destroy(dg_agg *a)
{
    if (!a) return;
    {
        std::lock_guard<std::mutex> g(a->mu);
        a->stop = true;
    }
    a->cv_in.notify_all();
    a->th.join(); /* drains what is queued first */
    delete a;
}

}  // extern "C"
