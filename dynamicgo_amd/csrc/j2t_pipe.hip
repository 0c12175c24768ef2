/*
 * j2t_pipe.hip — the host-memory paths around the device batch:
 *
 *  1. the batching aggregator behind BinaryConv.Do.
 *     The reference converts ONE message per call, from many goroutines at
 *     once (conv/j2t/conv_timing_test.go:76-99, b.RunParallel over
 *     BinaryConv.Do, conv/j2t/conv.go:53-77). A GPU needs batches, so callers
 *     reserve a place in the open batch with one atomic add, copy their JSON
 *     straight into its pinned upload buffer themselves (in parallel, no lock),
 *     and later copy their Thrift out of its pinned download buffer. A flusher
 *     thread seals a batch when it is full or its first message has waited
 *     max_wait_us, uploads it and launches convert + pack on the batch's own
 *     stream; a completer thread downloads [ret | packed offsets] and then
 *     exactly the packed bytes, and wakes the batch's callers. Up to
 *     AGG_INFLIGHT batches are in flight at once, so uploads, kernels and
 *     downloads of consecutive batches overlap.
 *
 *  2. dg_j2t_pipeline_host: one large host batch (pinned buffers) streamed
 *     through the same per-batch buffers in chunks: H2D, convert, pack, D2H
 *     of chunk k overlap those of chunks k-1 and k+1, all issued from C.
 *
 * Both use PipeBuf: one stream, its events, and the pinned and device
 * buffers of one batch in flight.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "host_internal.h"

namespace {

using Clock = std::chrono::steady_clock;

/* The slot of message i in a batch whose JSON prefix ends at byte e before
 * it: slot_off(e, i) = (4 e + 80 i) & ~7. Slot i is then at least
 * 4 len + 73 >= dg_slot_bound(len) bytes and 8-aligned, and a caller can
 * compute its slot's end from its own reservation alone. */
static inline uint64_t slot_off(uint64_t e, uint64_t i) { return (4 * e + 80 * i) & ~7ull; }

/* one batch in flight: a stream, two events, pinned and device buffers.
 * Upload layout: [in_off (cap_n+1) | out_off (cap_n+1) | JSON (cap_b + 64)];
 * download layout: [ret n | pack_off (n+1) | packed], n = the batch's count */
struct PipeBuf {
    int device = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev_hdr = nullptr, ev_done = nullptr;
    uint64_t cap_n = 0, cap_b = 0;
    uint8_t *h_up = nullptr; uint64_t h_up_cap = 0;
    uint8_t *h_down = nullptr; uint64_t h_down_cap = 0;
    uint8_t *d_up = nullptr; uint64_t d_up_cap = 0;
    uint8_t *d_out = nullptr; uint64_t d_out_cap = 0;
    uint8_t *d_down = nullptr; uint64_t d_down_cap = 0;
    uint32_t *d_ol = nullptr; uint64_t d_ol_cap = 0;

    uint64_t up_bytes(uint64_t n, uint64_t b) const { return 16 * (n + 1) + b + 64 + 16; }
    uint64_t *in_off() { return (uint64_t *)(void *)h_up; }
    uint64_t *out_off() { return (uint64_t *)(void *)h_up + cap_n + 1; }
    uint8_t *json() { return h_up + 16 * (cap_n + 1); }
    uint64_t slot_bytes(uint64_t n, uint64_t b) const { return slot_off(b, n) + 64; }
    static uint64_t down_head(uint64_t n) { return 16 * n + 8; }

    int init(int dev, uint64_t n, uint64_t b)
    {
        device = dev;
        cap_n = n;
        cap_b = b;
        HIPCHK(hipSetDevice(dev));
        HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&ev_hdr, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
        int rc;
        if ((rc = grow_pinned(h_up, h_up_cap, up_bytes(n, b)))) return rc;
        if ((rc = grow_pinned(h_down, h_down_cap, down_head(n) + b + 64))) return rc;
        if ((rc = grow(d_up, d_up_cap, up_bytes(n, b)))) return rc;
        if ((rc = grow(d_out, d_out_cap, slot_bytes(n, b)))) return rc;
        if ((rc = grow(d_down, d_down_cap, down_head(n) + slot_bytes(n, b)))) return rc;
        if ((rc = grow(d_ol, d_ol_cap, n + 1))) return rc;
        in_off()[0] = 0;
        out_off()[0] = 0;
        return DG_OK;
    }
    void release()
    {
        if (s) (void)hipStreamSynchronize(s);
        (void)hipHostFree(h_up);
        (void)hipHostFree(h_down);
        (void)hipFree(d_up);
        (void)hipFree(d_out);
        (void)hipFree(d_down);
        (void)hipFree(d_ol);
        if (ev_hdr) (void)hipEventDestroy(ev_hdr);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (s) (void)hipStreamDestroy(s);
        s = nullptr;
    }

    /* H2D of n messages (b JSON bytes, in h_up or at hjson), convert +
     * pack, D2H of [ret | pack_off]; ev_hdr follows. Device JSON pointer is
     * d_up + 16 (cap_n + 1), 16-aligned, with 64 zero bytes after the end. */
    int enqueue(dg_ctx *c, const dg_desc *d, uint32_t root, uint64_t flags, uint64_t n, uint64_t b, uint64_t max_len,
                const uint8_t *hjson = nullptr)
    {
        HIPCHK(hipSetDevice(device));
        const uint64_t jo = 16 * (cap_n + 1);
        HIPCHK(hipMemcpyAsync(d_up, h_up, 8 * (n + 1), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(d_up + 8 * (cap_n + 1), h_up + 8 * (cap_n + 1), 8 * (n + 1), hipMemcpyHostToDevice, s));
        if (hjson) {
            if (b) HIPCHK(hipMemcpyAsync(d_up + jo, hjson, b, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemsetAsync(d_up + jo + b, 0, 64, s));
        } else {
            HIPCHK(hipMemcpyAsync(d_up + jo, h_up + jo, b + 64, hipMemcpyHostToDevice, s));
        }
        uint64_t *d_ret = (uint64_t *)(void *)d_down, *d_po = d_ret + n;
        int rc = dg_i_convert_pack(c, d, root, d_up + jo, (const uint64_t *)(void *)d_up, n, flags, d_out,
                                   (const uint64_t *)(void *)(d_up + 8 * (cap_n + 1)), d_ol, d_ret,
                                   d_down + down_head(n), d_po, s, max_len);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(h_down, d_down, down_head(n), hipMemcpyDeviceToHost, s));
        HIPCHK(hipEventRecord(ev_hdr, s));
        return DG_OK;
    }
    /* after ev_hdr: D2H of the packed bytes to dst (pinned), ev_done follows */
    int download(uint64_t n, uint8_t *dst)
    {
        HIPCHK(hipSetDevice(device));
        const uint64_t total = ((const uint64_t *)(const void *)h_down)[2 * n];
        if (total) HIPCHK(hipMemcpyAsync(dst, d_down + down_head(n), total, hipMemcpyDeviceToHost, s));
        HIPCHK(hipEventRecord(ev_done, s));
        return DG_OK;
    }
    const uint64_t *ret() const { return (const uint64_t *)(const void *)h_down; }
    const uint64_t *pack_off(uint64_t n) const { return ret() + n; }
};

constexpr uint64_t SEALED = 1ull << 63;
constexpr int CNT_SHIFT = 40;
constexpr uint64_t CNT_MASK = (1ull << 23) - 1;
constexpr uint64_t BYTE_MASK = (1ull << CNT_SHIFT) - 1;
constexpr int AGG_INFLIGHT = 4;

/* one aggregator batch: lives in a ring of AGG_INFLIGHT, reused when its
 * last caller has copied its result out */
struct Batch {
    PipeBuf pb;
    /* SEALED | count << 40 | bytes: one fetch_add reserves (index, offset) */
    std::atomic<uint64_t> state{0};
    /* per reserved index: 0 pending, 1 filled, 2 failed (did not fit) */
    std::atomic<uint8_t> *status = nullptr;
    std::atomic<uint64_t> gen{0};        /* generation number of the current fill */
    std::atomic<int64_t> t_first{0};     /* ns timestamp of reservation 0 */
    std::atomic<int64_t> k_seal{-1};     /* reservations made before the seal (-1: not sealed yet) */
    uint32_t k_prev = 0;                 /* k_seal of the previous generation (status entries to clear) */
    uint32_t n = 0;                      /* messages in the sealed batch */
    uint64_t bytes = 0;
    std::atomic<uint32_t> consumed{0};
    int rc = DG_OK;
    uint8_t *h_packed = nullptr; uint64_t h_packed_cap = 0;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t done_gen = 0;               /* under mu: last generation whose results are readable */
    bool free_ = true;                   /* under the aggregator's mu: every caller is done with it */
};

}  // namespace

struct dg_agg {
    dg_ctx *ctx;
    const dg_desc *desc;
    uint32_t root;
    uint64_t flags;
    uint32_t max_batch;
    uint64_t max_bytes;
    std::chrono::nanoseconds max_wait;
    Batch b[AGG_INFLIGHT];
    std::atomic<Batch *> cur{nullptr};
    uint32_t cur_i = 0;
    std::mutex mu;                       /* cur changes, seal notices, frees, completer queue */
    std::condition_variable cv_flush;    /* flusher: a seal, a first reservation, a free batch, stop */
    std::condition_variable cv_cur;      /* callers: cur moved on */
    std::condition_variable cv_done;     /* completer: a batch in flight */
    std::deque<Batch *> inflight;
    bool stop = false;
    std::atomic<uint64_t> batches{0}, msgs{0};
    std::thread flusher, completer;

    static int64_t now_ns() { return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count(); }

    void seal(Batch *x)
    {
        const uint64_t prev = x->state.fetch_or(SEALED, std::memory_order_acq_rel);
        if (prev & SEALED) return;
        {
            std::lock_guard<std::mutex> g(mu);
            x->k_seal.store((int64_t)std::min<uint64_t>((prev >> CNT_SHIFT) & CNT_MASK, max_batch),
                            std::memory_order_release);
        }
        cv_flush.notify_one();
    }
    /* reserve a place for len bytes: true with (batch, gen, idx, off), or
     * false when the batch closed first (the caller waits for the next) */
    bool reserve(Batch *x, uint64_t len, uint64_t &gen, uint32_t &idx, uint64_t &off)
    {
        const uint64_t old = x->state.fetch_add((1ull << CNT_SHIFT) | len, std::memory_order_acq_rel);
        if (old & SEALED) return false;
        const uint64_t i = (old >> CNT_SHIFT) & CNT_MASK;
        off = old & BYTE_MASK;
        if (i < max_batch && off + len <= max_bytes) {
            idx = (uint32_t)i;
            gen = x->gen.load(std::memory_order_acquire);
            if (i == 0) {
                x->t_first.store(now_ns(), std::memory_order_release);
                {
                    std::lock_guard<std::mutex> g(mu); /* the flusher checks t_first under mu */
                }
                cv_flush.notify_one();
            }
            return true;
        }
        if (i < max_batch) x->status[i].store(2, std::memory_order_release);
        seal(x);
        return false;
    }
    void fill(Batch *x, uint32_t idx, uint64_t off, const uint8_t *json, uint64_t len)
    {
        PipeBuf &p = x->pb;
        if (len) memcpy(p.json() + off, json, len);
        p.in_off()[idx + 1] = off + len;
        p.out_off()[idx + 1] = slot_off(off + len, idx + 1);
        x->status[idx].store(1, std::memory_order_release);
        if (idx + 1 == max_batch) seal(x);
    }

    void run_flusher();
    void run_completer();
    void launch_batch(Batch *x);
};

void dg_agg::launch_batch(Batch *x)
{
    /* the callers that reserved before the seal are each filling or failing:
     * wait for every one of them (a failed one writes its status too), so
     * no caller touches this batch's staging once it is recycled */
    const uint32_t k = (uint32_t)x->k_seal.load(std::memory_order_acquire);
    x->k_prev = k;
    uint32_t n = k;
    for (uint32_t i = 0; i < k; i++) {
        uint8_t st;
        while ((st = x->status[i].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
        if (st == 2 && i < n) n = i;
    }
    x->n = n;
    x->rc = DG_OK;
    PipeBuf &p = x->pb;
    uint64_t max_len = 1;
    const uint64_t *io = p.in_off();
    for (uint32_t i = 0; i < n; i++) max_len = std::max<uint64_t>(max_len, io[i + 1] - io[i]);
    x->bytes = io[n];
    memset(p.json() + x->bytes, 0, 64);
    if (n) x->rc = p.enqueue(ctx, desc, root, flags, n, x->bytes, max_len);
    batches.fetch_add(n ? 1 : 0, std::memory_order_relaxed);
    msgs.fetch_add(n, std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(mu);
        inflight.push_back(x);
    }
    cv_done.notify_one();
}

void dg_agg::run_flusher()
{
    for (;;) {
        Batch *x = cur.load(std::memory_order_acquire);
        {
            std::unique_lock<std::mutex> g(mu);
            for (;;) {
                /* sealed: by a caller that did not fit, by the caller that
                 * took the last index, or below on the deadline / at stop */
                if (x->k_seal.load(std::memory_order_acquire) >= 0) break;
                const uint64_t st = x->state.load(std::memory_order_acquire);
                const bool any = ((st >> CNT_SHIFT) & CNT_MASK) != 0;
                if (stop && !any) {
                    inflight.push_back(nullptr); /* the completer's exit marker */
                    g.unlock();
                    cv_done.notify_one();
                    return;
                }
                const int64_t t0 = x->t_first.load(std::memory_order_acquire);
                if (stop || (t0 && now_ns() - t0 >= max_wait.count())) {
                    g.unlock();
                    seal(x);
                    g.lock();
                    continue;
                }
                if (t0) cv_flush.wait_for(g, std::chrono::nanoseconds(max_wait.count() - (now_ns() - t0)));
                else cv_flush.wait_for(g, std::chrono::milliseconds(5));
            }
        }
        launch_batch(x);
        /* the next batch of the ring, once its last caller has copied out */
        const uint32_t ni = (cur_i + 1) % AGG_INFLIGHT;
        Batch *y = &b[ni];
        {
            std::unique_lock<std::mutex> g(mu);
            cv_flush.wait(g, [&] { return y->free_; });
            y->free_ = false;
        }
        y->gen.fetch_add(1, std::memory_order_acq_rel);
        y->t_first.store(0, std::memory_order_relaxed);
        y->consumed.store(0, std::memory_order_relaxed);
        for (uint32_t i = 0; i < y->k_prev; i++) y->status[i].store(0, std::memory_order_relaxed);
        y->k_seal.store(-1, std::memory_order_relaxed);
        y->state.store(0, std::memory_order_release);
        {
            std::lock_guard<std::mutex> g(mu);
            cur.store(y, std::memory_order_release);
            cur_i = ni;
        }
        cv_cur.notify_all();
    }
}

void dg_agg::run_completer()
{
    for (;;) {
        Batch *x;
        {
            std::unique_lock<std::mutex> g(mu);
            cv_done.wait(g, [&] { return !inflight.empty(); });
            x = inflight.front();
            inflight.pop_front();
        }
        if (!x) return;
        PipeBuf &p = x->pb;
        if (x->n && x->rc == DG_OK) {
            hipError_t e = hipEventSynchronize(p.ev_hdr);
            if (e != hipSuccess) x->rc = set_err(DG_E_HIP, "aggregator batch: %s", hipGetErrorString(e));
        }
        if (x->n && x->rc == DG_OK) {
            const uint64_t total = p.pack_off(x->n)[x->n];
            x->rc = grow_pinned(x->h_packed, x->h_packed_cap, total + 64);
            if (x->rc == DG_OK) x->rc = p.download(x->n, x->h_packed);
            if (x->rc == DG_OK) {
                hipError_t e = hipEventSynchronize(p.ev_done);
                if (e != hipSuccess) x->rc = set_err(DG_E_HIP, "aggregator download: %s", hipGetErrorString(e));
            }
        }
        const bool empty = x->n == 0;
        {
            std::lock_guard<std::mutex> g(x->mu);
            x->done_gen = x->gen.load(std::memory_order_acquire);
        }
        x->cv.notify_all();
        if (empty) {
            std::lock_guard<std::mutex> g(mu);
            x->free_ = true;
            cv_flush.notify_one();
        }
    }
}

void dg_i_pipe_free(dg_ctx *c)
{
    for (void *q : c->pipe) {
        ((PipeBuf *)q)->release();
        delete (PipeBuf *)q;
    }
    c->pipe.clear();
}

extern "C" {

int dg_agg_create2(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, uint64_t flags, uint32_t max_batch,
                   uint64_t max_bytes, uint32_t max_wait_us, dg_agg **out)
{
    if (!ctx || !desc || !out || max_batch == 0 || max_batch > CNT_MASK / 2 || max_bytes == 0 ||
        max_bytes > (BYTE_MASK >> 2))
        return set_err(DG_E_INVALID, "bad args");
    dg_agg *a = new dg_agg();
    a->ctx = ctx;
    a->desc = desc;
    a->root = root_type;
    a->flags = flags;
    a->max_batch = max_batch;
    a->max_bytes = max_bytes;
    a->max_wait = std::chrono::microseconds(max_wait_us);
    for (Batch &x : a->b) {
        x.status = new std::atomic<uint8_t>[max_batch];
        for (uint32_t i = 0; i < max_batch; i++) x.status[i].store(0, std::memory_order_relaxed);
        int rc = x.pb.init(ctx->device, max_batch, max_bytes);
        if (rc == DG_OK) rc = grow_pinned(x.h_packed, x.h_packed_cap, max_bytes + 64);
        if (rc) {
            for (Batch &y : a->b) {
                y.pb.release();
                (void)hipHostFree(y.h_packed);
                delete[] y.status;
            }
            delete a;
            return rc;
        }
    }
    a->b[0].free_ = false;
    a->b[0].gen.store(1);
    a->cur.store(&a->b[0]);
    a->flusher = std::thread([a] { a->run_flusher(); });
    a->completer = std::thread([a] { a->run_completer(); });
    *out = a;
    return DG_OK;
}

int dg_agg_create(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, uint64_t flags, uint32_t max_batch,
                  uint32_t max_wait_us, dg_agg **out)
{
    /* room for max_batch messages of 512 B on average (at least 1 MiB) */
    const uint64_t mb = std::max<uint64_t>(1ull << 20, 512ull * max_batch);
    return dg_agg_create2(ctx, desc, root_type, flags, max_batch, mb, max_wait_us, out);
}

int dg_agg_submit(dg_agg *a, const uint8_t *json, size_t len, int nonblock, dg_agg_ticket *t)
{
    if (!a || (!json && len) || !t) return set_err(DG_E_INVALID, "bad args");
    static const uint8_t empty = 0;
    t->json = len ? json : &empty;
    t->len = len;
    if (len > a->max_bytes) { /* never fits a batch: converted alone by dg_agg_wait */
        t->batch = nullptr;
        return DG_OK;
    }
    for (;;) {
        Batch *x = a->cur.load(std::memory_order_acquire);
        uint64_t gen, off;
        uint32_t idx;
        if (a->reserve(x, len, gen, idx, off)) {
            a->fill(x, idx, off, t->json, len);
            t->batch = x;
            t->gen = gen;
            t->idx = idx;
            return DG_OK;
        }
        std::unique_lock<std::mutex> g(a->mu);
        if (a->stop) return set_err(DG_E_INVALID, "aggregator closed");
        if (a->cur.load(std::memory_order_acquire) != x) continue;
        if (nonblock) return DG_E_AGAIN; /* the next batch is not free yet */
        a->cv_cur.wait(g, [&] { return a->cur.load(std::memory_order_acquire) != x || a->stop; });
    }
}

int dg_agg_wait(dg_agg *a, dg_agg_ticket *t, uint8_t *out, size_t out_cap, size_t *out_len, uint64_t *ret)
{
    if (!a || !t || (!out && out_cap) || !out_len || !ret) return set_err(DG_E_INVALID, "bad args");
    Batch *x = (Batch *)t->batch;
    bool redo = x == nullptr;
    int rc = DG_OK;
    if (x) {
        {
            std::unique_lock<std::mutex> g(x->mu);
            x->cv.wait(g, [&] { return x->done_gen >= t->gen; });
        }
        rc = x->rc;
        if (rc == DG_OK) {
            const uint64_t r = x->pb.ret()[t->idx];
            if ((uint8_t)r == DG_ST_OUT_OVERFLOW) {
                redo = true; /* its slot was too small: alone, at its exact size */
            } else {
                const uint64_t *po = x->pb.pack_off(x->n);
                const uint64_t l = po[t->idx + 1] - po[t->idx];
                *ret = r;
                *out_len = l;
                if (l > out_cap) rc = DG_E_NOMEM; /* the caller retries with out_len bytes */
                else if (l) memcpy(out, x->h_packed + po[t->idx], l);
            }
        }
        if (x->consumed.fetch_add(1, std::memory_order_acq_rel) + 1 == x->n) {
            std::lock_guard<std::mutex> g(a->mu);
            x->free_ = true;
            a->cv_flush.notify_one();
        }
    }
    t->batch = nullptr;
    if (redo && rc == DG_OK) {
        rc = dg_j2t_do(a->ctx, a->desc, a->root, t->json, t->len, a->flags, out, out_cap, out_len, ret);
        if (rc == DG_E_NOMEM && *out_len <= out_cap) rc = DG_OK;
    }
    return rc;
}

int dg_agg_do(dg_agg *a, const uint8_t *json, size_t len, uint8_t *out, size_t out_cap, size_t *out_len,
              uint64_t *ret)
{
    dg_agg_ticket t;
    int rc = dg_agg_submit(a, json, len, 0, &t);
    if (rc) return rc;
    return dg_agg_wait(a, &t, out, out_cap, out_len, ret);
}

int dg_agg_stats(dg_agg *a, uint64_t *batches, uint64_t *msgs)
{
    if (!a) return set_err(DG_E_INVALID, "null aggregator");
    if (batches) *batches = a->batches.load();
    if (msgs) *msgs = a->msgs.load();
    return DG_OK;
}

void dg_agg_destroy(dg_agg *a)
{
    if (!a) return;
    {
        std::lock_guard<std::mutex> g(a->mu);
        a->stop = true;
    }
    a->cv_flush.notify_all();
    a->cv_cur.notify_all();
    a->flusher.join(); /* converts what is reserved first */
    a->completer.join();
    for (Batch &x : a->b) {
        x.pb.release();
        (void)hipHostFree(x.h_packed);
        delete[] x.status;
    }
    delete a;
}

/* One host batch streamed through PIPE_BUFS per-chunk buffers on their own
 * streams (see the file comment); the contract of dg_j2t_batch_host. */
constexpr int PIPE_BUFS = 3;

int dg_j2t_pipeline_host(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *json, const uint64_t *in_off,
                         uint64_t n, uint64_t flags, uint32_t chunks, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                         uint64_t *ret, uint64_t *out_need)
{
    if (!c || !d || (!json && n) || !in_off || !out_off || (!ret && n) || chunks == 0 || (!out && out_cap))
        return set_err(DG_E_INVALID, "bad args");
    if (n == 0) {
        out_off[0] = 0;
        if (out_need) *out_need = 0;
        return DG_OK;
    }
    chunks = (uint32_t)std::min<uint64_t>(chunks, n);
    std::vector<uint64_t> cb(chunks + 1);
    uint64_t cap_n = 0, cap_b = 0;
    for (uint32_t k = 0; k <= chunks; k++) cb[k] = n * k / chunks;
    for (uint32_t k = 0; k < chunks; k++) {
        cap_n = std::max(cap_n, cb[k + 1] - cb[k]);
        cap_b = std::max(cap_b, in_off[cb[k + 1]] - in_off[cb[k]]);
    }
    /* the buffers live in the context, reused across calls (grown on demand) */
    std::lock_guard<std::mutex> pg(c->pipe_mu);
    const int nb = (int)std::min<uint32_t>(PIPE_BUFS, chunks);
    if (c->pipe.size() < (size_t)nb || c->pipe_cap_n < cap_n || c->pipe_cap_b < cap_b) {
        for (void *q : c->pipe) {
            ((PipeBuf *)q)->release();
            delete (PipeBuf *)q;
        }
        c->pipe.clear();
        c->pipe_cap_n = std::max(cap_n, c->pipe_cap_n);
        c->pipe_cap_b = std::max(cap_b, c->pipe_cap_b);
        for (int i = 0; i < PIPE_BUFS; i++) {
            PipeBuf *q = new PipeBuf();
            c->pipe.push_back(q);
            int rc = q->init(c->device, c->pipe_cap_n, c->pipe_cap_b);
            if (rc) return rc;
        }
    }
    uint64_t cursor = 0, need = 0;
    bool fits = true;
    std::vector<uint64_t> redo;
    /* chunk k's results: header read, packed bytes downloaded to out (or
     * only counted once out_cap is exceeded) */
    auto drain = [&](uint32_t k) -> int {
        PipeBuf &p = *(PipeBuf *)c->pipe[k % nb];
        const uint64_t a = cb[k], m = cb[k + 1] - a;
        HIPCHK(hipEventSynchronize(p.ev_hdr));
        const uint64_t *r = p.ret(), *po = p.pack_off(m);
        const uint64_t total = po[m];
        memcpy(ret + a, r, 8 * m);
        for (uint64_t j = 0; j < m; j++) {
            out_off[a + j] = cursor + po[j];
            if ((uint8_t)r[j] == DG_ST_OUT_OVERFLOW) redo.push_back(a + j);
        }
        if (fits && cursor + total > out_cap) fits = false;
        if (fits) {
            int rc = p.download(m, out + cursor);
            if (rc) return rc;
        }
        cursor += total;
        return DG_OK;
    };
    for (uint32_t k = 0; k < chunks; k++) {
        if (k >= (uint32_t)nb) {
            int rc = drain(k - nb);
            if (rc) return rc;
        }
        PipeBuf &p = *(PipeBuf *)c->pipe[k % nb];
        if (k >= (uint32_t)nb) HIPCHK(hipEventSynchronize(p.ev_hdr)); /* its staging is free again */
        const uint64_t a = cb[k], m = cb[k + 1] - a, base = in_off[a];
        uint64_t *io = p.in_off(), *oo = p.out_off(), max_len = 1;
        for (uint64_t j = 0; j <= m; j++) {
            io[j] = in_off[a + j] - base;
            oo[j] = slot_off(io[j], j);
        }
        for (uint64_t j = 0; j < m; j++) max_len = std::max<uint64_t>(max_len, io[j + 1] - io[j]);
        int rc = p.enqueue(c, d, root, flags, m, io[m], max_len, json + base);
        if (rc) return rc;
    }
    for (uint32_t k = chunks > (uint32_t)nb ? chunks - nb : 0; k < chunks; k++) {
        int rc = drain(k);
        if (rc) return rc;
    }
    for (int i = 0; i < nb; i++) HIPCHK(hipStreamSynchronize(((PipeBuf *)c->pipe[i])->s));
    out_off[n] = cursor;
    need = cursor;
    if (!redo.empty()) {
        /* slot overflows (rare): each alone at its exact size, spliced in
         * place; later messages move up */
        std::vector<std::vector<uint8_t>> res(redo.size());
        uint64_t extra = 0;
        for (size_t q = 0; q < redo.size(); q++) {
            const uint64_t i = redo[q];
            size_t ol = 0;
            uint64_t r = 0;
            res[q].resize(4 * (in_off[i + 1] - in_off[i]) + 256);
            for (int t = 0; t < 2; t++) {
                int rc = dg_j2t_do(c, d, root, json + in_off[i], in_off[i + 1] - in_off[i], flags, res[q].data(),
                                   res[q].size(), &ol, &r);
                if (rc == DG_E_NOMEM && ol > res[q].size()) {
                    res[q].resize(ol);
                    continue;
                }
                if (rc) return rc;
                break;
            }
            res[q].resize(r == 0 ? ol : 0);
            ret[i] = r;
            extra += res[q].size();
        }
        need = cursor + extra;
        if (fits && need <= out_cap) {
            /* move every segment between reruns up by the bytes inserted before it */
            uint64_t shift = extra;
            uint64_t end = cursor;
            for (size_t q = redo.size(); q-- > 0;) {
                const uint64_t i = redo[q], at = out_off[i];
                shift -= res[q].size();
                memmove(out + at + shift + res[q].size(), out + at, end - at);
                memcpy(out + at + shift, res[q].data(), res[q].size());
                end = at;
            }
            uint64_t add = 0;
            size_t q = 0;
            for (uint64_t i = 0; i <= n; i++) {
                while (q < redo.size() && redo[q] < i) add += res[q++].size();
                out_off[i] += add;
            }
        } else {
            fits = false;
        }
    }
    if (out_need) *out_need = need;
    return fits ? DG_OK : set_err(DG_E_NOMEM, "output needs %llu bytes", (unsigned long long)need);
}

int dg_agg_drive(dg_agg *a, const uint8_t *arena, const uint64_t *in_off, uint64_t n, int threads, int window,
                 uint8_t *out, const uint64_t *out_off, uint64_t *out_len, uint64_t *ret, uint32_t *lat_ns,
                 double *seconds)
{
    if (!a || !arena || !in_off || threads < 1 || window < 1 || !out || !out_off || !out_len || !ret || !seconds)
        return set_err(DG_E_INVALID, "bad args");
    std::atomic<int> ready{0}, failed{0};
    std::atomic<bool> go{false};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        th.emplace_back([&, t] {
            /* messages [lo, hi) in order; at most `window` submitted and not
             * yet waited for: [h, i) */
            const uint64_t lo = n * t / threads, hi = n * (t + 1) / threads;
            std::vector<dg_agg_ticket> ring(window);
            std::vector<int64_t> t0(window);
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            uint64_t h = lo;
            auto finish = [&]() {
                const uint64_t j = h++;
                const int k = (int)((j - lo) % window);
                size_t ol = 0;
                int rc = dg_agg_wait(a, &ring[k], out + out_off[j], out_off[j + 1] - out_off[j], &ol, &ret[j]);
                if (lat_ns) lat_ns[j] = (uint32_t)std::min<int64_t>(dg_agg::now_ns() - t0[k], 0xffffffffll);
                out_len[j] = ol;
                if (rc) failed.fetch_add(1);
            };
            for (uint64_t i = lo; i < hi; i++) {
                while (i - h >= (uint64_t)window) finish();
                const int k = (int)((i - lo) % window);
                t0[k] = dg_agg::now_ns();
                for (;;) {
                    int rc = dg_agg_submit(a, arena + in_off[i], in_off[i + 1] - in_off[i], 1, &ring[k]);
                    if (rc == DG_OK) break;
                    if (rc != DG_E_AGAIN) {
                        failed.fetch_add(1);
                        ring[k].batch = nullptr;
                        break;
                    }
                    /* no open batch: the oldest one frees when its callers
                     * (this thread among them) take their results */
                    if (h < i) finish();
                    else std::this_thread::yield();
                }
            }
            while (h < hi) finish();
        });
    }
    while (ready.load() < threads) std::this_thread::yield();
    const auto ts = Clock::now();
    go.store(true, std::memory_order_release);
    for (auto &x : th) x.join();
    *seconds = std::chrono::duration<double>(Clock::now() - ts).count();
    return failed.load() ? set_err(DG_E_HIP, "%d aggregator calls failed", failed.load()) : DG_OK;
}

}  // extern "C"
