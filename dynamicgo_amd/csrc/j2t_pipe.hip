/*
 * j2t_pipe.hip — the host-memory paths around the device batch:
 *
 *  1. The batching aggregator behind BinaryConv.Do.
 *     The reference converts ONE message per call, from many goroutines at
 *     once (conv/j2t/conv_timing_test.go:76-99, b.RunParallel over
 *     BinaryConv.Do, conv/j2t/conv.go:53-77). A GPU needs batches. Every
 *     caller thread owns a sub-batch of the open batch (a pinned JSON region
 *     and its message ends), so a call touches no shared cache line: it
 *     copies its JSON into its own region and bumps its own count. A flusher
 *     thread seals the open batch (a seq_cst handshake with a per-thread busy
 *     flag), uploads every non-empty sub-batch, builds the batch's offsets on
 *     the device and launches convert + pack on the batch's own stream; a
 *     completer thread downloads [ret | packed offsets], then exactly the
 *     packed bytes, and wakes the callers, who copy their results out.
 *     the ring's batches (16) rotate, so uploads, kernels and downloads of
 *     consecutive batches overlap.
 *
 *  2. dg_j2t_pipeline_host: one large host batch (pinned buffers) streamed
 *     in chunks through PIPE_BUFS stream-private buffer sets: the upload of
 *     chunk k+1, the kernels of chunk k and the download of chunk k-1
 *     overlap, all issued from C; slot offsets are computed on the device.
 */
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include <linux/membarrier.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "host_internal.h"

namespace {

/* the seal handshake's asymmetric fence: callers pay no StoreLoad fence per
 * call; the flusher, once per batch, makes every thread of the process
 * execute one (Linux membarrier, private expedited) */
int sys_membarrier(int cmd) { return (int)syscall(__NR_membarrier, cmd, 0, 0); }

using Clock = std::chrono::steady_clock;

/* The slot of message i of a batch whose JSON before it ends at byte e:
 * slot_off(e, i) = (4 e + 80 i) & ~7. Slot i is then at least
 * 4 len + 73 >= dg_slot_bound(len) bytes and 8-aligned, and its offset
 * follows from (start, index) alone. */
__host__ __device__ inline uint64_t slot_off(uint64_t e, uint64_t i) { return (4 * e + 80 * i) & ~7ull; }

/* ---------------- device: offsets of a batch ---------------- */

typedef __attribute__((address_space(1))) uint8_t pgu8;
typedef __attribute__((address_space(1))) uint64_t pgu64;

/* one sub-batch of an aggregator batch: its messages are global indices
 * [gbase, gbase + n), its JSON bytes [jbase, jbase + bytes) */
struct SubRef {
    uint64_t gbase, jbase, n;
    const uint8_t *h;   /* the part's pinned host buffer: [ends (cap_n u64) | JSON] */
    uint64_t bytes;     /* its JSON bytes */
};

/* Gather of an aggregator batch: block (b, y) copies bytes [y G, y G + G)
 * of part b's JSON from pinned host memory (16-byte aligned loads over the
 * link, through LDS) to d_json + jbase, byte-exact at the words it shares
 * with its neighbours; blocks (b, 0) also turn the part's message ends into
 * the batch's in_off / out_off entries (and the last part's block writes
 * entry N and the 64 zero bytes after the JSON). One launch for the whole
 * upload, with enough blocks to keep many reads over the link in flight.
 * cap_n: the ends area of every part (u64 entries). */
constexpr uint64_t AGG_GATHER_BYTES = 16384; /* G: JSON bytes per gather block */
__global__ __launch_bounds__(256) void agg_gather_kernel(const SubRef *tab, uint64_t cap_n, uint8_t *d_json,
                                                         uint64_t N, uint64_t B, uint64_t *in_off, uint64_t *out_off)
{
    __shared__ __attribute__((aligned(16))) uint64_t st[4096 / 8 + 2];
    const SubRef r = tab[blockIdx.x];
    const uint64_t y0 = (uint64_t)blockIdx.y * AGG_GATHER_BYTES;
    if (y0 >= r.bytes && (blockIdx.y || !r.n)) return;
    if (blockIdx.y == 0) {
        const uint64_t *ends = (const uint64_t *)(const void *)r.h;
        for (uint64_t j = threadIdx.x; j < r.n; j += 256) {
            const uint64_t start = r.jbase + (j ? ends[j - 1] : 0);
            in_off[r.gbase + j] = start;
            out_off[r.gbase + j] = slot_off(start, r.gbase + j);
        }
        if (r.gbase + r.n == N) {
            if (threadIdx.x == 0) {
                in_off[N] = B;
                out_off[N] = slot_off(B, N);
            }
            if (threadIdx.x < 64) d_json[B + threadIdx.x] = 0;
        }
    }
    const uint8_t *src = r.h + 8 * cap_n; /* 16-aligned (cap_n even, see dg_agg_create2) */
    const uint64_t yend = y0 + AGG_GATHER_BYTES < r.bytes ? y0 + AGG_GATHER_BYTES : r.bytes;
    for (uint64_t c0 = y0; c0 < yend; c0 += 4096) {
        const uint64_t cn = yend - c0 < 4096 ? yend - c0 : 4096;
        __syncthreads();
        for (uint64_t k = threadIdx.x; k * 16 < cn; k += 256)
            ((uint4 *)(void *)st)[k] = ((const uint4 *)(const void *)(src + c0))[k];
        if (threadIdx.x < 2) st[(cn + 7) / 8 + threadIdx.x] = 0;
        __syncthreads();
        /* destination words of [jbase + c0, + cn) */
        const uintptr_t d0 = (uintptr_t)(d_json + r.jbase + c0), wb = d0 & ~(uintptr_t)7;
        const uint32_t lead = (uint32_t)(d0 - wb);
        const uint64_t nw = (lead + cn + 7) / 8;
        for (uint64_t k = threadIdx.x; k < nw; k += 256) {
            const int64_t off = (int64_t)k * 8 - lead; /* chunk offset of the word's first byte */
            pgu8 *w = (pgu8 *)(void *)(wb + k * 8);
            if (off >= 0 && off + 8 <= (int64_t)cn) {
                const uint32_t b = (uint32_t)off, sh = (b & 7) * 8;
                const uint64_t lo = st[b >> 3], hi = st[(b >> 3) + 1];
                *(pgu64 *)w = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
            } else {
                for (int q = 0; q < 8; q++) {
                    const int64_t o = off + q;
                    if (o >= 0 && o < (int64_t)cn) w[q] = ((const uint8_t *)(const void *)st)[o];
                }
            }
        }
    }
}

/* out_off of a chunk [a, a + m) of a host batch, from its raw offsets (in
 * device or pinned host memory), and the 64 zero bytes after its staged JSON
 * (pad; NULL when the kernels read the caller's pinned JSON in place) */
__global__ __launch_bounds__(256) void pipe_slots_kernel(const uint64_t *in_off, uint64_t m, uint64_t *out_off,
                                                         uint8_t *pad)
{
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j <= m) out_off[j] = slot_off(in_off[j] - in_off[0], j);
    if (pad && blockIdx.x == 0 && threadIdx.x < 8) ((uint64_t *)(void *)pad)[threadIdx.x] = 0;
}

/* A chunk's results into pinned host memory, after the previous chunk's:
 * base = *base_ptr (0 for the first chunk) is where its bytes start in dst.
 * The packing laid them out with dst's 16-byte phase at base (src_off[0] =
 * phase), so the copy is whole aligned 16-byte stores except at both ends,
 * where bytes of neighbouring chunks share a word (byte stores). Also
 * dst_off[i] = absolute offsets (dst_off[n] = the next chunk's base) and the
 * status words; nothing is written at or past dst_cap. */
__global__ __launch_bounds__(256) void pipe_copy_out_kernel(const uint8_t *src, const uint64_t *src_off, uint64_t n,
                                                            const uint64_t *ret_src, uint8_t *dst, uint64_t *dst_off,
                                                            uint64_t *ret_dst, const uint64_t *base_ptr,
                                                            uint64_t dst_cap, uint64_t *cur_out)
{
    __shared__ uint64_t s_base;
    if (threadIdx.x == 0) s_base = base_ptr ? *(volatile const uint64_t *)base_ptr : 0;
    __syncthreads();
    const uint64_t base = s_base;
    const uint64_t ph = ((uintptr_t)dst + base) & 15, wb = base - ph; /* src[x] -> dst[wb + x] */
    const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, nth = (uint64_t)gridDim.x * 256;
    for (uint64_t i = tid; i <= n; i += nth) {
        dst_off[i] = wb + src_off[i];
        if (i < n) ret_dst[i] = ret_src[i];
        else *cur_out = wb + src_off[i]; /* the next chunk's base, in device memory */
    }
    const uint64_t end = src_off[n];
    /* local bytes below dst_cap: dst_cap - wb without the wrap of wb = base - ph
     * when base < ph (the first chunk into a destination not 16-aligned) */
    const uint64_t lim = dst_cap + ph > base ? dst_cap + ph - base : 0;
    const uint64_t stop = end < lim ? end : lim;
    for (uint64_t w = tid; w * 16 < stop; w += nth) {
        const uint64_t lo = w * 16, hi = lo + 16;
        const uint64_t a = lo < ph ? ph : lo, b = hi < stop ? hi : stop;
        if (a == lo && b == hi) {
            *(uint4 *)(void *)(dst + wb + lo) = *(const uint4 *)(const void *)(src + lo);
        } else {
            for (uint64_t x = a; x < b; x++) dst[wb + x] = src[x];
        }
    }
}

/* device buffers of one batch in flight, grown on demand while idle:
 * [in_off | out_off] offsets, JSON, slots, out_len, ret */
struct DevBuf {
    uint64_t *d_off = nullptr; uint64_t off_cap = 0;   /* in_off (n+1) | out_off (n+1) */
    uint8_t *d_json = nullptr; uint64_t json_cap = 0;
    uint8_t *d_out = nullptr; uint64_t out_cap = 0;
    uint32_t *d_ol = nullptr; uint64_t ol_cap = 0;
    uint64_t *d_ret = nullptr; uint64_t ret_cap = 0;

    bool fits(uint64_t n, uint64_t b) const
    {
        return off_cap >= 2 * (n + 1) && json_cap >= b + 64 + 16 && out_cap >= slot_off(b, n) + 64 &&
               ol_cap >= n + 1 && ret_cap >= n + 1;
    }
    /* callers make sure no launch still uses the buffers when they grow.
     * Growth is sized for twice the batch that needed it (every buffer at
     * once): hipFree waits for the whole device, so a ring of batches whose
     * sizes wander must stop growing after its first few batches */
    int reserve(uint64_t n, uint64_t b, bool exact = false)
    {
        if (fits(n, b)) return DG_OK;
        int rc;
        if (!exact) {
            n = 2 * n + 64;
            b = 2 * b + 4096;
        }
        if ((rc = grow(d_off, off_cap, 2 * (n + 1)))) return rc;
        if ((rc = grow(d_json, json_cap, b + 64 + 16))) return rc;
        if ((rc = grow(d_out, out_cap, slot_off(b, n) + 64))) return rc;
        if ((rc = grow(d_ol, ol_cap, n + 1))) return rc;
        if ((rc = grow(d_ret, ret_cap, n + 1))) return rc;
        return DG_OK;
    }
    void release()
    {
        (void)hipFree(d_off);
        (void)hipFree(d_json);
        (void)hipFree(d_out);
        (void)hipFree(d_ol);
        (void)hipFree(d_ret);
        d_off = d_ret = nullptr;
        d_json = d_out = nullptr;
        d_ol = nullptr;
        off_cap = json_cap = out_cap = ol_cap = ret_cap = 0;
    }
    /* convert + pack n messages whose offsets are at in_off / out_off, JSON
     * at json. The packing writes straight into pinned host memory: bytes at
     * h_dst + h_dst_off[i] (positions from *base_in when chained, nothing
     * past dst_cap), after the event pack_after if set; then ret is
     * downloaded to h_ret and ev recorded. */
    int convert(dg_ctx *c, const dg_desc *d, uint32_t root, uint64_t flags, uint64_t n, const uint8_t *json,
                const uint64_t *in_off, const uint64_t *out_off, uint64_t max_len, hipStream_t s, uint64_t *h_ret,
                uint8_t *h_dst, uint64_t *h_dst_off, const uint64_t *base_in, uint64_t dst_cap, hipEvent_t pack_after,
                hipEvent_t ev)
    {
        int rc = dg_i_convert_pack(c, d, root, json, in_off, n, flags, d_out, out_off, d_ol, d_ret, h_dst, h_dst_off,
                                   s, max_len, base_in, dst_cap, pack_after, 0, h_ret);
        if (rc) return rc;
        HIPCHK(hipEventRecord(ev, s));
        return DG_OK;
    }
};

/* ---------------- the aggregator ---------------- */

constexpr int AGG_RING_MAX = 24; /* batches in the ring (dg_agg::ring, DG_AGG_RING, default 16): each batch stream
                                  * gets its own device scratch (DG_MAX_SCRATCH covers the ring + the context's own) */
constexpr int AGG_SLOTS = 256;  /* parts per batch */
constexpr int AGG_SHARED = 32;  /* the last AGG_SHARED parts are shared: a thread that finds the exclusive parts
                                 * taken writes one of these under its lock (no call converts alone for want of
                                 * a part, whatever the number of threads) */
constexpr int AGG_EXCL = AGG_SLOTS - AGG_SHARED;
constexpr int AGG_GEN_RING = 64; /* dg_agg_gateway_drive: parked callers by generation (> AGG_RING_MAX + 2) */
constexpr int AGG_EAGER_INFLIGHT = 1;
/* launch(): each batch's buffers are sized for the registered parts' caps
 * summed (no regrowth mid-run: gateway parts of 4096 calls grew buffers batch
 * after batch, 332 us per batch, r5y) while that exact size times the ring
 * stays within this budget of packed output (knob "exact_total"); above it a
 * batch grows lazily to twice what it needed. Every batch of the ring holds
 * about 1x the packed size in pinned host memory and ~5x in device memory. */
constexpr uint64_t AGG_EXACT_TOTAL = 4ull << 30;

/* one caller thread's part of one batch (its own cache lines) */
struct alignas(128) Sub {
    std::atomic<uint32_t> busy{0}; /* 1 while the owner writes a message (the seal handshake; for a shared part
                                    * also the lock among its writers) */
    std::atomic<uint32_t> n{0};    /* messages committed */
    uint64_t bytes = 0;            /* JSON bytes committed (owner-written) */
    uint64_t maxlen = 0;           /* its longest message (owner-written) */
    uint8_t *h = nullptr;          /* pinned: [ends (cap_n u64) | JSON (cap_b + 64)] */
    uint64_t gbase = 0;            /* set at the seal: its first global index */
    std::atomic<uint32_t> left{0}; /* results not yet taken */
    uint64_t *ends() const { return (uint64_t *)(void *)h; }
};

struct Batch {
    Sub sub[AGG_SLOTS];
    std::atomic<uint64_t> t_first{0}; /* ns timestamp of its first message (0: none yet) */
    std::atomic<uint32_t> seal_req{0};
    std::atomic<uint32_t> parts{0};   /* threads with a message in it (while open) */
    std::atomic<uint32_t> blocked{0}; /* ... of which wait on it (while open) */
    std::atomic<uint32_t> active{0};  /* non-empty sub-batches whose results are not all taken */
    uint64_t g = 0;                   /* generation it holds while open / in flight */
    uint64_t t_launched = 0;
    uint64_t n = 0, bytes = 0;
    int rc = DG_OK;
    hipStream_t s = nullptr;
    hipEvent_t ev_hdr = nullptr, ev_done = nullptr;
    DevBuf dv;
    uint8_t *h_hdr = nullptr; uint64_t h_hdr_cap = 0;       /* pinned [ret | pack_off] */
    uint8_t *h_packed = nullptr; uint64_t h_packed_cap = 0; /* pinned packed Thrift */
    SubRef *h_tab = nullptr;                                /* pinned sub-batch table */
    SubRef *d_tab = nullptr;
    std::atomic<uint64_t> done_g{0};  /* last generation whose results are readable */
    std::mutex mu;
    std::condition_variable cv;
    bool free_ = true;                /* under the aggregator's mu */
    const uint64_t *ret() const { return (const uint64_t *)(const void *)h_hdr; }
    const uint64_t *pack_off() const { return ret() + n; }
};

std::atomic<uint64_t> g_agg_ids{1};

/* live aggregators by id: a thread that exits hands its parts back to the
 * ones still alive (ThreadParts' destructor) */
std::mutex g_reg_mu;
std::unordered_map<uint64_t, dg_agg *> g_reg;

}  // namespace

struct dg_agg {
    dg_ctx *ctx;
    const dg_desc *desc;
    uint32_t root;
    uint64_t flags;
    uint32_t cap_n;   /* per caller thread per batch */
    uint64_t cap_b;
    std::chrono::nanoseconds max_wait;
    uint64_t id;
    Batch *b = nullptr;
    int ring = 16;                   /* batches in the ring: one filling, the rest converting or being taken (r4j: 16 threads 53.3M calls/s vs 48.5M at 8) */
    std::atomic<uint64_t> open{0};   /* the open generation; batch b[open % ring] */
    std::atomic<int> nslots{0};      /* exclusive parts handed out (<= AGG_EXCL) */
    std::atomic<int> nshared{0};     /* shared parts whose regions exist */
    std::atomic<uint32_t> shared_rr{0};
    /* depth > 0 (dg_agg_set_knob "depth"): the flusher also seals the open
     * batch as soon as it holds a message and fewer than `depth` batches
     * are converting -- the policy for callers that do not block in
     * dg_agg_wait (goroutines parked on a channel, an event loop) */
    std::atomic<int> depth{0};
    /* min_fill > 0 (knob "min_fill"): the depth rule seals only a batch that
     * holds at least this many calls (else max_wait or a full part does);
     * many callers with one call each refill a batch over a pipeline round
     * trip, and sealing at once made batches too small to fill the ring's
     * round trip (r5y: 65536 callers, 4428-call batches, the flusher waiting
     * 536 us a batch for a free one) */
    std::atomic<uint32_t> min_fill{0};
    std::atomic<uint64_t> exact_total{AGG_EXACT_TOTAL}; /* knob "exact_total" (bytes), see AGG_EXACT_TOTAL */
    uint64_t open_calls(const Batch *x) const
    {
        uint64_t k = 0;
        const int ns = nparts();
        for (int s = 0; s < ns; s++) k += x->sub[s].n.load(std::memory_order_relaxed);
        return k;
    }
    /* every generation <= done_upto is converted and readable (the completer
     * finishes batches in generation order); dg_agg_wait_gen blocks on it */
    std::atomic<uint64_t> done_upto{0};
    std::mutex gen_mu;
    std::condition_variable cv_gen;
    std::atomic<uint8_t> ready[AGG_SLOTS];
    std::mutex mu;                   /* open changes, frees, flusher wakeups, completer queue */
    std::condition_variable cv_flush, cv_open, cv_done;
    std::deque<Batch *> inflight;
    bool stop = false;
    bool asym = false; /* membarrier registered: callers use a compiler fence only */
    std::atomic<uint64_t> batches{0}, msgs{0};
    /* non-empty batches issued and not yet complete: a batch whose callers
     * all wait on it is sealed at once only while fewer than
     * AGG_EAGER_INFLIGHT are (else when the next one completes), so blocking
     * callers still coalesce while the GPU is busy */
    std::atomic<int> busy_batches{0};
    /* where the time goes (ns, summed; dg_agg_profile): 0 flusher waiting for
     * a seal, 1 waiting for a free batch, 2 in launch (uploads + kernel
     * issue), 3 completer waiting for the header, 4 for the packed bytes,
     * 5 seal-to-launched, 6 launched-to-done, 7 callers blocked in wait;
     * dg_agg_drive: 8 in submit, 9 in wait, 10 submits that met no open
     * batch */
    std::atomic<uint64_t> prof[16] = {}; /* 12-15: launch()'s parts: busy flags, buffers, gather issue, convert issue */
    std::thread flusher, completer;

    static uint64_t now_ns()
    {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
    }
    int slot(bool &shared);
    /* parts to scan at a seal: the exclusive ones handed out, then the shared ones */
    int nparts() const
    {
        const int sh = nshared.load(std::memory_order_seq_cst);
        return sh ? AGG_EXCL + sh : std::min(nslots.load(std::memory_order_seq_cst), AGG_EXCL);
    }
    std::vector<int> free_slots;     /* parts of exited threads (under mu) */
    void release_slot(int s)
    {
        std::lock_guard<std::mutex> g(mu);
        free_slots.push_back(s);
    }
    void wake_flusher()
    {
        { std::lock_guard<std::mutex> g(mu); }
        cv_flush.notify_one();
    }
    void run_flusher();
    void run_completer();
    int launch(Batch *x);
};

namespace {
/* the parts this thread holds, by aggregator id; handed back at thread exit */
struct ThreadParts {
    std::vector<std::pair<uint64_t, int>> v; /* (aggregator id, part); part | 0x10000 = shared */
    ~ThreadParts()
    {
        /* an exclusive part goes to the next new thread. Tickets this thread
         * submitted stay valid: dg_agg_wait may take them from any thread
         * (a goroutine resumes on another OS thread), and the next owner
         * appends behind them in the open batch */
        std::lock_guard<std::mutex> g(g_reg_mu);
        for (const auto &e : v) {
            auto it = g_reg.find(e.first);
            if (it != g_reg.end() && e.second >= 0 && e.second < AGG_EXCL) it->second->release_slot(e.second);
        }
    }
};
thread_local ThreadParts t_parts;
}  // namespace

/* this thread's slot (sub-batch index), registered on first use: an exited
 * thread's part, else new pinned regions in every batch of the ring; -1 when
 * all are taken */
int dg_agg::slot(bool &shared)
{
    for (const auto &e : t_parts.v)
        if (e.first == id) {
            shared = e.second >= AGG_EXCL;
            return e.second;
        }
    int s = -1;
    shared = false;
    {
        std::lock_guard<std::mutex> g(mu);
        if (!free_slots.empty()) {
            s = free_slots.back();
            free_slots.pop_back();
        }
    }
    if (s >= 0) {
        /* its regions exist */
    } else if ((s = nslots.fetch_add(1, std::memory_order_seq_cst)) >= AGG_EXCL) {
        nslots.fetch_sub(1);
        /* the exclusive parts are taken: a shared one, round robin; its
         * regions are made once, by whoever gets it first */
        shared = true;
        const int k = (int)(shared_rr.fetch_add(1, std::memory_order_relaxed) % AGG_SHARED);
        s = AGG_EXCL + k;
        std::lock_guard<std::mutex> g(mu);
        while (nshared.load(std::memory_order_relaxed) <= k) {
            const int j = AGG_EXCL + nshared.load(std::memory_order_relaxed);
            bool ok = true;
            (void)hipSetDevice(ctx->device);
            for (int r = 0; r < ring && ok; r++) {
                uint64_t cap = 0;
                uint8_t *h = nullptr;
                ok = grow_pinned(h, cap, 8 * cap_n + cap_b + 64) == DG_OK;
                b[r].sub[j].h = h;
            }
            if (!ok) {
                s = -1;
                break;
            }
            ready[j].store(1, std::memory_order_release);
            nshared.fetch_add(1, std::memory_order_seq_cst);
        }
    } else {
        bool ok = true;
        (void)hipSetDevice(ctx->device);
        for (int k = 0; k < ring && ok; k++) {
            uint64_t cap = 0;
            uint8_t *h = nullptr;
            ok = grow_pinned(h, cap, 8 * cap_n + cap_b + 64) == DG_OK;
            b[k].sub[s].h = h;
        }
        ready[s].store(ok ? 1 : 2, std::memory_order_release);
        if (!ok) s = -1;
    }
    t_parts.v.emplace_back(id, s);
    return s;
}

int dg_agg::launch(Batch *x)
{
    /* the sub-batches: every registered slot, once its owner is not in the
     * middle of a message (it saw the old generation open before the flip) */
    const int ns = nparts();
    uint32_t nsub = 0;
    uint64_t N = 0, B = 0;
    const uint64_t l0 = now_ns();
    for (int s = 0; s < ns; s++) {
        Sub &u = x->sub[s];
        while (u.busy.load(std::memory_order_seq_cst)) std::this_thread::yield();
        const uint32_t k = u.n.load(std::memory_order_acquire);
        u.left.store(k, std::memory_order_relaxed);
        if (!k) continue;
        u.gbase = N;
        x->h_tab[nsub++] = SubRef{N, B, k, u.h, u.bytes};
        N += k;
        B += u.bytes;
    }
    x->n = N;
    x->bytes = B;
    x->rc = DG_OK;
    x->active.store(nsub, std::memory_order_release);
    const uint64_t l1 = now_ns();
    prof[12].fetch_add(l1 - l0, std::memory_order_relaxed);
    if (!N) return DG_OK;
    HIPCHK(hipSetDevice(ctx->device));
    int rc;
    /* Buffers for the largest batch the registered parts can make (their
     * caps summed), so a batch never grows them again until a new thread
     * registers: hipFree / hipHostFree wait for the whole device, every batch
     * in flight. When that size over the whole ring exceeds exact_total
     * bytes, growth is for twice the batch that needed it instead. */
    const uint64_t Nx = (uint64_t)ns * cap_n, Bx = (uint64_t)ns * cap_b;
    const bool exact = slot_off(Bx, Nx) * (uint64_t)ring <= exact_total.load(std::memory_order_relaxed);
    const uint64_t Ng = exact ? Nx : 2 * N + 64, Bg = exact ? Bx : 2 * B + 4096;
    if ((rc = x->dv.reserve(exact ? Nx : N, exact ? Bx : B, exact))) return rc;
    if (x->h_hdr_cap < 16 * N + 8 && (rc = grow_pinned(x->h_hdr, x->h_hdr_cap, 16 * Ng + 8))) return rc;
    if (x->h_packed_cap < slot_off(B, N) + 64 && /* >= any packed size */
        (rc = grow_pinned(x->h_packed, x->h_packed_cap, slot_off(Bg, Ng) + 64)))
        return rc;
    /* the parts' longest message (the callers track it) picks the kernels */
    uint64_t max_len = 1;
    for (int s = 0; s < ns; s++)
        if (x->sub[s].n.load(std::memory_order_relaxed)) max_len = std::max<uint64_t>(max_len, x->sub[s].maxlen);
    /* one gather launch reads every part straight from pinned host memory
     * (the table too), then the offsets */
    uint64_t maxb = 0;
    for (uint32_t k = 0; k < nsub; k++) maxb = std::max<uint64_t>(maxb, x->h_tab[k].bytes);
    const uint32_t gy = (uint32_t)std::max<uint64_t>(1, (maxb + AGG_GATHER_BYTES - 1) / AGG_GATHER_BYTES);
    uint64_t *d_in = x->dv.d_off, *d_oo = d_in + N + 1;
    const uint64_t l2 = now_ns();
    hipLaunchKernelGGL(agg_gather_kernel, dim3(nsub, gy), dim3(256), 0, x->s, x->h_tab, (uint64_t)cap_n,
                       x->dv.d_json, N, B, d_in, d_oo);
    HIPCHK(hipGetLastError());
    const uint64_t l3 = now_ns();
    uint64_t *h_ret = (uint64_t *)(void *)x->h_hdr;
    rc = x->dv.convert(ctx, desc, root, flags, N, x->dv.d_json, d_in, d_oo, max_len, x->s, h_ret, x->h_packed,
                       h_ret + N, nullptr, 0, nullptr, x->ev_hdr);
    const uint64_t l4 = now_ns();
    prof[13].fetch_add(l2 - l1, std::memory_order_relaxed);
    prof[14].fetch_add(l3 - l2, std::memory_order_relaxed);
    prof[15].fetch_add(l4 - l3, std::memory_order_relaxed);
    return rc;
}

void dg_agg::run_flusher()
{
    for (;;) {
        const uint64_t g = open.load(std::memory_order_acquire);
        Batch *x = &b[g % ring];
        /* the next batch of the ring, once its callers have taken their
         * results -- waited for first, while x still fills, so that a free
         * slot and the seal are awaited together, not one after the other
         * (r5y: 65536 gateway callers, 244 us seal + 186-536 us free a batch) */
        Batch *y = &b[(g + 1) % ring];
        uint64_t t0 = now_ns();
        {
            std::unique_lock<std::mutex> lk(mu);
            cv_flush.wait(lk, [&] { return y->free_ || (stop && !x->t_first.load(std::memory_order_acquire)); });
            if (!y->free_) { /* stopping with nothing to convert (y's callers never came back) */
                inflight.push_back(nullptr);
                lk.unlock();
                cv_done.notify_one();
                return;
            }
            y->free_ = false;
        }
        uint64_t t1 = now_ns();
        prof[1].fetch_add(t1 - t0, std::memory_order_relaxed);
        {
            /* until a caller asks for the seal (its sub-batch is full), the
             * first message has waited max_wait, the depth rule, or stop */
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                if (x->seal_req.load(std::memory_order_acquire)) break;
                const uint64_t t0 = x->t_first.load(std::memory_order_acquire);
                const int dp = depth.load(std::memory_order_relaxed);
                bool poll = false; /* the depth rule waits for min_fill calls: look again shortly */
                if (dp > 0 && t0 && !stop && busy_batches.load(std::memory_order_seq_cst) < dp) {
                    const uint32_t mf = min_fill.load(std::memory_order_relaxed);
                    if (!mf || open_calls(x) >= mf) break;
                    poll = true;
                }
                if (stop) {
                    if (!t0) {
                        y->free_ = true; /* not taken after all */
                        inflight.push_back(nullptr); /* the completer's exit marker */
                        lk.unlock();
                        cv_done.notify_one();
                        return;
                    }
                    break;
                }
                if (t0) {
                    const uint64_t now = now_ns();
                    if (now - t0 >= (uint64_t)max_wait.count()) break;
                    const int64_t left = max_wait.count() - (int64_t)(now - t0);
                    cv_flush.wait_for(lk, std::chrono::nanoseconds(poll ? std::min<int64_t>(left, 10000) : left));
                } else {
                    cv_flush.wait_for(lk, std::chrono::milliseconds(20));
                }
            }
        }
        const uint64_t t1s = now_ns();
        prof[0].fetch_add(t1s - t1, std::memory_order_relaxed);
        t1 = t1s;
        const int ns = nparts();
        for (int s = 0; s < ns; s++) {
            y->sub[s].n.store(0, std::memory_order_relaxed);
            y->sub[s].bytes = 0;
            y->sub[s].maxlen = 0;
        }
        y->t_first.store(0, std::memory_order_relaxed);
        y->seal_req.store(0, std::memory_order_relaxed);
        y->parts.store(0, std::memory_order_relaxed);
        y->blocked.store(0, std::memory_order_relaxed);
        y->g = g + 1;
        /* the flip: callers that still see g finish their message first
         * (launch() waits for their busy flags) */
        {
            std::lock_guard<std::mutex> lk(mu);
            open.store(g + 1, std::memory_order_seq_cst);
        }
        /* every caller either sees g + 1 or has its busy flag visible to
         * launch() (the other half of the handshake in dg_agg_submit) */
        if (asym) (void)sys_membarrier(MEMBARRIER_CMD_PRIVATE_EXPEDITED);
        cv_open.notify_all();
        uint64_t t2 = now_ns();
        prof[1].fetch_add(t2 - t1, std::memory_order_relaxed);
        x->rc = launch(x);
        x->t_launched = now_ns();
        prof[2].fetch_add(x->t_launched - t2, std::memory_order_relaxed);
        prof[5].fetch_add(x->t_launched - t1, std::memory_order_relaxed);
        batches.fetch_add(x->n ? 1 : 0, std::memory_order_relaxed);
        if (x->n) busy_batches.fetch_add(1, std::memory_order_seq_cst); /* before the completer can see x */
        msgs.fetch_add(x->n, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(mu);
            inflight.push_back(x);
        }
        cv_done.notify_one();
    }
}

void dg_agg::run_completer()
{
    for (;;) {
        Batch *x;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv_done.wait(lk, [&] { return !inflight.empty(); });
            x = inflight.front();
            inflight.pop_front();
        }
        if (!x) return;
        const uint64_t c0 = now_ns();
        uint64_t c1 = c0;
        if (x->n && x->rc == DG_OK) {
            /* the packing wrote the bytes and offsets into pinned host
             * memory; ret followed them */
            hipError_t e = hipEventSynchronize(x->ev_hdr);
            c1 = now_ns();
            if (e != hipSuccess) x->rc = set_err(DG_E_HIP, "aggregator batch: %s", hipGetErrorString(e));
        }
        /* an empty batch has no caller to free it; a non-empty one is freed
         * by the caller that takes its last result (x may be reused as soon
         * as that happens: decide before publishing) */
        const bool empty = x->n == 0;
        const uint64_t c2 = now_ns();
        prof[3].fetch_add(c1 - c0, std::memory_order_relaxed);
        prof[4].fetch_add(c2 - c1, std::memory_order_relaxed);
        prof[6].fetch_add(c2 - x->t_launched, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(x->mu);
            x->done_g.store(x->g, std::memory_order_release);
        }
        x->cv.notify_all();
        {
            std::lock_guard<std::mutex> lk(gen_mu);
            done_upto.store(x->g, std::memory_order_release);
        }
        cv_gen.notify_all();
        if (!empty) {
            /* room in the pipeline: seal the open batch if all its callers wait on it */
            busy_batches.fetch_sub(1, std::memory_order_seq_cst);
            if (depth.load(std::memory_order_relaxed) > 0) wake_flusher(); /* room under the depth */
            Batch *o = &b[open.load(std::memory_order_seq_cst) % ring];
            const uint32_t parts = o->parts.load(std::memory_order_seq_cst);
            if (parts && o->blocked.load(std::memory_order_seq_cst) >= parts &&
                !o->seal_req.exchange(1, std::memory_order_acq_rel))
                wake_flusher();
        }
        if (empty) {
            std::lock_guard<std::mutex> lk(mu);
            x->free_ = true;
            cv_flush.notify_one();
        }
    }
}

/* ---------------- the pipelined host batch ---------------- */

namespace {

constexpr int PIPE_BUFS = 3;

/* one chunk in flight: a stream, events, device buffers, pinned header */
struct PipeBuf {
    hipStream_t s = nullptr;
    hipEvent_t ev_hdr = nullptr, ev_done = nullptr;
    DevBuf dv;
    uint8_t *d_packed = nullptr; uint64_t packed_cap = 0; /* [pack_off (n+1) | packed (16-aligned)] */
    int init(int dev)
    {
        HIPCHK(hipSetDevice(dev));
        HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&ev_hdr, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
        return DG_OK;
    }
    void release()
    {
        if (s) (void)hipStreamSynchronize(s);
        dv.release();
        (void)hipFree(d_packed);
        d_packed = nullptr;
        packed_cap = 0;
        if (ev_hdr) (void)hipEventDestroy(ev_hdr);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (s) (void)hipStreamDestroy(s);
        s = nullptr;
    }
};

}  // namespace

void dg_i_pipe_free(dg_ctx *c)
{
    for (void *q : c->pipe) {
        ((PipeBuf *)q)->release();
        delete (PipeBuf *)q;
    }
    c->pipe.clear();
    (void)hipFree(c->d_pipe_cur);
    c->d_pipe_cur = nullptr;
    c->pipe_cur_cap = 0;
    (void)hipHostFree(c->h_pipe_ovf);
    c->h_pipe_ovf = nullptr;
    c->h_pipe_ovf_cap = 0;
    (void)hipHostFree(c->h_pipe_out);
    (void)hipHostFree(c->h_pipe_aux);
    c->h_pipe_out = c->h_pipe_aux = nullptr;
    c->h_pipe_out_cap = c->h_pipe_aux_cap = 0;
}

extern "C" {

int dg_agg_create2(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, uint64_t flags, uint32_t max_batch,
                   uint64_t max_bytes, uint32_t max_wait_us, dg_agg **out)
{
    if (!ctx || !desc || !out || max_batch == 0 || max_bytes == 0) return set_err(DG_E_INVALID, "bad args");
    dg_agg *a = new dg_agg();
    a->ctx = ctx;
    a->desc = desc;
    a->root = root_type;
    a->flags = flags;
    a->cap_n = (max_batch + 1) & ~1u; /* even: each part's JSON area stays 16-aligned */
    a->cap_b = max_bytes;
    a->max_wait = std::chrono::microseconds(max_wait_us);
    a->id = g_agg_ids.fetch_add(1);
    a->asym = sys_membarrier(MEMBARRIER_CMD_REGISTER_PRIVATE_EXPEDITED) == 0;
    for (auto &r : a->ready) r.store(0, std::memory_order_relaxed);
    if (const char *e = getenv("DG_AGG_RING")) a->ring = std::max(2, std::min(AGG_RING_MAX, atoi(e)));
    a->b = new Batch[a->ring];
    int rc = DG_OK;
    (void)hipSetDevice(ctx->device);
    for (int k = 0; k < a->ring && rc == DG_OK; k++) {
        Batch &x = a->b[k];
        hipError_t e = hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&x.ev_hdr, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&x.ev_done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipHostMalloc((void **)&x.h_tab, sizeof(SubRef) * AGG_SLOTS, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc(&x.d_tab, sizeof(SubRef) * AGG_SLOTS);
        if (e != hipSuccess) rc = set_err(DG_E_HIP, "aggregator setup: %s", hipGetErrorString(e));
    }
    if (rc) {
        dg_agg_destroy(a);
        return rc;
    }
    /* generations start at 1: done_g == 0 means "nothing converted yet" */
    a->open.store(1);
    a->b[1].free_ = false;
    a->b[1].g = 1;
    {
        std::lock_guard<std::mutex> g(g_reg_mu);
        g_reg[a->id] = a;
    }
    a->flusher = std::thread([a] { a->run_flusher(); });
    a->completer = std::thread([a] { a->run_completer(); });
    *out = a;
    return DG_OK;
}

int dg_agg_create(dg_ctx *ctx, const dg_desc *desc, uint32_t root_type, uint64_t flags, uint32_t max_batch,
                  uint32_t max_wait_us, dg_agg **out)
{
    /* JSON room for max_batch messages of 512 B on average (at least 1 MiB) per thread */
    const uint64_t mb = std::max<uint64_t>(1ull << 20, 512ull * max_batch);
    return dg_agg_create2(ctx, desc, root_type, flags, max_batch, mb, max_wait_us, out);
}

int dg_agg_submit(dg_agg *a, const uint8_t *json, size_t len, int nonblock, dg_agg_ticket *t)
{
    if (!a || (!json && len) || !t) return set_err(DG_E_INVALID, "bad args");
    static const uint8_t empty = 0;
    t->json = len ? json : &empty;
    t->len = len;
    t->batch = nullptr;
    bool shared = false;
    const int s = len > a->cap_b ? -1 : a->slot(shared);
    if (s < 0) { /* converted alone by dg_agg_wait */
        a->prof[11].fetch_add(1, std::memory_order_relaxed);
        return DG_OK;
    }
    for (;;) {
        const uint64_t g = a->open.load(std::memory_order_seq_cst);
        Batch *x = &a->b[g % a->ring];
        Sub &u = x->sub[s];
        if (shared) { /* the part's lock among its writers, and the seal handshake (a locked RMW is a full fence) */
            for (uint32_t z = 0; !u.busy.compare_exchange_weak(z, 1, std::memory_order_seq_cst); z = 0)
                std::this_thread::yield();
        } else if (a->asym) {
            u.busy.store(1, std::memory_order_relaxed);
            std::atomic_signal_fence(std::memory_order_seq_cst); /* the flusher's membarrier is the fence */
        } else {
            u.busy.store(1, std::memory_order_seq_cst);
        }
        if (a->open.load(std::memory_order_seq_cst) == g) {
            const uint32_t j = u.n.load(std::memory_order_relaxed);
            if (j < a->cap_n && u.bytes + len <= a->cap_b) {
                if (len) memcpy(u.h + 8 * a->cap_n + u.bytes, t->json, len);
                u.bytes += len;
                if (len > u.maxlen) u.maxlen = len;
                u.ends()[j] = u.bytes;
                u.n.store(j + 1, std::memory_order_release);
                u.busy.store(0, std::memory_order_release);
                if (j == 0) {
                    x->parts.fetch_add(1, std::memory_order_acq_rel);
                    uint64_t z = 0;
                    if (x->t_first.compare_exchange_strong(z, dg_agg::now_ns(), std::memory_order_acq_rel))
                        a->wake_flusher();
                }
                t->batch = x;
                t->gen = g;
                t->idx = ((uint32_t)s << 24) | j; /* slot | index within its sub-batch */
                return DG_OK;
            }
            /* this thread's part of the open batch is full: seal it */
            u.busy.store(0, std::memory_order_release);
            if (!x->seal_req.load(std::memory_order_acquire) && !x->seal_req.exchange(1, std::memory_order_acq_rel))
                a->wake_flusher();
        } else {
            u.busy.store(0, std::memory_order_release);
            continue; /* the batch closed meanwhile: the next one is open */
        }
        if (a->open.load(std::memory_order_acquire) != g) continue;
        if (nonblock) return DG_E_AGAIN; /* the next batch is not open yet (no lock: callers poll this) */
        std::unique_lock<std::mutex> lk(a->mu);
        if (a->stop) return set_err(DG_E_INVALID, "aggregator closed");
        a->cv_open.wait(lk, [&] { return a->open.load(std::memory_order_acquire) != g || a->stop; });
    }
}

int dg_agg_ready(dg_agg *a, const dg_agg_ticket *t)
{
    if (!a || !t) return 0;
    const Batch *x = (const Batch *)t->batch;
    return !x || x->done_g.load(std::memory_order_acquire) >= t->gen;
}

int dg_agg_wait(dg_agg *a, dg_agg_ticket *t, uint8_t *out, size_t out_cap, size_t *out_len, uint64_t *ret)
{
    if (!a || !t || (!out && out_cap) || !out_len || !ret) return set_err(DG_E_INVALID, "bad args");
    Batch *x = (Batch *)t->batch;
    bool redo = x == nullptr;
    int rc = DG_OK;
    if (x) {
        /* waiting on the open batch: once every thread with a message in it
         * waits on it, nothing more will come from them, so seal it now */
        if (a->open.load(std::memory_order_acquire) == t->gen &&
            x->blocked.fetch_add(1, std::memory_order_seq_cst) + 1 >= x->parts.load(std::memory_order_seq_cst) &&
            a->busy_batches.load(std::memory_order_seq_cst) < AGG_EAGER_INFLIGHT &&
            !x->seal_req.exchange(1, std::memory_order_acq_rel))
            a->wake_flusher();
        if (x->done_g.load(std::memory_order_acquire) < t->gen) {
            const uint64_t w0 = dg_agg::now_ns();
            for (int spin = 0; x->done_g.load(std::memory_order_acquire) < t->gen; spin++) {
                if (spin < 64) {
                    std::this_thread::yield();
                    continue;
                }
                std::unique_lock<std::mutex> lk(x->mu);
                x->cv.wait(lk, [&] { return x->done_g.load(std::memory_order_acquire) >= t->gen; });
            }
            a->prof[7].fetch_add(dg_agg::now_ns() - w0, std::memory_order_relaxed);
        }
        Sub &u = x->sub[t->idx >> 24];
        rc = x->rc;
        if (rc == DG_OK) {
            const uint64_t i = u.gbase + (t->idx & 0xFFFFFFu);
            const uint64_t r = x->ret()[i];
            if ((uint8_t)r == DG_ST_OUT_OVERFLOW) {
                redo = true; /* its slot was too small: alone, at its exact size */
            } else {
                const uint64_t *po = x->pack_off();
                const uint64_t l = po[i + 1] - po[i];
                *ret = r;
                *out_len = l;
                if (l > out_cap) rc = DG_E_NOMEM; /* the caller retries with out_len bytes */
                else if (l) memcpy(out, x->h_packed + po[i], l);
            }
        }
        if (u.left.fetch_sub(1, std::memory_order_acq_rel) == 1 &&
            x->active.fetch_sub(1, std::memory_order_acq_rel) == 1) {
            std::lock_guard<std::mutex> lk(a->mu);
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

int dg_agg_profile(dg_agg *a, uint64_t *out, int n)
{
    if (!a || !out || n < 0 || n > 16) return set_err(DG_E_INVALID, "bad args");
    for (int i = 0; i < n; i++) out[i] = a->prof[i].load();
    return DG_OK;
}

void dg_agg_destroy(dg_agg *a)
{
    if (!a) return;
    {
        std::lock_guard<std::mutex> g(g_reg_mu);
        g_reg.erase(a->id);
    }
    if (a->flusher.joinable()) {
        {
            std::lock_guard<std::mutex> lk(a->mu);
            a->stop = true;
        }
        a->cv_flush.notify_all();
        a->cv_open.notify_all();
        a->flusher.join(); /* converts what is in the open batch first */
        a->completer.join();
    }
    if (a->b) {
        /* the context's scratches owned by (or last used on) the batch
         * streams go before the streams do: an event last recorded on a
         * destroyed stream is not safe to wait on later (HIP then reported
         * "operation not permitted on an event last recorded in a capturing
         * stream" from a later launch that grew a reused scratch) */
        std::vector<hipStream_t> ss;
        for (int k = 0; k < a->ring; k++)
            if (a->b[k].s) ss.push_back(a->b[k].s);
        dg_i_scratch_release(a->ctx, ss.data(), (int)ss.size());
        for (int k = 0; k < a->ring; k++) {
            Batch &x = a->b[k];
            if (x.s) (void)hipStreamSynchronize(x.s);
            for (Sub &u : x.sub) (void)hipHostFree(u.h);
            x.dv.release();
            (void)hipFree(x.d_tab);
            (void)hipHostFree(x.h_tab);
            (void)hipHostFree(x.h_hdr);
            (void)hipHostFree(x.h_packed);
            if (x.ev_hdr) (void)hipEventDestroy(x.ev_hdr);
            if (x.ev_done) (void)hipEventDestroy(x.ev_done);
            if (x.s) (void)hipStreamDestroy(x.s);
        }
        delete[] a->b;
    }
    delete a;
}

/* One host batch streamed through PIPE_BUFS per-chunk buffer sets on their
 * own streams (see the file comment); the contract of dg_j2t_batch_host.
 * Chunk k's device JSON pointer is its buffer minus the 16-aligned floor of
 * its first offset, so the kernels read the caller's offsets unchanged. Its
 * packing writes straight into the caller's pinned out / out_off (or pinned
 * staging copied out at the end when they are pageable), starting where
 * chunk k-1's packing ended: the packings are chained by events, everything
 * else of neighbouring chunks overlaps, and the host waits once. */
namespace {
bool host_pinned(const void *p, void **dev)
{
    hipPointerAttribute_t at;
    if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (at.type != hipMemoryTypeHost || !at.devicePointer) return false;
    *dev = at.devicePointer;
    return true;
}
}  // namespace

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
    for (uint32_t k = 0; k <= chunks; k++) cb[k] = n * k / chunks;
    std::lock_guard<std::mutex> pg(c->pipe_mu);
    HIPCHK(hipSetDevice(c->device));
    while (c->pipe.size() < (size_t)PIPE_BUFS) {
        PipeBuf *q = new PipeBuf();
        c->pipe.push_back(q);
        int rc = q->init(c->device);
        if (rc) return rc;
    }
    const int nb = (int)std::min<uint32_t>(PIPE_BUFS, chunks);
    /* where the results go: the caller's buffers if pinned, else staging */
    void *dv_out = nullptr, *dv_off = nullptr, *dv_ret = nullptr;
    const bool direct = out_cap > 0 && host_pinned(out, &dv_out) && host_pinned(out_off, &dv_off) &&
                        host_pinned(ret, &dv_ret);
    uint8_t *p_out = (uint8_t *)dv_out;
    uint64_t *p_off = (uint64_t *)dv_off, *p_ret = (uint64_t *)dv_ret;
    if (!direct) {
        int rc;
        if ((rc = grow_pinned(c->h_pipe_out, c->h_pipe_out_cap, out_cap + 64))) return rc;
        if ((rc = grow_pinned(c->h_pipe_aux, c->h_pipe_aux_cap, 16 * n + 16))) return rc;
        p_out = c->h_pipe_out;
        p_off = (uint64_t *)(void *)c->h_pipe_aux;
        p_ret = p_off + n + 1;
    }
    const uint32_t phase = (uint32_t)((uintptr_t)p_out & 15);
    /* chunk k's start in out, written by chunk k-1's copy-out: the next
     * chunk's kernels read it from device memory (one read per block), not
     * over the link */
    if (c->pipe_cur_cap < chunks + 1) {
        HIPCHK(hipDeviceSynchronize()); /* no chain of an earlier call still reads it */
        int rc;
        if ((rc = grow(c->d_pipe_cur, c->pipe_cur_cap, (uint64_t)chunks + 1))) return rc;
    }
    /* each chunk's packing counts its overflowed slots here, so the host
     * scans the status words (pinned: slow CPU reads) only when one did */
    {
        int rc;
        if ((rc = grow_pinned(c->h_pipe_ovf, c->h_pipe_ovf_cap, 8ull * chunks))) return rc;
    }
    uint64_t *h_ovf = (uint64_t *)(void *)c->h_pipe_ovf;
    /* zero copy: when the JSON arena (with the 16 readable bytes past its end
     * the kernels may touch) and the offsets are pinned, the kernels read
     * them over the link themselves -- no hipMemcpyAsync per chunk, and the
     * next chunk's reads overlap the previous chunk's copy-out */
    void *dv_json = nullptr, *dv_end = nullptr, *dv_in = nullptr, *dv_in_end = nullptr;
    const uint64_t jend = in_off[n] + 15;
    void *dv_in0 = nullptr;
    const bool in_pinned = host_pinned(in_off, &dv_in0);
    const bool zc = host_pinned(json, &dv_json) && host_pinned(json + jend, &dv_end) &&
                    (uint8_t *)dv_end - (uint8_t *)dv_json == (ptrdiff_t)jend && host_pinned(in_off, &dv_in) &&
                    host_pinned(in_off + n, &dv_in_end) && (uint64_t *)dv_in_end - (uint64_t *)dv_in == (ptrdiff_t)n &&
                    ((uintptr_t)dv_json & 15) == 0 && /* the flat kernel loads 16-byte words from the arena's base */
                    ((uintptr_t)dv_in & 7) == 0 && !getenv("DG_NO_ZERO_COPY");
    /* staged (DG_PIPE_STAGED=1, the r4i layout): pack into device memory,
     * then a copy-out kernel; else the packing writes the host buffers */
    static const bool staged = getenv("DG_PIPE_STAGED") != nullptr;
    if (getenv("DG_PIPE_DEBUG"))
        fprintf(stderr, "dg_j2t_pipeline_host: n=%llu chunks=%u direct=%d zero_copy=%d staged=%d\n",
                (unsigned long long)n, chunks, (int)direct, (int)zc, (int)staged);
    for (uint32_t k = 0; k < chunks; k++) {
        PipeBuf &p = *(PipeBuf *)c->pipe[k % nb];
        const uint64_t a = cb[k], m = cb[k + 1] - a, base = in_off[a], jb = base & ~15ull;
        /* the longest message picks the kernels; unknown (0) when the
         * offsets are pinned (read in place or uploaded): CPU reads of pinned
         * memory run at ~10 GB/s (a 64K batch's offsets cost 50 us), and the
         * kernels route long messages themselves */
        uint64_t max_len = 0;
        if (!zc && !in_pinned) {
            max_len = 1;
            for (uint64_t j = a; j < a + m; j++) max_len = std::max<uint64_t>(max_len, in_off[j + 1] - in_off[j]);
        }
        const uint64_t span = in_off[a + m] - jb;
        const uint64_t pk = 8 * (m + 1) + 16 + slot_off(span, m) + 64; /* pack_off + phase + packed */
        int rc;
        if (!p.dv.fits(m, span) || (staged && p.packed_cap < pk)) HIPCHK(hipStreamSynchronize(p.s)); /* free to grow */
        if ((rc = p.dv.reserve(m, span))) return rc;
        if (staged && (rc = grow(p.d_packed, p.packed_cap, pk))) return rc;
        uint64_t *d_in = p.dv.d_off, *d_oo = d_in + m + 1;
        uint64_t *d_po = (uint64_t *)(void *)p.d_packed;
        uint8_t *d_pk = p.d_packed + ((8 * (m + 1) + 15) & ~15ull);
        const uint8_t *j_base; /* the JSON the kernels read, in_off-relative */
        const uint64_t *j_in;
        if (zc) {
            j_base = (const uint8_t *)dv_json;
            j_in = (const uint64_t *)dv_in + a;
            hipLaunchKernelGGL(pipe_slots_kernel, dim3((uint32_t)((m + 256) / 256)), dim3(256), 0, p.s, j_in, m, d_oo,
                               (uint8_t *)nullptr);
        } else {
            HIPCHK(hipMemcpyAsync(d_in, in_off + a, 8 * (m + 1), hipMemcpyHostToDevice, p.s));
            if (span) HIPCHK(hipMemcpyAsync(p.dv.d_json, json + jb, span, hipMemcpyHostToDevice, p.s));
            hipLaunchKernelGGL(pipe_slots_kernel, dim3((uint32_t)((m + 256) / 256)), dim3(256), 0, p.s, d_in, m, d_oo,
                               p.dv.d_json + span);
            j_base = p.dv.d_json - jb;
            j_in = d_in;
        }
        HIPCHK(hipGetLastError());
        /* the packing needs the previous chunk's end (written by its pack or copy-out) */
        PipeBuf *prev = k ? (PipeBuf *)c->pipe[(k - 1) % nb] : nullptr;
        const uint64_t *base_ptr = k ? c->d_pipe_cur + k : nullptr;
        if (!staged) {
            /* the packing's coalesced stores are the download: straight into
             * out / out_off / ret (pinned), from the previous chunk's end */
            if ((rc = dg_i_convert_pack(c, d, root, j_base, j_in, m, flags, p.dv.d_out, d_oo, p.dv.d_ol, p.dv.d_ret,
                                        p_out, p_off + a, p.s, max_len, base_ptr ? base_ptr : c->d_zero, out_cap,
                                        prev ? prev->ev_hdr : nullptr, 0, p_ret + a, c->d_pipe_cur + k + 1,
                                        h_ovf + k)))
                return rc;
            HIPCHK(hipEventRecord(p.ev_hdr, p.s));
            continue;
        }
        if ((rc = dg_i_convert_pack(c, d, root, j_base, j_in, m, flags, p.dv.d_out, d_oo, p.dv.d_ol,
                                    p.dv.d_ret, d_pk, d_po, p.s, max_len, base_ptr ? base_ptr : c->d_zero, 0,
                                    prev ? prev->ev_hdr : nullptr, 1 | (int)(phase << 1), nullptr, nullptr,
                                    h_ovf + k)))
            return rc;
        const uint32_t cg = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((span / 16 + 255) / 256, (m + 256) / 256),
                                                         (uint64_t)c->n_cu * 4);
        hipLaunchKernelGGL(pipe_copy_out_kernel, dim3(cg), dim3(256), 0, p.s, d_pk, d_po, m, p.dv.d_ret, p_out,
                           p_off + a, p_ret + a, base_ptr, out_cap, c->d_pipe_cur + k + 1);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(p.ev_hdr, p.s));
    }
    for (int i = 0; i < nb; i++) HIPCHK(hipStreamSynchronize(((PipeBuf *)c->pipe[i])->s));
    /* the host's view of the offsets (a hipHostRegister'd buffer's device
     * alias need not equal its host address) */
    const uint64_t cursor = direct ? out_off[n] : p_off[n];
    bool fits = cursor <= out_cap;
    if (!direct) {
        memcpy(out_off, p_off, 8 * (n + 1));
        memcpy(ret, p_ret, 8 * n);
        if (fits && cursor) memcpy(out, p_out, cursor);
    }
    uint64_t need = cursor;
    std::vector<uint64_t> redo;
    for (uint32_t k = 0; k < chunks; k++)
        if (h_ovf[k])
            for (uint64_t i = cb[k]; i < cb[k + 1]; i++)
                if ((uint8_t)ret[i] == DG_ST_OUT_OVERFLOW) redo.push_back(i);
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

static const uint64_t DRIVE_SAMPLE = 8; /* power of two */

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
            uint64_t ts_sub = 0, ts_wait = 0, n_again = 0;
            /* the clock is read for every DRIVE_SAMPLE-th call only (about
             * 20 ns a read: five reads per call would be a fifth of a call's
             * host cost); the profile counters are scaled back up */
            auto sampled = [&](uint64_t j) { return (j & (DRIVE_SAMPLE - 1)) == 0; };
            auto finish = [&]() {
                const uint64_t j = h++;
                const int k = (int)((j - lo) % window);
                size_t ol = 0;
                const bool smp = sampled(j);
                const uint64_t w0 = smp ? dg_agg::now_ns() : 0;
                int rc = dg_agg_wait(a, &ring[k], out + out_off[j], out_off[j + 1] - out_off[j], &ol, &ret[j]);
                if (smp) {
                    const uint64_t w1 = dg_agg::now_ns();
                    ts_wait += (w1 - w0) * DRIVE_SAMPLE;
                    if (lat_ns) lat_ns[j] = (uint32_t)std::min<int64_t>(w1 - t0[k], 0xffffffffll);
                } else if (lat_ns) {
                    lat_ns[j] = 0;
                }
                out_len[j] = ol;
                if (rc) failed.fetch_add(1);
            };
            for (uint64_t i = lo; i < hi; i++) {
                while (i - h >= (uint64_t)window) finish();
                /* results already back are taken at once (an event loop's
                 * completions): their batches free early */
                while (h < i && dg_agg_ready(a, &ring[(int)((h - lo) % window)])) finish();
                const int k = (int)((i - lo) % window);
                const bool smp = sampled(i);
                if (smp) t0[k] = dg_agg::now_ns();
                for (;;) {
                    const uint64_t s0 = smp ? dg_agg::now_ns() : 0;
                    int rc = dg_agg_submit(a, arena + in_off[i], in_off[i + 1] - in_off[i], 1, &ring[k]);
                    if (smp) ts_sub += (dg_agg::now_ns() - s0) * DRIVE_SAMPLE;
                    if (rc == DG_OK) break;
                    n_again++;
                    if (rc != DG_E_AGAIN) {
                        failed.fetch_add(1);
                        ring[k].batch = nullptr;
                        break;
                    }
                    /* this thread's part of the open batch is full: the flip
                     * comes once the next batch of the ring is free, i.e.
                     * once its callers (this thread among them) have taken
                     * their results. Block on the oldest call rather than
                     * spin: spinning callers take the cores the flusher and
                     * completer need (r4k: 16 threads 46.1M calls/s spinning,
                     * 53.3M blocking in r4j; 64 threads 18.4M vs 42.2M) */
                    if (h < i) finish();
                    else std::this_thread::yield();
                }
            }
            while (h < hi) finish();
            a->prof[8].fetch_add(ts_sub, std::memory_order_relaxed);
            a->prof[9].fetch_add(ts_wait, std::memory_order_relaxed);
            a->prof[10].fetch_add(n_again, std::memory_order_relaxed);
        });
    }
    while (ready.load() < threads) std::this_thread::yield();
    const auto ts = Clock::now();
    go.store(true, std::memory_order_release);
    for (auto &x : th) x.join();
    *seconds = std::chrono::duration<double>(Clock::now() - ts).count();
    return failed.load() ? set_err(DG_E_HIP, "%d aggregator calls failed", failed.load()) : DG_OK;
}


int dg_agg_set_knob(dg_agg *a, const char *name, int64_t value)
{
    if (!a || !name) return set_err(DG_E_INVALID, "bad args");
    if (!strcmp(name, "depth")) {
        a->depth.store((int)std::max<int64_t>(0, std::min<int64_t>(value, a->ring - 2)), std::memory_order_relaxed);
    } else if (!strcmp(name, "min_fill")) {
        a->min_fill.store((uint32_t)std::max<int64_t>(0, std::min<int64_t>(value, 1ll << 30)), std::memory_order_relaxed);
    } else if (!strcmp(name, "exact_total")) {
        if (value < 0) return set_err(DG_E_INVALID, "exact_total < 0");
        a->exact_total.store((uint64_t)value, std::memory_order_relaxed);
    } else if (!strcmp(name, "max_wait_us")) {
        if (value < 0) return set_err(DG_E_INVALID, "max_wait_us < 0");
        std::lock_guard<std::mutex> g(a->mu);
        a->max_wait = std::chrono::microseconds(value);
    } else {
        return set_err(DG_E_INVALID, "unknown aggregator knob '%s'", name);
    }
    a->wake_flusher();
    return DG_OK;
}

int dg_agg_wait_gen(dg_agg *a, uint64_t after, uint32_t timeout_us, uint64_t *done)
{
    if (!a || !done) return set_err(DG_E_INVALID, "bad args");
    if (a->done_upto.load(std::memory_order_acquire) <= after && timeout_us) {
        std::unique_lock<std::mutex> lk(a->gen_mu);
        a->cv_gen.wait_for(lk, std::chrono::microseconds(timeout_us),
                           [&] { return a->done_upto.load(std::memory_order_acquire) > after; });
    }
    *done = a->done_upto.load(std::memory_order_acquire);
    return DG_OK;
}

uint64_t dg_agg_ticket_gen(const dg_agg_ticket *t) { return t && t->batch ? t->gen : 0; }

namespace {
#ifndef DG_GW_PREFETCH
#define DG_GW_PREFETCH 16
#endif
constexpr size_t GW_PREFETCH = DG_GW_PREFETCH; /* dg_agg_gateway_drive: results prefetched this many callers ahead
                                                * (r6: 16 vs 8) */
struct GwCaller {
    uint64_t next;  /* its next message */
    uint64_t cur;   /* the message in flight */
    uint64_t t0;    /* submit time (sampled messages) */
    dg_agg_ticket t;
    bool has;
};
struct alignas(64) GwWorker {
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<bool> idle{false};
};
}  // namespace

/* The gateway shape (see include/dgj2t.h): `callers` logical callers, each
 * with ONE call in flight at a time (a goroutine blocked in Do), multiplexed
 * over `workers` OS threads the way the Go runtime runs goroutines on its Ms
 * (each with its own run queue, a P); a poller thread (the binding's one
 * goroutine locked to an OS thread) blocks in dg_agg_wait_gen and publishes
 * each converted generation. A caller parks in its worker's own ring by the
 * generation of its call (no lock shared between workers: a shared park list
 * serialised the 16 workers at ~1.4 M calls/s, r5w) and is runnable again
 * once that generation is published. Nothing blocks an OS thread per call. */
int dg_agg_gateway_drive(dg_agg *a, const uint8_t *arena, const uint64_t *in_off, uint64_t n, int workers,
                         int callers, uint8_t *out, const uint64_t *out_off, uint64_t *out_len, uint64_t *ret,
                         uint32_t *lat_ns, double *seconds, uint64_t *stats)
{
    if (!a || !arena || !in_off || workers < 1 || callers < 1 || !out || !out_off || !out_len || !ret || !seconds)
        return set_err(DG_E_INVALID, "bad args");
    const uint32_t G = (uint32_t)std::min<uint64_t>((uint64_t)callers, std::max<uint64_t>(n, 1));
    /* every worker owns a range of the messages and must have callers to
     * serve it: with fewer callers (or messages) than workers, the extra
     * workers would own messages nobody submits and the drive never ends */
    workers = (int)std::min<uint64_t>((uint64_t)workers, G);
    std::vector<GwCaller> cs(G);
    for (uint32_t c = 0; c < G; c++) cs[c] = GwCaller{c, 0, 0, dg_agg_ticket{}, false};
    std::vector<GwWorker> wk(workers);
    std::atomic<uint64_t> processed{a->done_upto.load(std::memory_order_acquire)};
    std::atomic<uint64_t> completed{0}, n_again{0}, n_park{0}, n_wake{0};
    std::atomic<uint64_t> t_wait{0}, t_submit{0}, t_idle{0}, t_all{0}; /* ns summed over the workers */
    std::atomic<int> failed{0}, ready{0};
    std::atomic<bool> go{false};
    auto done_all = [&] { return completed.load(std::memory_order_acquire) >= n || failed.load() > 0; };
    std::vector<std::thread> th;
    for (int w = 0; w < workers; w++) {
        th.emplace_back([&, w] {
            std::vector<uint32_t> run, retry;
            std::vector<std::vector<uint32_t>> parked(AGG_GEN_RING);
            uint32_t nparked = 0;
            for (uint32_t c = (uint32_t)w; c < G; c += (uint32_t)workers) run.push_back(c);
            /* requests arrive at this worker in arena order: a runnable caller
             * takes the next one (a goroutine serving the next request), so
             * consecutive calls read consecutive JSON -- not message c, c + G,
             * ... of one caller, a cache miss per call */
            uint64_t nxt = n * (uint64_t)w / (uint64_t)workers;
            const uint64_t lim = n * (uint64_t)(w + 1) / (uint64_t)workers;
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            uint64_t seen = processed.load(std::memory_order_acquire), done_local = 0;
            uint64_t tw = 0, ts_ = 0, ti = 0, np_ = 0, na_ = 0; /* counted locally: no shared line per call */
            const uint64_t tw0 = dg_agg::now_ns();
            for (;;) {
                /* the callers of the generations published since the last look */
                const uint64_t pg = processed.load(std::memory_order_acquire);
                if (nparked)
                    for (uint64_t g = seen + 1; g <= pg && g <= seen + AGG_GEN_RING; g++) {
                        std::vector<uint32_t> &v = parked[g % AGG_GEN_RING];
                        run.insert(run.end(), v.begin(), v.end());
                        nparked -= (uint32_t)v.size();
                        v.clear();
                    }
                seen = pg;
                const bool only_retry = run.empty() && !retry.empty();
                run.insert(run.end(), retry.begin(), retry.end());
                retry.clear();
                if (run.empty()) {
                    if (done_all() || !nparked) break; /* !nparked: every caller of this worker is through */
                    const uint64_t i0 = dg_agg::now_ns();
                    {
                        std::unique_lock<std::mutex> lk(wk[w].mu);
                        wk[w].idle.store(true); /* seq_cst against the poller's store of processed, then load of idle */
                        wk[w].cv.wait_for(lk, std::chrono::milliseconds(1),
                                          [&] { return processed.load() > seen || done_all(); });
                        wk[w].idle.store(false, std::memory_order_relaxed);
                    }
                    ti += dg_agg::now_ns() - i0;
                    continue;
                }
                for (size_t k = 0; k < run.size(); k++) {
                    const uint32_t c = run[k];
                    GwCaller &C = cs[c];
                    if (k + 2 * GW_PREFETCH < run.size()) __builtin_prefetch(&cs[run[k + 2 * GW_PREFETCH]]);
                    if (k + GW_PREFETCH < run.size()) { /* a later caller's result: status, offsets (pinned, DMA-written: not in cache) */
                        /* only callers of published generations: a retried
                         * caller's batch may still be filling (its header and
                         * offsets not written yet, or being regrown) */
                        const GwCaller &D = cs[run[k + GW_PREFETCH]];
                        if (D.has && D.t.batch && D.t.gen <= seen) {
                            const Batch *x = (const Batch *)D.t.batch;
                            const uint64_t i = x->sub[D.t.idx >> 24].gbase + (D.t.idx & 0xFFFFFFu);
                            __builtin_prefetch(x->ret() + i);
                            __builtin_prefetch(x->pack_off() + i);
                        }
                    }
                    if (k + GW_PREFETCH / 2 < run.size()) { /* ... and, its offsets now cached, its packed bytes */
                        const GwCaller &D = cs[run[k + GW_PREFETCH / 2]];
                        if (D.has && D.t.batch && D.t.gen <= seen) {
                            const Batch *x = (const Batch *)D.t.batch;
                            const uint64_t i = x->sub[D.t.idx >> 24].gbase + (D.t.idx & 0xFFFFFFu);
                            const uint8_t *q = x->h_packed + x->pack_off()[i];
                            __builtin_prefetch(q);
                            __builtin_prefetch(q + 64);
                        }
                    }
                    if (C.has) { /* resumed: its generation is converted, dg_agg_wait does not block */
                        const uint64_t j = C.cur;
                        size_t ol = 0;
                        const uint64_t q0 = dg_agg::now_ns();
                        int rc = dg_agg_wait(a, &C.t, out + out_off[j], out_off[j + 1] - out_off[j], &ol, &ret[j]);
                        tw += dg_agg::now_ns() - q0;
                        out_len[j] = ol;
                        if (rc) failed.fetch_add(1);
                        if (lat_ns) lat_ns[j] = (j & (DRIVE_SAMPLE - 1)) == 0
                                                    ? (uint32_t)std::min<uint64_t>(dg_agg::now_ns() - C.t0, 0xffffffffull)
                                                    : 0;
                        C.has = false;
                        done_local++;
                    }
                    if (nxt >= lim) continue;
                    const uint64_t i = nxt;
                    if ((i & (DRIVE_SAMPLE - 1)) == 0) C.t0 = dg_agg::now_ns();
                    const uint64_t q1 = dg_agg::now_ns();
                    int rc = dg_agg_submit(a, arena + in_off[i], in_off[i + 1] - in_off[i], 1, &C.t);
                    ts_ += dg_agg::now_ns() - q1;
                    if (rc == DG_E_AGAIN) { /* no room in the open batch for this thread: later */
                        retry.push_back(c);
                        na_++;
                        continue;
                    }
                    if (rc) {
                        failed.fetch_add(1);
                        continue;
                    }
                    nxt++;
                    C.cur = i;
                    C.has = true;
                    if (!C.t.batch) { /* converted alone by dg_agg_wait: runnable at once */
                        retry.push_back(c);
                        continue;
                    }
                    /* park on its generation (the goroutine's channel receive) */
                    const uint64_t g = C.t.gen;
                    if (g <= processed.load(std::memory_order_acquire) || g > seen + AGG_GEN_RING) {
                        retry.push_back(c);
                    } else {
                        parked[g % AGG_GEN_RING].push_back(c);
                        nparked++;
                        np_++;
                    }
                }
                run.clear();
                if (done_local) {
                    completed.fetch_add(done_local, std::memory_order_acq_rel);
                    done_local = 0;
                }
                if (only_retry) std::this_thread::yield();
                if (done_all()) break;
            }
            n_park.fetch_add(np_);
            n_again.fetch_add(na_);
            t_wait.fetch_add(tw);
            t_submit.fetch_add(ts_);
            t_idle.fetch_add(ti);
            t_all.fetch_add(dg_agg::now_ns() - tw0);
        });
    }
    while (ready.load() < workers) std::this_thread::yield();
    const auto ts = Clock::now();
    go.store(true, std::memory_order_release);
    /* the poller: publish each converted generation, wake the idle workers */
    uint64_t last = processed.load();
    while (!done_all()) {
        uint64_t d = last;
        dg_agg_wait_gen(a, last, 1000, &d);
        if (d <= last) continue;
        processed.store(d);
        last = d;
        n_wake.fetch_add(1, std::memory_order_relaxed);
        for (auto &W : wk)
            if (W.idle.load()) {
                { std::lock_guard<std::mutex> lk(W.mu); }
                W.cv.notify_one();
            }
    }
    for (auto &W : wk) {
        { std::lock_guard<std::mutex> lk(W.mu); }
        W.cv.notify_all();
    }
    for (auto &x : th) x.join();
    *seconds = std::chrono::duration<double>(Clock::now() - ts).count();
    if (stats) {
        stats[0] = n_park.load();
        stats[1] = n_again.load();
        stats[2] = n_wake.load();
        stats[3] = G;
        stats[4] = t_wait.load(); /* ns in dg_agg_wait, summed over the workers */
        stats[5] = t_submit.load();
        stats[6] = t_idle.load();
        stats[7] = t_all.load();
    }
    return failed.load() ? set_err(DG_E_HIP, "%d gateway calls failed", failed.load()) : DG_OK;
}

}  // extern "C"
