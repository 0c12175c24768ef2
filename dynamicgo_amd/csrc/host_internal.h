/*
 * host_internal.h — what the C-ABI translation units share: the context,
 * descriptor and per-stream scratch records and the error helpers
 * (j2t_host.hip defines the functions, t2j_host.hip uses them).
 */
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/dgj2t.h"
#include "../../include/dgj2t_desc.h"

__attribute__((visibility("hidden"))) int set_err(int code, const char *fmt, ...);
#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return set_err(DG_E_HIP, "%s: %s", #x, hipGetErrorString(e_));  \
    } while (0)

/* Device scratch of one launch pipeline: the bail/big lists, their
 * self-resetting counters, the wave queue and the workspaces. Launches on the
 * SAME stream reuse it in stream order. Each stream a caller passes gets its
 * own scratch (up to DG_MAX_SCRATCH per context), so concurrent streams never
 * share lists or counters; past that cap a scratch is shared and the next
 * launch on another stream waits for its previous launch (hipStreamWaitEvent
 * on `done`), which keeps the ordering rule true in every case. */
constexpr int DG_MAX_SCRATCH = 40; /* an aggregator ring (<= AGG_RING_MAX = 24 streams) + the context's stream
                                    * + the in-flight side streams (<= 7) + the host pipeline's 3 */
constexpr uint32_t DG_NCOUNTS = 24;
constexpr uint32_t DG_J2T_COUNTS_BYTES = 6 * 4;
constexpr uint32_t DG_T2J_DEEP_COUNT = 8;
struct Scratch {
    hipStream_t owner = nullptr;   /* the stream it was created for */
    hipStream_t last = nullptr;    /* stream of the last launch that used it */
    bool used = false;
    hipEvent_t done = nullptr;     /* recorded after every launch that used it (no system-scope fence: ordering only) */
    uint8_t *ws_fast = nullptr;
    uint64_t ws_fast_lanes = 0;
    uint64_t *d_deep_list = nullptr;
    /* DG_NCOUNTS u32 counters, each owned by ONE path:
     * j2t: [0] bails, [1] large messages, [2] wave queue, [3] huge messages,
     *      [4] deep count, [5] blocks done (deep pass) -- [0..5] are reset by
     *      the launch's last kernel (list mode), or by a stream memset of
     *      DG_J2T_COUNTS_BYTES when an enqueue fails half way;
     * pack: [6] arrivals, [7] departures of dg_pack_device_scan, [12] its
     *      slot-overflow count (MsgFrame::ovf_out) -- self-reset;
     * t2j: [8] deep-pass queue length, [9] long messages, [10] the wave
     *      kernel's queue, [11] its bails; launches alternate between this
     *      set and [16..19] (t2j_set), and each launch's deep pass zeroes the
     *      other set, the one the previous launch used (no memset per
     *      launch). */
    uint32_t *d_counts = nullptr;
    uint32_t *d_bail_list = nullptr;
    uint64_t bail_cap = 0;
    uint32_t *d_big_list = nullptr;
    uint64_t big_cap = 0;
    uint8_t *ws_wave = nullptr;
    uint8_t *ws_deep = nullptr;
    uint64_t *d_sums = nullptr;    /* dg_pack_device_scan: per-block byte totals (n_cu) */
    uint8_t *d_frame = nullptr;    /* dg_pack_device_framed: header + footer bytes */
    std::vector<uint8_t> frame;    /* what d_frame holds */
    uint32_t *t2j_list = nullptr;  /* t2j: messages queued for the deep pass ([8] of d_counts counts them) */
    uint64_t t2j_list_cap = 0;
    uint32_t *t2j_big = nullptr;   /* t2j: long messages for the wave kernel ([9] counts them, [10] its queue) */
    uint64_t t2j_big_cap = 0;
    uint32_t *t2j_bail = nullptr;  /* t2j: the wave kernel's bails ([11] counts them) */
    uint64_t t2j_bail_cap = 0;
    uint32_t t2j_set = 0;          /* t2j: the counter set of the next launch (0: [8..11], 1: [16..19]) */
    /* a second stream of this scratch's launches (created on first use): the
     * t2j wave kernel runs on it beside the lane pass (Knobs::t2j_overlap) */
    hipStream_t side = nullptr;
    hipEvent_t side_go = nullptr, side_done = nullptr;
};
constexpr uint32_t FRAME_CAP = 4096;

/* routing knobs: env at dg_ctx_create, then dg_ctx_set_knob (include/dgj2t.h) */
struct Knobs {
    int64_t flat = -1;
    int64_t wave_min = 512;
    int64_t wave_occ = 0;
    int64_t small_mpw = 64;
    int64_t list_blocks = 16;
    int64_t t2j_spread = 0;
    int64_t t2j_overlap = 0;    /* t2j: 1 = the wave kernel on a second stream beside the lane pass; r4n t2j-c3: 65.1 GB/s with, 66.6 without (the lane pass is ~15 us of 1.21 ms, the route kernel adds 14) */
    int64_t t2j_wave_min = 256; /* t2j messages longer than this take the wave kernel (0: never); r4k t2j-c3: 128 / 192 / 256 / 384 / 512 / 1024 -> 66.1 / 66.5 / 66.3 / 59.4 / 53.7 / 23.3 GB/s */
    int64_t flat_wrap = -1;     /* the flat kernel's wrapped mode for roots that wrap a flat struct (0: off) */
};

struct dg_ctx {
    int device;
    hipStream_t stream;
    int n_cu = 0;
    Knobs knobs;
    uint32_t *d_pending = nullptr;
    unsigned long long *d_stats = nullptr; /* {bails, deeps} since the last dg_ctx_stats reset */
    std::vector<Scratch *> scratch;
    uint32_t rr = 0; /* round-robin pick once DG_MAX_SCRATCH scratches exist */
    std::mutex mu;
    /* staging for the host API */
    uint8_t *d_json = nullptr; uint64_t d_json_cap = 0;
    uint64_t *d_in_off = nullptr; uint64_t d_in_cap = 0;
    uint8_t *d_out = nullptr; uint64_t d_out_cap = 0;
    uint64_t *d_out_off = nullptr; uint64_t d_oo_cap = 0;
    uint32_t *d_out_len = nullptr; uint64_t d_ol_cap = 0;
    uint64_t *d_ret = nullptr; uint64_t d_ret_cap = 0;
    uint64_t *d_aux = nullptr; uint64_t d_aux_cap = 0;       /* t2j: per-message response-base spans */
    uint8_t *d_cb = nullptr; uint64_t d_cb_cap = 0;          /* t2j: callback answers (entries + bytes) */
    uint8_t *d_pack = nullptr; uint64_t d_pack_cap = 0;      /* packed Thrift (dg_pack_device_scan) */
    uint64_t *d_pack_off = nullptr; uint64_t d_po_cap = 0;
    uint8_t *h_up = nullptr; uint64_t h_up_cap = 0;          /* pinned: offsets + JSON, one H2D */
    uint8_t *h_down = nullptr; uint64_t h_down_cap = 0;      /* pinned: ret + out_len (+ packed bytes) */
    /* t2j deep pass: T2J_DEEP_DEPTH frames per lane, ONE per context (about
     * 100 MB, allocated by the first t2j launch), ordered across streams by
     * ws_t2j_done recorded after each deep pass on ws_t2j_last */
    uint8_t *ws_t2j = nullptr;
    hipEvent_t ws_t2j_done = nullptr;
    hipStream_t ws_t2j_last = nullptr;
    /* the t2j wave kernel's token regions (t2j_wave_ws_bytes, ~200 MB), one
     * per context, ordered across streams like ws_t2j */
    uint8_t *ws_t2w = nullptr;
    hipEvent_t ws_t2w_done = nullptr;
    hipStream_t ws_t2w_last = nullptr;
    /* dg_j2t_pipeline_host: its per-chunk buffers (j2t_pipe.hip PipeBuf),
     * kept across calls; pipe_mu serialises pipeline calls */
    std::mutex pipe_mu;
    std::vector<void *> pipe;
    uint8_t *h_pipe_out = nullptr; uint64_t h_pipe_out_cap = 0; /* pinned staging when the caller's */
    uint8_t *h_pipe_aux = nullptr; uint64_t h_pipe_aux_cap = 0; /* buffers are pageable */
    uint8_t *h_pipe_ovf = nullptr; uint64_t h_pipe_ovf_cap = 0; /* pipeline: slot overflows per chunk (pinned) */
    uint64_t *d_zero = nullptr;                                 /* 8 zero bytes (device) */
    uint64_t *d_pipe_cur = nullptr; uint64_t pipe_cur_cap = 0;  /* pipeline: chunk k's start in out (device) */
    /* dg_j2t_batch_device_inflight: the context's extra streams and their
     * fork/join events (created on first use) */
    std::vector<hipStream_t> side;
    std::vector<hipEvent_t> side_ev;
    hipEvent_t fork_ev = nullptr;
    /* dg_j2t_batch_device_ktime: while set, enqueue() records kt[0] before the
     * batch's first kernel, kt[1] after it, kt[2] after the wave kernel and
     * kt[3] after the list pass (timing events, on the launch stream) */
    hipEvent_t *kt = nullptr;
};

/* frees the context's pipeline buffers (j2t_pipe.hip) */
__attribute__((visibility("hidden"))) void dg_i_pipe_free(dg_ctx *c);

/* pinned host staging, grown on demand (hipHostMalloc is slow: keep it) */
static inline int grow_pinned(uint8_t *&p, uint64_t &cap, uint64_t want)
{
    if (cap >= want) return DG_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    uint64_t nc = std::max<uint64_t>(want, cap * 2);
    nc = std::max<uint64_t>(nc, 1 << 16);
    /* DG_HOST_NUMA=1: on the allocating thread's NUMA node (its policy)
     * instead of the driver's default placement */
    static const unsigned fl = getenv("DG_HOST_NUMA") ? hipHostMallocNumaUser : hipHostMallocDefault;
    HIPCHK(hipHostMalloc((void **)&p, nc, fl));
    cap = nc;
    return DG_OK;
}

struct dg_desc {
    dg_ctx *ctx;
    uint8_t *d_blob;
    size_t len;
    dg_desc_hdr hdr;
    uint8_t *d_side = nullptr;     /* t2j side table (dg_desc_attach_t2j) */
    std::vector<uint8_t> hblob;    /* host copy of the blob (launch decisions) */
    size_t side_len = 0;
};

template <class T>
static inline int grow(T *&p, uint64_t &cap, uint64_t want)
{
    if (cap >= want) return DG_OK;
    (void)hipFree(p);
    p = nullptr;
    uint64_t nc = std::max<uint64_t>(want, cap * 2);
    HIPCHK(hipMalloc(&p, nc * sizeof(T)));
    cap = nc;
    return DG_OK;
}

/* grow a scratch buffer: the old one may still be read by the scratch's
 * previous launch, so wait for it before freeing */
template <class T>
static inline int grow_x(Scratch *x, T *&p, uint64_t &cap, uint64_t want)
{
    if (cap >= want) return DG_OK;
    if (x->used) HIPCHK(hipEventSynchronize(x->done));
    return grow(p, cap, want);
}

/* before streams s[0..n) are destroyed: the device is synchronized, the
 * scratches they own are freed, and no other scratch keeps one of them as
 * the stream of its last launch (takes the ctx mutex) */
__attribute__((visibility("hidden"))) void dg_i_scratch_release(dg_ctx *c, const hipStream_t *s, int n);

/* the scratch for a launch on stream s (ctx mutex held) */
__attribute__((visibility("hidden"))) int scratch_for(dg_ctx *c, hipStream_t s, Scratch **out);

/* one batch converted and packed on stream s (takes the ctx mutex): message
 * i's Thrift at d_packed + d_pack_off[i], d_pack_off[n] = total; failed and
 * overflowed messages pack as nothing (their d_ret says why). Chained form:
 * positions start at *base_in, bytes past dst_cap are not written (0: no
 * limit); d_packed / d_pack_off may be pinned host memory; the packing
 * waits for pack_after (another stream's event) when it is set. base_mod16
 * = 1 | phase << 1: positions start at (*base_in + phase) & 15 instead.
 * cur_out (device, optional): the end position (the next chunk's base).
 * ovf_out (optional, e.g. pinned): the count of DG_ST_OUT_OVERFLOW messages. */
__attribute__((visibility("hidden"))) int dg_i_convert_pack(
    dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json, const uint64_t *d_in_off, uint64_t n,
    uint64_t flags, uint8_t *d_out, const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, uint8_t *d_packed,
    uint64_t *d_pack_off, hipStream_t s, uint64_t max_len, const uint64_t *base_in = nullptr, uint64_t dst_cap = 0,
    hipEvent_t pack_after = nullptr, int base_mod16 = 0, uint64_t *ret_dst = nullptr, uint64_t *cur_out = nullptr,
    uint64_t *ovf_out = nullptr);
