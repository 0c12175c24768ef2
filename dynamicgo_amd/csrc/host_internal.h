/*
 * host_internal.h — what the C-ABI translation units share: the context,
 * descriptor and per-stream scratch records and the error helpers
 * (j2t_host.hip defines the functions, t2j_host.hip uses them).
 */
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

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
constexpr int DG_MAX_SCRATCH = 8;
struct Scratch {
    hipStream_t owner = nullptr;   /* the stream it was created for */
    hipStream_t last = nullptr;    /* stream of the last launch that used it */
    bool used = false;
    hipEvent_t done = nullptr;     /* recorded after every launch that used it */
    uint8_t *ws_fast = nullptr;
    uint64_t ws_fast_lanes = 0;
    uint64_t *d_deep_list = nullptr;
    /* [0] bails, [1] large messages, [2] wave queue, [3] t2j deep count, [4] deep count,
     * [5] blocks done (deep pass): self-reset by the list-mode launch;
     * [6] arrivals, [7] departures of dg_pack_device_scan: self-reset */
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
    uint8_t *ws_t2j = nullptr;     /* t2j deep pass: T2J_DEEP_DEPTH frames per lane */
    uint32_t *t2j_list = nullptr;  /* t2j: messages queued for the deep pass ([3] of d_counts counts them) */
    uint64_t t2j_list_cap = 0;
};
constexpr uint32_t FRAME_CAP = 4096;

struct dg_ctx {
    int device;
    hipStream_t stream;
    int n_cu = 0;
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
};

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

/* the scratch for a launch on stream s (ctx mutex held) */
__attribute__((visibility("hidden"))) int scratch_for(dg_ctx *c, hipStream_t s, Scratch **out);
