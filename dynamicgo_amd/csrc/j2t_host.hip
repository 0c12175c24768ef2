/*
 * j2t_host.hip — the C ABI (include/dgj2t.h): contexts, descriptors, batch
 * launches and the host-buffer entry points. Kernels: j2t_machine.h.
 */
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "j2t_flat.h"
#include "host_internal.h"

/* ========================================================================== */
/* host side: C ABI                                                            */
/* ========================================================================== */
using namespace dg;

static thread_local char g_err[512];
int set_err(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

static const uint64_t FAST_WS_STRIDE = DCAP + WS_KEYCAP + (uint64_t)WS_REQCAP * 8;
static const uint64_t DEEP_WS_STRIDE = DCAP + DEEP_KEYCAP + (uint64_t)DEEP_REQCAP * 8 +
                                       (uint64_t)MAX_RECURSE * sizeof(Frame) + MAX_RECURSE / 8;

static void scratch_free(Scratch *x)
{
    if (!x) return;
    if (x->used) (void)hipEventSynchronize(x->done);
    (void)hipFree(x->ws_fast);
    (void)hipFree(x->d_deep_list);
    (void)hipFree(x->d_counts);
    (void)hipFree(x->d_bail_list);
    (void)hipFree(x->d_big_list);
    (void)hipFree(x->ws_wave);
    (void)hipFree(x->ws_deep);
    (void)hipFree(x->d_sums);
    (void)hipFree(x->d_frame);
    (void)hipFree(x->t2j_list);
    (void)hipFree(x->t2j_big);
    (void)hipFree(x->t2j_bail);
    if (x->side) (void)hipStreamSynchronize(x->side);
    if (x->side_go) (void)hipEventDestroy(x->side_go);
    if (x->side_done) (void)hipEventDestroy(x->side_done);
    if (x->side) (void)hipStreamDestroy(x->side);
    if (x->done) (void)hipEventDestroy(x->done);
    delete x;
}

static int scratch_new(dg_ctx *c, hipStream_t owner, Scratch **out)
{
    Scratch *x = new Scratch();
    x->owner = owner;
    /* `done` orders execution only: the host frees or overwrites a scratch
     * buffer after it, and a launch on another stream that takes the scratch
     * over waits for it. No host reads data through it, and a kernel's own
     * dispatch fences already publish its writes to the kernels after it (as
     * between the batch's kernels on one stream), so it carries no
     * system-scope fence: that fence cost every batch a 5-6 us gap before the
     * stream's next kernel (r8g trace; r8h/r8i: C2 in flight 336 -> 353 GB/s;
     * a device-scope release instead gained nothing). */
    hipError_t e = hipEventCreateWithFlags(&x->done, hipEventDisableTiming | hipEventDisableSystemFence);
    if (e == hipSuccess) e = hipMalloc(&x->d_counts, DG_NCOUNTS * 4);
    /* ordered before the owner stream's launches: a plain hipMemset runs on
     * the null stream, which a non-blocking stream (the aggregator's) does
     * not wait for -- its first batch then read uninitialised list counters
     * and left messages unconverted (ret 0, no bytes) */
    if (e == hipSuccess) e = hipMemsetAsync(x->d_counts, 0, DG_NCOUNTS * 4, owner);
    if (e == hipSuccess) e = hipMalloc(&x->ws_deep, DEEP_WS_STRIDE * DEEP_THREADS);
    if (e == hipSuccess) e = hipMalloc(&x->ws_wave, (size_t)c->n_cu * std::max(WV_BLOCKS_PER_CU, WV5_BLOCKS_PER_CU) * WV_WAVES * DCAP);
    if (e == hipSuccess) e = hipMalloc(&x->d_sums, (size_t)c->n_cu * 8);
    if (e == hipSuccess) e = hipMalloc(&x->d_frame, FRAME_CAP);
    if (e != hipSuccess) {
        scratch_free(x);
        return set_err(DG_E_HIP, "scratch allocation: %s", hipGetErrorString(e));
    }
    *out = x;
    return DG_OK;
}

void dg_i_scratch_release(dg_ctx *c, const hipStream_t *s, int n)
{
    if (!c || n <= 0) return;
    std::lock_guard<std::mutex> g(c->mu);
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize(); /* nothing is pending on any scratch after this */
    std::vector<Scratch *> keep;
    for (Scratch *x : c->scratch) {
        bool owned = false, last = false;
        for (int k = 0; k < n; k++) {
            owned |= x->owner == s[k];
            last |= x->last == s[k];
        }
        if (owned) {
            x->used = false; /* done (synchronized): scratch_free waits on nothing */
            scratch_free(x);
            continue;
        }
        if (last) {
            x->used = false;
            x->last = nullptr;
        }
        keep.push_back(x);
    }
    c->scratch.swap(keep);
    c->rr = 0;
    for (int k = 0; k < n; k++) { /* the t2j workspaces' last streams */
        if (c->ws_t2j_last == s[k]) c->ws_t2j_last = nullptr;
        if (c->ws_t2w_last == s[k]) c->ws_t2w_last = nullptr;
    }
}

/* The scratch for a launch on stream s (ctx mutex held); orders s after the
 * scratch's previous launch when that ran on another stream. */
int scratch_for(dg_ctx *c, hipStream_t s, Scratch **out)
{
    Scratch *x = nullptr;
    for (Scratch *y : c->scratch)
        if (y->owner == s) x = y;
    if (!x) {
        if ((int)c->scratch.size() < DG_MAX_SCRATCH) {
            int rc = scratch_new(c, s, &x);
            if (rc) return rc;
            c->scratch.push_back(x);
        } else {
            x = c->scratch[c->rr++ % c->scratch.size()];
        }
    }
    if (x->used && x->last != s) HIPCHK(hipStreamWaitEvent(s, x->done, 0));
    *out = x;
    return DG_OK;
}

#ifndef DG_SRC_HASH
#define DG_SRC_HASH "unknown"
#endif
/* provenance: the source hash dynamicgo_amd/build.py compiled this library
 * from (checked by _lib.lib() against the sources next to it) */
static const char g_build_info[] = "dgj2t-build:" DG_SRC_HASH " arch:gfx950";

static int64_t *knob_ref(dg_ctx *c, const char *name)
{
    Knobs &K = c->knobs;
    if (!strcmp(name, "flat")) return &K.flat;
    if (!strcmp(name, "wave_min")) return &K.wave_min;
    if (!strcmp(name, "wave_occ")) return &K.wave_occ;
    if (!strcmp(name, "small_mpw")) return &K.small_mpw;
    if (!strcmp(name, "list_blocks")) return &K.list_blocks;
    if (!strcmp(name, "t2j_spread")) return &K.t2j_spread;
    if (!strcmp(name, "t2j_wave_min")) return &K.t2j_wave_min;
    if (!strcmp(name, "t2j_overlap")) return &K.t2j_overlap;
    if (!strcmp(name, "flat_wrap")) return &K.flat_wrap;
    return nullptr;
}

extern "C" {

const char *dg_last_error(void) { return g_err; }

const char *dg_build_info(void) { return g_build_info; }

int dg_ctx_create(int device, dg_ctx **out)
{
    if (!out) return set_err(DG_E_INVALID, "null out");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_err(DG_E_INVALID, "device %d out of range (%d)", device, ndev);
    HIPCHK(hipSetDevice(device));
    dg_ctx *c = new dg_ctx();
    c->device = device;
    /* a blocking stream: ordered with the legacy default stream (handle 0), so
     * a caller passing stream NULL (torch's default stream) sees the results
     * in order */
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamDefault));
    HIPCHK(hipMalloc(&c->d_pending, 16));
    HIPCHK(hipMalloc(&c->d_zero, 16));
    HIPCHK(hipMemset(c->d_zero, 0, 16));
    HIPCHK(hipMalloc(&c->d_stats, 16 * 8));
    HIPCHK(hipMemset(c->d_stats, 0, 16 * 8));
    HIPCHK(hipDeviceSynchronize()); /* the memsets done before any stream (blocking or not) uses the buffers */
    HIPCHK(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device));
    /* routing knobs: the environment is read here, once per context */
    static const struct { const char *env; const char *name; } envk[] = {
        {"DG_FLAT", "flat"}, {"DG_WAVE_MIN", "wave_min"}, {"DG_WAVE_OCC", "wave_occ"},
        {"DG_SMALL_MPW", "small_mpw"}, {"DG_LIST_BLOCKS", "list_blocks"}, {"DG_T2J_SPREAD", "t2j_spread"},
        {"DG_T2J_WAVE_MIN", "t2j_wave_min"}, {"DG_T2J_OVERLAP", "t2j_overlap"}, {"DG_FLAT_WRAP", "flat_wrap"}};
    for (const auto &e : envk) {
        const char *v = getenv(e.env);
        if (v && *v) *knob_ref(c, e.name) = strtoll(v, nullptr, 10);
    }
    *out = c;
    return DG_OK;
}

int dg_ctx_set_knob(dg_ctx *c, const char *name, int64_t value)
{
    if (!c || !name) return set_err(DG_E_INVALID, "null ctx/name");
    std::lock_guard<std::mutex> g(c->mu);
    int64_t *k = knob_ref(c, name);
    if (!k) return set_err(DG_E_INVALID, "unknown knob '%s'", name);
    *k = value;
    return DG_OK;
}

int dg_ctx_get_knob(dg_ctx *c, const char *name, int64_t *value)
{
    if (!c || !name || !value) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    int64_t *k = knob_ref(c, name);
    if (!k) return set_err(DG_E_INVALID, "unknown knob '%s'", name);
    *value = *k;
    return DG_OK;
}

void dg_ctx_destroy(dg_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    dg_i_pipe_free(c);
    for (Scratch *x : c->scratch) scratch_free(x);
    c->scratch.clear();
    (void)hipFree(c->d_pending);
    (void)hipFree(c->d_zero);
    (void)hipFree(c->d_stats);
    (void)hipFree(c->d_json);
    (void)hipFree(c->d_in_off);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_out_off);
    (void)hipFree(c->d_out_len);
    (void)hipFree(c->d_ret);
    (void)hipFree(c->d_aux);
    (void)hipFree(c->d_cb);
    (void)hipFree(c->d_pack);
    (void)hipFree(c->d_pack_off);
    (void)hipHostFree(c->h_up);
    (void)hipHostFree(c->h_down);
    (void)hipFree(c->ws_t2j);
    if (c->ws_t2j_done) (void)hipEventDestroy(c->ws_t2j_done);
    (void)hipFree(c->ws_t2w);
    if (c->ws_t2w_done) (void)hipEventDestroy(c->ws_t2w_done);
    for (hipStream_t x : c->side) (void)hipStreamDestroy(x);
    for (hipEvent_t e : c->side_ev) (void)hipEventDestroy(e);
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

void *dg_ctx_stream(dg_ctx *c) { return c ? (void *)c->stream : nullptr; }

static int desc_finish(dg_ctx *c, const dg_desc_hdr &h, uint8_t *d_blob, size_t len, const void *host_blob,
                       dg_desc **out)
{
    if (h.magic != DG_DESC_MAGIC || h.version < 1 || h.version > DG_DESC_VERSION || h.total_len > len)
        return set_err(DG_E_DESC, "bad descriptor blob header");
    dg_desc *d = new dg_desc();
    d->ctx = c;
    d->d_blob = d_blob;
    d->len = len;
    d->hdr = h;
    d->hblob.assign((const uint8_t *)host_blob, (const uint8_t *)host_blob + h.total_len);
    *out = d;
    return DG_OK;
}

/* The flat-struct kernel applies: the root is a struct of at most 64 fields,
 * all scalars or strings, without HTTP-mapped fields under F_ENABLE_HM, and
 * the blob fits its LDS copy. */
static bool flat_root(const dg_desc *d, uint32_t root, uint64_t flags)
{
    const dg_desc_hdr &h = d->hdr;
    if (d->hblob.size() < h.total_len || h.version < 2 || h.total_len > FL_DESC || root >= h.n_types) return false;
    const uint8_t *b = d->hblob.data();
    const dg_type *T = (const dg_type *)(b + h.off_types);
    if (T[root].ttype != DG_T_STRUCT) return false;
    const dg_struct &sd = ((const dg_struct *)(b + h.off_structs))[T[root].st];
    if (sd.req_words != 1 || ((flags & DG_F_ENABLE_HM) && (sd.flags & DG_SF_HTTP_MAPPING))) return false;
    const dg_field *F = (const dg_field *)(b + h.off_fields);
    for (uint32_t k = 0; k < sd.n_fields; k++) {
        switch (T[F[sd.field_begin + k].type].ttype) {
        case DG_T_BOOL: case DG_T_BYTE: case DG_T_I16: case DG_T_I32: case DG_T_I64: case DG_T_DOUBLE: case DG_T_STRING:
            break;
        default:
            return false;
        }
    }
    return true;
}

/* Wrapped mode of the flat kernel (FlatParams::wrap): the root R is a
 * struct of at most 64 fields, one or more of them of a flat struct type W
 * (flat_root's conditions); a message that is one such member converts on
 * the flat kernel when nothing else of R needs writing at its '}' under these
 * flags (j2t_write_unset_fields, native/thrift.c:258-310: no REQUIRED field
 * left, none DEFAULT with F_WRITE_DEFAULT or OPTIONAL with F_WRITE_OPTIONAL,
 * no F_TRACE_BACK field cache), the member's field has no value mapping in
 * play and is not a skipped Base. Returns the fields allowed (bit = index in
 * R), 0 = not applicable. */
static uint64_t wrap_root(const dg_desc *d, uint32_t root, uint64_t flags, uint32_t *inner)
{
    const dg_desc_hdr &h = d->hdr;
    if (d->hblob.size() < h.total_len || h.version < 2 || h.total_len > FL_DESC || root >= h.n_types) return 0;
    const uint8_t *b = d->hblob.data();
    const dg_type *T = (const dg_type *)(b + h.off_types);
    if (T[root].ttype != DG_T_STRUCT) return 0;
    const dg_struct &rs = ((const dg_struct *)(b + h.off_structs))[T[root].st];
    if (rs.req_words != 1 || rs.n_fields > 64 || ((flags & DG_F_ENABLE_HM) && (rs.flags & DG_SF_HTTP_MAPPING))) return 0;
    const dg_field *F = (const dg_field *)(b + h.off_fields);
    const uint64_t req = ((const uint64_t *)(b + h.off_reqwords))[rs.req_begin];
    uint32_t w = DG_NONE;
    for (uint32_t k = 0; k < rs.n_fields && w == DG_NONE; k++) {
        const uint32_t t = F[rs.field_begin + k].type;
        if (T[t].ttype == DG_T_STRUCT && flat_root(d, t, flags)) w = t;
    }
    if (w == DG_NONE) return 0;
    uint64_t ok = 0;
    for (uint32_t k = 0; k < rs.n_fields; k++) {
        const dg_field &f = F[rs.field_begin + k];
        if (f.type != w || ((flags & DG_F_ENABLE_VM) && f.vm != DG_VM_NONE) ||
            ((f.flags & DG_FF_REQUEST_BASE) && (flags & DG_F_NO_WRITE_BASE)))
            continue;
        bool fine = true;
        for (uint32_t j = 0; j < rs.n_fields && fine; j++) {
            if (j == k || !((req >> j) & 1)) continue;
            const dg_field &g = F[rs.field_begin + j];
            if (g.flags & DG_FF_REQUEST_BASE) continue;
            if ((flags & DG_F_TRACE_BACK) || g.required == DG_REQ_REQUIRED ||
                ((flags & DG_F_WRITE_DEFAULT) && g.required == DG_REQ_DEFAULT) ||
                ((flags & DG_F_WRITE_OPTIONAL) && g.required == DG_REQ_OPTIONAL))
                fine = false;
        }
        if (fine) ok |= 1ull << k;
    }
    *inner = w;
    return ok;
}

int dg_desc_create(dg_ctx *c, const void *blob, size_t len, dg_desc **out)
{
    if (!c || !blob || !out || len < sizeof(dg_desc_hdr)) return set_err(DG_E_INVALID, "bad args");
    dg_desc_hdr h;
    memcpy(&h, blob, sizeof h);
    if (h.magic != DG_DESC_MAGIC || h.total_len > len) return set_err(DG_E_DESC, "bad descriptor blob");
    HIPCHK(hipSetDevice(c->device));
    uint8_t *d_blob;
    HIPCHK(hipMalloc(&d_blob, len));
    HIPCHK(hipMemcpy(d_blob, blob, len, hipMemcpyHostToDevice));
    return desc_finish(c, h, d_blob, len, blob, out);
}

int dg_desc_create_device(dg_ctx *c, const void *d_src, size_t len, dg_desc **out)
{
    if (!c || !d_src || !out || len < sizeof(dg_desc_hdr)) return set_err(DG_E_INVALID, "bad args");
    HIPCHK(hipSetDevice(c->device));
    uint8_t *d_blob;
    HIPCHK(hipMalloc(&d_blob, len));
    HIPCHK(hipMemcpy(d_blob, d_src, len, hipMemcpyDeviceToDevice));
    std::vector<uint8_t> hb(len);
    HIPCHK(hipMemcpy(hb.data(), d_blob, len, hipMemcpyDeviceToHost));
    dg_desc_hdr h;
    memcpy(&h, hb.data(), sizeof h);
    if (h.total_len > len) return set_err(DG_E_DESC, "bad descriptor blob");
    return desc_finish(c, h, d_blob, len, hb.data(), out);
}

void dg_desc_destroy(dg_desc *d)
{
    if (!d) return;
    (void)hipFree(d->d_blob);
    (void)hipFree(d->d_side);
    delete d;
}

uint32_t dg_desc_root(const dg_desc *d) { return d ? d->hdr.root_type : 0; }

int dg_ctx_stats(dg_ctx *c, uint64_t *bails, uint64_t *deeps, int reset)
{
    if (!c) return set_err(DG_E_INVALID, "null ctx");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    unsigned long long h[2];
    HIPCHK(hipMemcpy(h, c->d_stats, sizeof h, hipMemcpyDeviceToHost));
    if (bails) *bails = h[0];
    if (deeps) *deeps = h[1];
    if (reset) {
        HIPCHK(hipMemset(c->d_stats, 0, sizeof h));
        HIPCHK(hipDeviceSynchronize());
    }
    return DG_OK;
}

int dg_ctx_counters(dg_ctx *c, uint64_t *out, int n, int reset)
{
    if (!c || !out || n < 0 || n > 16) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, c->d_stats, (size_t)n * 8, hipMemcpyDeviceToHost));
    if (reset) {
        HIPCHK(hipMemset(c->d_stats, 0, 16 * 8));
        HIPCHK(hipDeviceSynchronize());
    }
    return DG_OK;
}

/* slots start at 128-byte boundaries: the L2 writes a partly written line
 * back whole, so an output that straddles a line boundary it did not need
 * to costs a line (C2: one line per message instead of two) */
uint64_t dg_slot_bound(uint64_t len) { return (4 * len + 64 + 127) & ~127ull; }

static int ensure_fast_ws(Scratch *x, uint64_t lanes)
{
    if (x->ws_fast_lanes >= lanes) return DG_OK;
    if (x->used) HIPCHK(hipEventSynchronize(x->done));
    (void)hipFree(x->ws_fast);
    (void)hipFree(x->d_deep_list);
    x->ws_fast = nullptr;
    x->d_deep_list = nullptr;
    x->ws_fast_lanes = 0;
    uint64_t want = std::max<uint64_t>(lanes, 1 << 16);
    HIPCHK(hipMalloc(&x->ws_fast, want * FAST_WS_STRIDE));
    HIPCHK(hipMalloc(&x->d_deep_list, want * 8));
    x->ws_fast_lanes = want;
    return DG_OK;
}

/* the host's callback answers of a batch (dg_cb_tables, dgj2t_defs.h):
 * HTTP-mapping entries (DG_F_HM_SPLIT) and value-mapping entries, device
 * pointers */
struct HMIn {
    const dg_hm_entry *tab;
    uint32_t n_hm;
    const uint8_t *bytes;
    const dg_cb_entry *vm = nullptr;
};

static int enqueue(dg_ctx *c, Scratch *x, const dg_desc *d, uint32_t root, const uint8_t *json,
                   const uint64_t *in_off, uint64_t n, uint64_t flags, uint8_t *out, const uint64_t *out_off,
                   uint32_t *out_len, uint64_t *ret, uint32_t *pending, hipStream_t s, uint64_t max_len,
                   const HMIn *hm)
{
    int rc = ensure_fast_ws(x, n);
    if (rc) return rc;
    const bool no_wave = (flags & DG_F_NO_WAVE_PATH) != 0;
    /* flat roots go to the field-major flat kernel when the batch's messages
     * fit it (max_len unknown: longer ones are listed for the wave kernel) */
    const Knobs &K = c->knobs;
    const bool use_flat = K.flat >= 0 ? K.flat != 0
                                      : (flags & DG_F_FLAT_PATH) != 0 ||
                                            (!(flags & DG_F_NO_FLAT_PATH) && (max_len == 0 || max_len <= FL_MAXLEN));
    const bool no_flat = (flags & DG_F_NO_FLAT_PATH) != 0 || K.flat == 0;
    auto mark = [&](int i) {
        if (c->kt) (void)hipEventRecord(c->kt[i], s);
    };
    flags &= ~(DG_F_NO_WAVE_PATH | DG_F_FLAT_PATH | DG_F_NO_FLAT_PATH);
    Params P;
    P.root = root;
    P.json = json;
    P.in_off = in_off;
    P.n = n;
    P.flag = flags;
    P.list = nullptr;
    P.list_count = nullptr;
    P.reset2 = nullptr;
    P.big_list = nullptr;
    P.big_count = nullptr;
    P.big_max = 0;
    P.huge_count = nullptr;
    P.huge_min = WV_HUGE_MIN;
    P.hm_tab = hm ? hm->tab : nullptr;
    P.hm_bytes = hm ? hm->bytes : nullptr;
    P.n_hm = hm ? hm->n_hm : 0;
    P.ans_tab = hm ? hm->vm : nullptr;
    P.out = out;
    P.out_off = out_off;
    P.out_len = out_len;
    P.ret = ret;
    P.pending = pending;
    P.deep_count = x->d_counts + 4;
    P.deep_list = x->d_deep_list;
    P.ws = x->ws_fast;
    P.ws_stride = FAST_WS_STRIDE;
    P.keycap = WS_KEYCAP;
    P.reqcap = WS_REQCAP;
    P.fast = d->hdr.version >= 2 && (flags & ~FAST_FLAGS) == 0;
    P.stats = c->d_stats;
    uint64_t blocks = (n + LANE_BLOCK - 1) / LANE_BLOCK;
    DeepParams DP;
    DP.ws = x->ws_deep;
    DP.ws_stride = DEEP_WS_STRIDE;
    DP.keycap = DEEP_KEYCAP;
    DP.reqcap = DEEP_REQCAP;
    DP.done = x->d_counts + 5;
    DP.blob = d->d_blob;
    DP.hdr = d->hdr;
    const uint64_t big_max = (uint64_t)K.wave_min; /* messages longer than this go to the wave kernel */
    const bool wave = P.fast && !no_wave && d->hdr.total_len <= WV_DESC && d->hdr.total_len <= DESC_LDS_BYTES &&
                      (max_len == 0 || max_len > big_max);
    /* the wave kernel's instance: 4 waves/SIMD with 2 KiB message staging
     * (C3 1.46 ms) beats the 5-wave one (96 VGPRs, 98 spilled, 128 B staging:
     * 1.55 ms) since keys ride in their values' lanes; the wave_occ knob
     * (4|5) forces one */
    const bool wave5 = K.wave_occ == 5;
    auto wave_launch = [&](hipStream_t st, const Params &Q, const WaveParams &W) {
        const uint64_t bpc = wave5 ? WV5_BLOCKS_PER_CU : WV_BLOCKS_PER_CU;
        const uint64_t wblocks = std::min<uint64_t>((n + WV_WAVES - 1) / WV_WAVES, (uint64_t)c->n_cu * bpc);
        if (wave5) launch_wave_kernel5(dim3((uint32_t)wblocks), st, Q, W);
        else launch_wave_kernel(dim3((uint32_t)wblocks), st, Q, W);
    };
    auto lane_launch = [&](dim3 g, const Params &Q) {
        if (d->hdr.total_len <= DESC_LDS_BYTES) launch_lane_kernel_lds(g, s, Q, DP);
        else launch_lane_kernel_glb(g, s, Q, DP);
    };
    const int mpw = (int)K.small_mpw; /* 0: lane kernel (in-kernel exact machine) */
    const bool small = P.fast && !no_wave && mpw > 0 && d->hdr.total_len <= SM_DESC;
    if (small) {
        /* 1. small kernel: lane-per-message fast path; declines -> bail list,
         *    messages longer than big_max -> big list (when the batch has any)
         * 2. wave kernel over the big list
         * 3. lane kernel in list mode: the exact machine on the bail list */
        if ((rc = grow_x(x, x->d_bail_list, x->bail_cap, n))) return rc;
        if ((rc = grow_x(x, x->d_big_list, x->big_cap, n))) return rc;
        const bool need_wave = max_len == 0 || max_len > big_max;
        Params P1 = P;
        if (need_wave) {
            P1.big_list = x->d_big_list;
            P1.big_count = x->d_counts + 1;
            P1.big_max = big_max;
            P1.huge_count = x->d_counts + 3;
        }
        SmallParams S;
        S.blob = d->d_blob;
        S.hdr = d->hdr;
        S.bail_count = x->d_counts;
        S.bail_list = x->d_bail_list;
        uint32_t inner = DG_NONE;
        const uint64_t wrap_ok = (K.flat_wrap != 0 && !no_flat && !flat_root(d, root, flags))
                                     ? wrap_root(d, root, flags, &inner)
                                     : 0;
        if ((use_flat && flat_root(d, root, flags)) || wrap_ok) {
            /* flat root struct: a lane group per message, a lane per field;
             * or a root whose messages wrap one flat struct (FlatParams::wrap) */
            FlatParams FP;
            FP.blob = d->d_blob;
            FP.hdr = d->hdr;
            FP.bail_count = x->d_counts;
            FP.bail_list = x->d_bail_list;
            FP.wrap = wrap_ok ? 1u : 0u;
            FP.wrap_inner = wrap_ok ? inner : 0u;
            FP.wrap_ok = wrap_ok;
            mark(0);
            launch_flat_kernel(dim3((uint32_t)((n + FL_MPB - 1) / FL_MPB)), s, P1, FP);
        } else {
            const uint64_t mpb = (uint64_t)SM_WAVES * (uint64_t)(mpw >= 64 ? 64 : mpw == 16 ? 16 : 32);
            mark(0);
            launch_small_kernel(mpw, dim3((uint32_t)((n + mpb - 1) / mpb)), s, P1, S);
        }
        HIPCHK(hipGetLastError());
        mark(1);
        if (need_wave) {
            WaveParams W;
            W.blob = d->d_blob;
            W.hdr = d->hdr;
            W.bail_count = x->d_counts;
            W.bail_list = x->d_bail_list;
            W.list = x->d_big_list;
            W.list_count = x->d_counts + 1;
            W.huge_count = x->d_counts + 3;
            W.list_cap = n;
            W.ws = x->ws_wave;
            W.queue = x->d_counts + 2;
            wave_launch(s, P, W);
            HIPCHK(hipGetLastError());
        }
        mark(2);
        Params P3 = P;
        P3.list = x->d_bail_list;
        P3.list_count = x->d_counts;
        P3.reset2 = x->d_counts + 1; /* P3.fast stays set: the small kernel's declines try the full fast path */
        const uint64_t lb = (uint64_t)std::max<int64_t>(1, K.list_blocks); /* list-pass grid */
        lane_launch(dim3((uint32_t)std::min<uint64_t>(blocks, lb)), P3);
        mark(3);
    } else if (!wave) {
        mark(0);
        lane_launch(dim3((uint32_t)blocks), P);
        mark(1);
        mark(2);
        mark(3);
    } else {
        /* 1. lane kernel: small messages (lane fast path + exact machine);
         *    messages longer than big_max are listed for the wave kernel
         * 2. wave kernel: the listed ones, one wavefront per message
         * 3. lane kernel in list mode: the wave kernel's bails, exact machine */
        if ((rc = grow_x(x, x->d_bail_list, x->bail_cap, n))) return rc;
        if ((rc = grow_x(x, x->d_big_list, x->big_cap, n))) return rc;
        Params P1 = P;
        P1.big_list = x->d_big_list;
        P1.big_count = x->d_counts + 1;
        P1.big_max = big_max;
        P1.huge_count = x->d_counts + 3;
        mark(0);
        lane_launch(dim3((uint32_t)blocks), P1);
        HIPCHK(hipGetLastError());
        mark(1);
        WaveParams W;
        W.blob = d->d_blob;
        W.hdr = d->hdr;
        W.bail_count = x->d_counts;
        W.bail_list = x->d_bail_list;
        W.list = x->d_big_list;
        W.list_count = x->d_counts + 1;
        W.huge_count = x->d_counts + 3;
        W.list_cap = n;
        W.ws = x->ws_wave;
        W.queue = x->d_counts + 2;
        wave_launch(s, P, W);
        HIPCHK(hipGetLastError());
        mark(2);
        Params P3 = P;
        P3.list = x->d_bail_list;
        P3.list_count = x->d_counts;
        P3.reset2 = x->d_counts + 1;
        P3.fast = 0;
        lane_launch(dim3((uint32_t)std::min<uint64_t>(blocks, 32)), P3);
        mark(3);
    }
    HIPCHK(hipGetLastError());
    return DG_OK;
}

/* One batch on stream s: the scratch for s, the kernels, then the scratch's
 * `done` event. If an enqueue fails half way, the counters the list-mode
 * launch would have reset are cleared on the stream, so the next launch on
 * this scratch starts clean. */
static int launch(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *json, const uint64_t *in_off,
                  uint64_t n, uint64_t flags, uint8_t *out, const uint64_t *out_off, uint32_t *out_len,
                  uint64_t *ret, uint32_t *pending, hipStream_t s, uint64_t max_len = 0,
                  const HMIn *hm = nullptr)
{
    if (n == 0) return DG_OK;
    if (root >= d->hdr.n_types) return set_err(DG_E_INVALID, "root type %u out of range", root);
    Scratch *x;
    int rc = scratch_for(c, s, &x);
    if (rc) return rc;
    rc = enqueue(c, x, d, root, json, in_off, n, flags, out, out_off, out_len, ret, pending, s, max_len, hm);
    if (rc) (void)hipMemsetAsync(x->d_counts, 0, DG_J2T_COUNTS_BYTES, s);
    HIPCHK(hipEventRecord(x->done, s));
    x->used = true;
    x->last = s;
    return rc;
}

int dg_j2t_batch_device(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json, const uint64_t *d_in_off,
                        uint64_t n, uint64_t flags, uint8_t *d_out, const uint64_t *d_out_off, uint32_t *d_out_len,
                        uint64_t *d_ret, uint32_t *d_pending, void *stream)
{
    if (!c || !d) return set_err(DG_E_INVALID, "null ctx/desc");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return launch(c, d, root, d_json, d_in_off, n, flags, d_out, d_out_off, d_out_len, d_ret, d_pending, s);
}

int dg_j2t_batch_device_ml(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json, const uint64_t *d_in_off,
                           uint64_t n, uint64_t flags, uint8_t *d_out, const uint64_t *d_out_off, uint32_t *d_out_len,
                           uint64_t *d_ret, uint32_t *d_pending, void *stream, uint64_t max_len)
{
    if (!c || !d) return set_err(DG_E_INVALID, "null ctx/desc");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return launch(c, d, root, d_json, d_in_off, n, flags, d_out, d_out_off, d_out_len, d_ret, d_pending, s, max_len);
}

int dg_j2t_batch_device_hm(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json, const uint64_t *d_in_off,
                           uint64_t n, uint64_t flags, const dg_hm_entry *d_hm_tab, uint32_t n_hm,
                           const uint8_t *d_hm_bytes, uint8_t *d_out, const uint64_t *d_out_off, uint32_t *d_out_len,
                           uint64_t *d_ret, uint32_t *d_pending, void *stream, uint64_t max_len)
{
    if (!c || !d || (d_hm_tab && n_hm && !d_hm_bytes)) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    HMIn hm{d_hm_tab, n_hm, d_hm_bytes};
    return launch(c, d, root, d_json, d_in_off, n, flags, d_out, d_out_off, d_out_len, d_ret, d_pending, s, max_len,
                  d_hm_tab ? &hm : nullptr);
}

int dg_j2t_batch_device_cb(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json, const uint64_t *d_in_off,
                           uint64_t n, uint64_t flags, const dg_cb_tables *cb, uint8_t *d_out, const uint64_t *d_out_off,
                           uint32_t *d_out_len, uint64_t *d_ret, uint32_t *d_pending, void *stream, uint64_t max_len)
{
    if (!c || !d || (cb && (cb->hm_tab || cb->ans_tab) && !cb->bytes)) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    HMIn hm{cb ? cb->hm_tab : nullptr, cb ? cb->n_hm : 0u, cb ? cb->bytes : nullptr, cb ? cb->ans_tab : nullptr};
    return launch(c, d, root, d_json, d_in_off, n, flags, d_out, d_out_off, d_out_len, d_ret, d_pending, s, max_len,
                  cb ? &hm : nullptr);
}

int dg_j2t_batch_device_iters(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json,
                              const uint64_t *d_in_off, uint64_t n, uint64_t flags, uint8_t *d_out,
                              const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, uint32_t *d_pending,
                              void *stream, uint64_t max_len, int iters)
{
    if (!c || !d || iters < 0) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    for (int k = 0; k < iters; k++) {
        int rc = launch(c, d, root, d_json, d_in_off, n, flags, d_out, d_out_off, d_out_len, d_ret, d_pending, s, max_len);
        if (rc) return rc;
    }
    return DG_OK;
}

int dg_j2t_batch_device_ktime(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json,
                              const uint64_t *d_in_off, uint64_t n, uint64_t flags, uint8_t *d_out,
                              const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, uint32_t *d_pending,
                              void *stream, uint64_t max_len, int iters, double *ms)
{
    if (!c || !d || iters < 1 || !ms) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    std::vector<hipEvent_t> ev((size_t)iters * 4, nullptr);
    int rc = DG_OK;
    /* timing events without the system-scope fence (HIP's flag for events
     * that only measure): with it each mark added the fence's L2 writeback to
     * the kernel before it (C2 flat kernel ~35.0 us against 33.1 under rocprof) */
    for (auto &e : ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) rc = set_err(DG_E_HIP, "hipEventCreate");
    for (int k = 0; k < iters && !rc; k++) {
        c->kt = &ev[(size_t)k * 4];
        rc = launch(c, d, root, d_json, d_in_off, n, flags, d_out, d_out_off, d_out_len, d_ret, d_pending, s, max_len);
    }
    c->kt = nullptr;
    ms[0] = ms[1] = ms[2] = 0;
    if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = set_err(DG_E_HIP, "hipStreamSynchronize");
    for (int k = 0; k < iters && !rc; k++)
        for (int i = 0; i < 3; i++) {
            float t = 0;
            if (hipEventElapsedTime(&t, ev[(size_t)k * 4 + i], ev[(size_t)k * 4 + i + 1]) != hipSuccess)
                rc = set_err(DG_E_HIP, "hipEventElapsedTime");
            ms[i] += t / iters;
        }
    for (auto &e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

int dg_j2t_batch_device_inflight(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json,
                                 const uint64_t *d_in_off, uint64_t n, uint64_t flags, const uint64_t *d_out_off,
                                 const dg_out_set *sets, int depth, void *stream, uint64_t max_len, int iters)
{
    if (!c || !d || !sets || depth < 1 || depth > 8 || iters < 0) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s0 = stream ? (hipStream_t)stream : c->stream;
    const int used = std::min(depth, std::max(iters, 1));
    while ((int)c->side.size() < used - 1) {
        hipStream_t x;
        hipEvent_t e;
        HIPCHK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence)); /* ordering only */
        c->side.push_back(x);
        c->side_ev.push_back(e);
    }
    /* fork / join events order the streams only (no host reads through them):
     * no system-scope fence, like the scratch's `done` */
    if (!c->fork_ev) HIPCHK(hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming | hipEventDisableSystemFence));
    if (used > 1) { /* fork: the side streams start after what `stream` holds */
        HIPCHK(hipEventRecord(c->fork_ev, s0));
        for (int j = 0; j < used - 1; j++) HIPCHK(hipStreamWaitEvent(c->side[j], c->fork_ev, 0));
    }
    int rc = DG_OK;
    for (int k = 0; k < iters && !rc; k++) {
        const int j = k % used;
        const dg_out_set &o = sets[j];
        rc = launch(c, d, root, d_json, d_in_off, n, flags, o.d_out, d_out_off, o.d_out_len, o.d_ret, o.d_pending,
                    j ? c->side[j - 1] : s0, max_len);
    }
    for (int j = 0; j < used - 1; j++) { /* join, also after an error */
        HIPCHK(hipEventRecord(c->side_ev[j], c->side[j]));
        HIPCHK(hipStreamWaitEvent(s0, c->side_ev[j], 0));
    }
    return rc;
}

/* dg_pack_device_scan / _framed without the context lock (the caller holds it) */
static int pack_scan_nolock(dg_ctx *c, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len,
                            const uint64_t *d_ret, uint64_t n, const uint8_t *hdr, uint32_t hdr_len, const uint8_t *ftr,
                            uint32_t ftr_len, uint8_t *d_dst, uint64_t *d_dst_off, hipStream_t s,
                            const uint64_t *base_in = nullptr, uint64_t dst_cap = 0, int base_mod16 = 0,
                            uint64_t *ret_dst = nullptr, uint64_t *cur_out = nullptr, uint64_t *ovf_out = nullptr);

/* Host batch: ONE pinned upload [in_off | out_off | JSON], the kernels, a
 * device packing pass (used slot prefixes back to back, failed messages
 * dropped), then ONE download of [ret | out_len | packed Thrift] when the
 * batch is small (<= HOST_ONE_TRIP slot bytes), else [ret | out_len] and
 * then exactly the packed bytes. Slot overflows (rare) are rerun together in
 * one exact-size launch on the same staging. */
static const uint64_t HOST_ONE_TRIP = 4ull << 20;

static int batch_host(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *json, const uint64_t *in_off,
                      uint64_t n, uint64_t flags, const HMIn *hm, uint64_t hm_len, uint8_t *out, uint64_t out_cap,
                      uint64_t *out_off, uint64_t *ret, uint64_t *out_need)
/* hm: host pointers (tab may be NULL with vm set, and the reverse) */
{
    if (!c || !d || (!json && n) || !in_off || !out_off || (!ret && n)) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    int rc;
    hipStream_t s = c->stream;
    const uint64_t base = in_off[0], bytes = in_off[n] - in_off[0];
    /* upload: [ioff (n+1) | soff (n+1) | HTTP-mapping table (n x n_hm),
     * value-mapping table (n), answer bytes (optional) | JSON + 64 zero bytes] */
    const uint64_t nhm = hm && hm->tab ? hm->n_hm : 0;
    const uint64_t nvm = hm && hm->vm ? 1 : 0;
    const uint64_t hmb = hm ? (hm_len + 7) & ~7ull : 0;
    const uint64_t hmw = hm ? 2 * n * nhm + n * nvm + hmb / 8 : 0; /* words */
    const uint64_t up_bytes = 16 * (n + 1) + 8 * hmw + bytes + 64;
    if ((rc = grow_pinned(c->h_up, c->h_up_cap, up_bytes))) return rc;
    uint64_t *ioff = (uint64_t *)(void *)c->h_up, *soff = ioff + n + 1;
    uint64_t *hhm = soff + n + 1;
    uint8_t *hj = (uint8_t *)(void *)(hhm + hmw);
    if (hm) {
        if (n * nhm) memcpy(hhm, hm->tab, 16 * n * nhm);
        if (n * nvm) memcpy(hhm + 2 * n * nhm, hm->vm, 8 * n);
        if (hm_len) memcpy(hhm + 2 * n * nhm + n * nvm, hm->bytes, hm_len);
    }
    uint64_t max_len = 1;
    soff[0] = 0;
    for (uint64_t i = 0; i <= n; i++) ioff[i] = in_off[i] - base;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t l = ioff[i + 1] - ioff[i];
        max_len = std::max<uint64_t>(max_len, l);
        soff[i + 1] = soff[i] + dg_slot_bound(l);
    }
    if (bytes) memcpy(hj, json + base, bytes);
    memset(hj + bytes, 0, 64);
    const uint64_t slots = soff[n];
    /* download: [ret (n u64) | out_len (n u32, padded to 8) | packed] */
    const uint64_t head = 8 * n + ((4 * n + 7) & ~7ull);
    const bool one_trip = slots <= HOST_ONE_TRIP;
    if ((rc = grow(c->d_json, c->d_json_cap, up_bytes))) return rc;
    if ((rc = grow(c->d_out, c->d_out_cap, slots + 64))) return rc;
    if ((rc = grow(c->d_pack, c->d_pack_cap, head + slots + 64))) return rc;
    if ((rc = grow(c->d_pack_off, c->d_po_cap, n + 1))) return rc;
    if ((rc = grow_pinned(c->h_down, c->h_down_cap, one_trip ? head + slots + 64 : head + 8))) return rc;
    const uint64_t *d_in = (const uint64_t *)(void *)c->d_json, *d_oo = d_in + n + 1;
    HMIn dhm{nullptr, (uint32_t)nhm, nullptr};
    if (hm) {
        dhm.tab = nhm ? (const dg_hm_entry *)(const void *)(d_oo + n + 1) : nullptr;
        dhm.vm = nvm ? (const dg_cb_entry *)(const void *)(d_oo + n + 1 + 2 * n * nhm) : nullptr;
        dhm.bytes = (const uint8_t *)(const void *)(d_oo + n + 1 + 2 * n * nhm + n * nvm);
    }
    const uint8_t *d_j = c->d_json + 16 * (n + 1) + 8 * hmw;
    uint64_t *d_ret = (uint64_t *)(void *)c->d_pack;
    uint32_t *d_ol = (uint32_t *)(void *)(c->d_pack + 8 * n);
    uint8_t *d_packed = c->d_pack + head;
    HIPCHK(hipMemcpyAsync(c->d_json, c->h_up, up_bytes, hipMemcpyHostToDevice, s));
    if ((rc = launch(c, d, root, d_j, d_in, n, flags, c->d_out, d_oo, d_ol, d_ret, nullptr, s, max_len,
                     hm ? &dhm : nullptr)))
        return rc;
    if ((rc = pack_scan_nolock(c, c->d_out, d_oo, d_ol, d_ret, n, nullptr, 0, nullptr, 0, d_packed, c->d_pack_off, s)))
        return rc;
    HIPCHK(hipMemcpyAsync(c->h_down, c->d_pack, one_trip ? head + slots : head, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const uint64_t *hret = (const uint64_t *)(void *)c->h_down;
    const uint32_t *hol = (const uint32_t *)(void *)(c->h_down + 8 * n);
    std::vector<uint32_t> olen(hol, hol + n);
    memcpy(ret, hret, n * 8);
    /* the packed bytes: failed and overflowed messages hold none */
    auto kept = [&](uint64_t i) {
        return ret[i] == 0 || (uint8_t)ret[i] == DG_ST_HM_END || (uint8_t)ret[i] == 24 /* ERR_VM_END's record */ ||
               (uint8_t)ret[i] == DG_ST_HM_END_AT || (uint8_t)ret[i] == DG_ST_CB_LIST;
    };
    uint64_t packed = 0;
    for (uint64_t i = 0; i < n; i++)
        if (kept(i)) packed += olen[i];
    /* overflowed messages: rerun together, each in a slot of the size it
     * reported (out_len carries it), on the same device staging (free now) */
    std::vector<uint64_t> redo;
    for (uint64_t i = 0; i < n; i++)
        if ((uint8_t)ret[i] == DG_ST_OUT_OVERFLOW) redo.push_back(i);
    std::vector<uint8_t> main_buf, rdown; /* host copies: main packed bytes (two-trip case), redo results */
    std::vector<uint64_t> redo_so;
    uint64_t rhead = 0;
    if (!redo.empty()) {
        const uint64_t m = redo.size();
        uint64_t rb = 0;
        for (uint64_t i : redo) rb += ioff[i + 1] - ioff[i];
        const uint64_t rhw = hm ? 2 * m * nhm + m * nvm + hmb / 8 : 0;
        std::vector<uint8_t> up(16 * (m + 1) + 8 * rhw + rb + 64, 0);
        uint64_t *io = (uint64_t *)(void *)up.data(), *so = io + m + 1, *rhm = so + m + 1;
        uint8_t *rj = (uint8_t *)(void *)(rhm + rhw);
        io[0] = so[0] = 0;
        if (hm && hm_len) memcpy(rhm + 2 * m * nhm + m * nvm, hm->bytes, hm_len);
        for (uint64_t k = 0; k < m; k++) {
            const uint64_t i = redo[k], l = ioff[i + 1] - ioff[i];
            if (hm && nhm) memcpy(rhm + 2 * k * nhm, hm->tab + i * nhm, 16 * nhm);
            if (hm && nvm) memcpy(rhm + 2 * m * nhm + k, hm->vm + i, 8);
            memcpy(rj + io[k], hj + ioff[i], l);
            io[k + 1] = io[k] + l;
            so[k + 1] = so[k] + (((uint64_t)olen[i] + 64 + 7) & ~7ull);
        }
        if (!one_trip) { /* the main batch's packed bytes, before the staging is reused */
            main_buf.resize(packed);
            if (packed) HIPCHK(hipMemcpy(main_buf.data(), d_packed, packed, hipMemcpyDeviceToHost));
        }
        rhead = 8 * m + ((4 * m + 7) & ~7ull);
        if ((rc = grow(c->d_json, c->d_json_cap, up.size()))) return rc;
        if ((rc = grow(c->d_out, c->d_out_cap, so[m] + 64))) return rc;
        const uint64_t *r_in = (const uint64_t *)(void *)c->d_json, *r_oo = r_in + m + 1;
        uint64_t *r_ret = (uint64_t *)(void *)c->d_pack; /* rhead <= head: d_pack is large enough */
        uint32_t *r_ol = (uint32_t *)(void *)(c->d_pack + 8 * m);
        HIPCHK(hipMemcpyAsync(c->d_json, up.data(), up.size(), hipMemcpyHostToDevice, s));
        HMIn rhmd{nhm ? (const dg_hm_entry *)(const void *)(r_oo + m + 1) : nullptr, (uint32_t)nhm,
                  (const uint8_t *)(const void *)(r_oo + m + 1 + 2 * m * nhm + m * nvm),
                  nvm ? (const dg_cb_entry *)(const void *)(r_oo + m + 1 + 2 * m * nhm) : nullptr};
        if ((rc = launch(c, d, root, c->d_json + 16 * (m + 1) + 8 * rhw, r_in, m, flags, c->d_out, r_oo, r_ol, r_ret,
                         nullptr, s, max_len, hm ? &rhmd : nullptr)))
            return rc;
        rdown.resize(rhead + so[m]);
        HIPCHK(hipMemcpyAsync(rdown.data(), c->d_pack, rhead, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(rdown.data() + rhead, c->d_out, so[m], hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        redo_so.assign(so, so + m + 1);
        for (uint64_t k = 0; k < m; k++) {
            const uint64_t i = redo[k];
            memcpy(&ret[i], rdown.data() + 8 * k, 8);
            memcpy(&olen[i], rdown.data() + 8 * m + 4 * k, 4);
            if ((uint8_t)ret[i] == DG_ST_OUT_OVERFLOW)
                return set_err(DG_E_NOMEM, "message %llu overflowed its exact-size slot", (unsigned long long)i);
        }
    }
    uint64_t total = 0;
    out_off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (!kept(i)) olen[i] = 0;
        total += olen[i];
        out_off[i + 1] = total;
    }
    if (out_need) *out_need = total;
    if (total > out_cap || (!out && total)) return set_err(DG_E_NOMEM, "output needs %llu bytes", (unsigned long long)total);
    if (redo.empty()) {
        /* the packed bytes ARE the output layout */
        if (one_trip) {
            if (total) memcpy(out, c->h_down + head, total);
        } else if (total) {
            HIPCHK(hipMemcpy(out, d_packed, total, hipMemcpyDeviceToHost));
        }
        return DG_OK;
    }
    /* interleave: the main batch's packed bytes in order, the redo slots */
    const uint8_t *mp = one_trip ? c->h_down + head : main_buf.data();
    uint64_t pp = 0;
    size_t rk = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (rk < redo.size() && redo[rk] == i) {
            if (olen[i]) memcpy(out + out_off[i], rdown.data() + rhead + redo_so[rk], olen[i]);
            rk++;
        } else if (olen[i]) {
            memcpy(out + out_off[i], mp + pp, olen[i]);
            pp += olen[i];
        }
    }
    return DG_OK;
}

int dg_j2t_batch_host(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *json, const uint64_t *in_off,
                      uint64_t n, uint64_t flags, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *ret,
                      uint64_t *out_need)
{
    return batch_host(c, d, root, json, in_off, n, flags, nullptr, 0, out, out_cap, out_off, ret, out_need);
}

int dg_j2t_batch_host_hm(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *json, const uint64_t *in_off,
                         uint64_t n, uint64_t flags, const dg_hm_entry *hm_tab, uint32_t n_hm, const uint8_t *hm_bytes,
                         uint64_t hm_len, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *ret,
                         uint64_t *out_need)
{
    if ((hm_tab && n_hm && n && !hm_tab) || (hm_len && !hm_bytes)) return set_err(DG_E_INVALID, "bad args");
    for (uint64_t k = 0; hm_tab && k < n * n_hm; k++)
        if (hm_tab[k].len != DG_HM_ERR && (uint64_t)hm_tab[k].off + hm_tab[k].len > hm_len)
            return set_err(DG_E_INVALID, "HTTP-mapping entry %llu outside the bytes", (unsigned long long)k);
    HMIn hm{hm_tab, n_hm, hm_bytes};
    return batch_host(c, d, root, json, in_off, n, flags, hm_tab ? &hm : nullptr, hm_len, out, out_cap, out_off, ret,
                      out_need);
}

int dg_j2t_batch_host_cb(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *json, const uint64_t *in_off,
                         uint64_t n, uint64_t flags, const dg_cb_tables *cb, uint8_t *out, uint64_t out_cap,
                         uint64_t *out_off, uint64_t *ret, uint64_t *out_need)
{
    if (!cb) return batch_host(c, d, root, json, in_off, n, flags, nullptr, 0, out, out_cap, out_off, ret, out_need);
    if ((cb->len && !cb->bytes) || (cb->hm_tab && cb->n_hm && !n)) return set_err(DG_E_INVALID, "bad args");
    for (uint64_t k = 0; cb->hm_tab && k < n * cb->n_hm; k++)
        if (cb->hm_tab[k].len != DG_HM_ERR && (uint64_t)cb->hm_tab[k].off + cb->hm_tab[k].len > cb->len)
            return set_err(DG_E_INVALID, "HTTP-mapping entry %llu outside the bytes", (unsigned long long)k);
    for (uint64_t i = 0; cb->ans_tab && i < n; i++) {
        /* the answers must lie inside the bytes (the kernel walks them unchecked) */
        uint64_t at = cb->ans_tab[i].off;
        for (uint32_t k = 0; k < cb->ans_tab[i].count; k++) {
            if (at + 4 > cb->len) return set_err(DG_E_INVALID, "value-mapping entry %llu outside the bytes", (unsigned long long)i);
            uint32_t l;
            memcpy(&l, cb->bytes + at, 4);
            at += 4 + (uint64_t)l;
            if (at > cb->len) return set_err(DG_E_INVALID, "value-mapping entry %llu outside the bytes", (unsigned long long)i);
        }
    }
    HMIn hm{cb->hm_tab, cb->hm_tab ? cb->n_hm : 0u, cb->bytes, cb->ans_tab};
    return batch_host(c, d, root, json, in_off, n, flags, (cb->hm_tab || cb->ans_tab) ? &hm : nullptr, cb->len, out,
                      out_cap, out_off, ret, out_need);
}

int dg_j2t_do(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *json, size_t len, uint64_t flags,
              uint8_t *out, size_t out_cap, size_t *out_len, uint64_t *ret)
{
    uint64_t in_off[2] = {0, len};
    uint64_t oo[2];
    uint64_t need = 0;
    static const uint8_t empty = 0;
    int rc = dg_j2t_batch_host(c, d, root, len ? json : &empty, in_off, 1, flags, out, out_cap, oo, ret, &need);
    if (out_len) *out_len = need;
    return rc;
}

int dg_pack_device(dg_ctx *c, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len, uint64_t n,
                   uint8_t *d_dst, const uint64_t *d_dst_off, void *stream)
{
    if (!c || (n && (!d_out || !d_out_off || !d_out_len || !d_dst || !d_dst_off))) return set_err(DG_E_INVALID, "bad args");
    if (n == 0) return DG_OK;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    uint64_t blocks = std::min<uint64_t>((n + 3) / 4, (uint64_t)c->n_cu * 8);
    launch_pack_kernel(dim3((uint32_t)blocks), s, d_out, d_out_off, d_out_len, n, d_dst, d_dst_off);
    HIPCHK(hipGetLastError());
    return DG_OK;
}

static int pack_scan_nolock(dg_ctx *c, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len,
                            const uint64_t *d_ret, uint64_t n, const uint8_t *hdr, uint32_t hdr_len, const uint8_t *ftr,
                            uint32_t ftr_len, uint8_t *d_dst, uint64_t *d_dst_off, hipStream_t s,
                            const uint64_t *base_in, uint64_t dst_cap, int base_mod16, uint64_t *ret_dst,
                            uint64_t *cur_out, uint64_t *ovf_out)
{
    if (n == 0) {
        if (ovf_out) HIPCHK(hipMemsetAsync(ovf_out, 0, 8, s));
        if (base_in && !base_mod16) HIPCHK(hipMemcpyAsync(d_dst_off, base_in, 8, hipMemcpyDefault, s));
        else HIPCHK(hipMemsetAsync(d_dst_off, 0, 8, s));
        if (cur_out) HIPCHK(hipMemcpyAsync(cur_out, d_dst_off, 8, hipMemcpyDefault, s));
        return DG_OK;
    }
    Scratch *x;
    int rc = scratch_for(c, s, &x);
    if (rc) return rc;
    MsgFrame fr{};
    fr.ret = d_ret; /* failed messages pack as nothing */
    fr.base_in = base_in;
    fr.dst_cap = dst_cap;
    fr.base_mod16 = base_mod16 ? 1u : 0u;
    fr.phase_add = (uint32_t)(base_mod16 >> 1) & 15; /* dg_i_convert_pack: 1 | phase << 1 */
    fr.ret_dst = ret_dst;
    fr.cur_out = cur_out;
    fr.ovf_out = d_ret ? ovf_out : nullptr;
    if (hdr) {
        /* header at 0, footer 8-aligned after it; both followed by >= 16 readable bytes */
        const uint32_t fo = (hdr_len + 7) & ~7u;
        std::vector<uint8_t> tmp(fo + ftr_len + 16, 0);
        memcpy(tmp.data(), hdr, hdr_len);
        if (ftr_len) memcpy(tmp.data() + fo, ftr, ftr_len);
        if (tmp != x->frame) {
            /* a new header/footer (a new method): wait until the scratch's
             * last launch is done reading the old one, then upload */
            if (x->used) HIPCHK(hipEventSynchronize(x->done));
            HIPCHK(hipMemcpy(x->d_frame, tmp.data(), tmp.size(), hipMemcpyHostToDevice));
            x->frame = tmp;
        }
        fr.hdr = x->d_frame;
        fr.hdr_len = hdr_len;
        fr.ftr = x->d_frame + fo;
        fr.ftr_len = ftr_len;
    }
    /* every block must be resident at once (they wait for each other): at
     * most one block per CU */
    const uint64_t G = std::min<uint64_t>((n + 255) / 256, (uint64_t)c->n_cu);
    launch_pack_scan_kernel(dim3((uint32_t)G), s, d_out, d_out_off, d_out_len, n, d_dst, d_dst_off, x->d_sums,
                            x->d_counts + 6, fr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) (void)hipMemsetAsync(x->d_counts + 6, 0, 8, s);
    HIPCHK(hipEventRecord(x->done, s));
    x->used = true;
    x->last = s;
    if (e != hipSuccess) return set_err(DG_E_HIP, "pack scan launch: %s", hipGetErrorString(e));
    return DG_OK;
}

static int pack_scan(dg_ctx *c, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len,
                     const uint64_t *d_ret, uint64_t n, const uint8_t *hdr, uint32_t hdr_len, const uint8_t *ftr,
                     uint32_t ftr_len, uint8_t *d_dst, uint64_t *d_dst_off, void *stream)
{
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return pack_scan_nolock(c, d_out, d_out_off, d_out_len, d_ret, n, hdr, hdr_len, ftr, ftr_len, d_dst, d_dst_off, s);
}

}  // extern "C"

/* conversion + packing of one batch on stream s (failed and overflowed
 * messages pack as nothing), for the pipelined host paths (j2t_pipe.hip) */
int dg_i_convert_pack(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json, const uint64_t *d_in_off,
                      uint64_t n, uint64_t flags, uint8_t *d_out, const uint64_t *d_out_off, uint32_t *d_out_len,
                      uint64_t *d_ret, uint8_t *d_packed, uint64_t *d_pack_off, hipStream_t s, uint64_t max_len,
                      const uint64_t *base_in, uint64_t dst_cap, hipEvent_t pack_after, int base_mod16,
                      uint64_t *ret_dst, uint64_t *cur_out, uint64_t *ovf_out)
{
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    int rc = launch(c, d, root, d_json, d_in_off, n, flags, d_out, d_out_off, d_out_len, d_ret, nullptr, s, max_len);
    if (rc) return rc;
    if (pack_after) HIPCHK(hipStreamWaitEvent(s, pack_after, 0));
    return pack_scan_nolock(c, d_out, d_out_off, d_out_len, d_ret, n, nullptr, 0, nullptr, 0, d_packed, d_pack_off, s,
                            base_in, dst_cap, base_mod16, ret_dst, cur_out, ovf_out);
}

extern "C" {

int dg_pack_device_scan(dg_ctx *c, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len,
                        uint64_t n, uint8_t *d_dst, uint64_t *d_dst_off, void *stream)
{
    if (!c || !d_dst_off || (n && (!d_out || !d_out_off || !d_out_len || !d_dst))) return set_err(DG_E_INVALID, "bad args");
    return pack_scan(c, d_out, d_out_off, d_out_len, nullptr, n, nullptr, 0, nullptr, 0, d_dst, d_dst_off, stream);
}

int dg_pack_device_framed(dg_ctx *c, const uint8_t *d_out, const uint64_t *d_out_off, const uint32_t *d_out_len,
                          const uint64_t *d_ret, uint64_t n, const uint8_t *hdr, uint32_t hdr_len, const uint8_t *ftr,
                          uint32_t ftr_len, uint8_t *d_dst, uint64_t *d_dst_off, void *stream)
{
    if (!c || !d_dst_off || !hdr || (ftr_len && !ftr) || ((hdr_len + 7) & ~7u) + ftr_len + 16 > FRAME_CAP ||
        (n && (!d_out || !d_out_off || !d_out_len || !d_ret || !d_dst)))
        return set_err(DG_E_INVALID, "bad args");
    return pack_scan(c, d_out, d_out_off, d_out_len, d_ret, n, hdr, hdr_len, ftr, ftr_len, d_dst, d_dst_off, stream);
}

int dg_bench_device(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_json, const uint64_t *d_in_off,
                    uint64_t n, uint64_t flags, uint8_t *d_out, const uint64_t *d_out_off, uint32_t *d_out_len,
                    uint64_t *d_ret, int iters, float *ms)
{
    if (!c || !d || iters < 1 || !ms) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, c->stream));
    for (int k = 0; k < iters; k++) {
        int rc = launch(c, d, root, d_json, d_in_off, n, flags, d_out, d_out_off, d_out_len, d_ret, c->d_pending,
                        c->stream);
        if (rc) return rc;
    }
    HIPCHK(hipEventRecord(e1, c->stream));
    HIPCHK(hipEventSynchronize(e1));
    HIPCHK(hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return DG_OK;
}

}  // extern "C"
