/*
 * t2j_host.hip — the C ABI of the reverse path, Thrift binary -> JSON
 * (include/dgj2t.h dg_desc_attach_t2j / dg_t2j_*; the reference's
 * t2j.BinaryConv.Do / DoInto, conv/t2j/conv.go:50-95). Kernels: t2j_device.h.
 */
#include <string.h>

#include "host_internal.h"
#include "t2j_device.h"

using namespace dg;

static const uint64_t T2J_DEEP_WS =
    (uint64_t)T2J_DEEP_BLOCKS * T2J_BLOCK * (T2J_DEEP_DEPTH * sizeof(T2JFrame) + (uint64_t)T2J_WIDE_WORDS * 8);

/* lanes per message of the LDS-frame pass (t2j_kern.hip) from the batch's
 * longest message: short messages want full waves, ~1 KB ones sparse waves;
 * unknown or huge (a mixed batch) keep the middle. the t2j_spread knob (1|2|4) forces. */
static uint32_t t2j_spread(const dg_ctx *c, uint64_t max_len)
{
    const int64_t v = c->knobs.t2j_spread;
    if (v) return v == 1 || v == 4 ? (uint32_t)v : 2u;
    if (max_len == 0 || max_len > 16384) return 2;
    return max_len <= 512 ? 1 : 4;
}

/* one batch on stream s. With the wave path (a descriptor that fits LDS and
 * messages that may be long): the lane pass converts the short messages and
 * lists the long ones, the wave kernel converts those (t2j_wave.h), the lane
 * pass in list mode converts the wave kernel's bails. Then the deep pass over
 * what the lane passes queued (it also zeroes the counter set the previous
 * launch used); the scratch's `done`
 * event after. */
static int t2j_launch(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *src, const uint64_t *in_off,
                      uint64_t n, uint64_t opts, uint8_t *out, const uint64_t *out_off, uint32_t *out_len,
                      uint64_t *ret, hipStream_t s, uint64_t max_len, uint64_t *aux = nullptr,
                      const dg_cb_entry *ans = nullptr, const uint8_t *ans_bytes = nullptr)
{
    if (n == 0) return DG_OK;
    if (!d->d_side) return set_err(DG_E_DESC, "descriptor has no t2j side table (dg_desc_attach_t2j)");
    if (root >= d->hdr.n_types) return set_err(DG_E_INVALID, "root type %u out of range", root);
    if (n > 0xFFFFFFFFull) return set_err(DG_E_INVALID, "batch of %llu messages", (unsigned long long)n);
    Scratch *x;
    int rc = scratch_for(c, s, &x);
    if (rc) return rc;
    if ((rc = grow_x(x, x->t2j_list, x->t2j_list_cap, n))) return rc;
    if (!c->ws_t2j) {
        HIPCHK(hipMalloc(&c->ws_t2j, T2J_DEEP_WS));
        /* ordering only (the next deep pass on another stream): no system-scope fence */
        HIPCHK(hipEventCreateWithFlags(&c->ws_t2j_done, hipEventDisableTiming | hipEventDisableSystemFence));
    }
    const uint64_t wmin = (uint64_t)c->knobs.t2j_wave_min;
    /* the root-level Go-side options run on the lane kernel only */
    const bool wave = !(opts & (DG_T2J_CONVERT_EXC | DG_T2J_SKIP_RESP_BASE | DG_T2J_HM)) && wmin > 0 && d->hdr.total_len <= 16384 && d->hdr.n_fields <= 1024 && /* T2W_FX */
                      d->hdr.n_types < 4096 && /* a token's type index */
                      d->side_len <= 12288 /* T2W_SIDE */ && (max_len == 0 || max_len > wmin);
    if (wave) {
        if ((rc = grow_x(x, x->t2j_big, x->t2j_big_cap, n))) return rc;
        if ((rc = grow_x(x, x->t2j_bail, x->t2j_bail_cap, n))) return rc;
        if (!c->ws_t2w) HIPCHK(hipMalloc(&c->ws_t2w, t2j_wave_ws_bytes((uint32_t)c->n_cu * T2W_BPC)));
    }
    /* overlapped form: the wave kernel (and its bails' list pass) on the
     * scratch's second stream, beside the lane pass over the short ones, so
     * the lane pass fills the CUs the persistent wave grid leaves idle */
    const bool ovl = wave && c->knobs.t2j_overlap != 0;
    if (ovl && !x->side) {
        HIPCHK(hipStreamCreateWithFlags(&x->side, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&x->side_go, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&x->side_done, hipEventDisableTiming));
    }
    hipStream_t ws = ovl ? x->side : s; /* the wave kernel's stream */
    if (wave) {
        /* one token workspace per context, like the deep workspace: a wave
         * pass on another stream waits for the previous one */
        if (c->ws_t2w_last && c->ws_t2w_last != ws) HIPCHK(hipStreamWaitEvent(ws, c->ws_t2w_done, 0));
    }
    /* this launch's counter set; its deep pass zeroes the other one */
    uint32_t *const cnt = x->d_counts + (x->t2j_set ? 16u : DG_T2J_DEEP_COUNT);
    uint32_t *const cnt_next = x->d_counts + (x->t2j_set ? DG_T2J_DEEP_COUNT : 16u);
    T2JParams P;
    memset(&P, 0, sizeof P);
    P.root = root;
    P.opts = opts;
    P.src = src;
    P.in_off = in_off;
    P.n = n;
    P.out = out;
    P.out_off = out_off;
    P.out_len = out_len;
    P.ret = ret;
    P.blob = d->d_blob;
    P.hdr = d->hdr;
    P.side = d->d_side;
    P.deep_list = x->t2j_list;
    P.deep_count = cnt;
    P.reset_counts = cnt_next;
    P.ws = c->ws_t2j;
    P.stats = c->d_stats;
    P.aux = (opts & DG_T2J_SKIP_RESP_BASE) ? aux : nullptr;
    P.ans_tab = (opts & DG_T2J_HM) ? ans : nullptr;
    P.ans_bytes = ans_bytes;
    hipError_t e = hipSuccess;
    if (wave) {
        T2JParams P1 = P;
        P1.big_list = x->t2j_big;
        P1.big_count = cnt + 1;
        P1.big_min = wmin;
        if (ovl) {
            launch_t2j_route(n, s, P1); /* the long ones, by length */
            if ((e = hipGetLastError()) == hipSuccess) e = hipEventRecord(x->side_go, s);
            if (e == hipSuccess) e = hipStreamWaitEvent(ws, x->side_go, 0);
            P1.skip_big = 1;
            P1.big_list = nullptr;
            P1.big_count = nullptr;
        }
        if (e == hipSuccess) launch_t2j_pass(n, s, P1, 1); /* the short ones: full waves */
        T2WParams W;
        W.list = x->t2j_big;
        W.count = cnt + 1;
        W.queue = cnt + 2;
        W.bail_list = x->t2j_bail;
        W.bail_count = cnt + 3;
        const uint32_t wblocks = (uint32_t)c->n_cu * T2W_BPC; /* the token regions are sized for it */
        W.tok = c->ws_t2w;
        W.side_len = (uint32_t)d->side_len;
        if (e == hipSuccess && (e = hipGetLastError()) == hipSuccess) {
            launch_t2j_wave(wblocks, ws, P, W);
            e = hipGetLastError();
        }
        if (e == hipSuccess) {
            T2JParams P3 = P;
            P3.list = x->t2j_bail;
            P3.list_count = W.bail_count;
            launch_t2j_list(64, ws, P3);
            e = hipGetLastError();
        }
        if (e == hipSuccess) {
            if (!c->ws_t2w_done) e = hipEventCreateWithFlags(&c->ws_t2w_done, hipEventDisableTiming | hipEventDisableSystemFence);
            if (e == hipSuccess) e = hipEventRecord(c->ws_t2w_done, ws);
            if (e == hipSuccess) c->ws_t2w_last = ws;
        }
        if (ovl && e == hipSuccess) { /* the deep pass takes both passes' queue */
            e = hipEventRecord(x->side_done, ws);
            if (e == hipSuccess) e = hipStreamWaitEvent(s, x->side_done, 0);
        }
    } else {
        launch_t2j_pass(n, s, P, t2j_spread(c, max_len));
        e = hipGetLastError();
    }
    /* the deep workspace is one per context: a deep pass on another stream
     * than the previous one waits for it (deep messages are rare; the LDS
     * passes of different streams still overlap) */
    if (e == hipSuccess && c->ws_t2j_last && c->ws_t2j_last != s) e = hipStreamWaitEvent(s, c->ws_t2j_done, 0);
    if (e == hipSuccess) {
        launch_t2j_deep(s, P);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(c->ws_t2j_done, s);
    if (e == hipSuccess) c->ws_t2j_last = s;
    if (e == hipSuccess) {
        x->t2j_set ^= 1u;
    } else { /* the deep pass may not have run: both sets cleared */
        (void)hipMemsetAsync(cnt, 0, 16, s);
        (void)hipMemsetAsync(cnt_next, 0, 16, s);
    }
    HIPCHK(hipEventRecord(x->done, s));
    x->used = true;
    x->last = s;
    if (e != hipSuccess) return set_err(DG_E_HIP, "t2j launch: %s", hipGetErrorString(e));
    return DG_OK;
}

extern "C" {

int dg_desc_attach_t2j(dg_desc *d, const void *side, size_t len)
{
    if (!d || !side || len < sizeof(dg_t2j_hdr)) return set_err(DG_E_INVALID, "bad args");
    dg_t2j_hdr h;
    memcpy(&h, side, sizeof h);
    if (h.magic != DG_T2J_MAGIC || h.version != 1 || h.total_len > len || h.n_fields != d->hdr.n_fields ||
        (uint64_t)h.off_fields + (uint64_t)h.n_fields * sizeof(dg_t2j_field) > len ||
        (uint64_t)h.off_pool + h.pool_len > len || (h.off_pool & 7))
        return set_err(DG_E_DESC, "bad t2j side table");
    /* every key range inside the pool (the kernel reads them unchecked) */
    const dg_t2j_field *f = (const dg_t2j_field *)((const uint8_t *)side + h.off_fields);
    for (uint32_t k = 0; k < h.n_fields; k++)
        if ((uint64_t)f[k].key_off + f[k].key_len > h.pool_len || (uint64_t)f[k].name_off + f[k].name_len > h.pool_len ||
            (f[k].key_off & 7) || (f[k].name_off & 7))
            return set_err(DG_E_DESC, "t2j side table: field %u key out of range", k);
    std::lock_guard<std::mutex> g(d->ctx->mu);
    HIPCHK(hipSetDevice(d->ctx->device));
    uint8_t *p;
    HIPCHK(hipMalloc(&p, len + 16)); /* the kernel reads whole words past a key's end */
    HIPCHK(hipMemcpy(p, side, len, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(p + len, 0, 16));
    HIPCHK(hipDeviceSynchronize()); /* before launches on non-blocking streams read it */
    if (d->d_side) {
        HIPCHK(hipDeviceSynchronize()); /* launches in flight may read the old table */
        (void)hipFree(d->d_side);
    }
    d->d_side = p;
    d->side_len = len;
    return DG_OK;
}

/* 128-byte slots, like dg_slot_bound: t2j-c2's writes were 380 B per
 * message (every line its 208 B of JSON touched) at 8-byte alignment */
uint64_t dg_t2j_slot_bound(uint64_t len) { return (3 * len + 64 + 127) & ~127ull; }

int dg_t2j_batch_device_ml(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_thrift,
                           const uint64_t *d_in_off, uint64_t n, uint64_t opts, uint8_t *d_out,
                           const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, void *stream,
                           uint64_t max_len)
{
    if (!c || !d) return set_err(DG_E_INVALID, "null ctx/desc");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return t2j_launch(c, d, root, d_thrift, d_in_off, n, opts, d_out, d_out_off, d_out_len, d_ret, s, max_len);
}

int dg_t2j_batch_device_aux(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_thrift,
                            const uint64_t *d_in_off, uint64_t n, uint64_t opts, uint8_t *d_out,
                            const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, uint64_t *d_aux,
                            void *stream, uint64_t max_len)
{
    if (!c || !d || ((opts & DG_T2J_SKIP_RESP_BASE) && !d_aux)) return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return t2j_launch(c, d, root, d_thrift, d_in_off, n, opts, d_out, d_out_off, d_out_len, d_ret, s, max_len, d_aux);
}

int dg_t2j_batch_device_cb(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_thrift,
                           const uint64_t *d_in_off, uint64_t n, uint64_t opts, uint8_t *d_out,
                           const uint64_t *d_out_off, uint32_t *d_out_len, uint64_t *d_ret, uint64_t *d_aux,
                           const dg_cb_entry *d_ans, const uint8_t *d_ans_bytes, void *stream, uint64_t max_len)
{
    if (!c || !d || ((opts & DG_T2J_SKIP_RESP_BASE) && !d_aux) || (d_ans && !d_ans_bytes))
        return set_err(DG_E_INVALID, "bad args");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return t2j_launch(c, d, root, d_thrift, d_in_off, n, opts, d_out, d_out_off, d_out_len, d_ret, s, max_len, d_aux,
                      d_ans, d_ans_bytes);
}

int dg_t2j_batch_device(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *d_thrift, const uint64_t *d_in_off,
                        uint64_t n, uint64_t opts, uint8_t *d_out, const uint64_t *d_out_off, uint32_t *d_out_len,
                        uint64_t *d_ret, void *stream)
{
    return dg_t2j_batch_device_ml(c, d, root, d_thrift, d_in_off, n, opts, d_out, d_out_off, d_out_len, d_ret, stream,
                                  0);
}

static int t2j_batch_host(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *thrift, const uint64_t *in_off,
                          uint64_t n, uint64_t opts, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *ret,
                          uint64_t *out_need, uint64_t *aux, const dg_cb_tables *cb)
{
    if (!c || !d || (!thrift && n) || !in_off || !out_off || (!ret && n) ||
        ((opts & DG_T2J_SKIP_RESP_BASE) && n && !aux) || (cb && cb->ans_tab && cb->len && !cb->bytes))
        return set_err(DG_E_INVALID, "bad args");
    const dg_cb_entry *ans = cb && (opts & DG_T2J_HM) ? cb->ans_tab : nullptr;
    for (uint64_t i = 0; ans && i < n; i++) /* one byte per answer, inside the bytes (read unchecked) */
        if (ans[i].off + ans[i].count > cb->len)
            return set_err(DG_E_INVALID, "callback answers of message %llu outside the bytes", (unsigned long long)i);
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    const uint64_t base = in_off[0];
    std::vector<uint64_t> ioff(n + 1), soff(n + 1);
    std::vector<uint32_t> olen(n);
    std::vector<uint8_t> stage;
    hipStream_t s = c->stream;
    int rc;
    /* pass 0: every message in a dg_t2j_slot_bound slot; pass 1: the
     * overflowed ones again, each in a slot of exactly the size it reported */
    std::vector<uint64_t> todo(n);
    for (uint64_t i = 0; i < n; i++) todo[i] = i;
    std::vector<uint64_t> slot_of(n, 0); /* stage offset of message i's final bytes */
    uint64_t max_len = 0;
    for (uint64_t i = 0; i < n; i++) max_len = std::max<uint64_t>(max_len, in_off[i + 1] - in_off[i]);
    for (int pass = 0; pass < 2 && !todo.empty(); pass++) {
        const uint64_t m = todo.size();
        std::vector<uint64_t> io(m + 1), so(m + 1);
        io[0] = so[0] = 0;
        for (uint64_t k = 0; k < m; k++) {
            const uint64_t i = todo[k], len = in_off[i + 1] - in_off[i];
            io[k + 1] = io[k] + len;
            so[k + 1] = so[k] + (pass == 0 ? dg_t2j_slot_bound(len) : ((uint64_t)olen[i] + 64 + 7) & ~7ull);
        }
        if ((rc = grow(c->d_json, c->d_json_cap, io[m] + 64))) return rc;
        if ((rc = grow(c->d_in_off, c->d_in_cap, m + 1))) return rc;
        if ((rc = grow(c->d_out, c->d_out_cap, so[m] + 64))) return rc;
        if ((rc = grow(c->d_out_off, c->d_oo_cap, m + 1))) return rc;
        if ((rc = grow(c->d_out_len, c->d_ol_cap, m + 1))) return rc;
        if ((rc = grow(c->d_ret, c->d_ret_cap, m + 1))) return rc;
        if (aux && (rc = grow(c->d_aux, c->d_aux_cap, m + 1))) return rc;
        if (ans) { /* [m entries | the answer bytes] */
            if ((rc = grow(c->d_cb, c->d_cb_cap, 8 * m + cb->len + 8))) return rc;
            std::vector<dg_cb_entry> e(m);
            for (uint64_t k = 0; k < m; k++) e[k] = ans[todo[k]];
            HIPCHK(hipMemcpyAsync(c->d_cb, e.data(), 8 * m, hipMemcpyHostToDevice, s));
            if (cb->len) HIPCHK(hipMemcpyAsync(c->d_cb + 8 * m, cb->bytes, cb->len, hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s)); /* e is a local */
        }
        if (pass == 0) {
            HIPCHK(hipMemcpyAsync(c->d_json, thrift + base, io[m], hipMemcpyHostToDevice, s));
        } else {
            for (uint64_t k = 0; k < m; k++)
                HIPCHK(hipMemcpyAsync(c->d_json + io[k], thrift + in_off[todo[k]], io[k + 1] - io[k],
                                      hipMemcpyHostToDevice, s));
        }
        HIPCHK(hipMemsetAsync(c->d_json + io[m], 0, 64, s));
        HIPCHK(hipMemcpyAsync(c->d_in_off, io.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_out_off, so.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
        if ((rc = t2j_launch(c, d, root, c->d_json, c->d_in_off, m, opts, c->d_out, c->d_out_off, c->d_out_len,
                             c->d_ret, s, max_len, aux ? c->d_aux : nullptr,
                             ans ? (const dg_cb_entry *)(const void *)c->d_cb : nullptr, ans ? c->d_cb + 8 * m : nullptr)))
            return rc;
        std::vector<uint64_t> r(m), ax(aux ? m : 0);
        std::vector<uint32_t> l(m);
        if (aux) HIPCHK(hipMemcpyAsync(ax.data(), c->d_aux, m * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(r.data(), c->d_ret, m * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(l.data(), c->d_out_len, m * 4, hipMemcpyDeviceToHost, s));
        const uint64_t off0 = stage.size();
        stage.resize(off0 + so[m]);
        HIPCHK(hipMemcpyAsync(stage.data() + off0, c->d_out, so[m], hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        std::vector<uint64_t> next;
        for (uint64_t k = 0; k < m; k++) {
            const uint64_t i = todo[k];
            ret[i] = r[k];
            olen[i] = l[k];
            if (aux) aux[i] = ax[k];
            slot_of[i] = off0 + so[k];
            if ((uint8_t)r[k] == DG_ST_OUT_OVERFLOW) {
                if (pass == 1)
                    return set_err(DG_E_NOMEM, "message %llu overflowed its exact-size slot", (unsigned long long)i);
                next.push_back(i);
            }
        }
        todo.swap(next);
    }
    uint64_t total = 0;
    out_off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (ret[i] != 0 && (uint8_t)ret[i] != DG_T2J_E_EXCEPTION && (uint8_t)ret[i] != DG_T2J_E_CALLBACK)
            olen[i] = 0; /* kept: the exception's JSON, a stop's record */
        total += olen[i];
        out_off[i + 1] = total;
    }
    if (out_need) *out_need = total;
    if (total > out_cap || (!out && total)) return set_err(DG_E_NOMEM, "output needs %llu bytes", (unsigned long long)total);
    for (uint64_t i = 0; i < n; i++)
        if (olen[i]) memcpy(out + out_off[i], stage.data() + slot_of[i], olen[i]);
    return DG_OK;
}

int dg_t2j_batch_host(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *thrift, const uint64_t *in_off,
                      uint64_t n, uint64_t opts, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *ret,
                      uint64_t *out_need)
{
    return t2j_batch_host(c, d, root, thrift, in_off, n, opts, out, out_cap, out_off, ret, out_need, nullptr, nullptr);
}

int dg_t2j_batch_host_aux(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *thrift, const uint64_t *in_off,
                          uint64_t n, uint64_t opts, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *ret,
                          uint64_t *out_need, uint64_t *aux)
{
    return t2j_batch_host(c, d, root, thrift, in_off, n, opts, out, out_cap, out_off, ret, out_need, aux, nullptr);
}

int dg_t2j_batch_host_cb(dg_ctx *c, const dg_desc *d, uint32_t root, const uint8_t *thrift, const uint64_t *in_off,
                         uint64_t n, uint64_t opts, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *ret,
                         uint64_t *out_need, uint64_t *aux, const dg_cb_tables *cb)
{
    return t2j_batch_host(c, d, root, thrift, in_off, n, opts, out, out_cap, out_off, ret, out_need, aux, cb);
}

}  // extern "C"
