/*
 * j2t_machine.h — the exact machine and the lane kernel (device side).
 *
 * Kernel map (one launch per batch):
 *  j2t_lane_kernel  one lane per message; the block's JSON span is staged in
 *                   LDS. Phase 1: each lane runs the fast path (j2t_fast.h) on
 *                   its own message. Phase 2: the messages the fast path
 *                   bailed on are compacted onto the first lanes and redone by
 *                   the exact machine (Machine<S>::run, a restatement of
 *                   j2t_fsm_exec native/thrift.c:765-1187) with a stack of
 *                   LDS_DEPTH frames; messages that outgrow it are listed as
 *                   DG_ST_DEEP and the LAST block to finish redoes them
 *                   (deep_pass) with a MAX_RECURSE (4096) stack in device
 *                   workspace.
 * The kernel is instantiated in j2t_kern_lds.hip (descriptor copied to LDS)
 * and j2t_kern_glb.hip (descriptor read from global memory), so the two
 * compile in parallel; j2t_host.hip holds the C ABI.
 */
#pragma once
#include <hip/hip_runtime.h>

#include "j2t_device.h"
#include "j2t_fast.h"

namespace dg {

constexpr int FAST_DEPTH = 24;      /* frames per lane in the fast kernel */
constexpr int FAST_SKIP_WORDS = 1;  /* 64 skip levels */
constexpr int WS_KEYCAP = 1024;     /* unquoted-key buffer per lane (reference key cache: 1 KB) */
constexpr int WS_REQCAP = 256;      /* multi-word requires arena per lane (words) */
constexpr int DEEP_THREADS = 256;   /* lanes of the deep pass (= LANE_BLOCK) */
constexpr int DEEP_KEYCAP = 1 << 20;
constexpr int DEEP_REQCAP = 1 << 16;

struct Params {
    uint32_t root;
    const uint8_t *json;
    const uint64_t *in_off;
    uint64_t n;
    uint64_t flag;
    uint8_t *out;
    const uint64_t *out_off;
    uint32_t *out_len;
    uint64_t *ret;
    uint32_t *pending;
    uint32_t *deep_count; /* DG_ST_DEEP messages appended here by the fast kernel */
    uint64_t *deep_list;
    uint8_t *ws;       /* per-lane workspace base */
    uint64_t ws_stride;/* bytes per lane */
    uint32_t keycap, reqcap;
    uint32_t fast;     /* run the fast path first (descriptor v2, flags within FAST_FLAGS) */
    unsigned long long *stats; /* {messages bailed to the exact machine, messages redone deep} */
    const uint32_t *list;      /* list mode: convert only these messages (exact machine) */
    uint32_t *list_count;      /* device count of `list` (self-reset by the last block) */
    uint32_t *reset2;          /* two more counters the last block resets (list mode: large-message count, wave queue) */
    uint32_t *big_list;        /* messages longer than big_max are left to the wave kernel via this list */
    uint32_t *big_count;
    uint64_t big_max;
    uint32_t *huge_count;      /* messages longer than huge_min go to the END of big_list (taken first) */
    uint64_t huge_min;
    const dg_hm_entry *hm_tab; /* DG_F_HM_SPLIT: n_hm entries per message (dgj2t_defs.h), or NULL: the root's
                                  mapped fields only, all written by the host */
    const uint8_t *hm_bytes;   /* the host's callback answers (dg_cb_tables.bytes) */
    uint32_t n_hm;
    const dg_cb_entry *ans_tab; /* non-inline value mapping: one entry per message (dgj2t_defs.h), or NULL */
};

/* List message i (len bytes) for the wave kernel. Huge ones are written from
 * the end of the list and the wave kernel's queue hands them out first: a
 * C4-size message keeps a wave busy for about a millisecond, so one taken
 * last would set the kernel's tail. */
DGI void list_big(const Params &P, uint64_t i, uint64_t len)
{
    if (P.huge_count && len > P.huge_min) {
        const uint32_t q = __hip_atomic_fetch_add(P.huge_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        P.big_list[P.n - 1 - q] = (uint32_t)i;
    } else {
        const uint32_t q = __hip_atomic_fetch_add(P.big_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        P.big_list[q] = (uint32_t)i;
    }
}

/* Append v to list[*count] for every active lane with want, one atomic per
 * wave (ballot + prefix): t2j-c3's routing pass spent 0.28 ms on 65 536
 * single-counter atomics. Call with every active lane, not under want. */
DGI void wave_push(uint32_t *list, uint32_t *count, bool want, uint32_t v, bool from_end = false, uint64_t n = 0)
{
    const uint64_t m = __builtin_amdgcn_ballot_w64(want);
    if (!m) return;
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t q = 0;
    if (lane == leader)
        q = __hip_atomic_fetch_add(count, (uint32_t)__builtin_popcountll(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    q = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)leader) + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
    if (want) list[from_end ? n - 1 - q : q] = v;
}

/* list_big for every active lane at once (want: this lane's message goes) */
DGI void list_big_w(const Params &P, bool want, uint64_t i, uint64_t len)
{
    const bool huge = want && P.huge_count && len > P.huge_min;
    wave_push(P.big_list, P.big_count, want && !huge, (uint32_t)i);
    if (P.huge_count) wave_push(P.big_list, P.huge_count, huge, (uint32_t)i, true, P.n);
}

#ifdef DG_PROFILE
#define PROF_DECL uint64_t prof[16] = {0};
#define PROF(k, stmt)                                    \
    do {                                                 \
        uint64_t t0_ = __builtin_amdgcn_s_memtime();     \
        stmt;                                            \
        prof[k] += __builtin_amdgcn_s_memtime() - t0_;   \
    } while (0)
#else
#define PROF_DECL
#define PROF(k, stmt) stmt
#endif

/* Frame stack: frame k of this lane at base[k * stride] (LDS: frame-major
 * across the block, so a wave at equal depth touches consecutive slots). */
template <class FP>
struct FStack {
    FP base;
    uint32_t stride;
    DGI auto &operator[](uint32_t k) const { return base[k * stride]; }
};

/* The FSM of one message over source type S (LDS- or global-backed) and
 * frame storage FP (LDS or device workspace). */
template <class S, class FP, class DV>
struct Machine {
    DV D;
    S src;
    Out out;
    uint64_t flag;
    FStack<FP> vt;
    uint32_t sp, cap;
    gu64 *skipbits;
    uint32_t skipcap;
    Workspace ws;
    uint32_t reqlen;
    uint32_t field_cache_len;
    const dg_hm_entry *hm_row; /* this message's HTTP-mapping entries (Params::hm_tab), or NULL */
    const uint8_t *hm_bytes;
    const dg_cb_entry *ans_row; /* this message's value-mapping answers (Params::ans_tab), or NULL */
    uint32_t ans_seen;          /* non-inline value-mapping values met so far */
    uint64_t ans_at;            /* hm_bytes offset of the next answer */
    uint32_t ncb;               /* DG_F_CB_COLLECT: callbacks recorded in this pass */
    uint32_t cb_need;           /* ... the slot bytes the first record needs when it does not fit */
    uint64_t slot_cap;          /* ... the slot's size (out.cap is 0 once one is: the output is dropped) */
    Out rec;                    /* ... their records, from the slot's start */
    JState jt;
    PROF_DECL

    DGI dg_type TY(uint32_t t) const { return ldrec(&D.T[t]); }

    DGI uint64_t push(uint32_t st, uint32_t td, int64_t p)
    {
        if (sp >= MAX_RECURSE) return pack(E_RECURSE_MAX, sp, (uint64_t)p);
        if (sp >= cap) return pack0(DG_ST_DEEP, 0);
        auto &x = vt[sp++];
        x.st = st;
        x.td = td;
        return 0;
    }

    /* requires bits of struct frame x (bm_* native/map.c:134-154) */
    template <class FR>
    DGI bool bm_is_set(const FR &x, const dg_struct &sd, uint32_t k) const
    {
        if (sd.req_words == 1) return (x.u >> k) & 1;
        return (ws.reqarena[(uint32_t)x.u + (k >> 6)] >> (k & 63)) & 1;
    }
    template <class FR>
    DGI void bm_set_req(FR &x, const dg_struct &sd, uint32_t k, int req)
    {
        uint64_t m = 1ull << (k & 63);
        bool set = req == DG_REQ_DEFAULT || req == DG_REQ_REQUIRED;
        if (!set && req != DG_REQ_OPTIONAL) return;
        if (sd.req_words == 1) {
            x.u = set ? (x.u | m) : (x.u & ~m);
        } else {
            gu64 *w = &ws.reqarena[(uint32_t)x.u + (k >> 6)];
            *w = set ? (*w | m) : (*w & ~m);
        }
    }

    /* tb_write_empty native/thrift.c:171-203 */
    DGI uint64_t write_empty(uint32_t td, int64_t p)
    {
        const dg_type t = TY(td);
        switch (t.ttype) {
        case DG_T_BOOL:
        case DG_T_BYTE: out.w8(0); return 0;
        case DG_T_I16: out.w16(0); return 0;
        case DG_T_I32: out.w32(0); return 0;
        case DG_T_I64:
        case DG_T_DOUBLE: out.w64(0); return 0;
        case DG_T_STRING: out.w32(0); return 0;
        case DG_T_LIST:
        case DG_T_SET:
            out.w8(TY(t.elem).ttype);
            out.w32(0);
            return 0;
        case DG_T_MAP:
            out.w8(TY(t.key).ttype);
            out.w8(TY(t.elem).ttype);
            out.w32(0);
            return 0;
        case DG_T_STRUCT: out.w8(0); return 0;
        default: return pack(E_UNSUPPORT_THRIFT_TYPE, t.ttype, (uint64_t)p);
        }
    }
    /* tb_write_default_or_empty native/thrift.c:205-217 */
    DGI uint64_t write_default_or_empty(const dg_field &f, int64_t p)
    {
        if (f.dflt_len != DG_NONE) {
            for (uint32_t i = 0; i < f.dflt_len; i++) out.w8(D.P[f.dflt_off + i]);
            return 0;
        }
        return write_empty(f.type, p);
    }

    /* j2t_write_unset_fields native/thrift.c:258-310 */
    template <class FR>
    DGI uint64_t write_unset_fields(const FR &x, const dg_struct &sd, int64_t p)
    {
        bool wr = flag & DG_F_WRITE_REQUIRE, wd = flag & DG_F_WRITE_DEFAULT;
        bool wo = flag & DG_F_WRITE_OPTIONAL, tb = flag & DG_F_TRACE_BACK;
        for (uint32_t w = 0; w < sd.req_words; w++) {
            uint64_t bits = sd.req_words == 1 ? x.u : ws.reqarena[(uint32_t)x.u + w];
            while (bits) {
                uint32_t k = w * 64 + __builtin_ctzll(bits);
                bits &= bits - 1;
                const dg_field f = ldrec(&D.F[sd.field_begin + k]);
                if (f.flags & DG_FF_REQUEST_BASE) continue;
                if (tb && (f.required == DG_REQ_REQUIRED || sp == 1)) field_cache_len++;
                else if (!wr && f.required == DG_REQ_REQUIRED)
                    return pack(E_NULL_REQUIRED, f.id, (uint64_t)p);
                else if ((wr && f.required == DG_REQ_REQUIRED) || (wd && f.required == DG_REQ_DEFAULT) ||
                         (wo && f.required == DG_REQ_OPTIONAL)) {
                    out.w8(TY(f.type).ttype);
                    out.w16(f.id);
                    uint64_t r = write_default_or_empty(f, p);
                    if (r) return r;
                }
            }
        }
        return 0;
    }

    /* ERR_HM_END (native/thrift.c:898-903): unset fields went to the Go
     * handler's field cache. At the root under DG_F_HM_SPLIT the host serves
     * it (handleUnmatchedFields, conv/j2t/impl_amd64.go:71-115): the output so
     * far, then the root's remaining requires words (big-endian u64; the
     * cached fields are their set bits, in field order), status
     * DG_ST_HM_END with value = the word count. Elsewhere: the reference's
     * code (a nested struct's callback needs the Go FSM to resume). */
    template <class FR>
    DGI uint64_t hm_end(const FR &x, const dg_struct &sd, uint32_t si, int64_t p)
    {
        if (!(flag & DG_F_HM_SPLIT)) return pack0(E_HM_END, (uint64_t)p);
        if (sp == 1) {
            for (uint32_t w = 0; w < sd.req_words; w++) out.w64(sd.req_words == 1 ? x.u : ws.reqarena[(uint32_t)x.u + w]);
            return pack(DG_ST_HM_END, sd.req_words, (uint64_t)p);
        }
        /* nested: the host's handleUnmatchedFields answer (fields + STOP), or
         * stop for it (dgj2t_defs.h dg_cb_entry) */
        field_cache_len = 0;
        if (take_answer()) return 0;
        if (flag & DG_F_CB_COLLECT) {
            if (!cb_room(16 + 8 * sd.req_words)) return cb_full(16 + 8 * sd.req_words);
            rec.w64(pack(DG_ST_HM_END_AT, sd.req_words, (uint64_t)p));
            rec.w64(si);
            for (uint32_t w = 0; w < sd.req_words; w++) {
                uint64_t bits = sd.req_words == 1 ? x.u : ws.reqarena[(uint32_t)x.u + w], m = 0;
                while (bits) {
                    const uint32_t b = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    const dg_field f = ldrec(&D.F[sd.field_begin + w * 64 + b]);
                    if (!(f.flags & DG_FF_REQUEST_BASE) && f.required == DG_REQ_REQUIRED) m |= 1ull << b;
                }
                rec.w64(m);
            }
            ncb++;
            return 0;
        }
        out.set_len(0);
        out.w64(si);
        for (uint32_t w = 0; w < sd.req_words; w++) {
            uint64_t bits = sd.req_words == 1 ? x.u : ws.reqarena[(uint32_t)x.u + w], m = 0;
            while (bits) { /* the fields write_unset_fields cached (native/thrift.c:281-294) */
                const uint32_t b = __builtin_ctzll(bits);
                bits &= bits - 1;
                const dg_field f = ldrec(&D.F[sd.field_begin + w * 64 + b]);
                if (!(f.flags & DG_FF_REQUEST_BASE) && f.required == DG_REQ_REQUIRED) m |= 1ull << b;
            }
            out.w64(m);
        }
        return pack(DG_ST_HM_END_AT, sd.req_words, (uint64_t)p);
    }

    /* DG_F_CB_COLLECT: room for a callback record of `bytes` in the slot.
     * The first one switches the output off (out.cap = 0: later writes are
     * only counted) and starts the records at the slot's start. A callback's
     * answer is output bytes only -- the reference's FSM resumes after the
     * value or the struct either way (conv/j2t/impl_amd64.go:71-155) -- so
     * converting on without it meets the same later callbacks and errors. */
    DGI bool cb_room(uint32_t bytes)
    {
        if (ncb == 0) {
            slot_cap = out.cap;
            rec.init((uint8_t *)(void *)out.b, slot_cap);
            out.cap = 0;
        }
        return rec.len + bytes <= slot_cap;
    }

    /* a record does not fit the slot: the records so far go to the host, or,
     * when there are none, the slot is too small even for the first one and
     * the host reruns the message with a slot of the bytes needed (as for
     * any output overflow) instead of getting an empty record list */
    DGI uint64_t cb_full(uint32_t bytes)
    {
        if (ncb) return pack(DG_ST_CB_LIST, ncb, 0);
        out.cap = slot_cap;
        cb_need = bytes;
        return pack(DG_ST_OUT_OVERFLOW, bytes, 0);
    }

    /* the host's next callback answer (dg_cb_entry), if it has one: written */
    DGI bool take_answer()
    {
        if (!ans_row || ans_seen >= ans_row->count) return false;
        const uint32_t n = (uint32_t)hm_bytes[ans_at] | ((uint32_t)hm_bytes[ans_at + 1] << 8) |
                           ((uint32_t)hm_bytes[ans_at + 2] << 16) | ((uint32_t)hm_bytes[ans_at + 3] << 24);
        for (uint32_t b = 0; b < n; b++) out.w8(hm_bytes[ans_at + 4 + b]);
        ans_at += 4 + (uint64_t)n;
        ans_seen++;
        return true;
    }

    /* j2t_number native/thrift.c:312-365 */
    template <class S2>
    DGI uint64_t j2t_number(uint32_t td, S2 &s, int64_t &p)
    {
        int64_t s0 = p;
        vnumber(s, p, jt, ws.dbuf);
        if (jt.vt < 0) return pack((uint32_t)-jt.vt, (uint64_t)s0, (uint64_t)p);
        bool isint = jt.vt == V_INTEGER;
        switch (TY(td).ttype) {
        case DG_T_BYTE: out.w8(isint ? (uint8_t)jt.iv : (uint8_t)cvt32(jt.dv)); return 0;
        case DG_T_I16: out.w16(isint ? (uint16_t)jt.iv : (uint16_t)cvt32(jt.dv)); return 0;
        case DG_T_I32: out.w32(isint ? (uint32_t)jt.iv : (uint32_t)cvt32(jt.dv)); return 0;
        case DG_T_I64: out.w64(isint ? (uint64_t)jt.iv : (uint64_t)cvt64(jt.dv)); return 0;
        case DG_T_DOUBLE: out.w64((uint64_t)__double_as_longlong(jt.dv)); return 0;
        }
        return pack(E_DISMATCH_TYPE, v2(TY(td).ttype, V_INTEGER), (uint64_t)p);
    }

    /* j2t_string native/thrift.c:367-399 */
    DGI uint64_t j2t_string(int64_t &p)
    {
        int64_t s0 = p;
        bool esc;
        int64_t e;
        PROF(8, e = advance_string(src, s0, esc));
        if (e < 0) return pack((uint32_t)-e, (uint64_t)s0, (uint64_t)p);
        p = e;
        int64_t n = e - s0 - 1;
        if (flag & DG_F_VALIDATE_UTF8) {
            int64_t u = utf8_check(src, s0, n);
            if (u >= 0) return pack(E_INVAL, src.raw(s0 + u), (uint64_t)(s0 + u));
        }
        if (esc) {
            uint64_t lp = out.alloc(4);
            OutSink sink{&out};
            int64_t l;
            PROF(9, l = unquote(src, s0, n, sink));
            if (l < 0) return pack((uint32_t)-l, (uint64_t)s0, (uint64_t)p);
            out.put32(lp, (uint32_t)l);
        } else {
            PROF(11, out.w32((uint32_t)n));
            PROF(10, copy_src(s0, n));
        }
        return 0;
    }

    /* copy src[s0, s0+n) to the output (string bodies, tb_write_string) */
    DGI void copy_src(int64_t s0, int64_t n)
    {
#ifdef DG_ABL_NOSTR
        out.len += n;
        return;
#endif
        int64_t i = 0;
        for (; i + 8 <= n; i += 8) out.wle(src.get8(s0 + i), 8);
        for (; i < n; i++) out.w8(src.raw(s0 + i));
    }

    /* j2t_binary native/thrift.c:401-420 */
    DGI uint64_t j2t_binary(int64_t &p)
    {
        int64_t s0 = p;
        bool esc;
        int64_t e = advance_string(src, s0, esc);
        if (e < 0) return pack((uint32_t)-e, (uint64_t)s0, (uint64_t)p);
        p = e;
        int64_t n = e - s0 - 1;
        uint64_t back = out.alloc(4);
        int64_t l;
        PROF(12, l = b64decode(out, src, s0, n));
        if (l < 0) return pack(E_DECODE_BASE64, (uint64_t)(-l - 1), (uint64_t)p);
        out.put32(back, (uint32_t)l);
        return 0;
    }

    /* A JSON object key: raw in the source, or unquoted into the lane's key
     * buffer (the reference's key cache, native/thrift.c:480-498). */
    struct Key {
        bool inbuf;
        int64_t s0;
        int64_t n;
        uint32_t hash;
    };
    DGI uint8_t key_byte(const Key &k, int64_t i) { return k.inbuf ? ws.keybuf[i] : src.raw(k.s0 + i); }

    /* j2t_map_key native/thrift.c:422-447 */
    DGI uint64_t j2t_map_key(const Key &k, uint32_t kt, int64_t p)
    {
        switch (TY(kt).ttype) {
        case DG_T_STRING:
            out.w32((uint32_t)k.n);
            if (k.inbuf) {
                for (int64_t i = 0; i < k.n; i++) out.w8(ws.keybuf[i]);
            } else {
                copy_src(k.s0, k.n);
            }
            return 0;
        case DG_T_BYTE:
        case DG_T_I16:
        case DG_T_I32:
        case DG_T_I64:
        case DG_T_DOUBLE: {
            int64_t q = 0;
            if (k.inbuf) {
                SrcT<glb_u64> kb;
                kb.init((glb_u64 *)ws.keybuf, 0, k.n);
                return j2t_number(kt, kb, q);
            }
            S kv = src.sub(k.s0, k.n);
            return j2t_number(kt, kv, q);
        }
        default:
            return pack(E_UNSUPPORT_THRIFT_TYPE, TY(kt).ttype, (uint64_t)p);
        }
    }

    /* exact-match field lookup (j2t_find_field_key native/thrift.c:449-468) */
    DGI int32_t find_field(const dg_struct &sd, const Key &k)
    {
#ifdef DG_ABL_NOKEY
        return (int32_t)(sd.field_begin + (k.hash % sd.n_fields));
#endif
        uint32_t j = k.hash & sd.name_mask;
        for (;;) {
            const dg_name nm = ldrec(&D.N[sd.name_begin + j]);
            if (nm.field == DG_NONE) return -1;
            if (nm.hash == k.hash && nm.key_len == (uint32_t)k.n) {
                bool eq = true;
                for (int64_t i = 0; i < k.n; i++) {
                    if (D.P[nm.key_off + i] != key_byte(k, i)) {
                        eq = false;
                        break;
                    }
                }
                if (eq) return (int32_t)nm.field;
            }
            j = (j + 1) & sd.name_mask;
        }
    }

    /* j2t_read_key native/thrift.c:470-504 */
    DGI uint64_t read_key(int64_t &p, Key &k)
    {
        int64_t s0 = p;
        bool esc;
        int64_t e = advance_string(src, s0, esc);
        if (e < 0) return pack((uint32_t)-e, (uint64_t)s0, (uint64_t)p);
        p = e;
        k.s0 = s0;
        k.n = e - s0 - 1;
        k.inbuf = false;
        if (esc) {
            BufSink sink{ws.keybuf, (int64_t)ws.keycap, false};
            int64_t l = unquote(src, s0, k.n, sink);
            if (l < 0) return pack((uint32_t)-l, (uint64_t)s0, (uint64_t)p);
            if (sink.over) return pack0(DG_ST_DEEP, 0);
            k.inbuf = true;
            k.n = l;
        }
        uint32_t h = DG_NAME_HASH_SEED;
        for (int64_t i = 0; i < k.n; i++) h = DG_NAME_HASH_STEP(h, key_byte(k, i));
        k.hash = h;
        return 0;
    }

    /* j2t_key native/thrift.c:668-763 */
    DGI uint64_t j2t_key(int64_t &p, uint32_t dc, bool obj0, uint64_t &unwindPos, int32_t &lastField)
    {
        Key key;
        uint64_t r;
        int64_t ks = p;
        PROF(1, r = read_key(p, key));
        if (r) return r;
        int64_t kn = key.n;
        const dg_type t = TY(dc);
        if (t.ttype == DG_T_MAP) {
            if ((flag & DG_F_VALIDATE_UTF8) && TY(t.key).ttype == DG_T_STRING) {
                int64_t u = utf8_check(src, ks, p - ks - 1);
                if (u >= 0) return pack(E_INVAL, src.raw(ks + u), (uint64_t)(ks + u));
            }
            unwindPos = out.len;
            r = j2t_map_key(key, t.key, p);
            if (r) return r;
            if (obj0) {
                set_size(vt[sp - 1], 0);
                return push(J_ELEM, t.elem, p);
            }
            auto &x = vt[sp - 1];
            x.st = J_ELEM;
            x.td = t.elem;
            return 0;
        }
        auto &pex = vt[obj0 ? sp - 1 : sp - 2];
        const dg_struct sd = ldrec(&D.S[t.st]);
        int32_t fi;
        PROF(2, fi = find_field(sd, key));
        if (fi < 0 || ((ldrec(&D.F[fi]).flags & DG_FF_REQUEST_BASE) && (flag & DG_F_NO_WRITE_BASE))) {
            if (fi < 0 && (flag & DG_F_ALLOW_UNKNOWN) == 0) return pack(E_UNKNOWN_FIELD, (uint64_t)kn, (uint64_t)p);
            if (obj0) return push(J_ELEM | ST_SKIP, DG_NONE, p);
            auto &x = vt[sp - 1];
            x.st = J_ELEM | ST_SKIP;
            x.td = DG_NONE;
            return 0;
        }
        const dg_field f = ldrec(&D.F[fi]);
        uint32_t k = (uint32_t)fi - sd.field_begin;
        if ((flag & DG_F_ENABLE_HM) && (f.flags & DG_FF_HTTP_MAPPING) && !bm_is_set(pex, sd, k)) {
            if (obj0) return push(J_ELEM | ST_SKIP, f.type, p);
            auto &x = vt[sp - 1];
            x.st = J_ELEM | ST_SKIP;
            x.td = f.type;
            return 0;
        }
        uint32_t vm = ST_VM;
        if ((flag & DG_F_ENABLE_VM) == 0 || f.vm == DG_VM_NONE) {
            vm = ST_FIELD;
            unwindPos = out.len;
            lastField = fi;
            out.w8(TY(f.type).ttype);
            out.w16(f.id);
        }
        if (obj0) {
            r = push(J_ELEM | vm, f.type, p);
            if (r) return r;
        } else {
            auto &x = vt[sp - 1];
            x.st = J_ELEM | vm;
            x.td = f.type;
        }
        vt[sp - 1].u = (uint32_t)fi;
        /* the object frame is vt[sp-2] in both cases once the ELEM is on top */
        bm_set_req(vt[sp - 2], sd, k, DG_REQ_OPTIONAL);
        return 0;
    }

    /* j2t_field_vm native/thrift.c:506-666 */
    DGI uint64_t field_vm(int64_t &p, uint32_t fidx)
    {
        const dg_field f = ldrec(&D.F[fidx]);
        uint8_t ft = TY(f.type).ttype;
        if (f.vm <= DG_VM_INLINE_MAX) {
            out.w8(ft);
            out.w16(f.id);
            if (f.vm != DG_VM_JSCONV) return pack(E_UNSUPPORT_VM_TYPE, f.vm, (uint64_t)p);
            uint8_t ch = src.at(p - 1);
            if (ch == '"') {
                if (ft == DG_T_STRING) return j2t_string(p);
                if (src.at(p) == '"') {
                    uint64_t r = write_default_or_empty(f, p);
                    if (r) return r;
                    p += 1;
                    return 0;
                }
            } else {
                if (ch != '-' && (ch < '0' || ch > '9')) return pack(E_INVAL, sx8_64(ch), (uint64_t)p);
                p -= 1;
            }
            int64_t s0 = p;
            vnumber(src, p, jt, ws.dbuf);
            if (jt.vt != V_INTEGER && jt.vt != V_DOUBLE) return pack(E_NUMBER_FMT, (uint64_t)jt.vt, (uint64_t)p);
            bool isint = jt.vt == V_INTEGER;
            switch (ft) {
            case DG_T_STRING:
                out.w32((uint32_t)(p - s0));
                copy_src(s0, p - s0);
                return 0;
            case DG_T_I64: out.w64(isint ? (uint64_t)jt.iv : (uint64_t)cvt64(jt.dv)); break;
            case DG_T_I32: out.w32(isint ? (uint32_t)jt.iv : (uint32_t)cvt32(jt.dv)); break;
            case DG_T_I16:
                out.w16(isint ? (uint16_t)jt.iv : (uint16_t)cvt32(jt.dv));
                /* the reference misses a break here (native/thrift.c:590-603) */
                out.w8(isint ? (uint8_t)jt.iv : (uint8_t)cvt32(jt.dv));
                break;
            case DG_T_BYTE: out.w8(isint ? (uint8_t)jt.iv : (uint8_t)cvt32(jt.dv)); break;
            case DG_T_DOUBLE: out.w64((uint64_t)__double_as_longlong(jt.dv)); break;
            default: return pack(E_UNSUPPORT_THRIFT_TYPE, ft, (uint64_t)p);
            }
            if (ch == '"') {
                if (src.at(p) != '"') return pack(E_INVAL, sx8_64(src.at(p)), (uint64_t)p);
                p += 1;
            }
            return 0;
        }
        /* non-inline value mapping: skip the value, then the Go host's
         * handleValueMapping (conv/j2t/impl_amd64.go:117-155) on its text */
        p -= 1;
        int64_t s0 = p;
        SkipRes sr = skip_one(src, p, skipbits, skipcap);
        p = sr.p;
        if (sr.r == SKIP_DEEP) return pack0(DG_ST_DEEP, 0);
        if (sr.r < 0) return pack((uint32_t)-sr.r, (uint64_t)s0, (uint64_t)p);
        /* agw.body_dynamic on a STRING field: field header, then the raw value
         * text as a binary (thrift/annotation/value_mapping.go:101-106); the
         * host rejects a value that ends the input (impl_amd64.go:132) */
        if (f.vm == DG_VM_BODY_DYNAMIC && ft == DG_T_STRING && p < src.n) {
            out.w8(ft);
            out.w16(f.id);
            out.w32((uint32_t)(p - s0));
            copy_src(s0, p - s0);
            return 0;
        }
        if (take_answer()) return 0; /* the host's answer for this value (dg_cb_entry) */
        if (flag & DG_F_CB_COLLECT) { /* recorded; the machine converts on */
            if (!cb_room(24)) return cb_full(24);
            rec.w64(pack0(E_VM_END, (uint64_t)p));
            rec.w64((uint64_t)s0);
            rec.w64((uint64_t)fidx);
            ncb++;
            return 0;
        }
        /* ERR_VM_END for the host: the value's start and the field, in the slot */
        out.set_len(0);
        out.w64((uint64_t)s0);
        out.w64((uint64_t)fidx);
        return pack0(E_VM_END, (uint64_t)p);
    }

    /* j2t_fsm_exec native/thrift.c:765-1187 */
    DGI uint64_t run(uint32_t root)
    {
        int64_t p = 0;
        bool null_val = false;
        uint64_t unwindPos = 0;
        int32_t lastField = -1;
        sp = 1;
        vt[0].st = J_VAL;
        vt[0].td = root;
        while (sp) {
            if (sp >= MAX_RECURSE) return pack(E_RECURSE_MAX, sp, (uint64_t)p);
            auto &x = vt[sp - 1];
            uint32_t dc = x.td;
            uint32_t st = x.st;
            uint8_t ch;
            PROF(0, ch = advance_ns(src, p));
            switch (st & 0xffff) {
            default:
                sp--;
                break;
            case J_ARR_0:
                if (ch == ']') {
                    out.put32(fbp(x), 0);
                    sp--;
                    continue;
                }
                set_size(x, 0);
                x.st = J_ARR;
                p -= 1;
                {
                    uint64_t r = push(J_VAL, TY(dc).elem, p);
                    if (r) return r;
                }
                continue;
            case J_ARR:
                if (ch == ']' || ch == ',') {
                    if (!null_val) set_size(x, fsize(x) + 1);
                    else null_val = false;
                    if (ch == ']') {
                        out.put32(fbp(x), fsize(x));
                        sp--;
                        continue;
                    }
                    uint64_t r = push(J_VAL, TY(dc).elem, p);
                    if (r) return r;
                    continue;
                }
                return pack(E_INVAL, v2(sx8(ch), J_ARR), (uint64_t)p);
            case J_OBJ_0:
                if (ch == '}') {
                    const dg_type t = TY(dc);
                    if (t.ttype == DG_T_STRUCT) {
                        const dg_struct sd = ldrec(&D.S[t.st]);
                        uint64_t r;
                        PROF(6, r = write_unset_fields(x, sd, p - 1));
                        if (r) return r;
                        if (sd.req_words > 1) reqlen -= sd.req_words;
                        if ((flag & DG_F_ENABLE_HM) && field_cache_len > 0) {
                            uint64_t r2 = hm_end(x, sd, t.st, p);
                            if (r2) return r2;
                        } else {
                            out.w8(0);
                        }
                    } else {
                        out.put32(fbp(x), 0);
                    }
                    sp--;
                    continue;
                }
                if (ch == '"') {
                    x.st = J_OBJ;
                    uint64_t r = j2t_key(p, dc, true, unwindPos, lastField);
                    if (r) return r;
                    continue;
                }
                return pack(E_INVAL, v2(sx8(ch), J_OBJ_0), (uint64_t)p);
            case J_OBJ:
                if (ch == '}') {
                    const dg_type t = TY(dc);
                    if (t.ttype == DG_T_STRUCT) {
                        const dg_struct sd = ldrec(&D.S[t.st]);
                        if (null_val) {
                            null_val = false;
                            bm_set_req(x, sd, (uint32_t)lastField - sd.field_begin, ldrec(&D.F[lastField]).required);
                            out.set_len(unwindPos);
                        }
                        uint64_t r;
                        PROF(6, r = write_unset_fields(x, sd, p - 1));
                        if (r) return r;
                        if (sd.req_words > 1) reqlen -= sd.req_words;
                        if ((flag & DG_F_ENABLE_HM) && field_cache_len > 0) {
                            uint64_t r2 = hm_end(x, sd, t.st, p);
                            if (r2) return r2;
                        } else {
                            out.w8(0);
                        }
                    } else {
                        if (!null_val) set_size(x, fsize(x) + 1);
                        else {
                            null_val = false;
                            out.set_len(unwindPos);
                        }
                        out.put32(fbp(x), fsize(x));
                    }
                    sp--;
                    continue;
                }
                if (ch == ',') {
                    const dg_type t = TY(dc);
                    if (t.ttype == DG_T_MAP) {
                        if (!null_val) set_size(x, fsize(x) + 1);
                        else {
                            null_val = false;
                            out.set_len(unwindPos);
                        }
                    } else if (null_val) {
                        null_val = false;
                        const dg_struct sd = ldrec(&D.S[t.st]);
                        bm_set_req(x, sd, (uint32_t)lastField - sd.field_begin, ldrec(&D.F[lastField]).required);
                        out.set_len(unwindPos);
                    }
                    uint64_t r = push(J_KEY, dc, p);
                    if (r) return r;
                    continue;
                }
                return pack(E_INVAL, v2(sx8(ch), J_OBJ), (uint64_t)p);
            case J_KEY: {
                if (ch != '"') return pack(E_INVAL, v2('"', J_KEY), (uint64_t)p);
                uint64_t r = j2t_key(p, dc, false, unwindPos, lastField);
                if (r) return r;
                continue;
            }
            case J_ELEM:
                if (ch != ':') return pack(E_INVAL, v2(':', J_ELEM), (uint64_t)p);
                x.st = J_VAL | (st & 0xffff0000u);
                continue;
            }
            /* J_VAL, already dropped */
            if (st & ST_SKIP) {
                p -= 1;
                int64_t s0 = p;
                SkipRes sr = skip_one(src, p, skipbits, skipcap);
                p = sr.p;
                if (sr.r == SKIP_DEEP) return pack0(DG_ST_DEEP, 0);
                if (sr.r < 0) return pack((uint32_t)-sr.r, (uint64_t)s0, (uint64_t)p);
                continue;
            }
            if ((flag & DG_F_ENABLE_VM) && (st & ST_VM)) {
                uint64_t r = field_vm(p, (uint32_t)x.u);
                if (r) return r;
                continue;
            }
            const dg_type t = TY(dc);
            switch (ch) {
            case '0': case '1': case '2': case '3': case '4':
            case '5': case '6': case '7': case '8': case '9': case '-': {
                p -= 1;
                uint64_t r;
                PROF(3, r = j2t_number(dc, src, p));
                if (r) return r;
                break;
            }
            case 'n': {
                int64_t s0 = p;
                int64_t r = advance_dword(src, p, 1, p - 1, VS_NULL);
                if (r < 0) return pack((uint32_t)-r, (uint64_t)s0, (uint64_t)p);
                null_val = true;
                break;
            }
            case 't':
            case 'f': {
                int64_t s0 = p;
                int64_t r = ch == 't' ? advance_dword(src, p, 1, p - 1, VS_TRUE) : advance_dword(src, p, 0, p - 1, VS_ALSE);
                if (r < 0) return pack((uint32_t)-r, (uint64_t)s0, (uint64_t)p);
                if (t.ttype != DG_T_BOOL) return pack(E_DISMATCH_TYPE, v2(t.ttype, DG_T_BOOL), (uint64_t)p);
                out.w8(ch == 't' ? 1 : 0);
                break;
            }
            case '[': {
                if (t.ttype != DG_T_LIST && t.ttype != DG_T_SET)
                    return pack(E_DISMATCH_TYPE2, ((uint32_t)t.ttype << 16) | (DG_T_SET << 8) | DG_T_LIST, (uint64_t)p);
                out.w8(TY(t.elem).ttype);
                uint64_t bp = out.alloc(4);
                uint64_t r = push(J_ARR_0, dc, p);
                if (r) return r;
                vt[sp - 1].u = (uint32_t)bp;
                break;
            }
            case '{': {
                if (t.ttype != DG_T_STRUCT && t.ttype != DG_T_MAP)
                    return pack(E_DISMATCH_TYPE2, ((uint32_t)t.ttype << 16) | (DG_T_MAP << 8) | DG_T_STRUCT, (uint64_t)p);
                if (t.ttype == DG_T_STRUCT) {
                    const dg_struct sd = ldrec(&D.S[t.st]);
                    uint64_t r = push(J_OBJ_0, dc, p);
                    if (r) return r;
                    auto &nx = vt[sp - 1];
                    /* bm_malloc_reqs native/thrift.c:232-250 */
                    if (sd.req_words == 1) {
                        nx.u = D.R[sd.req_begin];
                    } else {
                        if (reqlen + sd.req_words > ws.reqcap) return pack0(DG_ST_DEEP, 0);
                        nx.u = reqlen;
                        for (uint32_t w = 0; w < sd.req_words; w++) ws.reqarena[reqlen + w] = D.R[sd.req_begin + w];
                        reqlen += sd.req_words;
                    }
                    if ((flag & DG_F_ENABLE_HM) && (sd.flags & DG_SF_HTTP_MAPPING)) {
                        /* ERR_HM (native/thrift.c:1119-1123) -> handleHttpMappings; pre-split
                         * (DG_F_HM_SPLIT): the host wrote the root's mapped fields, which
                         * reqs.Set(id, Optional) marks as set (conv/j2t/impl.go:284) */
                        if (!(flag & DG_F_HM_SPLIT)) return pack0(E_HM, (uint64_t)(p - 1));
                        uint64_t mask = ~0ull;
                        if (hm_row) {
                            /* the host's handleHttpMappings for this struct (the same bytes for
                             * every instance: they depend on the request and the struct only) */
                            uint32_t slot = 0;
                            for (uint32_t s = 0; s < t.st; s++)
                                if (ldrec(&D.S[s]).flags & DG_SF_HTTP_MAPPING) slot++;
                            const dg_hm_entry e = hm_row[slot];
                            if (e.len == DG_HM_ERR) return pack(DG_ST_HM_ERR, slot, (uint64_t)(p - 1));
                            for (uint32_t b = 0; b < e.len; b++) out.w8(hm_bytes[(uint64_t)e.off + b]);
                            mask = e.mask;
                        } else if (sp != 1) {
                            return pack0(E_HM, (uint64_t)(p - 1)); /* root only: vt[0] */
                        }
                        /* a mapped field the host wrote is reqs.Set(id, Optional) (its JSON key is
                         * skipped); one it did not (ReadHttpValueFallback, not in the request) is
                         * reqs.Set(id, Required): read from the body (impl.go:276-284) */
                        for (uint32_t k = 0; k < sd.n_fields; k++)
                            if (ldrec(&D.F[sd.field_begin + k]).flags & DG_FF_HTTP_MAPPING)
                                bm_set_req(nx, sd, k, k >= 64 || ((mask >> k) & 1) ? DG_REQ_OPTIONAL : DG_REQ_REQUIRED);
                    }
                } else {
                    out.w8(TY(t.key).ttype);
                    out.w8(TY(t.elem).ttype);
                    uint64_t bp = out.alloc(4);
                    uint64_t r = push(J_OBJ_0, dc, p);
                    if (r) return r;
                    vt[sp - 1].u = (uint32_t)bp;
                }
                break;
            }
            case '"': {
                uint64_t r;
                if (t.ttype == DG_T_STRING) {
                    if ((flag & DG_F_NO_BASE64) == 0 && (t.flags & DG_TF_BINARY)) PROF(5, r = j2t_binary(p));
                    else PROF(4, r = j2t_string(p));
                    if (r) return r;
                } else if ((flag & DG_F_ENABLE_I2S) && (t.ttype == DG_T_I64 || t.ttype == DG_T_I32 || t.ttype == DG_T_I16 ||
                                                         t.ttype == DG_T_BYTE || t.ttype == DG_T_DOUBLE)) {
                    if (src.at(p) == '"') {
                        r = write_empty(dc, p);
                        if (r) return r;
                    } else {
                        r = j2t_number(dc, src, p);
                        if (r) return r;
                        if (p >= src.n) return pack(E_EOF, 0, (uint64_t)p);
                        if (src.at(p) != '"') return pack(E_INVAL, v2(sx8(src.at(p)), J_VAL), (uint64_t)p);
                    }
                    p += 1;
                } else {
                    return pack(E_DISMATCH_TYPE, v2(t.ttype, DG_T_STRING), (uint64_t)p);
                }
                break;
            }
            case 0:
                return pack(E_EOF, 0, (uint64_t)p);
            default:
                return pack(E_INVAL, v2(sx8(ch), J_VAL), (uint64_t)p);
            }
        }
        return 0;
    }
};

/* BinaryConv.do prelude/epilogue (conv/j2t/impl.go:38-91, conv.go:70-77) around
 * the FSM for message i read through `src`. Returns the status; writes olen. */
template <class S, class FP, class DV>
DGI uint64_t convert_one(const Params &P, const DV &dv, uint64_t i, const S &src, FStack<FP> frames, uint32_t depth,
                         gu64 *skipbits, uint32_t skipcap, const Workspace &ws, uint32_t &olen)
{
    uint64_t oa = P.out_off[i], ob = P.out_off[i + 1];
    Machine<S, FP, DV> m;
    m.D = dv;
    m.src = src;
    m.out.init(P.out + oa, ob - oa);
    m.flag = P.flag;
    m.vt = frames;
    m.cap = depth;
    m.skipbits = skipbits;
    m.skipcap = skipcap;
    m.ws = ws;
    m.reqlen = 0;
    m.field_cache_len = 0;
    m.hm_row = P.hm_tab ? P.hm_tab + i * P.n_hm : nullptr;
    m.hm_bytes = P.hm_bytes;
    m.ans_row = P.ans_tab ? P.ans_tab + i : nullptr;
    m.ans_seen = 0;
    m.ans_at = m.ans_row ? m.ans_row->off : 0;
    m.ncb = 0;
    m.cb_need = 0;
    uint64_t r;
    if (m.src.n == 0) { /* empty body -> STOP (conv/j2t/impl.go:52-82) */
        m.out.w8(0);
        r = 0;
    } else if (dv.T[P.root].ttype == DG_T_STRING && m.src.raw(0) != '"') {
        /* unquoted STRING root: json.EncodeString then unquote == identity
         * (conv/j2t/impl.go:85-88; native/parsing.c:28-62 escapes only '"',
         * '\\' and control bytes, all restored by unquote) */
        m.out.w32((uint32_t)m.src.n);
        m.copy_src(0, m.src.n);
        r = 0;
    } else {
#ifdef DG_PROFILE
        uint64_t t0 = __builtin_amdgcn_s_memtime();
        r = m.run(P.root);
        m.prof[7] = __builtin_amdgcn_s_memtime() - t0;
        for (int k = 0; k < 16; k++) *(uint64_t *)(P.out + oa + 8 * k) = m.prof[k];
        olen = 128;
        return 0;
#else
        r = m.run(P.root);
#endif
    }
    if (m.ncb && (uint8_t)r != DG_ST_DEEP) {
        /* DG_F_CB_COLLECT: the recorded callbacks, whatever came after them
         * (an error there is met again once the host has served them) */
        m.rec.finish();
        olen = (uint32_t)m.rec.len;
        return pack(DG_ST_CB_LIST, m.ncb < 0xFFFFFFu ? m.ncb : 0xFFFFFFu, 0);
    }
    if (m.cb_need && (uint8_t)r == DG_ST_OUT_OVERFLOW) { /* cb_full: no room for the first record */
        olen = m.cb_need;
        return r;
    }
    /* HM_END: the host completes the output; VM_END / HM_END_AT: the callback's record */
    const bool keep = r == 0 || (uint8_t)r == DG_ST_HM_END || (uint8_t)r == E_VM_END || (uint8_t)r == DG_ST_HM_END_AT;
    if (keep) m.out.finish();
    if (keep && m.out.len > m.out.cap) {
        /* the bytes needed travel in out_len (32 bits); the 24-bit value field
         * of the status word only carries them saturated */
        const uint64_t need = m.out.len;
        olen = need > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)need;
        return pack(DG_ST_OUT_OVERFLOW, need > 0xFFFFFFull ? 0xFFFFFFull : need, 0);
    }
    olen = keep ? (uint32_t)m.out.len : 0;
    return r;
}

DGI Workspace lane_ws(const Params &P, uint64_t lane)
{
    Workspace w;
    gu8 *base = (gu8 *)(void *)(P.ws + lane * P.ws_stride);
    w.dbuf = base;
    w.keybuf = base + DCAP;
    w.keycap = P.keycap;
    w.reqarena = (gu64 *)(base + DCAP + P.keycap);
    w.reqcap = P.reqcap;
    return w;
}

DGI SrcT<glb_u64> global_src(const Params &P, uint64_t i)
{
    uint64_t a = P.in_off[i], b = P.in_off[i + 1];
    SrcT<glb_u64> s;
    s.init((glb_u64 *)(const void *)(P.json + (a & ~7ull)), (int64_t)(a & 7), (int64_t)(b - a));
    return s;
}

DGI void finish(const Params &P, uint64_t i, uint64_t r, uint32_t olen)
{
    P.ret[i] = r;
    P.out_len[i] = olen;
    if ((uint8_t)r == DG_ST_OUT_OVERFLOW && P.pending) atomicAdd(P.pending, 1u);
}

/* Deep pass: messages that outgrew the fast stack, redone by the LAST block
 * to finish, with a MAX_RECURSE stack in device workspace. The list and its
 * counter are published with agent-scope atomics behind each producer
 * block's release fence; the last block acquires once. */
template <class DV>
DGI void deep_pass(const Params &P, const DV &dv, uint32_t *done, uint32_t nblocks)
{
    __shared__ uint32_t s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence(); /* release this block's results */
        uint32_t prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == nblocks - 1;
        if (s_last) __threadfence(); /* acquire every other block's */
    }
    __syncthreads();
    if (!s_last) return;
    uint32_t cnt = __hip_atomic_load(P.deep_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0 && cnt) atomicAdd(&P.stats[1], (unsigned long long)cnt);
    uint64_t lane = threadIdx.x;
    Workspace ws = lane_ws(P, lane);
    FStack<Frame *> frames{(Frame *)(P.ws + lane * P.ws_stride + DCAP + P.keycap + (uint64_t)P.reqcap * 8), 1};
    gu64 *skipbits = (gu64 *)(void *)(frames.base + MAX_RECURSE);
    for (uint64_t k = lane; k < cnt; k += blockDim.x) {
        uint64_t i = __hip_atomic_load(&P.deep_list[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t olen;
        uint64_t r = convert_one(P, dv, i, global_src(P, i), frames, MAX_RECURSE, skipbits, MAX_RECURSE, ws, olen);
        finish(P, i, r, olen);
    }
    __syncthreads();
    if (threadIdx.x == 0) { /* self-reset for the next launch on this context */
        if (P.list_count) __hip_atomic_store(P.list_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (P.reset2) {
            __hip_atomic_store(P.reset2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(P.reset2 + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(P.reset2 + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __hip_atomic_store(P.deep_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

constexpr uint32_t LANE_BLOCK = 256;
constexpr uint32_t STAGE_BYTES = 64 * 1024; /* LDS staging of the block's JSON bytes */
constexpr uint32_t LDS_DEPTH = 8;           /* frames per lane in LDS: 8 x 256 x 16 B = 32 KiB */
constexpr uint32_t DESC_LDS_BYTES = 48 * 1024; /* descriptors up to this size are copied to LDS */

struct DeepParams {
    uint8_t *ws;
    uint64_t ws_stride;
    uint32_t keycap, reqcap;
    uint32_t *done;
    const uint8_t *blob; /* descriptor blob (device) */
    dg_desc_hdr hdr;
};

/* One lane per message. The block's messages are contiguous in the arena:
 * when their span fits, it is staged into LDS with coalesced 16-byte loads
 * and every lane parses from LDS through its 8-byte register window. With
 * LDS_DESC the descriptor tables are copied to LDS too. */
template <bool LDS_DESC>
__global__ __launch_bounds__(LANE_BLOCK) __attribute__((amdgpu_waves_per_eu(1, 1))) void j2t_lane_kernel(Params P, DeepParams DP)
{
    __shared__ __attribute__((aligned(16))) uint64_t stage[STAGE_BYTES / 8 + 2]; /* +16 B: word reads past the end */
    __shared__ __attribute__((aligned(16))) Frame lframes[LDS_DEPTH * LANE_BLOCK];
    __shared__ __attribute__((aligned(16))) uint64_t ldesc[LDS_DESC ? DESC_LDS_BYTES / 8 : 2];
    __shared__ uint64_t s_p10u[20];
    __shared__ double s_p10d[23];
    __shared__ uint32_t s_nbail;
    __shared__ uint16_t s_bail[LANE_BLOCK];
    __shared__ uint32_t s_cnt;
    if (P.list) {
        /* list mode: the messages the wave kernel bailed on, on the exact
         * machine only, grid-strided over the device-side count */
        if (threadIdx.x == 0) {
            s_cnt = __hip_atomic_load(P.list_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (blockIdx.x == 0 && s_cnt) atomicAdd(&P.stats[0], (unsigned long long)s_cnt);
        }
        __syncthreads();
        if (s_cnt == 0) {
            /* nothing declined (the common case): no descriptor copy, no deep
             * pass, no fences; every block saw the same zero count (nothing
             * writes it during this launch), block 0 resets the counters the
             * earlier launches of the pipeline left (list count is 0, the deep
             * count and `done` are only ever raised by list work) */
            if (blockIdx.x == 0 && threadIdx.x == 0 && P.reset2) {
                __hip_atomic_store(P.reset2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(P.reset2 + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(P.reset2 + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
        }
        if constexpr (LDS_DESC) {
            const uint4 *g = (const uint4 *)DP.blob;
            uint4 *l = (uint4 *)ldesc;
            for (uint32_t k = threadIdx.x; k < (DP.hdr.total_len + 15) / 16; k += LANE_BLOCK) l[k] = g[k];
        }
        if (P.fast) {
            if (threadIdx.x < 20) {
                uint64_t v = 1;
                for (uint32_t k = 0; k < threadIdx.x; k++) v *= 10;
                s_p10u[threadIdx.x] = v;
            }
            if (threadIdx.x < 23) s_p10d[threadIdx.x] = P10[threadIdx.x];
        }
        __syncthreads();
        auto dvl = [&]() {
            if constexpr (LDS_DESC) return desc_view<3>((const __attribute__((address_space(3))) uint8_t *)(void *)ldesc, DP.hdr);
            else return desc_view<1>((const __attribute__((address_space(1))) uint8_t *)(const void *)DP.blob, DP.hdr);
        }();
        const uint32_t cnt = s_cnt;
        for (uint64_t k = (uint64_t)blockIdx.x * LANE_BLOCK + threadIdx.x; k < cnt; k += (uint64_t)gridDim.x * LANE_BLOCK) {
            uint64_t j = P.list[k];
            if (P.fast) {
                /* the small kernel's declines: the full fast path first (unknown-field
                 * skips, numeric map keys, default writes), then the exact machine */
                Out out;
                out.init(P.out + P.out_off[j], P.out_off[j + 1] - P.out_off[j]);
                FastTabs tb{(const __attribute__((address_space(3))) uint64_t *)(void *)s_p10u,
                            (lds_f64 *)(void *)s_p10d};
                SrcT<glb_u64> s = global_src(P, j);
                if (fast_convert(dvl, s, out, P.flag, P.root, (LFFrame *)(void *)&lframes[threadIdx.x], LANE_BLOCK, tb)) {
                    finish(P, j, 0, (uint32_t)out.len);
                    continue;
                }
            }
            FStack<LFrame *> frames{(LFrame *)(void *)&lframes[threadIdx.x], LANE_BLOCK};
            Workspace ws = lane_ws(P, j);
            uint32_t olen;
            uint64_t r = convert_one(P, dvl, j, global_src(P, j), frames, LDS_DEPTH, nullptr, 64, ws, olen);
            finish(P, j, r, olen);
            if ((uint8_t)r == DG_ST_DEEP) {
                uint32_t q = __hip_atomic_fetch_add(P.deep_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&P.deep_list[q], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        Params Q = P;
        Q.ws = DP.ws;
        Q.ws_stride = DP.ws_stride;
        Q.keycap = DP.keycap;
        Q.reqcap = DP.reqcap;
        deep_pass(Q, dvl, DP.done, gridDim.x);
        return;
    }
    uint64_t b0 = (uint64_t)blockIdx.x * LANE_BLOCK;
    uint64_t b1 = b0 + LANE_BLOCK < P.n ? b0 + LANE_BLOCK : P.n;
    uint64_t lo = P.in_off[b0], hi = P.in_off[b1];
    uint64_t base = lo & ~15ull;
    uint64_t words = (hi - base + 15) >> 4;
    bool staged = words * 16 <= STAGE_BYTES;
    if (staged) {
        const uint4 *g = (const uint4 *)(P.json + base);
        uint4 *l = (uint4 *)stage;
        for (uint64_t k = threadIdx.x; k < words; k += LANE_BLOCK) l[k] = g[k];
    }
    if constexpr (LDS_DESC) {
        const uint4 *g = (const uint4 *)DP.blob;
        uint4 *l = (uint4 *)ldesc;
        for (uint32_t k = threadIdx.x; k < (DP.hdr.total_len + 15) / 16; k += LANE_BLOCK) l[k] = g[k];
    }
    if (threadIdx.x < 20) {
        uint64_t v = 1;
        for (uint32_t k = 0; k < threadIdx.x; k++) v *= 10;
        s_p10u[threadIdx.x] = v;
    }
    if (threadIdx.x < 23) s_p10d[threadIdx.x] = P10[threadIdx.x];
    if (threadIdx.x == 0) s_nbail = 0;
    __syncthreads();
    auto dv = [&]() {
        if constexpr (LDS_DESC) return desc_view<3>((const __attribute__((address_space(3))) uint8_t *)(void *)ldesc, DP.hdr);
        else return desc_view<1>((const __attribute__((address_space(1))) uint8_t *)(const void *)DP.blob, DP.hdr);
    }();
    uint64_t i = b0 + threadIdx.x;
    /* phase 1: the fast path on this lane's own message */
    if (i < b1) {
        bool done = false;
        const uint64_t len_i = P.in_off[i + 1] - P.in_off[i];
        const bool big = P.big_list && len_i > P.big_max;
        list_big_w(P, big, i, len_i); /* a large message: the wave kernel (one wavefront per message) takes it */
        if (big) {
            done = true;
        } else if (P.fast) {
            uint64_t oa = P.out_off[i], ob = P.out_off[i + 1];
            Out out;
            out.init(P.out + oa, ob - oa);
            FastTabs tb{(const __attribute__((address_space(3))) uint64_t *)(void *)s_p10u,
                        (lds_f64 *)(void *)s_p10d};
            LFFrame *ff = (LFFrame *)(void *)&lframes[threadIdx.x];
            if (staged) {
                uint64_t a = P.in_off[i], b = P.in_off[i + 1];
                SrcT<lds_u64> s;
                s.init((lds_u64 *)(void *)stage, (int64_t)(a - base), (int64_t)(b - a));
                done = fast_convert(dv, s, out, P.flag, P.root, ff, LANE_BLOCK, tb);
            } else {
                SrcT<glb_u64> s = global_src(P, i);
                done = fast_convert(dv, s, out, P.flag, P.root, ff, LANE_BLOCK, tb);
            }
            if (done) finish(P, i, 0, (uint32_t)out.len);
        }
        if (!done) {
            uint32_t k = atomicAdd(&s_nbail, 1u);
            s_bail[k] = (uint16_t)threadIdx.x;
        }
    }
    __syncthreads();
    /* phase 2: the exact machine on the block's bailed messages, compacted
     * onto the first lanes */
    uint32_t nbail = s_nbail;
    if (threadIdx.x == 0 && nbail && P.fast) atomicAdd(&P.stats[0], (unsigned long long)nbail);
    if (threadIdx.x < nbail) {
        uint64_t j = b0 + s_bail[threadIdx.x];
        FStack<LFrame *> frames{(LFrame *)(void *)&lframes[threadIdx.x], LANE_BLOCK};
        gu64 *skipbits = nullptr; /* 64 skip levels in a register */
        Workspace ws = lane_ws(P, j);
        uint32_t olen;
        uint64_t r;
        if (staged) {
            uint64_t a = P.in_off[j], b = P.in_off[j + 1];
            SrcT<lds_u64> s;
            s.init((lds_u64 *)(void *)stage, (int64_t)(a - base), (int64_t)(b - a));
            r = convert_one(P, dv, j, s, frames, LDS_DEPTH, skipbits, 64, ws, olen);
        } else {
            r = convert_one(P, dv, j, global_src(P, j), frames, LDS_DEPTH, skipbits, 64, ws, olen);
        }
        finish(P, j, r, olen);
        if ((uint8_t)r == DG_ST_DEEP) {
            uint32_t k = __hip_atomic_fetch_add(P.deep_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&P.deep_list[k], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    Params Q = P;
    Q.ws = DP.ws;
    Q.ws_stride = DP.ws_stride;
    Q.keycap = DP.keycap;
    Q.reqcap = DP.reqcap;
    deep_pass(Q, dv, DP.done, gridDim.x);
}

/* launchers, one per translation unit */
void launch_lane_kernel_lds(dim3 grid, hipStream_t s, const Params &P, const DeepParams &DP);
void launch_lane_kernel_glb(dim3 grid, hipStream_t s, const Params &P, const DeepParams &DP);

}  // namespace dg
