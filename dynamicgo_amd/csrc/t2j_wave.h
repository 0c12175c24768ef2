/*
 * t2j_wave.h — the reverse path (conv/t2j, Thrift binary -> JSON) with one
 * wavefront per message, for messages longer than T2W_MIN bytes.
 *
 * Why: the lane-per-message kernel (t2j_device.h) walks 16-64 messages per
 * wave, and every lane is at a different kind of field at any moment, so the
 * wave executes the union of all their paths (t2j-c3: 3.7 ms, 0.008 of HBM
 * roofline). Here a message is split into tokens and the 64 lanes work on
 * them together:
 *
 *  1. Walk (lane 0): Thrift is length-prefixed, so the structure is found by
 *     reading only headers, lengths and sizes -- never a string body. Lane 0
 *     walks the message like doRecurse (conv/t2j/impl.go:189-393) and emits
 *     one token per JSON value: its separator and key (struct field: the
 *     pre-encoded "alias": of the side table; map entry: the key's Thrift
 *     position), its type and the Thrift position of its value; containers
 *     give an open and a close token. 64 tokens make a page.
 *  2. Page (all lanes, one token each): the JSON length of every token
 *     (numbers formatted into registers: i64toa, Schubfach f64toa; string
 *     escapes counted by 8-byte scan tasks spread over the wave; base64 4/3),
 *     one prefix sum, then every lane writes its bytes at its offset
 *     (byte-exact at shared words). Long string and base64 bodies become
 *     chunk tasks over the 64 lanes.
 *
 * The same bytes as t2j_convert, byte for byte. Anything outside the common
 * error-free shape BAILS to the lane kernel, which converts the message from
 * scratch with the exact code and reports errors: truncation, invalid or
 * mismatched wire types, unknown fields, value mapping, NaN/Inf without
 * EncodeNullJSONForInfOrNan, unset fields that would be written or are
 * REQUIRED, structs of more than 64 fields, nesting beyond T2W_MAXD, a
 * non-struct root, slot overflow.
 */
#pragma once
#include "t2j_device.h"
#include "j2t_wave.h"

namespace dg {

constexpr uint32_t T2W_MSG = 2048;  /* messages up to this (minus 16) are staged in LDS */
constexpr uint32_t T2W_MAXD = 16;   /* nesting the walker handles */
constexpr uint32_t T2W_MIN = 512;   /* messages longer than this take the wave kernel */
constexpr uint32_t T2W_CH = 16;     /* string body bytes per copy task */
constexpr uint32_t T2W_B64 = 24;    /* base64 input bytes per task (32 characters) */

enum : uint32_t { TK_VAL = 0, TK_OPEN_OBJ = 1, TK_OPEN_ARR = 2, TK_CLOSE_OBJ = 3, TK_CLOSE_ARR = 4 };
enum : uint32_t { TKF_COMMA = 8, TKF_KEYF = 16, TKF_KEYM = 32 };

/* one open container. The walker keeps the innermost one in registers and
 * the ones around it in LDS. */
struct T2WFrame {
    uint32_t kind; /* TF_STRUCT / TF_LIST / TF_MAP */
    uint32_t n;    /* list/map: elements; struct: predicted next field index */
    uint32_t i;    /* list/map: elements done; struct: a field was written */
    uint32_t fb;   /* struct: first field (global index) */
    uint32_t nf;   /* struct: fields */
    uint32_t st;   /* struct: struct index */
    uint32_t etd;  /* list/map: element / value type index */
    uint32_t ett;  /* list/map: its ttype | type flags << 8; map: | key ttype << 16 */
    uint64_t u;    /* struct: requires bits still unset */
};

struct T2WLds {
    uint8_t kind[64];   /* TK_* | TKF_* */
    uint8_t kt[64];     /* map entries: the key's Thrift type */
    uint32_t pos[64];   /* Thrift position of the value */
    uint32_t aux[64];   /* TKF_KEYF: field index; TKF_KEYM: Thrift position of the key */
    uint32_t td[64];    /* value type index */
    uint32_t xk[64];    /* escape bytes the map key string adds (scan tasks) */
    uint32_t xv[64];    /* ... the value string adds */
    uint32_t cinc[64];  /* tasks: inclusive prefix of per-lane task counts */
    uint32_t ck[64];    /* scan: chunks of the key string (the rest are the value's) */
    uint32_t cs[64];    /* scan: key string start; write: body source start */
    uint32_t cn[64];    /* scan: key string length; write: body length | 1 << 31 base64 */
    uint32_t cvs[64];   /* scan: value string start; write: body output offset in the slot */
    uint32_t cvn[64];   /* scan: value string length */
    T2WFrame fr[T2W_MAXD];
};

/* up to 32 bytes of output in registers (numbers, literals) */
struct RegOut {
    uint64_t w0, w1, w2, w3;
    uint32_t len;
    DGI void init()
    {
        w0 = w1 = w2 = w3 = 0;
        len = 0;
    }
    DGI void wle(uint64_t v, uint32_t n)
    {
        if (n < 8) v &= (1ull << (n << 3)) - 1;
        const uint32_t k = len >> 3, sh = (len & 7) << 3;
        const uint64_t lo = v << sh, hi = sh ? v >> (64 - sh) : 0;
        if (k == 0) { w0 |= lo; w1 |= hi; }
        else if (k == 1) { w1 |= lo; w2 |= hi; }
        else if (k == 2) { w2 |= lo; w3 |= hi; }
        else w3 |= lo;
        len += n;
    }
    DGI void w8(uint8_t c) { wle(c, 1); }
    template <class O>
    DGI void flush(O &o) const
    {
        uint32_t n = len;
        if (n) o.wle(w0, n < 8 ? n : 8);
        if (n > 8) o.wle(w1, n - 8 < 8 ? n - 8 : 8);
        if (n > 16) o.wle(w2, n - 16 < 8 ? n - 16 : 8);
        if (n > 24) o.wle(w3, n - 24);
    }
};

/* extra bytes the quote of 8 source bytes adds (native/parsing.c:28-63):
 * '"' '\\' \t \n \r one each, other bytes < 0x20 five each */
DGI uint32_t quote_extra(uint64_t w, uint32_t nb)
{
    const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    const uint32_t cl = ~((lo & 0x7F7F7F7Fu) + 0x60606060u) & ~lo & 0x80808080u;
    const uint32_t ch = ~((hi & 0x7F7F7F7Fu) + 0x60606060u) & ~hi & 0x80808080u;
    const uint64_t ctl = (uint64_t)cl | ((uint64_t)ch << 32);
    uint64_t one = eqbytes(w, '"') | eqbytes(w, '\\') | eqbytes(w, '\t') | eqbytes(w, '\n') | eqbytes(w, '\r');
    uint64_t five = ctl & ~one;
    if (nb < 8) {
        const uint64_t m = (1ull << (nb << 3)) - 1;
        one &= m;
        five &= m;
    }
    return (uint32_t)__builtin_popcountll(one) + 5u * (uint32_t)__builtin_popcountll(five);
}

/* big-endian k-byte read at byte i of a message view */
template <class S>
DGI uint64_t be_at(S &src, int64_t i, uint32_t k)
{
    return __builtin_bswap64(src.get8(i)) >> ((8 - k) << 3);
}

/* HandleRequires (thrift/utils.go:149-176) would write nothing and report no
 * error for these unset fields */
template <class DV>
DGI bool unsets_silent(const DV &D, const dg_struct &sd, uint64_t bits, uint64_t opts)
{
    while (bits) {
        const uint32_t k = (uint32_t)__builtin_ctzll(bits);
        bits &= bits - 1;
        const dg_field fd = ldrec(&D.F[sd.field_begin + k]);
        if (fd.required == DG_REQ_REQUIRED) return false;
        if (fd.required == DG_REQ_DEFAULT && (opts & DG_T2J_WRITE_DEFAULT)) return false;
        if (fd.required == DG_REQ_OPTIONAL && ((opts & DG_T2J_WRITE_OPTIONAL) || fd.dflt_len != DG_NONE)) return false;
    }
    return true;
}

/* per field, packed in LDS by the kernel: id | ttype << 16 | (type flags |
 * 0x80 when it has a value mapping) << 24 | type index << 32 */
DGI uint32_t fx_id(uint64_t v) { return (uint32_t)(v & 0xFFFF); }
DGI uint32_t fx_tt(uint64_t v) { return (uint32_t)(v >> 16) & 0xFF; }
DGI uint32_t fx_fl(uint64_t v) { return (uint32_t)(v >> 24) & 0xFF; }
DGI uint32_t fx_td(uint64_t v) { return (uint32_t)(v >> 32); }
constexpr uint32_t T2W_FX = 1024; /* fields the LDS table holds (descriptors with more take the lane kernel) */

/* the walker's next tokens, up to 64 (lane 0): returns the count, or -1 to
 * bail; `done` when the root struct closed. State across pages: p, the
 * frames (sp of them, the innermost in `cur`), `started`. */
template <class S, class DV>
DGI int32_t t2w_walk(const DV &D, const __attribute__((address_space(3))) uint64_t *fx, S &src, int64_t &p,
                     uint32_t &sp, T2WFrame &cur, T2WLds &L, uint64_t opts, bool &done, bool &started, uint32_t root)
{
    const int64_t n = src.n;
    uint32_t nt = 0;
    auto emit = [&](uint32_t kind, uint32_t pos, uint32_t aux, uint32_t td, uint32_t kt) {
        L.kind[nt] = (uint8_t)kind;
        L.kt[nt] = (uint8_t)kt;
        L.pos[nt] = pos;
        L.aux[nt] = aux;
        L.td[nt] = td;
        nt++;
    };
    /* a value of type td (ttype tt) at p: scalars and strings become one
     * token (p moves past them), containers an open token and a frame */
    auto value = [&](uint32_t td, uint32_t tt, uint32_t flags, uint32_t aux, uint32_t kt) -> bool {
        const uint32_t fs = num_bytes((uint8_t)tt) ? num_bytes((uint8_t)tt) : tt == DG_T_BOOL ? 1u : 0u;
        if (fs) {
            if (p + fs > n) return false;
            emit(TK_VAL | flags, (uint32_t)p, aux, td, kt);
            p += fs;
            return true;
        }
        if (tt == DG_T_STRING) {
            if (p + 4 > n) return false;
            const int64_t sz = (int32_t)be_at(src, p, 4);
            if (sz < 0 || p + 4 + sz > n) return false;
            emit(TK_VAL | flags, (uint32_t)p, aux, td, kt);
            p += 4 + sz;
            return true;
        }
        if (sp >= T2W_MAXD) return false;
        const dg_type t = ldrec(&D.T[td]);
        T2WFrame f;
        f.i = 0;
        f.u = 0;
        f.fb = f.nf = f.st = 0;
        f.etd = f.ett = 0;
        if (tt == DG_T_STRUCT) {
            const dg_struct sd = ldrec(&D.S[t.st]);
            if (sd.req_words != 1) return false;
            f.kind = TF_STRUCT;
            f.n = 0;
            f.fb = sd.field_begin;
            f.nf = sd.n_fields;
            f.st = t.st;
            f.u = D.R[sd.req_begin];
            emit(TK_OPEN_OBJ | flags, 0, aux, td, kt);
        } else if (tt == DG_T_LIST || tt == DG_T_SET) {
            if (p + 5 > n) return false;
            const uint64_t w = __builtin_bswap64(src.get8(p)); /* et | count (big-endian) */
            const uint8_t et = (uint8_t)(w >> 56);
            const int64_t cnt = (int32_t)(uint32_t)(w >> 24);
            const dg_type e = ldrec(&D.T[t.elem]);
            if (cnt < 0 || et != e.ttype) return false;
            p += 5;
            f.kind = TF_LIST;
            f.n = (uint32_t)cnt;
            f.etd = t.elem;
            f.ett = e.ttype | ((uint32_t)e.flags << 8);
            emit(TK_OPEN_ARR | flags, 0, aux, td, kt);
        } else if (tt == DG_T_MAP) {
            if (p + 6 > n) return false;
            const uint64_t w = __builtin_bswap64(src.get8(p)); /* kt | vt | count */
            const uint8_t k = (uint8_t)(w >> 56), v = (uint8_t)(w >> 48);
            const int64_t cnt = (int32_t)(uint32_t)(w >> 16);
            const dg_type kd = ldrec(&D.T[t.key]), vd = ldrec(&D.T[t.elem]);
            if (cnt < 0 || k != kd.ttype || v != vd.ttype) return false;
            if (!(k == DG_T_STRING || num_bytes(k)) || k == DG_T_DOUBLE) return false; /* buildinTypeToKey's */
            p += 6;
            f.kind = TF_MAP;
            f.n = (uint32_t)cnt;
            f.etd = t.elem;
            f.ett = vd.ttype | ((uint32_t)vd.flags << 8) | ((uint32_t)k << 16);
            emit(TK_OPEN_OBJ | flags, 0, aux, td, kt);
        } else {
            return false;
        }
        if (sp) L.fr[sp - 1] = cur;
        cur = f;
        sp++;
        return true;
    };
    auto pop = [&]() {
        sp--;
        if (sp) cur = L.fr[sp - 1];
    };
    if (!started) { /* the root: a struct (other roots take the lane kernel) */
        started = true;
        if (ldrec(&D.T[root]).ttype != DG_T_STRUCT || !value(root, DG_T_STRUCT, 0, 0, 0)) return -1;
    }
    while (nt < 64) {
        if (sp == 0) {
            done = true;
            break;
        }
        if (cur.kind == TF_STRUCT) {
            if (p + 1 > n) return -1;
            const uint64_t w = src.get8(p); /* type, id (big-endian) */
            const uint64_t h = cur.n < cur.nf ? fx[cur.fb + cur.n] : 0ull; /* the predicted field */
            const uint8_t t = (uint8_t)w;
            if (t == 0) { /* STOP: unset fields must write nothing */
                if (cur.u && !unsets_silent(D, ldrec(&D.S[cur.st]), cur.u, opts)) return -1;
                p += 1;
                emit(TK_CLOSE_OBJ, 0, 0, 0, 0);
                pop();
                continue;
            }
            if (p + 3 > n) return -1;
            const uint32_t id = (uint32_t)(((w >> 8) & 0xFF) << 8 | ((w >> 16) & 0xFF));
            uint32_t k = cur.n;
            uint64_t v = h;
            if (cur.n >= cur.nf || fx_id(h) != id) { /* fields are sorted by id */
                uint32_t lo = 0, hi = cur.nf;
                k = 0xFFFFFFFFu;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    const uint64_t x = fx[cur.fb + mid];
                    if (fx_id(x) == id) {
                        k = mid;
                        v = x;
                        break;
                    }
                    if (fx_id(x) < id) lo = mid + 1;
                    else hi = mid;
                }
                if (k == 0xFFFFFFFFu) return -1; /* unknown field (skip or error): the lane kernel */
            }
            if (fx_tt(v) != t) return -1;
            if ((opts & DG_T2J_ENABLE_VM) && (fx_fl(v) & 0x80)) return -1;
            cur.u &= ~(1ull << k);
            cur.n = k + 1;
            const uint32_t comma = cur.i ? TKF_COMMA : 0u;
            cur.i = 1;
            p += 3;
            if (!value(fx_td(v), t, comma | TKF_KEYF, cur.fb + k, 0)) return -1;
        } else if (cur.kind == TF_LIST) {
            if (cur.i == cur.n) {
                emit(TK_CLOSE_ARR, 0, 0, 0, 0);
                pop();
                continue;
            }
            const uint32_t comma = cur.i ? TKF_COMMA : 0u;
            cur.i++;
            if (!value(cur.etd, cur.ett & 0xFF, comma, 0, 0)) return -1;
        } else {
            if (cur.i == cur.n) {
                emit(TK_CLOSE_OBJ, 0, 0, 0, 0);
                pop();
                continue;
            }
            const uint32_t comma = cur.i ? TKF_COMMA : 0u;
            cur.i++;
            const uint8_t kt = (uint8_t)(cur.ett >> 16);
            const int64_t kp = p;
            if (kt == DG_T_STRING) {
                if (p + 4 > n) return -1;
                const int64_t sz = (int32_t)be_at(src, p, 4);
                if (sz < 0 || p + 4 + sz > n) return -1;
                p += 4 + sz;
            } else {
                if (p + num_bytes(kt) > n) return -1;
                p += num_bytes(kt);
            }
            if (!value(cur.etd, cur.ett & 0xFF, comma | TKF_KEYM, (uint32_t)kp, kt)) return -1;
        }
    }
    return (int32_t)nt;
}

/* the JSON of a number/bool token, into registers; false: bail */
template <class S>
DGI bool t2w_scalar(S &src, int64_t p, uint8_t tt, uint64_t opts, RegOut &r)
{
    switch (tt) {
    case DG_T_BOOL:
        if (be_at(src, p, 1) == 1) r.wle('t' | ('r' << 8) | ('u' << 16) | ('e' << 24), 4);
        else r.wle('f' | ('a' << 8) | ('l' << 16) | ('s' << 24) | (0x65ull << 32), 5);
        return true;
    case DG_T_BYTE: {
        const uint8_t v = (uint8_t)be_at(src, p, 1);
        emit_i64(r, (opts & DG_T2J_BYTE_AS_UINT8) ? (int64_t)v : (int64_t)(int8_t)v);
        return true;
    }
    case DG_T_I16: emit_i64(r, (int16_t)be_at(src, p, 2)); return true;
    case DG_T_I32: emit_i64(r, (int32_t)be_at(src, p, 4)); return true;
    case DG_T_I64: {
        const int64_t v = (int64_t)be_at(src, p, 8);
        if (opts & DG_T2J_INT64_AS_STRING) r.w8('"');
        emit_i64(r, v);
        if (opts & DG_T2J_INT64_AS_STRING) r.w8('"');
        return true;
    }
    case DG_T_DOUBLE: {
        const uint64_t u = be_at(src, p, 8);
        if (((u >> 52) & 0x7FF) == 0x7FF) {
            if (!(opts & DG_T2J_NULL_FOR_NAN_INF)) return false; /* the error: the lane kernel reports it */
            r.wle('n' | ('u' << 8) | ('l' << 16) | ('l' << 24), 4);
            return true;
        }
        emit_f64(r, __longlong_as_double((long long)u));
        return true;
    }
    }
    return false;
}

/* a map key that is a number: its digits in registers (buildinTypeToKey) */
template <class S>
DGI void t2w_numkey(S &src, int64_t p, uint8_t kt, uint64_t opts, RegOut &r)
{
    switch (kt) {
    case DG_T_BYTE: {
        const uint8_t v = (uint8_t)be_at(src, p, 1);
        emit_i64(r, (opts & DG_T2J_BYTE_AS_UINT8) ? (int64_t)v : (int64_t)(int8_t)v);
        break;
    }
    case DG_T_I16: emit_i64(r, (int16_t)be_at(src, p, 2)); break;
    case DG_T_I32: emit_i64(r, (int32_t)be_at(src, p, 4)); break;
    default: emit_i64(r, (int64_t)be_at(src, p, 8)); break;
    }
}

/* one message (a wave): false = bail */
template <class S, class DV>
DGI bool t2w_run(const T2JParams &P, const DV &D, const __attribute__((address_space(3))) uint64_t *fx,
                 const T2JSide &X, uint64_t m, T2WLds &L, S src, uint32_t lane)
{
    const uint64_t opts = P.opts;
    const uint64_t oa = P.out_off[m], cap = P.out_off[m + 1] - oa;
    gu8 *ob = (gu8 *)(void *)(P.out + oa);
    const bool b64 = !(opts & DG_T2J_NO_BASE64);
    int64_t p = 0; /* walker state (lane 0) */
    uint32_t sp = 0;
    T2WFrame cur{};
    bool done = false, started = false;
    uint64_t O = 0; /* output bytes so far */
    for (;;) {
        int32_t nt = 0;
        if (lane == 0) nt = t2w_walk(D, fx, src, p, sp, cur, L, opts, done, started, P.root);
        nt = __builtin_amdgcn_readfirstlane(nt);
        if (nt < 0) return false;
        const bool fin = __builtin_amdgcn_readfirstlane(done ? 1 : 0) != 0;
        __builtin_amdgcn_wave_barrier();
        const bool act = lane < (uint32_t)nt;
        const uint32_t kd = act ? L.kind[lane] : 0u;
        const uint32_t kind = kd & 7;
        const uint32_t pos = act ? L.pos[lane] : 0u, aux = act ? L.aux[lane] : 0u, td = act ? L.td[lane] : 0u;
        const uint32_t kt = act ? L.kt[lane] : 0u;
        const bool keyf = act && (kd & TKF_KEYF), keym = act && (kd & TKF_KEYM), comma = act && (kd & TKF_COMMA);
        const bool isval = act && kind == TK_VAL;
        const dg_type vt = ldrec(&D.T[isval ? td : 0u]);
        const uint8_t tt = isval ? vt.ttype : 0;
        const bool isstr = isval && tt == DG_T_STRING;
        const bool isbin = isstr && b64 && (vt.flags & DG_TF_BINARY);
        const bool kstr = keym && kt == DG_T_STRING;
        const uint32_t vn = isstr ? (uint32_t)be_at(src, pos, 4) : 0u;
        const uint32_t kn = kstr ? (uint32_t)be_at(src, aux, 4) : 0u;
        /* escapes: 8-byte scan tasks over the wave, counts summed per token */
        {
            const uint32_t kc = kstr ? (kn + 7) / 8 : 0u, vc = isstr && !isbin ? (vn + 7) / 8 : 0u;
            const uint32_t cinc = wave_incl_sum(kc + vc, lane);
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)cinc, 63);
            L.xk[lane] = 0;
            L.xv[lane] = 0;
            if (T) {
                L.cinc[lane] = cinc;
                L.ck[lane] = kc;
                L.cs[lane] = aux + 4;
                L.cn[lane] = kn;
                L.cvs[lane] = pos + 4;
                L.cvn[lane] = vn;
                __builtin_amdgcn_wave_barrier();
                for (uint32_t c = lane; c < T; c += 64) {
                    uint32_t l = 0;
#pragma unroll
                    for (uint32_t step = 32; step; step >>= 1)
                        if (L.cinc[l + step - 1] <= c) l += step;
                    const uint32_t own = c - (l ? L.cinc[l - 1] : 0u); /* task index within lane l */
                    const bool iskey = own < L.ck[l];
                    const uint32_t j = iskey ? own : own - L.ck[l];
                    const uint32_t len = iskey ? L.cn[l] : L.cvn[l];
                    const uint32_t s0 = (iskey ? L.cs[l] : L.cvs[l]) + j * 8;
                    const uint32_t nb = len - j * 8 < 8 ? len - j * 8 : 8u;
                    const uint32_t x = quote_extra(src.get8(s0), nb);
                    if (x) atomicAdd(iskey ? &L.xk[l] : &L.xv[l], x);
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        const uint32_t xk = L.xk[lane], xv = L.xv[lane];
        /* lengths */
        RegOut rv, rk;
        rv.init();
        rk.init();
        bool bad = false;
        uint32_t klen = 0, vlen = 0;
        dg_t2j_field xf{};
        if (keyf) {
            xf = ldrec(&X.X[aux]);
            klen = xf.key_len;
        } else if (kstr) {
            klen = kn + xk + 3; /* "key": */
        } else if (keym) {
            rk.w8('"');
            t2w_numkey(src, aux, (uint8_t)kt, opts, rk);
            rk.wle('"' | (':' << 8), 2);
            klen = rk.len;
        }
        bool chunked = false;
        if (isstr) {
            if (isbin) {
                vlen = 2 + (vn + 2) / 3 * 4;
                chunked = vn > T2W_B64;
            } else {
                vlen = 2 + vn + xv;
                chunked = xv == 0 && vn > T2W_CH;
            }
        } else if (isval) {
            if (!t2w_scalar(src, pos, tt, opts, rv)) bad = true;
            vlen = rv.len;
        } else if (act) {
            vlen = 1;
        }
        if (ballot(bad)) return false;
        const uint32_t ln = (comma ? 1u : 0u) + klen + vlen;
        const uint32_t incl = wave_incl_sum(ln, lane);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (O + tot > cap) return false; /* slot overflow: the lane kernel reports it */
        const uint64_t at = O + incl - ln;
        /* the token's bytes; a chunked body is left to the tasks below */
        {
            WOut w;
            w.init(ob + at);
            if (comma) w.w8(',');
            if (keyf) {
                const __attribute__((address_space(1))) uint64_t *kw =
                    (const __attribute__((address_space(1))) uint64_t *)(X.P + xf.key_off);
                uint32_t i = 0;
                for (; i + 8 <= xf.key_len; i += 8) w.wle(kw[i >> 3], 8);
                if (i < xf.key_len) w.wle(kw[i >> 3], xf.key_len - i);
            } else if (kstr) {
                w.w8('"');
                if (xk) emit_quoted(w, src, (int64_t)aux + 4, kn);
                else fast_copy(src, (int64_t)aux + 4, (int64_t)kn, w);
                w.wle('"' | (':' << 8), 2);
            } else if (keym) {
                rk.flush(w);
            }
            if (act && !isval) {
                w.w8(kind == TK_OPEN_OBJ ? '{' : kind == TK_OPEN_ARR ? '[' : kind == TK_CLOSE_OBJ ? '}' : ']');
            } else if (isstr) {
                w.w8('"');
                if (!chunked) {
                    if (isbin) emit_base64(w, src, (int64_t)pos + 4, vn);
                    else if (xv) emit_quoted(w, src, (int64_t)pos + 4, vn);
                    else fast_copy(src, (int64_t)pos + 4, (int64_t)vn, w);
                    w.w8('"');
                }
            } else if (isval) {
                rv.flush(w);
            }
            w.finish();
            if (chunked) {
                WOut q; /* the closing quote after the body */
                q.init(ob + at + ln - 1);
                q.w8('"');
                q.finish();
            }
        }
        /* chunked bodies: copy / base64 tasks over the wave */
        {
            const uint32_t nch = !chunked ? 0u : isbin ? (vn + T2W_B64 - 1) / T2W_B64 : (vn + T2W_CH - 1) / T2W_CH;
            const uint32_t cinc = wave_incl_sum(nch, lane);
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)cinc, 63);
            if (T) {
                L.cinc[lane] = cinc;
                L.cs[lane] = pos + 4;
                L.cn[lane] = vn | (isbin ? 0x80000000u : 0u);
                L.cvs[lane] = (uint32_t)(at + ln - vlen + 1); /* after the opening quote */
                __builtin_amdgcn_wave_barrier();
                for (uint32_t c = lane; c < T; c += 64) {
                    uint32_t l = 0;
#pragma unroll
                    for (uint32_t step = 32; step; step >>= 1)
                        if (L.cinc[l + step - 1] <= c) l += step;
                    const uint32_t k = c - (l ? L.cinc[l - 1] : 0u);
                    const uint32_t bn = L.cn[l], blen = bn & 0x7FFFFFFFu;
                    WOut w;
                    if (bn >> 31) {
                        const uint32_t s0 = k * T2W_B64, n = blen - s0 < T2W_B64 ? blen - s0 : T2W_B64;
                        w.init(ob + L.cvs[l] + (uint64_t)k * (T2W_B64 / 3 * 4));
                        emit_base64(w, src, (int64_t)L.cs[l] + s0, (int64_t)n);
                    } else {
                        const uint32_t s0 = k * T2W_CH, n = blen - s0 < T2W_CH ? blen - s0 : T2W_CH;
                        w.init(ob + L.cvs[l] + s0);
                        fast_copy(src, (int64_t)L.cs[l] + s0, (int64_t)n, w);
                    }
                    w.finish();
                }
            }
        }
        O += tot;
        if (fin) break;
    }
    if (lane == 0) {
        P.ret[m] = 0;
        P.out_len[m] = (uint32_t)O;
    }
    return true;
}

}  // namespace dg
