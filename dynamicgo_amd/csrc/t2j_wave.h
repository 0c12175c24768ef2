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
#ifndef DG_T2W_CH
#define DG_T2W_CH 8
#endif
#ifndef DG_T2W_B64
#define DG_T2W_B64 12
#endif
constexpr uint32_t T2W_CH = DG_T2W_CH;   /* string body bytes per copy task (8/12: t2j-c3 1.67 -> 1.59 ms vs 16/24; 4/6 no better) */
constexpr uint32_t T2W_B64 = DG_T2W_B64; /* base64 input bytes per task (4/3 as many characters) */

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
    uint32_t xk[64];    /* escape bytes the map key string adds (scan tasks) */
    uint32_t xv[64];    /* ... the value string adds */
    uint32_t cinc[64];  /* tasks: inclusive prefix of per-lane task counts */
    uint32_t ck[64];    /* tasks: the map key's (the rest are the value's) */
    uint32_t cs[64];    /* key string source */
    uint32_t cn[64];    /* scan: key string length; write: key text output offset */
    uint32_t cvs[64];   /* value string / body source */
    uint32_t cvn[64];   /* scan: value string length; write: body output offset */
};
#ifndef DG_T2W_MPT
#define DG_T2W_MPT 16
#endif
/* messages a wave takes at once (one walker lane each). r4m, t2j-c3: 16 /
 * 32 / 64 -> 1.21 / 1.49 / 2.33 ms (at 64 the frames and token rings cut
 * the kernel to 2 waves/SIMD) */
constexpr uint32_t T2W_MPT = DG_T2W_MPT;

/* the t2j side table (keys) copied to LDS by the wave kernel */
struct T2WSide {
    const __attribute__((address_space(3))) dg_t2j_field *X;
    const __attribute__((address_space(3))) uint8_t *P;
};
constexpr uint32_t T2W_SIDE = 12288; /* side tables up to this many bytes take the wave path */

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
        /* masks, not an indexed array: the words stay in registers */
        const uint64_t m0 = k == 0 ? ~0ull : 0ull, m1 = k == 1 ? ~0ull : 0ull, m2 = k == 2 ? ~0ull : 0ull,
                       m3 = k == 3 ? ~0ull : 0ull;
        w0 |= lo & m0;
        w1 |= (lo & m1) | (hi & m0);
        w2 |= (lo & m2) | (hi & m1);
        w3 |= (lo & m3) | (hi & m2);
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

/* Token sink of the batched walk: this lane's region of the wave's token
 * buffer (global memory, T2W_TOKCAP tokens). A token is 8 bytes (16 before:
 * the tokens' round trip through L2/HBM was most of t2j-c3's traffic):
 *   pos (bits 0-20)   Thrift position of the value (messages < 2 MiB)
 *   aux (21-41)       TKF_KEYF: field index; TKF_KEYM: Thrift position of the key
 *   td  (42-53)       value type index (the wave path takes < 4096 types)
 *   kind (54-59)      TK_* | TKF_*
 *   kt  (60-63)       map key ttype */
typedef uint64_t T2WTok;
constexpr uint32_t T2W_POSBITS = 21;
DGI uint64_t t2w_tok(uint32_t kind, uint32_t pos, uint32_t aux, uint32_t td, uint32_t kt)
{
    return (uint64_t)pos | ((uint64_t)aux << 21) | ((uint64_t)td << 42) | ((uint64_t)kind << 54) | ((uint64_t)kt << 60);
}
constexpr uint32_t T2W_TOKCAP = 192; /* tokens per message (more: the lane kernel) */
constexpr uint32_t T2W_RING = T2W_MPT >= 64 ? 4 : 8; /* tokens a walker keeps in LDS before writing them out together */
constexpr uint32_t T2W_BD = 3;       /* frames kept in LDS per lane (the innermost is in registers) */

/* One lane walks its whole message (doRecurse's order, conv/t2j/impl.go:
 * 189-393) into tokens: returns the count, or -1 to bail. Parent frames
 * live in LDS at frs[d * T2W_MPT] (d < T2W_BD), the innermost in registers.
 * Tokens collect in the lane's LDS ring (ring[j * T2W_MPT], j < T2W_RING)
 * and go to global memory T2W_RING at a time: a global store ahead of the
 * walk's next (dependent) load would make that load wait for the store's
 * acknowledgement too (one vmcnt counts both). */
typedef __attribute__((address_space(3))) uint64_t lds_tok;
static_assert(T2W_RING * T2W_MPT * sizeof(T2WTok) <= T2W_MSG && T2W_TOKCAP % T2W_RING == 0, "ring in the stage");
/* bytes [p, p + 16) of the message as two little-endian words: three
 * aligned words read at once (the third only when it lies within the 16
 * readable bytes past the message, wmax) */
template <class S>
DGI void t2w_win(const S &src, int64_t p, int64_t wmax, uint64_t &lo, uint64_t &hi)
{
    const int64_t b = src.off0 + p, k = b >> 3;
    const uint32_t sh = (uint32_t)(b & 7) << 3;
    const uint64_t a0 = src.w8[k], a1 = src.w8[k + 1], a2r = src.w8[k + 2 <= wmax ? k + 2 : wmax];
    const uint64_t a2 = k + 2 <= wmax ? a2r : 0ull;
    lo = sh ? (a0 >> sh) | (a1 << (64 - sh)) : a0;
    hi = sh ? (a1 >> sh) | (a2 << (64 - sh)) : a1;
}

template <class S, class DV>
DGI int32_t t2w_walk(const DV &D, const __attribute__((address_space(3))) uint64_t *fx, S &src,
                     T2WFrame *frs, T2WTok *tok, lds_tok *ring, uint32_t root, uint64_t opts)
{
    const int64_t n = src.n;
    const int64_t wmax = (src.off0 + n + 8) >> 3; /* the last word inside the 16 readable bytes past the end */
    int64_t p = 0;
    uint32_t sp = 0, nt = 0;
    if (n >= ((int64_t)1 << T2W_POSBITS)) return -1; /* positions must fit a token */
    T2WFrame cur{};
    auto emit = [&](uint32_t kind, uint32_t pos, uint32_t aux, uint32_t td, uint32_t kt) -> bool {
        if (nt >= T2W_TOKCAP) return false;
        ring[(nt % T2W_RING) * T2W_MPT] = t2w_tok(kind, pos, aux, td, kt);
        nt++;
        if (nt % T2W_RING == 0) {
#pragma unroll
            for (uint32_t j = 0; j < T2W_RING; j++) tok[nt - T2W_RING + j] = ring[j * T2W_MPT];
        }
        return true;
    };
    auto push = [&](const T2WFrame &f) {
        if (sp) frs[(sp - 1) * T2W_MPT] = cur;
        cur = f;
        sp++;
    };
    auto pop = [&]() {
        sp--;
        if (sp) cur = frs[(sp - 1) * T2W_MPT];
    };
    /* the root struct */
    {
        const dg_type rt = ldrec(&D.T[root]);
        if (rt.ttype != DG_T_STRUCT) return -1;
        const dg_struct sd = ldrec(&D.S[rt.st]);
        if (sd.req_words != 1 || !emit(TK_OPEN_OBJ, 0, 0, root, 0)) return -1;
        T2WFrame f{};
        f.kind = TF_STRUCT;
        f.fb = sd.field_begin;
        f.nf = sd.n_fields;
        f.st = rt.st;
        f.u = D.R[sd.req_begin];
        push(f);
    }
    /* One step per token, with ONE window read, ONE value decoder and ONE
     * emit: the 16 walkers of a wave sit at different kinds of steps, and the
     * wave runs the union of their paths, so every duplicated site (a read,
     * the token ring's flush) would be paid once per kind. */
    while (sp) {
        uint64_t lo, hi;
        t2w_win(src, p, wmax, lo, hi);
        uint32_t ek = 0, eaux = 0, ekt = 0; /* the token: kind | flags, key, map key type */
        uint32_t act = 0;                   /* 1: a closer (pop), 2: an opener (push) */
        bool isv = false;                   /* a value follows at p: type vtd / vtt, first 8 bytes vw */
        uint32_t vtd = 0, vtt = 0;
        uint64_t vw = lo;
        if (cur.kind == TF_STRUCT) {
            if (p + 1 > n) return -1;
            const uint8_t t = (uint8_t)lo; /* type, id (big-endian) */
            if (t == 0) {                  /* STOP: unset fields must write nothing */
                if (cur.u && !unsets_silent(D, ldrec(&D.S[cur.st]), cur.u, opts)) return -1;
                p += 1;
                ek = TK_CLOSE_OBJ;
                act = 1;
            } else {
                if (p + 3 > n) return -1;
                const uint64_t h = cur.n < cur.nf ? fx[cur.fb + cur.n] : 0ull; /* the predicted field */
                const uint32_t id = (uint32_t)(((lo >> 8) & 0xFF) << 8 | ((lo >> 16) & 0xFF));
                uint32_t k = cur.n;
                uint64_t v = h;
                if (cur.n >= cur.nf || fx_id(h) != id) { /* fields are sorted by id */
                    uint32_t lo_ = 0, hi_ = cur.nf;
                    k = 0xFFFFFFFFu;
                    while (lo_ < hi_) {
                        const uint32_t mid = (lo_ + hi_) >> 1;
                        const uint64_t x = fx[cur.fb + mid];
                        if (fx_id(x) == id) {
                            k = mid;
                            v = x;
                            break;
                        }
                        if (fx_id(x) < id) lo_ = mid + 1;
                        else hi_ = mid;
                    }
                    if (k == 0xFFFFFFFFu) return -1; /* unknown field (skip or error): the lane kernel */
                }
                if (fx_tt(v) != t) return -1;
                if ((opts & DG_T2J_ENABLE_VM) && (fx_fl(v) & 0x80)) return -1;
                cur.u &= ~(1ull << k);
                cur.n = k + 1;
                ek = (cur.i ? TKF_COMMA : 0u) | TKF_KEYF;
                cur.i = 1;
                p += 3;
                eaux = cur.fb + k;
                isv = true;
                vtd = fx_td(v);
                vtt = t;
                vw = (lo >> 24) | (hi << 40);
            }
        } else if (cur.i == cur.n) {
            ek = cur.kind == TF_LIST ? TK_CLOSE_ARR : TK_CLOSE_OBJ;
            act = 1;
        } else {
            ek = cur.i ? TKF_COMMA : 0u;
            cur.i++;
            if (cur.kind == TF_MAP) {
                ekt = (uint8_t)(cur.ett >> 16);
                eaux = (uint32_t)p;
                if (ekt == DG_T_STRING) {
                    if (p + 4 > n) return -1;
                    const int64_t sz = (int32_t)__builtin_bswap32((uint32_t)lo);
                    if (sz < 0 || p + 4 + sz > n) return -1;
                    p += 4 + sz;
                    uint64_t h2;
                    t2w_win(src, p, wmax, vw, h2); /* the value after the key's body */
                } else {
                    const uint32_t nb = num_bytes((uint8_t)ekt);
                    if (p + nb > n) return -1;
                    p += nb;
                    vw = nb >= 8 ? hi : (lo >> (8 * nb)) | (hi << (64 - 8 * nb));
                }
                ek |= TKF_KEYM;
            }
            isv = true;
            vtd = cur.etd;
            vtt = cur.ett & 0xFF;
        }
        /* the value: scalars and strings are one token (p moves past them),
         * containers an open token and a frame */
        uint32_t epos = 0, etd = 0;
        T2WFrame f;
        if (isv) {
            etd = vtd;
            const uint32_t fs = num_bytes((uint8_t)vtt) ? num_bytes((uint8_t)vtt) : vtt == DG_T_BOOL ? 1u : 0u;
            if (fs) {
                if (p + fs > n) return -1;
                epos = (uint32_t)p;
                p += fs;
            } else if (vtt == DG_T_STRING) {
                if (p + 4 > n) return -1;
                const int64_t sz = (int32_t)__builtin_bswap32((uint32_t)vw);
                if (sz < 0 || p + 4 + sz > n) return -1;
                epos = (uint32_t)p;
                p += 4 + sz;
            } else {
                if (sp > T2W_BD) return -1;
                const dg_type t = ldrec(&D.T[vtd]);
                f.i = 0;
                f.u = 0;
                f.fb = f.nf = f.st = 0;
                f.etd = f.ett = 0;
                if (vtt == DG_T_STRUCT) {
                    const dg_struct sd = ldrec(&D.S[t.st]);
                    if (sd.req_words != 1) return -1;
                    f.kind = TF_STRUCT;
                    f.n = 0;
                    f.fb = sd.field_begin;
                    f.nf = sd.n_fields;
                    f.st = t.st;
                    f.u = D.R[sd.req_begin];
                    ek |= TK_OPEN_OBJ;
                } else if (vtt == DG_T_LIST || vtt == DG_T_SET) {
                    if (p + 5 > n) return -1;
                    const uint64_t wb = __builtin_bswap64(vw); /* et | count (big-endian) */
                    const uint8_t et = (uint8_t)(wb >> 56);
                    const int64_t cnt = (int32_t)(uint32_t)(wb >> 24);
                    const dg_type e = ldrec(&D.T[t.elem]);
                    if (cnt < 0 || et != e.ttype) return -1;
                    p += 5;
                    f.kind = TF_LIST;
                    f.n = (uint32_t)cnt;
                    f.etd = t.elem;
                    f.ett = e.ttype | ((uint32_t)e.flags << 8);
                    ek |= TK_OPEN_ARR;
                } else if (vtt == DG_T_MAP) {
                    if (p + 6 > n) return -1;
                    const uint64_t wb = __builtin_bswap64(vw); /* kt | vt | count */
                    const uint8_t k = (uint8_t)(wb >> 56), v = (uint8_t)(wb >> 48);
                    const int64_t cnt = (int32_t)(uint32_t)(wb >> 16);
                    const dg_type kd = ldrec(&D.T[t.key]), vd = ldrec(&D.T[t.elem]);
                    if (cnt < 0 || k != kd.ttype || v != vd.ttype) return -1;
                    if (!(k == DG_T_STRING || num_bytes(k)) || k == DG_T_DOUBLE) return -1; /* buildinTypeToKey's */
                    p += 6;
                    f.kind = TF_MAP;
                    f.n = (uint32_t)cnt;
                    f.etd = t.elem;
                    f.ett = vd.ttype | ((uint32_t)vd.flags << 8) | ((uint32_t)k << 16);
                    ek |= TK_OPEN_OBJ;
                } else {
                    return -1;
                }
                act = 2;
            }
        }
        if (!emit(ek, epos, eaux, etd, ekt)) return -1;
        if (act == 1) pop();
        else if (act == 2) push(f);
    }
    for (uint32_t j = nt & ~(T2W_RING - 1); j < nt; j++) tok[j] = ring[(j % T2W_RING) * T2W_MPT];
    return (int32_t)nt;
}

#ifdef DG_T2W_PROF
#define T2P_DECL uint64_t t2p_t = __builtin_readcyclecounter(); uint64_t t2p_acc[6] = {0};
#define T2P(k) do { uint64_t t_ = __builtin_readcyclecounter(); t2p_acc[k] += t_ - t2p_t; t2p_t = t_; } while (0)
#define T2P_FLUSH() do { if (lane == 0 && P.stats) for (int k_ = 0; k_ < 6; k_++) atomicAdd(&P.stats[2 + k_], (unsigned long long)t2p_acc[k_]); } while (0)
#define T2P_ARG , uint64_t &t2p_t, uint64_t *t2p_acc
#define T2P_PASS , t2p_t, t2p_acc
#else
#define T2P_DECL
#define T2P(k)
#define T2P_FLUSH()
#define T2P_ARG
#define T2P_PASS
#endif

/* a number/bool at byte p of Thrift type tt as JSON in registers. Integers
 * and doubles share ONE 24-digit conversion (Dig24) and its writes: the
 * lanes of a page format both kinds at once, so separate i64toa and f64toa
 * paths would each be paid by the whole wave (f64toa, native/fastfloat.c:
 * 349-404; i64toa, native/fastint.c:212-231). false: bail (NaN/Inf without
 * the option) */
template <class S>
DGI bool t2w_number(S &src, int64_t p, uint8_t tt, uint64_t opts, bool quote64, RegOut &r)
{
    const uint32_t nb = tt == DG_T_BOOL || tt == DG_T_BYTE ? 1u : tt == DG_T_I16 ? 2u : tt == DG_T_I32 ? 4u : 8u;
    const uint64_t u = be_at(src, p, nb);
    if (tt == DG_T_BOOL) {
        if (u == 1) r.wle('t' | ('r' << 8) | ('u' << 16) | ('e' << 24), 4);
        else r.wle('f' | ('a' << 8) | ('l' << 16) | ('s' << 24) | (0x65ull << 32), 5);
        return true;
    }
    bool neg, dec = false;
    uint64_t mag;
    int32_t exp = 0;
    if (tt == DG_T_DOUBLE) {
        const uint64_t rsig = u & 0x000FFFFFFFFFFFFFull;
        const int32_t rexp = (int32_t)((u >> 52) & 0x7FF);
        if (rexp == 0x7FF) {
            if (!(opts & DG_T2J_NULL_FOR_NAN_INF)) return false; /* the error: the lane kernel reports it */
            r.wle('n' | ('u' << 8) | ('l' << 16) | ('l' << 24), 4);
            return true;
        }
        neg = (u >> 63) != 0;
        const uint64_t c = rexp ? rsig | 0x0010000000000000ull : rsig;
        const int32_t q = rexp ? rexp - 1075 : -1074;
        if ((u << 1) == 0) {
            mag = 0; /* "0" / "-0" */
        } else if (rexp && q <= 0 && q >= -52 && (c & ((1ull << -q) - 1)) == 0) {
            mag = c >> -q; /* an integer */
        } else {
            f64_to_dec(rsig, rexp, c, q, mag, exp);
            dec = true;
        }
    } else {
        /* sign-extend (BYTE as unsigned with ByteAsUint8) */
        const int64_t v = tt == DG_T_BYTE ? ((opts & DG_T2J_BYTE_AS_UINT8) ? (int64_t)u : (int64_t)(int8_t)u)
                          : tt == DG_T_I16 ? (int64_t)(int16_t)u
                          : tt == DG_T_I32 ? (int64_t)(int32_t)u
                                           : (int64_t)u;
        neg = v < 0;
        mag = neg ? 0ull - (uint64_t)v : (uint64_t)v;
    }
    if (quote64) r.w8('"');
    if (neg) r.w8('-');
    Dig24 D;
    D.init(mag); /* mag == 0: first = 23, the last '0' */
    if (dec) f64_write_dec(r, D, exp);
    else D.put(r, D.first, 24 - D.first);
    if (quote64) r.w8('"');
    return true;
}

/* one page of a message: up to 64 tokens, one per lane (tok = this page's
 * first token); O = the message's output bytes so far. false: bail. */
template <class S, class DV>
DGI bool t2w_page(const T2JParams &P, const DV &D, const T2WSide &X, T2WLds &L, S &src, const T2WTok *tok,
                  bool act, gu8 *ob, uint64_t cap, uint64_t &O, uint32_t lane T2P_ARG)
{
    const uint64_t opts = P.opts;
    const bool b64 = !(opts & DG_T2J_NO_BASE64);
        const T2WTok tk = act ? tok[lane] : 0ull;
        const uint32_t kd = (uint32_t)(tk >> 54) & 63u;
        const uint32_t kind = kd & 7;
        const uint32_t pos = (uint32_t)tk & 0x1FFFFFu, aux = (uint32_t)(tk >> 21) & 0x1FFFFFu;
        const uint32_t td = (uint32_t)(tk >> 42) & 0xFFFu;
        const uint32_t kt = (uint32_t)(tk >> 60);
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
        T2P(1);
        /* numbers in registers: the map key's (iteration 0), then the value's,
         * through one call site */
        RegOut rk, rv;
        rk.init();
        rv.init();
        bool bad = false;
        const bool knum = keym && !kstr, vnum = isval && !isstr;
#pragma nounroll
        for (uint32_t it = 0; it < 2; it++) {
            const bool want = it == 0 ? knum : vnum;
            if (!ballot(want)) continue;
            if (want) {
                RegOut r;
                r.init();
                if (it == 0) r.w8('"');
                if (!t2w_number(src, it == 0 ? aux : pos, it == 0 ? (uint8_t)kt : tt, opts,
                                it == 1 && tt == DG_T_I64 && (opts & DG_T2J_INT64_AS_STRING), r))
                    bad = true;
                if (it == 0) {
                    r.wle('"' | (':' << 8), 2);
                    rk = r;
                } else {
                    rv = r;
                }
            }
        }
        if (ballot(bad)) return false;
        T2P(2);
        uint32_t klen = 0, koff = 0;
        if (keyf) {
            const dg_t2j_field xf = ldrec(&X.X[aux]);
            klen = xf.key_len;
            koff = xf.key_off;
        } else if (kstr) {
            klen = kn + xk + 3; /* "key": */
        } else if (keym) {
            klen = rk.len;
        }
        uint32_t vlen = 0;
        bool tasks = false; /* the body goes to copy / base64 tasks */
        if (isstr) {
            vlen = isbin ? 2 + (vn + 2) / 3 * 4 : 2 + vn + xv;
            tasks = isbin || xv == 0;
        } else if (isval) {
            vlen = rv.len;
        } else if (act) {
            vlen = 1;
        }
        const uint32_t ln = (comma ? 1u : 0u) + klen + vlen;
        const uint32_t incl = wave_incl_sum(ln, lane);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (O + tot > cap) return false; /* slot overflow: the lane kernel reports it */
        const uint64_t at = O + incl - ln;
        /* the token's bytes: comma, key, value; string bodies with escapes
         * (rare) by their lane through ONE emit_quoted call site, the others
         * skipped here and written by the tasks below */
        {
            uint64_t wb = at; /* where w was (re)started */
            WOut w;
            w.init(ob + wb);
            if (comma) w.w8(',');
            if (keyf) {
                const __attribute__((address_space(3))) uint64_t *kw =
                    (const __attribute__((address_space(3))) uint64_t *)(X.P + koff);
                uint32_t i = 0;
                for (; i + 8 <= klen; i += 8) w.wle(kw[i >> 3], 8);
                if (i < klen) w.wle(kw[i >> 3], klen - i);
            } else if (knum) {
                rk.flush(w);
            }
#pragma nounroll
            for (uint32_t it = 0; it < 2; it++) {
                if (it == 1) { /* the value: brackets and numbers first */
                    if (act && !isval) w.w8(kind == TK_OPEN_OBJ ? '{' : kind == TK_OPEN_ARR ? '[' : kind == TK_CLOSE_OBJ ? '}' : ']');
                    else if (vnum) rv.flush(w);
                }
                const bool has = it == 0 ? kstr : isstr;
                if (!ballot(has)) continue;
                if (has) {
                    const bool serial = it == 0 ? xk != 0 : !tasks;
                    const uint32_t n = it == 0 ? kn : vn;
                    w.w8('"');
                    if (serial) {
                        emit_quoted(w, src, (int64_t)(it == 0 ? aux : pos) + 4, n);
                    } else { /* the tasks write the n body bytes (or their base64) */
                        const uint64_t skip = it == 1 && isbin ? (uint64_t)(vn + 2) / 3 * 4 : n;
                        w.finish();
                        wb += w.len + skip;
                        w.init(ob + wb);
                    }
                    if (it == 0) w.wle('"' | (':' << 8), 2);
                    else w.w8('"');
                }
            }
            w.finish();
        }
        T2P(3);
        /* bodies without escapes -- map key text, string values (copies) --
         * and binary values (base64): tasks over the wave */
        {
            const uint32_t kcn = kstr && !xk ? (kn + T2W_CH - 1) / T2W_CH : 0u;
            const uint32_t vcn = !tasks ? 0u : isbin ? (vn + T2W_B64 - 1) / T2W_B64 : (vn + T2W_CH - 1) / T2W_CH;
            const uint32_t cinc = wave_incl_sum(kcn + vcn, lane);
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)cinc, 63);
            if (T) {
                L.cinc[lane] = cinc;
                L.ck[lane] = kcn;
                L.cs[lane] = aux + 4;                                      /* key text source */
                L.cn[lane] = (uint32_t)(at + (comma ? 1u : 0u) + 1);       /* key text output */
                L.cvs[lane] = pos + 4;                                     /* value body source */
                L.cvn[lane] = (uint32_t)(at + ln - vlen + 1);              /* value body output */
                L.xk[lane] = kn;
                L.xv[lane] = vn | (isbin ? 0x80000000u : 0u);
                __builtin_amdgcn_wave_barrier();
                for (uint32_t c = lane; c < T; c += 64) {
                    uint32_t l = 0;
#pragma unroll
                    for (uint32_t step = 32; step; step >>= 1)
                        if (L.cinc[l + step - 1] <= c) l += step;
                    const uint32_t own = c - (l ? L.cinc[l - 1] : 0u);
                    const bool iskey = own < L.ck[l];
                    const uint32_t k = iskey ? own : own - L.ck[l];
                    const uint32_t bn = iskey ? L.xk[l] : L.xv[l], blen = bn & 0x7FFFFFFFu;
                    const bool bin = !iskey && (bn >> 31);
                    const uint32_t step = bin ? T2W_B64 : T2W_CH;
                    const uint32_t s0 = k * step, n = blen - s0 < step ? blen - s0 : step;
                    const uint64_t dst = (iskey ? L.cn[l] : L.cvn[l]) + (uint64_t)k * (bin ? T2W_B64 / 3 * 4 : T2W_CH);
                    const int64_t src0 = (int64_t)(iskey ? L.cs[l] : L.cvs[l]) + s0;
                    WOut w;
                    w.init(ob + dst);
                    if (bin) emit_base64(w, src, src0, (int64_t)n);
                    else fast_copy(src, src0, (int64_t)n, w);
                    w.finish();
                }
            }
        }
        O += tot;
        T2P(5);
        return true;
}

/* Up to 64 messages (one wave, msgs[0 .. nm)): every lane walks its message
 * into its token region, then the wave formats the messages one by one, a
 * page of 64 tokens at a time. Bailed messages are listed for the lane
 * kernel. */
template <class DV>
DGI void t2w_batch(const T2JParams &P, const T2WParams &W, const DV &D,
                   const __attribute__((address_space(3))) uint64_t *fx, const T2WSide &X, uint64_t mine,
                   uint32_t nm, T2WLds &L, T2WFrame *frs, T2WTok *tokw,
                   __attribute__((address_space(3))) uint64_t *mbuf, uint32_t lane)
{
    T2P_DECL
    int32_t ntok = -1;
    if (lane < nm) {
        const uint64_t a = P.in_off[mine], b = P.in_off[mine + 1];
        SrcT<glb_u64> s;
        s.init((glb_u64 *)(const void *)(P.src + (a & ~7ull)), (int64_t)(a & 7), (int64_t)(b - a));
        /* the walk's token rings live in the message stage (unused until the formatting) */
        if (b - a > 0 && b - a <= 0x7FFFFFFF) ntok = t2w_walk(D, fx, s, frs + lane, tokw + (uint64_t)lane * T2W_TOKCAP,
                                                                 (lds_tok *)(void *)mbuf + lane, P.root, P.opts);
    }
    __builtin_amdgcn_wave_barrier();
    T2P(0);
#pragma nounroll
    for (uint32_t i = 0; i < nm; i++) {
        const int32_t nti = __builtin_amdgcn_readlane(ntok, (int)i);
        const uint64_t m = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mine, (int)i);
        bool ok = nti >= 0;
        if (ok) {
            /* the message staged in the wave's LDS buffer when it fits (the
             * pages read it at random), else read through L2; one generic
             * instantiation for both (I-cache) */
            const uint64_t a = P.in_off[m], b = P.in_off[m + 1];
            const uint64_t words = (b - a + (a & 7) + 7) >> 3;
            const uint64_t *base;
            if (words + 2 <= T2W_MSG / 8) {
                const glb_u64 *g = (const glb_u64 *)(const void *)(P.src + (a & ~7ull));
                for (uint64_t j = lane; j < words; j += 64) mbuf[j] = g[j];
                if (lane < 2) mbuf[words + lane] = 0;
                base = (const uint64_t *)(void *)mbuf;
            } else {
                base = (const uint64_t *)(const void *)(P.src + (a & ~7ull));
            }
            __builtin_amdgcn_wave_barrier();
            SrcT<const uint64_t> src;
            src.init(base, (int64_t)(a & 7), (int64_t)(b - a));
            const uint64_t oa = P.out_off[m], cap = P.out_off[m + 1] - oa;
            gu8 *ob = (gu8 *)(void *)(P.out + oa);
            uint64_t O = 0;
            const T2WTok *tk = tokw + (uint64_t)i * T2W_TOKCAP;
            for (int32_t base = 0; base < nti && ok; base += 64)
                ok = t2w_page(P, D, X, L, src, tk + base, lane < (uint32_t)(nti - base), ob, cap, O, lane T2P_PASS);
            if (ok && lane == 0) {
                P.ret[m] = 0;
                P.out_len[m] = (uint32_t)O;
            }
        }
        if (!ok && lane == 0) W.bail_list[atomicAdd(W.bail_count, 1u)] = (uint32_t)m;
        __builtin_amdgcn_wave_barrier(); /* mbuf is reused by the next message */
    }
    T2P(4);
    T2P_FLUSH();
}

}  // namespace dg
