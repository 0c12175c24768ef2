/*
 * t2j_device.h — the reverse path, Thrift binary -> JSON (conv/t2j), on the
 * GPU: one lane per message.
 *
 * Thrift binary is length-prefixed, so a message is walked front to back
 * with no scanning: every lane runs the reference's doRecurse
 * (conv/t2j/impl.go:189-393) iteratively over a small frame stack in LDS
 * (messages nested deeper than T2J_LDS_DEPTH are reported DG_ST_DEEP and
 * rerun by the same code with the frames in device memory). The JSON bytes
 * are the reference's, byte for byte:
 *   numbers   i64toa (native/fastint.c:212-231) and f64toa, the Schubfach
 *             shortest round-trip formatter (native/fastfloat.c:288-404,
 *             R. Giulietti, "The Schubfach way to render doubles", 2022);
 *   strings   quote with flags 0 (native/parsing.c:28-63, 487): '"' and '\\'
 *             backslashed, \t \n \r short, other bytes < 0x20 as \u00xx;
 *   binary    standard padded base64 (base64x.StdEncoding);
 *   keys      pre-encoded on the host (the t2j side table,
 *             include/dgj2t_desc.h dg_t2j_*);
 *   unsets    thrift/utils.go:149-176 HandleRequires + writeDefaultOrEmpty
 *             (conv/t2j/impl.go:440-468);
 *   js_conv   thrift/annotation/value_mapping.go:143-214 (numbers quoted).
 * Errors are status words (include/dgj2t_defs.h DG_T2J_E_*), code | pos << 8
 * | value << 40, pos = the Thrift read offset where the reference's read
 * failed.
 */
#pragma once
#include "j2t_device.h"
#include "t2j_tables.h"

namespace dg {

constexpr uint32_t T2J_LDS_DEPTH = 12;   /* frames per lane in LDS */
constexpr uint32_t T2J_DEEP_DEPTH = 4096; /* frames per lane in the deep rerun */
constexpr uint32_t T2J_WIDE_WORDS = 1024; /* deep rerun: requires words per lane for structs of > 64 fields */
constexpr uint32_t T2J_BLOCK = 256;
constexpr int T2J_SKIP_DEPTH = 1023;     /* MaxSkipDepth, thrift/binary_skip.go:24 */

enum : uint32_t { RD_EOF = 1, RD_BAD_TYPE = 2, RD_BAD_SIZE = 3, RD_DEPTH = 4 };
enum : uint32_t { TF_STRUCT = 1, TF_LIST = 2, TF_MAP = 3, TF_SKIP_STRUCT = 4, TF_SKIP_LIST = 5, TF_SKIP_MAP = 6 };

/* one open container (24 B) */
struct T2JFrame {
    uint32_t kind; /* TF_* */
    uint32_t td;   /* type index; skip frames: element wire type(s) */
    uint32_t n;    /* elements (list/map) */
    uint32_t i;    /* elements done; struct: fields written (comma) */
    uint64_t u;    /* struct: requires bits by field index; skip frames: maxDepth */
};

struct T2JSide {
    const __attribute__((address_space(1))) dg_t2j_field *X;
    const __attribute__((address_space(1))) uint8_t *P;
};

DGI uint64_t t2j_err(uint32_t code, uint64_t pos, uint64_t val) { return (val << 40) | (pos << 8) | code; }

/* ---------------- encoders ---------------- */

/* 4 decimal digits of y < 10000 as ASCII, first digit lowest */
DGI uint32_t dig4(uint32_t y)
{
    const uint32_t hi = y / 100, lo = y - hi * 100;
    const uint32_t a = hi / 10, b = hi - a * 10, c = lo / 10, d = lo - c * 10;
    return 0x30303030u | a | (b << 8) | (c << 16) | (d << 24);
}
/* 8 decimal digits of x < 10^8 with leading zeros, first digit lowest */
DGI uint64_t dig8(uint32_t x)
{
    const uint32_t a = x / 10000, b = x - a * 10000;
    return (uint64_t)dig4(a) | ((uint64_t)dig4(b) << 32);
}
/* x < 10^8 without leading zeros: the 8 digits with leading zeros, shifted
 * past the leading '0' bytes (at least one digit stays) */
template <class O>
DGI void emit_small(O &o, uint32_t x)
{
    const uint64_t d = dig8(x);
    const uint64_t z = d ^ 0x3030303030303030ull; /* nonzero bytes: digits 1-9 */
    const uint32_t lead = z ? ((uint32_t)__builtin_ctzll(z) >> 3) : 7u;
    o.wle(d >> (lead << 3), 8 - lead);
}
/* the decimal digits of sig (< 10^24) as a 24-byte ASCII string with
 * leading zeros, held in three words (byte i of the string = byte i & 7 of
 * word i >> 3), and the positions of its first and last nonzero digits */
struct Dig24 {
    uint64_t w0, w1, w2;
    uint32_t first, last;
    DGI void init(uint64_t sig)
    {
        const uint64_t a = sig / 100000000ull;
        const uint32_t b = (uint32_t)(sig - a * 100000000ull);
        const uint32_t a1 = (uint32_t)(a / 100000000ull), a0 = (uint32_t)(a - (uint64_t)a1 * 100000000ull);
        w0 = dig8(a1);
        w1 = dig8(a0);
        w2 = dig8(b);
        const uint64_t z0 = w0 ^ 0x3030303030303030ull, z1 = w1 ^ 0x3030303030303030ull,
                       z2 = w2 ^ 0x3030303030303030ull;
        first = z0 ? (uint32_t)__builtin_ctzll(z0) >> 3
                   : z1 ? 8 + ((uint32_t)__builtin_ctzll(z1) >> 3) : 16 + ((uint32_t)__builtin_ctzll(z2 | (1ull << 63)) >> 3);
        last = z2 ? 16 + ((63 - (uint32_t)__builtin_clzll(z2)) >> 3)
                  : z1 ? 8 + ((63 - (uint32_t)__builtin_clzll(z1)) >> 3) : ((63 - (uint32_t)__builtin_clzll(z0 | 1)) >> 3);
    }
    /* string bytes [from, from + len) (from + len <= 24): the string shifted
     * by `from` bytes, straight-line (no indexed words: they would live in
     * scratch), then up to three writes */
    template <class O>
    DGI void put(O &o, uint32_t from, uint32_t len) const
    {
        const uint32_t k = from >> 3, b = (from & 7) << 3;
        const uint64_t x0 = k == 0 ? w0 : k == 1 ? w1 : w2, x1 = k == 0 ? w1 : k == 1 ? w2 : 0ull,
                       x2 = k == 0 ? w2 : 0ull;
        const uint64_t s0 = b ? (x0 >> b) | (x1 << (64 - b)) : x0, s1 = b ? (x1 >> b) | (x2 << (64 - b)) : x1,
                       s2 = b ? x2 >> b : x2;
        if (len) o.wle(s0, len < 8 ? len : 8u);
        if (len > 8) o.wle(s1, len - 8 < 8 ? len - 8 : 8u);
        if (len > 16) o.wle(s2, len - 16);
    }
};

/* k <= 24 ASCII zeros */
template <class O>
DGI void put_zeros(O &o, uint32_t k)
{
    const uint64_t z = 0x3030303030303030ull;
    if (k) o.wle(z, k < 8 ? k : 8u);
    if (k > 8) o.wle(z, k - 8 < 8 ? k - 8 : 8u);
    if (k > 16) o.wle(z, k - 16);
}

/* u64toa (native/fastint.c:221-231): decimal, no leading zeros. Straight
 * line (the 24-digit string, then its digits from the first nonzero one):
 * lanes formatting numbers of different lengths take the same path. */
template <class O>
DGI void emit_u64(O &o, uint64_t v)
{
    Dig24 D;
    D.init(v); /* v == 0: first = 23, the last '0' */
    D.put(o, D.first, 24 - D.first);
}
/* i64toa (native/fastint.c:212-219) */
template <class O>
DGI void emit_i64(O &o, int64_t v)
{
    if (v >= 0) {
        emit_u64(o, (uint64_t)v);
    } else {
        o.w8('-');
        emit_u64(o, 0ull - (uint64_t)v);
    }
}

/* Schubfach: the shortest decimal sig * 10^exp in the rounding interval of
 * c * 2^q (native/fastfloat.c:288-347) */
DGI uint64_t round_odd(uint64_t ghi, uint64_t glo, uint64_t cp)
{
    const uint64_t x_hi = __umul64hi(cp, glo);
    const uint64_t y_lo0 = cp * ghi;
    const uint64_t y_lo = y_lo0 + x_hi;
    const uint64_t y_hi = __umul64hi(cp, ghi) + (y_lo < y_lo0 ? 1ull : 0ull);
    return y_hi | (y_lo > 1 ? 1ull : 0ull);
}
DGI void f64_to_dec(uint64_t rsig, int32_t rexp, uint64_t c, int32_t q, uint64_t &sig, int32_t &dexp)
{
    const bool even = !(c & 1);
    const bool irregular = rsig == 0 && rexp > 1;
    const uint64_t cbl = 4 * c - 2 + (irregular ? 1 : 0), cb = 4 * c, cbr = 4 * c + 2;
    const int32_t k = (q * 1262611 - (irregular ? 524031 : 0)) >> 22;
    const int32_t h = q + (((-k) * 1741647) >> 19) + 1;
    const uint64_t ghi = DG_POW10_CEIL[-k + 292][0], glo = DG_POW10_CEIL[-k + 292][1];
    const uint64_t vbl = round_odd(ghi, glo, cbl << h);
    const uint64_t vb = round_odd(ghi, glo, cb << h);
    const uint64_t vbr = round_odd(ghi, glo, cbr << h);
    const uint64_t lower = vbl + (even ? 0 : 1), upper = vbr - (even ? 0 : 1);
    const uint64_t s = vb / 4;
    if (s >= 10) {
        const uint64_t sp = s / 10;
        const bool up_in = lower <= 40 * sp, wp_in = 40 * sp + 40 <= upper;
        if (up_in != wp_in) {
            sig = sp + (wp_in ? 1 : 0);
            dexp = k + 1;
            return;
        }
    }
    const bool u_in = lower <= 4 * s, w_in = 4 * s + 4 <= upper;
    if (u_in != w_in) {
        sig = s + (w_in ? 1 : 0);
        dexp = k;
        return;
    }
    const uint64_t mid = 4 * s + 2;
    const bool up = vb > mid || (vb == mid && (s & 1) != 0);
    sig = s + (up ? 1 : 0);
    dexp = k;
}

/* the shortest digits sig * 10^exp (sig's digits in D) in f64toa's layout
 * (native/fastfloat.c:349-404): an integer, a decimal, or d.ddde[+-]x when
 * the decimal exponent is < -6 or > 20 (write_dec :241-259) */
template <class O>
DGI void f64_write_dec(O &o, const Dig24 &D, int32_t exp)
{
    const uint32_t cnt = 24 - D.first; /* d[i] = string byte D.first + i */
    const int32_t dot = (int32_t)cnt + exp;
    const int32_t sci = dot - 1;
    const uint32_t nd = D.last - D.first + 1; /* digits without trailing zeros */
    if (sci < -6 || sci > 20) { /* format_exponent :168-203 */
        D.put(o, D.first, 1);
        if (nd > 1) {
            o.w8('.');
            D.put(o, D.first + 1, nd - 1);
        }
        int32_t e = exp + (int32_t)cnt - 1;
        if (e < 0) {
            o.wle('e' | ('-' << 8), 2);
            e = -e;
        } else {
            o.wle('e' | ('+' << 8), 2);
        }
        emit_small(o, (uint32_t)e);
        return;
    }
    if (dot < (int32_t)cnt) { /* format_decimal :205-239 */
        if (dot <= 0) {
            o.wle('0' | ('.' << 8), 2);
            put_zeros(o, (uint32_t)-dot);
            D.put(o, D.first, nd);
            return;
        }
        if ((int32_t)nd > dot) {
            D.put(o, D.first, (uint32_t)dot);
            o.w8('.');
            D.put(o, D.first + (uint32_t)dot, nd - (uint32_t)dot);
        } else {
            D.put(o, D.first, nd);
            put_zeros(o, (uint32_t)dot - nd);
        }
        return;
    }
    D.put(o, D.first, cnt); /* integer digits, then zeros up to the point */
    put_zeros(o, (uint32_t)(dot - (int32_t)cnt));
}

/* f64toa (native/fastfloat.c:349-404) for a finite double: the shortest
 * round-trip digits, written as an integer, a decimal, or d.ddde[+-]x when
 * the decimal exponent is < -6 or > 20 (write_dec :241-259) */
template <class O>
DGI void emit_f64(O &o, double fp)
{
    const uint64_t raw = (uint64_t)__double_as_longlong(fp);
    const bool neg = (raw >> 63) != 0;
    const uint64_t rsig = raw & 0x000FFFFFFFFFFFFFull;
    const int32_t rexp = (int32_t)((raw >> 52) & 0x7FF);
    if (neg) o.w8('-');
    if ((raw << 1) == 0) {
        o.w8('0');
        return;
    }
    uint64_t c;
    int32_t q;
    if (rexp != 0) {
        c = rsig | 0x0010000000000000ull;
        q = rexp - 1075;
        if (q <= 0 && q >= -52 && (c & ((1ull << -q) - 1)) == 0) { /* an integer */
            emit_u64(o, c >> -q);
            return;
        }
    } else {
        c = rsig;
        q = -1074;
    }
    uint64_t sig;
    int32_t exp;
    f64_to_dec(rsig, rexp, c, q, sig, exp);
    Dig24 D;
    D.init(sig);
    f64_write_dec(o, D, exp);
}

/* quote (native/parsing.c:487, flags 0) of src[s0, s0+n): 8 bytes per step
 * when none of them needs an escape */
template <class S, class O>
DGI void emit_quoted(O &o, S &src, int64_t s0, int64_t n)
{
    int64_t i = 0;
    while (i < n) {
        const uint64_t w = src.get8(s0 + i);
        const int64_t rem = n - i;
        const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
        /* bytes < 0x20 (top bit clear, + 0x60 does not reach 0x80), '"', '\\' */
        const uint32_t cl = ~((lo & 0x7F7F7F7Fu) + 0x60606060u) & ~lo & 0x80808080u;
        const uint32_t ch = ~((hi & 0x7F7F7F7Fu) + 0x60606060u) & ~hi & 0x80808080u;
        uint64_t m = ((uint64_t)cl | ((uint64_t)ch << 32)) | eqbytes(w, '"') | eqbytes(w, '\\');
        if (rem < 8) m &= (1ull << (rem << 3)) - 1;
        if (m == 0) {
            const uint32_t k = rem < 8 ? (uint32_t)rem : 8u;
            o.wle(w, k);
            i += k;
            continue;
        }
        const uint32_t j = (uint32_t)__builtin_ctzll(m) >> 3;
        if (j) o.wle(w, j);
        const uint8_t c = (uint8_t)(w >> (j << 3));
        if (c == '"') o.wle('\\' | ('"' << 8), 2);
        else if (c == '\\') o.wle('\\' | ('\\' << 8), 2);
        else if (c == '\t') o.wle('\\' | ('t' << 8), 2);
        else if (c == '\n') o.wle('\\' | ('n' << 8), 2);
        else if (c == '\r') o.wle('\\' | ('r' << 8), 2);
        else {
            const uint32_t h1 = c >> 4, h2 = c & 15;
            const uint64_t x1 = h1 < 10 ? '0' + h1 : 'a' + h1 - 10, x2 = h2 < 10 ? '0' + h2 : 'a' + h2 - 10;
            o.wle('\\' | ('u' << 8) | ('0' << 16) | ('0' << 24) | (x1 << 32) | (x2 << 40), 6);
        }
        i += j + 1;
    }
}

DGI uint64_t b64c(uint32_t v) /* one standard-alphabet character */
{
    return v < 26 ? 'A' + v : v < 52 ? 'a' + v - 26 : v < 62 ? '0' + v - 52 : v == 62 ? '+' : '/';
}
/* standard padded base64 of src[s0, s0+n) (base64x.StdEncoding; the
 * reference's b64encode, native/base64.c:173, mode 0) */
template <class S, class O>
DGI void emit_base64(O &o, S &src, int64_t s0, int64_t n)
{
    int64_t i = 0;
    for (; i + 3 <= n; i += 3) {
        const uint64_t w = src.get8(s0 + i);
        const uint32_t t = ((uint32_t)(w & 0xFF) << 16) | ((uint32_t)((w >> 8) & 0xFF) << 8) | (uint32_t)((w >> 16) & 0xFF);
        o.wle(b64c(t >> 18) | (b64c((t >> 12) & 63) << 8) | (b64c((t >> 6) & 63) << 16) | (b64c(t & 63) << 24), 4);
    }
    if (i < n) {
        const uint64_t w = src.get8(s0 + i);
        const uint32_t b0 = (uint32_t)(w & 0xFF), b1 = n - i > 1 ? (uint32_t)((w >> 8) & 0xFF) : 0u;
        const uint32_t t = (b0 << 16) | (b1 << 8);
        const uint64_t c2 = n - i > 1 ? b64c((t >> 6) & 63) : '=';
        o.wle(b64c(t >> 18) | (b64c((t >> 12) & 63) << 8) | (c2 << 16) | ((uint64_t)'=' << 24), 4);
    }
}

/* ---------------- the walk ---------------- */

template <class S>
struct T2JRd {
    S src;
    int64_t p;
    DGI bool need(int64_t k) const { return p + k <= (int64_t)src.n; }
    DGI uint8_t u8() { return src.raw(p++); }
    DGI uint64_t be(uint32_t k) /* k <= 8 bytes, big-endian */
    {
        const uint64_t w = src.get8(p);
        p += k;
        return __builtin_bswap64(w) >> ((8 - k) << 3);
    }
};

DGI bool ttype_valid(uint8_t t) /* thrift/descriptor.go:60-67 */
{
    return t <= 17 && ((0x3FD5Fu >> t) & 1); /* 0 1 2 3 4 6 8 10 11 12 13 14 15 16 17 */
}
DGI uint32_t fixed_size(uint8_t t) /* typeSize, thrift/binary_skip.go:26-41 */
{
    switch (t) {
    case 2: case 3: return 1;
    case 6: return 2;
    case 8: return 4;
    case 4: case 10: return 8;
    }
    return 0;
}

template <class DV>
DGI int32_t t2j_field(const DV &D, const dg_struct &sd, uint32_t hint, uint16_t id)
{
    if (hint < sd.n_fields && ldrec(&D.F[sd.field_begin + hint]).id == id) return (int32_t)(sd.field_begin + hint);
    uint32_t lo = 0, hi = sd.n_fields; /* fields are sorted by id */
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        const uint16_t fid = ldrec(&D.F[sd.field_begin + m]).id;
        if (fid == id) return (int32_t)(sd.field_begin + m);
        if (fid < id) lo = m + 1;
        else hi = m;
    }
    return -1;
}

#ifndef DG_T2J_GROUPS
#define DG_T2J_GROUPS 0
#endif
#if DG_T2J_GROUPS
/* JSON output of one lane: Out's 8-byte word assembly, completed words held
 * in registers until the 64-byte aligned group they belong to is complete,
 * then stored as four 16-byte stores issued together. 64 lanes writing 64
 * slots 16 bytes at a time left L2 lines partly written long enough to be
 * written back more than once (t2j-c2: 24.5 MB written for 13.6 MB of JSON
 * and status words); whole groups staged through LDS wrote 16.6 MB but cost
 * 14 % of the kernel (r4o/r4p). Here the group is 8 named registers shifted
 * one word per completed word (constant register indices: no scratch). */
struct JOut {
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    gu8 *b;
    uint64_t cap;
    uint64_t len;
    uint64_t wbuf;  /* the word holding position len */
    uint64_t g0, g1, g2, g3, g4, g5, g6, g7; /* the open group's completed words, newest in g7 */
    uint32_t gb;    /* the slot's first word's position in its 64-byte group (0..7) */
    bool wide;      /* slot base 8-aligned: word and 16-byte stores allowed */

    DGI void init(uint8_t *base, uint64_t c)
    {
        b = (gu8 *)(void *)base;
        cap = c;
        len = 0;
        wbuf = 0;
        g0 = g1 = g2 = g3 = g4 = g5 = g6 = g7 = 0;
        wide = ((uintptr_t)base & 7) == 0;
        gb = wide ? (uint32_t)(((uintptr_t)base >> 3) & 7) : 0u;
    }
    DGI void store_word(uint64_t wi, uint64_t v)
    {
        const uint64_t a = wi << 3;
        if (wide && a + 8 <= cap) *(gu64 *)(b + a) = v;
        else if (a < cap) Out::store_bytes(b, a, cap, v);
    }
    DGI uint64_t load_word(uint64_t wi) const
    {
        const uint64_t a = wi << 3;
        if (wide && a + 8 <= cap) return *(const gu64 *)(b + a);
        return a < cap ? Out::load_bytes(b, a, cap) : 0;
    }
    /* the open group's newest k words (k <= 8) end at word e (exclusive):
     * word e - k + m = g_{8-k+m}; words before the slot or past cap are not
     * written */
    static __device__ __noinline__ void group_edge(gu8 *b, uint64_t cap, bool wide, int64_t e, uint32_t k,
                                                   uint64_t x0, uint64_t x1, uint64_t x2, uint64_t x3, uint64_t x4,
                                                   uint64_t x5, uint64_t x6, uint64_t x7)
    {
        const uint64_t g[8] = {x0, x1, x2, x3, x4, x5, x6, x7};
        for (uint32_t m = 8 - k; m < 8; m++) {
            const int64_t wi = e - 8 + (int64_t)m;
            if (wi < 0) continue;
            const uint64_t a = (uint64_t)wi << 3;
            if (wide && a + 8 <= cap) *(gu64 *)(b + a) = g[m];
            else if (a < cap) Out::store_bytes(b, a, cap, g[m]);
        }
    }
    DGI void wle(uint64_t v, uint32_t n)
    {
        const uint32_t used = (uint32_t)(len & 7);
        const uint32_t sh = used << 3;
        if (n < 8) v &= (1ull << (n << 3)) - 1;
        const uint64_t lo = (wbuf & ((1ull << sh) - 1)) | (v << sh);
        const uint64_t hi = used ? (v >> (64 - sh)) : 0;
        const uint64_t wi = len >> 3;
        len += n;
        if (used + n >= 8) {
            g0 = g1;
            g1 = g2;
            g2 = g3;
            g3 = g4;
            g4 = g5;
            g5 = g6;
            g6 = g7;
            g7 = lo;
            if (((gb + (uint32_t)wi) & 7) == 7) { /* the group is complete */
                if (wide && wi >= 7 && (wi + 1) * 8 <= cap) {
                    __attribute__((address_space(1))) u64x2 *q =
                        (__attribute__((address_space(1))) u64x2 *)(void *)(b + (wi - 7) * 8); /* 64-byte aligned */
                    u64x2 p0, p1, p2, p3;
                    p0.x = g0; p0.y = g1;
                    p1.x = g2; p1.y = g3;
                    p2.x = g4; p2.y = g5;
                    p3.x = g6; p3.y = g7;
                    q[0] = p0;
                    q[1] = p1;
                    q[2] = p2;
                    q[3] = p3;
                } else {
                    group_edge(b, cap, wide, (int64_t)wi + 1, 8, g0, g1, g2, g3, g4, g5, g6, g7);
                }
            }
            wbuf = hi;
        } else {
            wbuf = lo;
        }
    }
    DGI void w8(uint8_t v) { wle(v, 1); }
    /* truncate to x; the converter only ever truncates to 0 (a stop's
     * record or an exception's JSON replaces the output) */
    DGI void set_len(uint64_t x)
    {
        if (x == 0) {
            len = 0;
            wbuf = 0;
            return;
        }
        finish(); /* general case (unused): flush, then read the partial word back */
        len = x;
        wbuf = (x & 7) ? load_word(x >> 3) : 0;
    }
    /* the open group's completed words, and the partial word */
    DGI void finish()
    {
        const uint64_t lw = len >> 3;
        const uint32_t k = (gb + (uint32_t)lw) & 7; /* completed words of the open group */
        if (k) group_edge(b, cap, wide, (int64_t)lw, k, g0, g1, g2, g3, g4, g5, g6, g7);
        if (len & 7) store_word(lw, wbuf);
    }
};
#else
/* JSON output of one lane: Out's 8-byte word assembly, with completed words
 * stored in aligned 16-byte pairs (one dwordx4 store per lane per 16 bytes,
 * the width the L2 write counters and write-back handle whole; 8-byte stores
 * of 64 lanes into 64 slots showed as 29.9 MB written on t2j-c2 for 13.6 MB
 * of JSON). The first word of a pair waits in `wlo`. */
struct JOut {
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    gu8 *b;
    uint64_t cap;
    uint64_t len;
    uint64_t wbuf;  /* the word holding position len */
    uint64_t wlo;   /* the completed first word of the pair holding len */
    uint32_t sk;    /* the slot's first word within its 16-byte pair (0 or 1) */
    bool wide;      /* slot base 8-aligned: word and pair stores allowed */

    DGI void init(uint8_t *base, uint64_t c)
    {
        b = (gu8 *)(void *)base;
        cap = c;
        len = 0;
        wbuf = wlo = 0;
        wide = ((uintptr_t)base & 7) == 0;
        sk = wide ? (uint32_t)(((uintptr_t)base >> 3) & 1) : 0u;
    }
    DGI void store_word(uint64_t wi, uint64_t v)
    {
        const uint64_t a = wi << 3;
        if (wide && a + 8 <= cap) *(gu64 *)(b + a) = v;
        else if (a < cap) Out::store_bytes(b, a, cap, v);
    }
    DGI uint64_t load_word(uint64_t wi) const
    {
        const uint64_t a = wi << 3;
        if (wide && a + 8 <= cap) return *(const gu64 *)(b + a);
        return a < cap ? Out::load_bytes(b, a, cap) : 0;
    }
    static __device__ __noinline__ void pair_edge(gu8 *b, uint64_t cap, bool wide, uint64_t wi, uint64_t w0, uint64_t w1)
    {
        for (uint32_t j = 0; j < 2; j++) {
            if (wi + j < 1) continue;
            const uint64_t a = (wi + j - 1) << 3, v = j ? w1 : w0;
            if (wide && a + 8 <= cap) *(gu64 *)(b + a) = v;
            else if (a < cap) Out::store_bytes(b, a, cap, v);
        }
    }
    DGI void wle(uint64_t v, uint32_t n)
    {
        const uint32_t used = (uint32_t)(len & 7);
        const uint32_t sh = used << 3;
        if (n < 8) v &= (1ull << (n << 3)) - 1;
        const uint64_t lo = (wbuf & ((1ull << sh) - 1)) | (v << sh);
        const uint64_t hi = used ? (v >> (64 - sh)) : 0;
        const uint64_t wi = len >> 3;
        len += n;
        if (used + n >= 8) {
            if (((sk + (uint32_t)wi) & 1) == 0) {
                wlo = lo;
            } else if (wide && wi >= 1 && (wi + 1) * 8 <= cap) {
                u64x2 p;
                p.x = wlo;
                p.y = lo;
                /* (non-temporal stores here: 44.6 MB written on t2j-c2 instead of 24.7, r4m;
                 * whole 64-byte groups staged in LDS, branch wip-jout-groups: 16.6 MB
                 * written, but the kernel 52.4 -> 59.7 us, r4o/r4p) */
                *(__attribute__((address_space(1))) u64x2 *)(void *)(b + (wi - 1) * 8) = p; /* 16-byte aligned */
            } else {
                pair_edge(b, cap, wide, wi, wlo, lo);
            }
            wbuf = hi;
        } else {
            wbuf = lo;
        }
    }
    DGI void w8(uint8_t v) { wle(v, 1); }
    /* truncate to x <= len */
    DGI void set_len(uint64_t x)
    {
        const uint64_t xw = x >> 3, lw = len >> 3;
        if (((sk + xw) >> 1) != ((sk + lw) >> 1)) { /* x's pair is stored already: take it back */
            if (((sk + (uint32_t)xw) & 1) && xw >= 1) wlo = load_word(xw - 1);
            wbuf = (x & 7) ? load_word(xw) : 0;
        } else if (xw != lw) {
            wbuf = (x & 7) ? wlo : 0;
        }
        len = x;
    }
    /* the waiting first word of the open pair, and the partial word */
    DGI void finish()
    {
        const uint64_t lw = len >> 3;
        if (((sk + (uint32_t)lw) & 1) && lw >= 1) store_word(lw - 1, wlo);
        if (len & 7) store_word(lw, wbuf);
    }
};

#endif

/* side-table bytes [off, off+len) (8-aligned, 16 readable past the end) */
DGI void emit_side(JOut &o, const T2JSide &X, uint32_t off, uint32_t len)
{
    const __attribute__((address_space(1))) uint64_t *w = (const __attribute__((address_space(1))) uint64_t *)(X.P + off);
    uint32_t i = 0;
    for (; i + 8 <= len; i += 8) o.wle(w[i >> 3], 8);
    if (i < len) o.wle(w[i >> 3], len - i);
}

/* one message. FP: frame storage (LDS or device workspace), `cap` frames. */
/* the Thrift size of a fixed-size scalar, 0 otherwise */
DGI uint32_t num_bytes(uint8_t tt)
{
    switch (tt) {
    case DG_T_BYTE: return 1;
    case DG_T_I16: return 2;
    case DG_T_I32: return 4;
    case DG_T_I64:
    case DG_T_DOUBLE: return 8;
    }
    return 0;
}

/* DefaultValue().JSONValue() of a scalar or string IDL constant
 * (thrift/idl.go:834-955: EncodeInt64 / EncodeFloat64 / EncodeString /
 * true|false), from its Thrift bytes in the descriptor pool */
template <class DV>
DGI void emit_default(JOut &o, const DV &D, const dg_field &fd, uint8_t tt)
{
    auto byte = [&](uint32_t k) -> uint64_t { return (uint8_t)D.P[fd.dflt_off + k]; };
    if (tt == DG_T_BOOL) {
        if (byte(0) == 1) o.wle('t' | ('r' << 8) | ('u' << 16) | ('e' << 24), 4);
        else o.wle('f' | ('a' << 8) | ('l' << 16) | ('s' << 24) | (0x65ull << 32), 5);
        return;
    }
    if (tt == DG_T_STRING) {
        const uint32_t n = (uint32_t)((byte(0) << 24) | (byte(1) << 16) | (byte(2) << 8) | byte(3));
        const uintptr_t a = (uintptr_t)(const void *)&D.P[fd.dflt_off + 4];
        SrcT<const uint64_t> ps;
        ps.init((const uint64_t *)(a & ~(uintptr_t)7), (int64_t)(a & 7), (int64_t)n);
        o.w8('"');
        emit_quoted(o, ps, 0, n);
        o.w8('"');
        return;
    }
    const uint32_t nb = num_bytes(tt);
    uint64_t u = 0;
    for (uint32_t k = 0; k < nb; k++) u = (u << 8) | byte(k);
    switch (tt) {
    case DG_T_BYTE: emit_i64(o, (int8_t)u); break;
    case DG_T_I16: emit_i64(o, (int16_t)u); break;
    case DG_T_I32: emit_i64(o, (int32_t)u); break;
    case DG_T_I64: emit_i64(o, (int64_t)u); break;
    default: emit_f64(o, __longlong_as_double((long long)u)); break;
    }
}

/* GO: the root-level Go-side options are compiled in (DG_T2J_CONVERT_EXC,
 * DG_T2J_SKIP_RESP_BASE, DG_T2J_HM); the plain instance keeps the lane
 * kernel's registers at occupancy 4 (113 vs 139 VGPRs) */
template <bool GO, class S, class FP, class DV>
DGI uint64_t t2j_convert(const DV &D, const T2JSide &X, S src, uint32_t root, uint64_t opts, JOut &o, FP fr,
                         uint32_t fstride, uint32_t cap, gu64 *wide = nullptr, uint32_t widecap = 0,
                         uint64_t *aux = nullptr, const dg_cb_entry *ans = nullptr, const uint8_t *ans_bytes = nullptr)
{
    if (!GO) {
        opts &= ~(uint64_t)(DG_T2J_CONVERT_EXC | DG_T2J_SKIP_RESP_BASE | DG_T2J_HM);
        aux = nullptr;
        ans = nullptr;
    }
    T2JRd<S> r{src, 0};
    uint32_t sp = 0;
    uint32_t wlen = 0; /* words of `wide` in use: requires bitmaps of open structs of > 64 fields */
    auto F = [&](uint32_t k) -> auto & { return fr[k * fstride]; };
    /* the root struct's Go-side options (conv/t2j/impl.go:74-187): the
     * exception field being converted (DG_T2J_CONVERT_EXC), a response-base
     * value being skipped (DG_T2J_SKIP_RESP_BASE, its span to aux) */
    bool exc = false;
    bool base_pend = false;
    int64_t base_s0 = 0;
    if (aux) *aux = ~0ull;
    /* DG_T2J_HM: the host's answers to writeHttpValue, one byte per call in
     * call order (dg_cb_entry): 0 = the response took the value, 1 = write it
     * to the JSON as well, 2 = still open: convert the container value to
     * JSON and stop with it (the calls its conversion makes follow it). A
     * call past the answers stops the message at the value. */
    uint32_t ans_seen = 0; /* calls so far */
    auto take = [&](uint8_t &a) -> bool {
        const uint32_t k = ans_seen++;
        if (!ans || k >= ans->count) return false;
        a = ans_bytes[ans->off + k];
        return true;
    };
    uint32_t cb_fi = ~0u, cb_sp = 0, cb_idx = 0;
    int64_t cb_s0 = 0;
    /* a stop's record: its payload (a mapped container's JSON, else nothing)
     * and a 16-byte trailer: kind (1 mapped value, 2 unset mapped field) |
     * resp << 8 | the call's index << 16, the field's index, the value's span */
    auto stop = [&](uint32_t kind, uint32_t idx, uint32_t fi, int64_t s0, int64_t s1) -> uint64_t {
        if (idx > 0xFFFF) return t2j_err(DG_T2J_E_DEPTH, r.p, idx); /* more calls than a record counts */
        o.wle((uint64_t)kind | ((uint64_t)idx << 16) | ((uint64_t)fi << 32), 8);
        o.wle((uint64_t)(uint32_t)s0 | ((uint64_t)(uint32_t)s1 << 32), 8);
        return t2j_err(DG_T2J_E_CALLBACK, r.p, kind & 0xFF);
    };
    /* bit k: frame k is a struct with a ResponseSetter: the root (do()), a
     * root field's struct value (doRecurse(resp), conv/t2j/impl.go:167) and
     * the value writeHttpValue converts to JSON (impl.go:565); their fields'
     * values and container elements get nil (impl.go:327,360,383) */
    uint64_t respm = 0;
    bool push_resp = (opts & DG_T2J_HM) != 0; /* the next struct value pushed gets one: first the root */
    auto resp_level = [&]() -> bool { return sp - 1 < 64 && ((respm >> (sp - 1)) & 1); };

    /* the value of type td at the reader: scalars written, containers opened
     * (their header read and checked, the frame pushed) */
    auto value = [&](uint32_t td) -> uint64_t {
        const dg_type t = ldrec(&D.T[td]);
        switch (t.ttype) {
        case DG_T_BOOL:
            if (!r.need(1)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            if (r.u8() == 1) o.wle('t' | ('r' << 8) | ('u' << 16) | ('e' << 24), 4);
            else o.wle('f' | ('a' << 8) | ('l' << 16) | ('s' << 24) | (0x65ull << 32), 5);
            return 0;
        case DG_T_BYTE: {
            if (!r.need(1)) return t2j_err(DG_T2J_E_WRITE, r.p, RD_EOF);
            const uint8_t v = r.u8();
            emit_i64(o, (opts & DG_T2J_BYTE_AS_UINT8) ? (int64_t)v : (int64_t)(int8_t)v);
            return 0;
        }
        case DG_T_I16:
            if (!r.need(2)) return t2j_err(DG_T2J_E_WRITE, r.p, RD_EOF);
            emit_i64(o, (int16_t)r.be(2));
            return 0;
        case DG_T_I32:
            if (!r.need(4)) return t2j_err(DG_T2J_E_WRITE, r.p, RD_EOF);
            emit_i64(o, (int32_t)r.be(4));
            return 0;
        case DG_T_I64: {
            if (!r.need(8)) return t2j_err(DG_T2J_E_WRITE, r.p, RD_EOF);
            const int64_t v = (int64_t)r.be(8);
            if (opts & DG_T2J_INT64_AS_STRING) {
                o.w8('"');
                emit_i64(o, v);
                o.w8('"');
            } else {
                emit_i64(o, v);
            }
            return 0;
        }
        case DG_T_DOUBLE: {
            if (!r.need(8)) return t2j_err(DG_T2J_E_WRITE, r.p, RD_EOF);
            const uint64_t u = r.be(8);
            if (((u >> 52) & 0x7FF) == 0x7FF) {
                if (!(opts & DG_T2J_NULL_FOR_NAN_INF)) return t2j_err(DG_T2J_E_NAN_INF, r.p, 0);
                o.wle('n' | ('u' << 8) | ('l' << 16) | ('l' << 24), 4);
                return 0;
            }
            emit_f64(o, __longlong_as_double((long long)u));
            return 0;
        }
        case DG_T_STRING: {
            if (!r.need(4)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const int32_t sz = (int32_t)r.be(4);
            if (sz < 0 || !r.need(sz)) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE);
            const int64_t s0 = r.p;
            r.p += sz;
            o.w8('"');
            if ((t.flags & DG_TF_BINARY) && !(opts & DG_T2J_NO_BASE64)) emit_base64(o, r.src, s0, sz); /* EncodeBaniry */
            else emit_quoted(o, r.src, s0, sz);
            o.w8('"');
            return 0;
        }
        case DG_T_STRUCT: {
            if (sp >= cap) return pack0(DG_ST_DEEP, 0);
            const dg_struct sd = ldrec(&D.S[t.st]);
            uint64_t u = D.R[sd.req_begin];
            if (sd.req_words != 1) {
                /* > 64 fields: the bitmap lives in the deep pass's per-lane
                 * words (a stack: structs close in reverse order) */
                if (!wide) return pack0(DG_ST_DEEP, 0);
                if (wlen + sd.req_words > widecap) return t2j_err(DG_T2J_E_DEPTH, r.p, T2J_DEEP_DEPTH);
                for (uint32_t w = 0; w < sd.req_words; w++) wide[wlen + w] = D.R[sd.req_begin + w];
                u = wlen;
                wlen += sd.req_words;
            }
            if (sp < 64) respm = push_resp ? respm | (1ull << sp) : respm & ~(1ull << sp);
            auto &f = F(sp++);
            f.kind = TF_STRUCT;
            f.td = td;
            f.n = 0; /* predicted next field index */
            f.i = 0;
            f.u = u;
            o.w8('{');
            return 0;
        }
        case DG_T_LIST:
        case DG_T_SET: {
            if (!r.need(1)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint8_t et = r.u8();
            if (!ttype_valid(et)) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_TYPE);
            if (!r.need(4)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const int32_t n = (int32_t)r.be(4);
            if (n < 0) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE);
            const uint8_t want = ldrec(&D.T[t.elem]).ttype;
            if (et != want) return t2j_err(DG_T2J_E_DISMATCH_TYPE, r.p, ((uint32_t)want << 8) | et);
            if (sp >= cap) return pack0(DG_ST_DEEP, 0);
            auto &f = F(sp++);
            f.kind = TF_LIST;
            f.td = td;
            f.n = (uint32_t)n;
            f.i = 0;
            o.w8('[');
            return 0;
        }
        case DG_T_MAP: {
            if (!r.need(1)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint8_t kt = r.u8();
            if (!ttype_valid(kt)) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_TYPE);
            if (!r.need(1)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint8_t vt = r.u8();
            if (!ttype_valid(vt)) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_TYPE);
            if (!r.need(4)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const int32_t n = (int32_t)r.be(4);
            if (n < 0) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE);
            const uint8_t wk = ldrec(&D.T[t.key]).ttype, wv = ldrec(&D.T[t.elem]).ttype;
            if (kt != wk) return t2j_err(DG_T2J_E_DISMATCH_TYPE, r.p, ((uint32_t)wk << 8) | kt);
            if (vt != wv) return t2j_err(DG_T2J_E_DISMATCH_TYPE, r.p, ((uint32_t)wv << 8) | vt);
            if (sp >= cap) return pack0(DG_ST_DEEP, 0);
            auto &f = F(sp++);
            f.kind = TF_MAP;
            f.td = td;
            f.n = (uint32_t)n;
            f.i = 0;
            o.w8('{');
            return 0;
        }
        }
        return t2j_err(DG_T2J_E_UNSUPPORTED, r.p, t.ttype);
    };

    /* one element inside a skipped container, or skipType
     * (thrift/binary_skip.go:109-210) of wire type t with budget `depth`:
     * fixed sizes are skipn'd before any depth check, list/map strings are
     * skipstr'd directly (str_direct), everything else is skipType(t, depth):
     * containers continue as a skip frame */
    auto skip = [&](uint8_t t, uint32_t depth, bool str_direct) -> uint64_t {
        const uint32_t fs = fixed_size(t);
        if (fs) {
            if (!r.need(fs)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            r.p += fs;
            return 0;
        }
        if (!(str_direct && t == DG_T_STRING) && (int32_t)depth <= 0) return t2j_err(DG_T2J_E_READ, r.p, RD_DEPTH);
        if (t == DG_T_STRING) { /* skipstr (:80-95): the size as uint32 in a 64-bit int */
            if (!r.need(4)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint64_t sz = (uint32_t)__builtin_bswap32((uint32_t)r.src.get8(r.p));
            if (r.p + 4 + (int64_t)sz > (int64_t)r.src.n) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            r.p += 4 + (int64_t)sz;
            return 0;
        }
        if (t == DG_T_STRUCT) {
            if (sp >= cap) return pack0(DG_ST_DEEP, 0);
            auto &f = F(sp++);
            f.kind = TF_SKIP_STRUCT;
            f.u = depth;
            return 0;
        }
        if (t == DG_T_MAP) {
            if (!r.need(6)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint8_t kt = r.u8(), vt = r.u8();
            const int32_t sz = (int32_t)r.be(4);
            if (sz < 0) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE);
            const uint32_t ks = fixed_size(kt), vs = fixed_size(vt);
            if (ks && vs) {
                const int64_t k = (int64_t)sz * (int64_t)(ks + vs);
                if (!r.need(k)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                r.p += k;
                return 0;
            }
            if (sp >= cap) return pack0(DG_ST_DEEP, 0);
            auto &f = F(sp++);
            f.kind = TF_SKIP_MAP;
            f.td = kt | ((uint32_t)vt << 8);
            f.n = (uint32_t)sz * 2; /* keys and values alternate */
            f.i = 0;
            f.u = depth;
            return 0;
        }
        if (t == DG_T_LIST || t == DG_T_SET) {
            if (!r.need(5)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint8_t vt = r.u8();
            const int32_t sz = (int32_t)r.be(4);
            if (sz < 0) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE);
            const uint32_t vs = fixed_size(vt);
            if (vs) {
                const int64_t k = (int64_t)sz * (int64_t)vs;
                if (!r.need(k)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                r.p += k;
                return 0;
            }
            if (sp >= cap) return pack0(DG_ST_DEEP, 0);
            auto &f = F(sp++);
            f.kind = TF_SKIP_LIST;
            f.td = vt;
            f.n = (uint32_t)sz;
            f.i = 0;
            f.u = depth;
            return 0;
        }
        return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE); /* default: errInvalidDataSize */
    };

    /* handleUnsets -> HandleRequires (thrift/utils.go:149-176), ascending id */
    auto unsets = [&](auto &f, const dg_struct &sd, bool resp) -> uint64_t {
        for (uint32_t w = 0; w < sd.req_words; w++) {
            uint64_t bits = sd.req_words == 1 ? f.u : (uint64_t)wide[(uint32_t)f.u + w];
            while (bits) {
                const uint32_t k = w * 64 + (uint32_t)__builtin_ctzll(bits);
                bits &= bits - 1;
                const dg_field fd = ldrec(&D.F[sd.field_begin + k]);
                if (fd.required == DG_REQ_REQUIRED && !(opts & DG_T2J_WRITE_REQUIRE))
                    return t2j_err(DG_T2J_E_MISS_REQUIRED, r.p, fd.id);
                if ((fd.required == DG_REQ_DEFAULT && !(opts & DG_T2J_WRITE_DEFAULT)) ||
                    (fd.required == DG_REQ_OPTIONAL && !(opts & DG_T2J_WRITE_OPTIONAL) && fd.dflt_len == DG_NONE))
                    continue;
                const uint8_t ftt = ldrec(&D.T[fd.type]).ttype;
                if ((opts & DG_T2J_HM) && (fd.flags & DG_FF_HTTP_MAPPING)) {
                    /* handleUnsets (impl.go:401-429): writeHttpValue of the default first, at
                     * every level (resp may be nil there) */
                    uint8_t a;
                    if (!take(a)) {
                        o.set_len(0);
                        return stop(2 | (resp ? 0x100u : 0u), ans_seen - 1, sd.field_begin + k, 0, 0);
                    }
                    if (a == 0) continue;
                }
                if (fd.dflt_len != DG_NONE && !(ftt == DG_T_BOOL || num_bytes(ftt) || ftt == DG_T_STRING))
                    return t2j_err(DG_T2J_E_NEEDS_HOST, r.p, fd.id); /* a container constant's JSONValue() */
                if (f.i) o.w8(',');
                f.i = 1;
                const dg_t2j_field xf = ldrec(&X.X[sd.field_begin + k]);
                emit_side(o, X, xf.name_off, xf.name_len); /* "name": */
                if (fd.dflt_len != DG_NONE) {
                    /* DefaultValue().JSONValue() (thrift/idl.go:834-955): EncodeInt64 /
                     * EncodeFloat64 / EncodeString / true|false of the IDL constant, here
                     * from its Thrift bytes in the descriptor pool */
                    emit_default(o, D, fd, ftt);
                    continue;
                }
                switch (ftt) { /* writeDefaultOrEmpty conv/t2j/impl.go:440-468 */
                case DG_T_BOOL: o.wle('f' | ('a' << 8) | ('l' << 16) | ('s' << 24) | (0x65ull << 32), 5); break;
                case DG_T_BYTE: case DG_T_I16: case DG_T_I32: case DG_T_I64: case DG_T_DOUBLE: o.w8('0'); break;
                case DG_T_STRING: o.wle('"' | ('"' << 8), 2); break;
                case DG_T_LIST: case DG_T_SET: o.wle('[' | (']' << 8), 2); break;
                case DG_T_MAP: case DG_T_STRUCT: o.wle('{' | ('}' << 8), 2); break;
                default: return t2j_err(DG_T2J_E_UNSUPPORTED, r.p, ldrec(&D.T[fd.type]).ttype);
                }
            }
        }
        return 0;
    };

    uint64_t e = value(root);
    push_resp = false;
    if (e) return e;
    while (sp) {
        if (cb_fi != ~0u && sp == cb_sp) return stop(1 | 0x100u, cb_idx, cb_fi, cb_s0, r.p); /* the mapped value read */
        auto &f = F(sp - 1);
        switch (f.kind) {
        case TF_STRUCT: {
            const dg_type st = ldrec(&D.T[f.td]);
            const dg_struct sd = ldrec(&D.S[st.st]);
            if (sp == 1) {
                if (base_pend) { /* the skipped response base ends here */
                    *aux = (uint64_t)base_s0 | ((uint64_t)r.p << 32);
                    base_pend = false;
                }
                if (exc) { /* the exception field is done: unsets, then the error (impl.go:173-187) */
                    if ((e = unsets(f, sd, resp_level()))) return e;
                    return t2j_err(DG_T2J_E_EXCEPTION, r.p, 0);
                }
            }
            if (!r.need(1)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint8_t t = r.u8();
            if (!ttype_valid(t)) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_TYPE);
            if (t == 0) {
                if ((e = unsets(f, sd, resp_level()))) return e;
                o.w8('}');
                if (sd.req_words != 1) wlen -= sd.req_words;
                sp--;
                continue;
            }
            if (!r.need(2)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint16_t id = (uint16_t)r.be(2);
            const int32_t fi = t2j_field(D, sd, f.n, id);
            if (fi < 0) {
                if (opts & DG_T2J_DISALLOW_UNKNOWN) return t2j_err(DG_T2J_E_UNKNOWN_FIELD, r.p, id);
                if ((e = skip(t, T2J_SKIP_DEPTH, false))) return e;
                continue;
            }
            const uint32_t k = (uint32_t)fi - sd.field_begin;
            if (sd.req_words == 1) f.u &= ~(1ull << k);
            else wide[(uint32_t)f.u + (k >> 6)] &= ~(1ull << (k & 63));
            f.n = k + 1;
            const dg_field fd = ldrec(&D.F[fi]);
            if (sp == 1 && (opts & DG_T2J_SKIP_RESP_BASE) && (fd.flags & DG_FF_RESPONSE_BASE) && aux) {
                /* readResponseBase (impl.go:54-72): SkipType(STRUCT), no key */
                base_s0 = r.p;
                if ((e = skip(DG_T_STRUCT, T2J_SKIP_DEPTH, false))) return e;
                base_pend = true;
                continue;
            }
            if ((fd.flags & DG_FF_HTTP_MAPPING) && (opts & DG_T2J_HM) && resp_level()) {
                /* writeHttpValue (impl.go:132-142, 296-306): the host's answer, or a stop
                 * with the value's span (and a container's JSON, impl.go:561-574) */
                uint8_t a;
                const uint8_t dt = ldrec(&D.T[fd.type]).ttype;
                if (!take(a)) { /* a new call: the host reads the value at the stop's position */
                    o.set_len(0);
                    return stop(1 | 0x100u, ans_seen - 1, (uint32_t)fi, r.p, r.p);
                }
                if (a == 2 && (dt == DG_T_STRUCT || dt == DG_T_MAP || dt == DG_T_LIST || dt == DG_T_SET)) {
                    /* the call needs the value's JSON (doRecurse(resp), impl.go:561-574):
                     * converted here, the calls it makes answered after this one's */
                    cb_s0 = r.p;
                    cb_fi = (uint32_t)fi;
                    cb_sp = sp;
                    cb_idx = ans_seen - 1;
                    o.set_len(0);
                    push_resp = true;
                    e = value(fd.type);
                    push_resp = false;
                    if (e) return e;
                    continue; /* stops when the frames are back at cb_sp */
                }
                if (a == 0) { /* the response took it: the value is consumed */
                    if ((e = skip(dt, T2J_SKIP_DEPTH, false))) return e;
                    continue;
                }
            }
            if (f.i) o.w8(',');
            f.i = 1;
            const dg_t2j_field xf = ldrec(&X.X[fi]);
            emit_side(o, X, xf.key_off, xf.key_len); /* "alias": */
            if (sp == 1 && (opts & DG_T2J_CONVERT_EXC) && id != 0) { /* only the exception field's data */
                o.set_len(0);
                exc = true;
            }
            if ((opts & DG_T2J_ENABLE_VM) && fd.vm == DG_VM_BODY_DYNAMIC) {
                /* agwBodyDynamic.Read (thrift/annotation/value_mapping.go:84-99): the raw bytes */
                const uint8_t ft = ldrec(&D.T[fd.type]).ttype;
                if (ft != DG_T_STRING) return t2j_err(DG_T2J_E_CONVERT, r.p, 0x200u | ft);
                if (!r.need(4)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                const int32_t sz = (int32_t)r.be(4);
                if (sz < 0 || !r.need(sz)) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE);
                int32_t q = 0;
                for (; q + 8 <= sz; q += 8) o.wle(r.src.get8(r.p + q), 8);
                if (q < sz) o.wle(r.src.get8(r.p + q), (uint32_t)(sz - q));
                r.p += sz;
                continue;
            }
            if ((opts & DG_T2J_ENABLE_VM) && fd.vm != DG_VM_NONE) {
                /* apiJSConv.Read (thrift/annotation/value_mapping.go:143-214) */
                if (fd.vm != DG_VM_JSCONV) return t2j_err(DG_T2J_E_NEEDS_HOST, r.p, fd.vm);
                const uint8_t ft = ldrec(&D.T[fd.type]).ttype;
                uint8_t et = ft;
                int32_t cnt = 1;
                if (ft == DG_T_LIST) {
                    o.w8('[');
                    if (!r.need(1)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                    et = r.u8();
                    if (!ttype_valid(et)) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_TYPE);
                    if (!r.need(4)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                    cnt = (int32_t)r.be(4);
                    if (cnt < 0) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE);
                }
                for (int32_t j = 0; j < cnt; j++) { /* appendInt */
                    o.w8('"');
                    switch (et) {
                    case DG_T_BYTE:
                        if (!r.need(1)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                        emit_i64(o, (int64_t)r.u8()); /* ReadByte: 0..255 */
                        break;
                    case DG_T_I16:
                        if (!r.need(2)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                        emit_i64(o, (int16_t)r.be(2));
                        break;
                    case DG_T_I32:
                        if (!r.need(4)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                        emit_i64(o, (int32_t)r.be(4));
                        break;
                    case DG_T_I64:
                        if (!r.need(8)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                        emit_i64(o, (int64_t)r.be(8));
                        break;
                    case DG_T_DOUBLE: {
                        if (!r.need(8)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                        const uint64_t u = r.be(8);
                        if (((u >> 52) & 0x7FF) != 0x7FF) emit_f64(o, __longlong_as_double((long long)u)); /* f64toa: nothing for inf/nan */
                        break;
                    }
                    case DG_T_STRING: {
                        if (!r.need(4)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
                        const int32_t sz = (int32_t)r.be(4);
                        if (sz < 0 || !r.need(sz)) return t2j_err(DG_T2J_E_READ, r.p, RD_BAD_SIZE);
                        for (int32_t b = 0; b < sz; b++) o.w8(r.src.raw(r.p + b)); /* raw, not escaped */
                        r.p += sz;
                        break;
                    }
                    default:
                        return t2j_err(DG_T2J_E_UNSUPPORTED, r.p, et);
                    }
                    o.w8('"');
                    if (ft == DG_T_LIST && j != cnt - 1) o.w8(',');
                }
                if (ft == DG_T_LIST) o.w8(']');
                continue;
            }
            push_resp = sp == 1 && (respm & 1); /* do() passes resp to its fields' values */
            e = value(fd.type);
            push_resp = false;
            if (e) return e;
            continue;
        }
        case TF_LIST: {
            if (f.i == f.n) {
                o.w8(']');
                sp--;
                continue;
            }
            if (f.i) o.w8(',');
            f.i++;
            if ((e = value(ldrec(&D.T[f.td]).elem))) return e;
            continue;
        }
        case TF_MAP: {
            if (f.i == f.n) {
                o.w8('}');
                sp--;
                continue;
            }
            if (f.i) o.w8(',');
            f.i++;
            const dg_type mt = ldrec(&D.T[f.td]);
            const uint8_t kt = ldrec(&D.T[mt.key]).ttype;
            o.w8('"'); /* buildinTypeToKey (conv/t2j/impl.go:470-530) */
            switch (kt) {
            case DG_T_BYTE: {
                if (!r.need(1)) return t2j_err(DG_T2J_E_CONVERT, r.p, RD_EOF);
                const uint8_t v = r.u8();
                emit_i64(o, (opts & DG_T2J_BYTE_AS_UINT8) ? (int64_t)v : (int64_t)(int8_t)v);
                break;
            }
            case DG_T_I16:
                if (!r.need(2)) return t2j_err(DG_T2J_E_CONVERT, r.p, RD_EOF);
                emit_i64(o, (int16_t)r.be(2));
                break;
            case DG_T_I32:
                if (!r.need(4)) return t2j_err(DG_T2J_E_CONVERT, r.p, RD_EOF);
                emit_i64(o, (int32_t)r.be(4));
                break;
            case DG_T_I64:
                if (!r.need(8)) return t2j_err(DG_T2J_E_CONVERT, r.p, RD_EOF);
                emit_i64(o, (int64_t)r.be(8));
                break;
            case DG_T_STRING: {
                if (!r.need(4)) return t2j_err(DG_T2J_E_CONVERT, r.p, RD_EOF);
                const int32_t sz = (int32_t)r.be(4);
                if (sz < 0 || !r.need(sz)) return t2j_err(DG_T2J_E_CONVERT, r.p, RD_BAD_SIZE);
                emit_quoted(o, r.src, r.p, sz); /* json.NoQuote */
                r.p += sz;
                break;
            }
            default:
                return t2j_err(DG_T2J_E_CONVERT, r.p, 0x100u | kt); /* wrapped as ErrConvert */
            }
            o.wle('"' | (':' << 8), 2);
            if ((e = value(mt.elem))) return e;
            continue;
        }
        case TF_SKIP_STRUCT: {
            const uint32_t depth = (uint32_t)f.u;
            if (!r.need(1)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            const uint8_t tp = r.u8();
            if (tp == 0) {
                sp--;
                continue;
            }
            if (!r.need(2)) return t2j_err(DG_T2J_E_READ, r.p, RD_EOF);
            r.p += 2;
            if ((e = skip(tp, depth - 1, false))) return e;
            continue;
        }
        case TF_SKIP_LIST:
        case TF_SKIP_MAP: {
            if (f.i == f.n) {
                sp--;
                continue;
            }
            const uint8_t et = f.kind == TF_SKIP_LIST ? (uint8_t)f.td : (uint8_t)(f.i & 1 ? f.td >> 8 : f.td);
            f.i++;
            if ((e = skip(et, (uint32_t)f.u - 1, true))) return e;
            continue;
        }
        }
    }
    return 0;
}

struct T2JParams {
    uint32_t root;
    uint64_t opts;
    const uint8_t *src;       /* Thrift arena */
    const uint64_t *in_off;   /* n + 1 */
    uint64_t n;
    uint8_t *out;             /* JSON slots */
    const uint64_t *out_off;
    uint32_t *out_len;        /* JSON bytes; DG_ST_OUT_OVERFLOW: bytes needed */
    uint64_t *ret;
    const uint8_t *blob;      /* descriptor (device) */
    dg_desc_hdr hdr;
    const uint8_t *side;      /* t2j side table (device) */
    uint64_t *aux;            /* DG_T2J_SKIP_RESP_BASE: per message the response base's span (or NULL) */
    const dg_cb_entry *ans_tab; /* DG_T2J_HM: per message the host's writeHttpValue answers (or NULL) */
    const uint8_t *ans_bytes;
    uint32_t *deep_list;      /* messages nested beyond the LDS frames */
    uint32_t *deep_count;     /* their number */
    uint32_t *reset_counts;   /* the deep pass zeroes these 4 counters: the set the previous launch used */
    uint8_t *ws;              /* deep pass: T2J_DEEP_DEPTH frames per lane */
    /* the wave path (t2j_wave.h): the lane pass lists messages longer than
     * big_min (when big_list is set) instead of converting them; list mode
     * (list set): the lane pass converts list[0 .. *list_count) instead of
     * all n */
    uint32_t *big_list;
    uint32_t *big_count;
    uint64_t big_min;
    uint32_t skip_big;        /* messages longer than big_min are skipped, not listed (t2j_route_kernel listed them) */
    const uint32_t *list;
    const uint32_t *list_count;
    unsigned long long *stats; /* DG_T2W_PROF builds: phase cycles of the wave kernel (dg_ctx_counters 2..) */
};

DGI T2JSide t2j_side(const uint8_t *side)
{
    const dg_t2j_hdr xh = *(const dg_t2j_hdr *)side;
    return T2JSide{(const __attribute__((address_space(1))) dg_t2j_field *)(const void *)(side + xh.off_fields),
                   (const __attribute__((address_space(1))) uint8_t *)(const void *)(side + xh.off_pool)};
}

/* finish one message: overflow check, status and length */
DGI void t2j_store(const T2JParams &P, uint64_t i, uint64_t r, JOut &o)
{
    uint32_t olen = 0;
    if (r == 0 || (uint8_t)r == DG_T2J_E_EXCEPTION || (uint8_t)r == DG_T2J_E_CALLBACK) { /* kept: the exception's JSON, the stop's record */
        o.finish();
        if (o.len > o.cap) {
            const uint64_t need = o.len;
            olen = need > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)need;
            r = pack(DG_ST_OUT_OVERFLOW, need > 0xFFFFFFull ? 0xFFFFFFull : need, 0);
        } else {
            olen = (uint32_t)o.len;
        }
    }
    P.ret[i] = r;
    P.out_len[i] = olen;
}

constexpr uint32_t T2J_DEEP_BLOCKS = 4; /* 1024 lanes x 96 KiB of frames */

void launch_t2j_pass(uint64_t n, hipStream_t s, const T2JParams &P, uint32_t spread); /* spread 1, 2 or 4 */

/* the wave path (t2j_wave.h) */
constexpr uint32_t T2W_WAVES = 4; /* waves (messages in flight) per block */
struct T2WParams {
    const uint32_t *list;  /* the lane pass's long messages */
    const uint32_t *count;
    uint32_t *queue;       /* next list entry to take (zeroed by the host after the launch) */
    uint32_t *bail_list;   /* messages left to the lane kernel's list mode */
    uint32_t *bail_count;
    uint8_t *tok;          /* token regions, t2j_wave_ws_bytes(blocks) */
    uint32_t side_len;     /* the side table's bytes (copied to LDS) */
};
uint64_t t2j_wave_ws_bytes(uint32_t blocks);
constexpr uint32_t T2W_BPC = 4; /* wave-kernel blocks per CU in the grid */
void launch_t2j_list(uint32_t blocks, hipStream_t s, const T2JParams &P); /* list mode, 1 lane per message */
void launch_t2j_route(uint64_t n, hipStream_t s, const T2JParams &P);      /* big_list by length only */
void launch_t2j_wave(uint32_t blocks, hipStream_t s, const T2JParams &P, const T2WParams &W);
void launch_t2j_deep(hipStream_t s, const T2JParams &P);

}  // namespace dg
