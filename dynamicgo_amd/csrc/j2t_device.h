/*
 * j2t_device.h — device-side JSON -> Thrift-binary transcoder for gfx950.
 *
 * One LANE per message: the 64 lanes of a wavefront run
 * 64 independent push-down automata over their own messages. Same-schema
 * batches keep lanes in the same FSM state most of the time, so divergence is
 * bounded by value-length differences, not by control structure.
 *
 * Semantics follow the reference's j2t_fsm_exec (native/thrift.c:765-1187)
 * bit-for-bit, including packed error words; each routine cites the reference
 * code it reproduces. Differences are purely structural:
 *  - no re-entry: the output slot is pre-sized; writes past it are dropped and
 *    the message is reported DG_ST_OUT_OVERFLOW with the length it needs
 *    (the reference grows the Go buffer and re-enters, conv/j2t/impl_amd64.go:
 *    199-226, which is transparent to the caller);
 *  - the state stack and requires bitmaps live in a small per-lane stack; a
 *    message that outgrows it is reported DG_ST_DEEP and redone by the deep
 *    kernel with a 4096-entry stack in device workspace (MAX_RECURSE,
 *    native/native.h:72);
 *  - src[len] reads as 0 (see oracle/ref_harness.c).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/dgj2t_defs.h"
#include "../../include/dgj2t_desc.h"
#include "dg_tables.h"

namespace dg {

#define DGI __device__ __forceinline__
#define DGN __device__ __noinline__

/* reference error codes (native/native.h:47-70) */
enum : uint32_t {
    E_EOF = 1, E_INVAL = 2, E_ESCAPE = 3, E_UNICODE = 4, E_NUMBER_FMT = 6, E_RECURSE_MAX = 7,
    E_FLOAT_INF = 8, E_DISMATCH_TYPE = 9, E_NULL_REQUIRED = 10, E_UNSUPPORT_THRIFT_TYPE = 11,
    E_UNKNOWN_FIELD = 12, E_DISMATCH_TYPE2 = 13, E_DECODE_BASE64 = 14, E_HM = 19,
    E_UNSUPPORT_VM_TYPE = 20, E_HM_END = 21, E_VM_END = 24
};
enum : int64_t { V_DOUBLE = 8, V_INTEGER = 9 };
enum : uint32_t { J_VAL = 0, J_ARR = 1, J_OBJ = 2, J_KEY = 3, J_ELEM = 4, J_ARR_0 = 5, J_OBJ_0 = 6 };
constexpr uint32_t ST_FIELD = 1u << 16, ST_SKIP = 1u << 17, ST_VM = 1u << 18;
constexpr uint32_t MAX_RECURSE = 4096;
constexpr uint32_t VS_NULL = 0x6c6c756e, VS_TRUE = 0x65757274, VS_ALSE = 0x65736c61;

/* WRAP_ERR_POS / WRAP_ERR0 / WRAP_ERR2 (native/thrift.h:226-242) */
DGI uint64_t pack(uint32_t e, uint64_t v, uint64_t p) { return (v << 40) | (p << 8) | (uint8_t)e; }
DGI uint64_t pack0(uint32_t e, uint64_t v) { return (v << 8) | (uint8_t)e; }
DGI uint32_t v2(uint32_t vh, uint8_t vl) { return (vh << 8) | vl; }
DGI uint32_t sx8(uint8_t c) { return (uint32_t)(int32_t)(int8_t)c; } /* (uint32_t)(char) */
DGI uint64_t sx8_64(uint8_t c) { return (uint64_t)(int64_t)(int8_t)c; }

/* The descriptor tables, in global memory (DescView) or copied to LDS by the
 * kernel prologue (DescViewT<3>); records are read by value. */
template <int AS>
struct DescViewT {
    const __attribute__((address_space(AS))) dg_type *T;
    const __attribute__((address_space(AS))) dg_struct *S;
    const __attribute__((address_space(AS))) dg_field *F;
    const __attribute__((address_space(AS))) dg_name *N;
    const __attribute__((address_space(AS))) uint64_t *R;
    const __attribute__((address_space(AS))) uint8_t *P;
};
typedef DescViewT<1> DescView;

/* read a descriptor record (multiple of 8 bytes) by value from any address space */
template <class T, int AS>
DGI typename std::remove_cv<T>::type ldrec(const __attribute__((address_space(AS))) T *p)
{
    static_assert(sizeof(T) % 8 == 0, "record size");
    const __attribute__((address_space(AS))) uint64_t *q = (const __attribute__((address_space(AS))) uint64_t *)p;
    uint64_t tmp[sizeof(T) / 8];
#pragma unroll
    for (unsigned k = 0; k < sizeof(T) / 8; k++) tmp[k] = q[k];
    typename std::remove_cv<T>::type v;
    __builtin_memcpy(&v, tmp, sizeof(T));
    return v;
}

/* views of a dg_desc v1 blob at `base` (section offsets from its header) */
template <int AS>
DGI DescViewT<AS> desc_view(const __attribute__((address_space(AS))) uint8_t *base, const dg_desc_hdr &h)
{
    DescViewT<AS> v;
    v.T = (const __attribute__((address_space(AS))) dg_type *)(base + h.off_types);
    v.S = (const __attribute__((address_space(AS))) dg_struct *)(base + h.off_structs);
    v.F = (const __attribute__((address_space(AS))) dg_field *)(base + h.off_fields);
    v.N = (const __attribute__((address_space(AS))) dg_name *)(base + h.off_names);
    v.R = (const __attribute__((address_space(AS))) uint64_t *)(base + h.off_reqwords);
    v.P = base + h.off_pool;
    return v;
}

/* J2TState (native/thrift.h:164-170) without jp (no re-entry): 16 bytes.
 * u = J2TExtra: container {bp: low 32, size: high 32}; struct {inline
 * requires bits, or arena offset in the low 32}; field {field index}. */
struct Frame {
    uint32_t st; /* J_* | ST_* */
    uint32_t td; /* type index */
    uint64_t u;
};
template <class FR> DGI uint32_t fbp(const FR &x) { return (uint32_t)x.u; }
template <class FR> DGI uint32_t fsize(const FR &x) { return (uint32_t)(x.u >> 32); }
template <class FR> DGI void set_size(FR &x, uint32_t v) { x.u = (x.u & 0xffffffffull) | ((uint64_t)v << 32); }
typedef __attribute__((address_space(3))) Frame LFrame;

/* address-space-typed pointers: LDS (ds_*) or global (global_*), never flat */
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef const __attribute__((address_space(3))) uint64_t lds_u64;
typedef const __attribute__((address_space(1))) uint64_t glb_u64;

/* Per-lane workspace in device memory (rare paths only). */
struct Workspace {
    gu8 *dbuf;     /* 800 B big-decimal digits (internal/types/types.go:268) */
    gu8 *keybuf;   /* unquoted-key buffer (reference key cache) */
    uint32_t keycap;
    gu64 *reqarena;/* multi-word requires bitmaps */
    uint32_t reqcap;   /* words */
};


/* One message's bytes, read through a cached, aligned 8-byte window. `w8` is
 * the 8-aligned word at or below the message start, `off0` the start's byte
 * offset from it. Reads at i >= n yield 0. Whole aligned words are read, so
 * up to 7 bytes before/after the message must be readable (arena padding). */
template <class W, class I = int64_t>
struct SrcT {
    typedef I idx;   /* position type: int32_t when the whole source is an LDS window */
    const W *w8;
    I off0;
    I n;
    I tag;
    uint64_t word;
    DGI void init(const W *words, I off, I len)
    {
        w8 = words;
        off0 = off;
        n = len;
        tag = -1;
        word = 0;
    }
    DGI uint64_t wordk(I k)
    {
        if (k != tag) {
            tag = k;
            word = w8[k];
        }
        return word;
    }
    DGI uint8_t raw(I i)
    {
        I b = off0 + i;
        return (uint8_t)(wordk(b >> 3) >> ((b & 7) << 3));
    }
    DGI uint8_t at(I i) { return (std::make_unsigned_t<I>)i < (std::make_unsigned_t<I>)n ? raw(i) : 0; }
    /* 8 bytes at [i, i+8) (caller guarantees i + 8 <= n), first byte lowest */
    DGI uint64_t get8(I i)
    {
        I b = off0 + i;
        I k = b >> 3;
        uint32_t sh = (uint32_t)(b & 7) << 3;
        uint64_t lo = wordk(k);
        if (sh == 0) return lo;
        uint64_t hi = wordk(k + 1);
        return (lo >> sh) | (hi << (64 - sh));
    }
    /* sub-view [s0, s0+len) of this message (same memory) */
    DGI SrcT sub(I s0, I len) const
    {
        SrcT r;
        r.init(w8, off0 + s0, len);
        return r;
    }
};

/* exact per-byte zero flags (0x80 in each zero byte, no false positives) */
/* SWAR on gfx950: the VALU is 32 bits wide and takes 32-bit literal
 * constants inline, while a 64-bit constant needs an SGPR pair (and under the
 * kernels' SGPR pressure, spill lanes: v_readlane/v_writelane churn in the
 * inner loops). So the byte-parallel helpers work on 32-bit halves with
 * replicated-byte literals; no carry ever crosses a byte, let alone a half. */
DGI uint32_t zb32(uint32_t v) { return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu); }
DGI uint64_t zbytes(uint64_t v)
{
    return (uint64_t)zb32((uint32_t)v) | ((uint64_t)zb32((uint32_t)(v >> 32)) << 32);
}
/* 0x80 in each byte of w equal to c */
DGI uint64_t eqbytes(uint64_t w, uint8_t c)
{
    const uint32_t cc = (uint32_t)c * 0x01010101u;
    return (uint64_t)zb32((uint32_t)w ^ cc) | ((uint64_t)zb32((uint32_t)(w >> 32) ^ cc) << 32);
}
/* 0xFF in every byte whose top bit is set in m (m: 0x80 flags only) */
DGI uint32_t ff32(uint32_t m) { return (m << 1) - (m >> 7); }

/* Thrift output with a hard slot bound and 8-byte write combining.
 * Bytes are assembled in `wbuf` (the word holding position len) and stored
 * as whole aligned words; back-patches of already-stored words (list/map
 * sizes, string lengths) go straight to memory. Writes past `cap` are
 * dropped while `len` keeps counting: the required size is reported on
 * overflow. */
struct Out {
    gu8 *b;
    uint64_t cap;
    uint64_t len;
    uint64_t wbuf;
    bool wide; /* slot base 8-aligned: word stores allowed */

    DGI void init(uint8_t *base, uint64_t c)
    {
        b = (gu8 *)(void *)base;
        cap = c;
        len = 0;
        wbuf = 0;
        wide = ((uintptr_t)base & 7) == 0;
    }
    /* the byte-wise edge cases (unaligned slot, last partial word of the
     * slot) are out of line: every write site inlines only the word store */
    static __device__ __noinline__ void store_bytes(gu8 *b, uint64_t a, uint64_t cap, uint64_t v)
    {
        for (int k = 0; k < 8; k++)
            if (a + k < cap) b[a + k] = (uint8_t)(v >> (8 * k));
    }
    static __device__ __noinline__ uint64_t load_bytes(const gu8 *b, uint64_t a, uint64_t cap)
    {
        uint64_t v = 0;
        for (int k = 0; k < 8; k++)
            if (a + k < cap) v |= (uint64_t)b[a + k] << (8 * k);
        return v;
    }
    DGI void store_word(uint64_t wi, uint64_t v)
    {
        uint64_t a = wi << 3;
        if (wide && a + 8 <= cap) *(gu64 *)(b + a) = v;
        else if (a < cap) store_bytes(b, a, cap, v);
    }
    DGI uint64_t load_word(uint64_t wi) const
    {
        uint64_t a = wi << 3;
        if (wide && a + 8 <= cap) return *(const gu64 *)(b + a);
        return a < cap ? load_bytes(b, a, cap) : 0;
    }
    /* append n (1..8) bytes given little-endian in v (first byte lowest) */
    DGI void wle(uint64_t v, uint32_t n)
    {
#ifdef DG_ABL_NOOUT
        len += n;
        wbuf ^= v;
        return;
#endif
        uint32_t used = (uint32_t)(len & 7);
        uint32_t sh = used << 3;
        if (n < 8) v &= (1ull << (n << 3)) - 1;
        uint64_t lo = (wbuf & ((1ull << sh) - 1)) | (v << sh);
        uint64_t hi = used ? (v >> (64 - sh)) : 0;
        uint64_t wi = len >> 3;
        len += n;
        if (used + n >= 8) {
            store_word(wi, lo);
            wbuf = hi;
        } else {
            wbuf = lo;
        }
    }
    DGI void w8(uint8_t v) { wle(v, 1); }
    DGI void w16(uint16_t v) { wle(__builtin_bswap16(v), 2); }
    DGI void w32(uint32_t v) { wle(__builtin_bswap32(v), 4); }
    DGI void w64(uint64_t v) { wle(__builtin_bswap64(v), 8); }
    /* reserve k (<= 8) bytes to be back-patched; returns their position */
    DGI uint64_t alloc(uint32_t k)
    {
        uint64_t s = len;
        wle(0, k);
        return s;
    }
    /* overwrite one already-written byte */
    DGI void patch8(uint64_t q, uint8_t v)
    {
        if (q >= (len & ~7ull)) {
            uint32_t sh = (uint32_t)(q & 7) << 3;
            wbuf = (wbuf & ~(0xFFull << sh)) | ((uint64_t)v << sh);
        } else if (q < cap) {
            b[q] = v;
        }
    }
    DGI void put32(uint64_t at, uint32_t v)
    {
        patch8(at, v >> 24);
        patch8(at + 1, v >> 16);
        patch8(at + 2, v >> 8);
        patch8(at + 3, v);
    }
    /* truncate to x <= len (the reference's buf->len = unwindPos) */
    DGI void set_len(uint64_t x)
    {
        if ((x >> 3) != (len >> 3)) wbuf = (x & 7) ? load_word(x >> 3) : 0;
        len = x;
    }
    DGI void finish()
    {
        if (len & 7) store_word(len >> 3, wbuf);
    }
};

/* x86 cvttsd2si (the reference's double->int casts, native/thrift.c:324-359) */
DGI int32_t cvt32(double d) { return (d > -2147483649.0 && d < 2147483648.0) ? (int32_t)d : INT32_MIN; }
DGI int64_t cvt64(double d)
{
    return (d >= -9223372036854775808.0 && d < 9223372036854775808.0) ? (int64_t)d : INT64_MIN;
}

/* ' ', '\t', '\n', '\r' as one shift of a 33-bit mask: no short-circuit
 * branches (a chain of || compiled to a branch tree with exec-mask SALU per
 * test, and sank the loads feeding it into the branches) */
DGI bool isspace_(uint8_t c) { return ((0x100002600ull >> (c & 63)) & (uint64_t)(c < 33)) != 0; }

/* advance_ns native/scanning.c:64-105 (+ lspace native/fastbytes.c:25-123):
 * 4 scalar probes, then a scan; note *p is left unchanged when the scan
 * reaches EOF (the reference returns before updating it). */
template <class S>
DGI uint8_t advance_ns(S &s, int64_t &p)
{
    int64_t vi = p;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (vi < s.n) {
            uint8_t c = s.raw(vi);
            if (!isspace_(c)) {
                p = vi + 1;
                return c;
            }
        }
        vi++;
    }
    if (vi >= s.n) {
        p = vi;
        return 0;
    }
    while (vi < s.n) {
        uint8_t c = s.raw(vi);
        if (!isspace_(c)) {
            p = vi + 1;
            return c;
        }
        vi++;
    }
    return 0;
}

/* advance_dword native/scanning.c:107-128 (long vs size_t compare: unsigned) */
template <class S>
DGI int64_t advance_dword(S &s, int64_t &p, int64_t dec, int64_t ret, uint32_t val)
{
    if ((uint64_t)p > (uint64_t)(s.n + dec - 4)) {
        p = s.n;
        return -(int64_t)E_EOF;
    }
    uint32_t w = (uint32_t)s.at(p - dec) | ((uint32_t)s.at(p - dec + 1) << 8) |
                 ((uint32_t)s.at(p - dec + 2) << 16) | ((uint32_t)s.at(p - dec + 3) << 24);
    if (w == val) {
        p += 4 - dec;
        return ret;
    }
    p -= dec;
    while (s.at(p) == (val & 0xff)) {
        val >>= 8;
        ++p;
    }
    return -(int64_t)E_INVAL;
}

/* advance_string native/scanning.c:130-375: index after the closing quote;
 * esc = whether a backslash occurs inside the string. 8 bytes per step: the
 * window word is tested for '"' and '\\' with exact SWAR byte compares. */
template <class S>
DGI int64_t advance_string(S &s, int64_t p0, bool &esc)
{
    typedef typename S::idx I;
    esc = false;
    const I p = (I)p0;
    if (s.n == p) return -(int64_t)E_EOF;
    I i = p;
    while (i < s.n) {
        I b = s.off0 + i;
        I k = b >> 3;
        uint64_t w = s.wordk(k);
        uint64_t m = eqbytes(w, '"') | eqbytes(w, '\\');
        m &= ~0ull << ((b & 7) << 3);
        I lim = s.n - (k * 8 - s.off0); /* bytes of this word inside the message */
        if (lim < 8) m &= (1ull << (lim << 3)) - 1;
        if (m == 0) {
            i = (k + 1) * 8 - s.off0;
            continue;
        }
        int j = __builtin_ctzll(m) >> 3;
        I pos = k * 8 + j - s.off0;
        if ((uint8_t)(w >> (j << 3)) == '"') return pos + 1;
        esc = true;
        if (pos + 1 >= s.n) return -(int64_t)E_EOF;
        i = pos + 2;
    }
    return -(int64_t)E_EOF;
}

DGI int hexv(uint8_t c)
{
    if (c >= '0' && c <= '9') return c - '0';
    uint8_t l = c | 0x20;
    if (l >= 'a' && l <= 'f') return l - 'a' + 10;
    return -1;
}
template <class S>
DGI bool hex4(S &s, int64_t i, uint32_t &v)
{
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int h = hexv(s.at(i + k));
        if (h < 0) return false;
        r = (r << 4) | (uint32_t)h;
    }
    v = r;
    return true;
}

/* unquote native/parsing.c:702-945 with flags == 0, over src[s0, s0+nb).
 * Writes through `dst` (an Out at a position, or a plain buffer); returns
 * the unquoted length or -errcode. */
template <class S, class Sink>
DGI int64_t unquote(S &src, int64_t s0, int64_t nb, Sink &dst)
{
    int64_t o = 0, i = s0;
    while (nb > 0) {
        uint8_t c0 = src.raw(i);
        if (c0 != '\\') {
            dst(o++, c0);
            i++;
            nb--;
            continue;
        }
        i += 2;
        nb -= 2;
        if (nb < 0) return -(int64_t)E_EOF;
        uint8_t c = src.raw(i - 1);
        uint8_t cc;
        switch (c) { /* _UnquoteTab native/parsing.c:565-575 */
        case '/': cc = '/'; break;
        case '"': cc = '"'; break;
        case 'b': cc = '\b'; break;
        case 'f': cc = '\f'; break;
        case 'n': cc = '\n'; break;
        case 'r': cc = '\r'; break;
        case 't': cc = '\t'; break;
        case '\\': cc = '\\'; break;
        case 'u': cc = 0xff; break;
        default: return -(int64_t)E_ESCAPE;
        }
        if (cc != 0xff) {
            dst(o++, cc);
            continue;
        }
        if (nb < 4) return -(int64_t)E_EOF;
        uint32_t r0, r1;
        if (!hex4(src, i, r0)) return -(int64_t)E_INVAL;
        i += 4;
        nb -= 4;
        if (r0 <= 0x7f) {
            dst(o++, (uint8_t)r0);
            continue;
        }
        if (r0 <= 0x7ff) {
            dst(o++, 0xc0 | (r0 >> 6));
            dst(o++, 0x80 | (r0 & 0x3f));
            continue;
        }
        if (r0 < 0xd800 || r0 > 0xdfff) {
            dst(o++, 0xe0 | (r0 >> 12));
            dst(o++, 0x80 | ((r0 >> 6) & 0x3f));
            dst(o++, 0x80 | (r0 & 0x3f));
            continue;
        }
        if (nb < 6 || r0 > 0xdbff || src.raw(i) != '\\' || src.raw(i + 1) != 'u') return -(int64_t)E_UNICODE;
        if (!hex4(src, i + 2, r1)) return -(int64_t)E_INVAL;
        i += 6;
        nb -= 6;
        if (r1 < 0xdc00 || r1 > 0xdfff) return -(int64_t)E_UNICODE;
        r0 = ((r0 - 0xd800) << 10) + (r1 - 0xdc00) + 0x10000;
        dst(o++, 0xf0 | (r0 >> 18));
        dst(o++, 0x80 | ((r0 >> 12) & 0x3f));
        dst(o++, 0x80 | ((r0 >> 6) & 0x3f));
        dst(o++, 0x80 | (r0 & 0x3f));
    }
    return o;
}

struct OutSink {
    Out *o;
    DGI void operator()(int64_t, uint8_t v) { o->w8(v); } /* sequential */
};
struct BufSink {
    gu8 *b;
    int64_t cap;
    bool over;
    DGI void operator()(int64_t i, uint8_t v)
    {
        if (i < cap) b[i] = v;
        else over = true;
    }
};

/* Extension DG_F_VALIDATE_UTF8: offset of the first invalid UTF-8 sequence in
 * src[s0, s0+n) as utf8_validate (native/utf8.c:101-212) defines validity, or
 * -1. ASCII runs are skipped 8 bytes at a time. */
template <class S>
DGI int64_t utf8_check(S &src, int64_t s0, int64_t n)
{
    int64_t i = 0;
    while (i < n) {
        if (i + 8 <= n) {
            uint64_t hb = src.get8(s0 + i) & 0x8080808080808080ull;
            if (hb == 0) {
                i += 8;
                continue;
            }
            i += __builtin_ctzll(hb) >> 3;
        } else if (src.raw(s0 + i) < 0x80) {
            i++;
            continue;
        }
        uint8_t c = src.raw(s0 + i);
        int size;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) {
            size = 2;
        } else if (c >= 0xE0 && c <= 0xEF) {
            size = 3;
            if (c == 0xE0) lo = 0xA0;
            else if (c == 0xED) hi = 0x9F;
        } else if (c >= 0xF0 && c <= 0xF4) {
            size = 4;
            if (c == 0xF0) lo = 0x90;
            else if (c == 0xF4) hi = 0x8F;
        } else {
            return i;
        }
        if (n - i < size) return i;
        uint8_t c1 = src.raw(s0 + i + 1);
        if (c1 < lo || c1 > hi) return i;
        for (int k = 2; k < size; k++) {
            uint8_t ck = src.raw(s0 + i + k);
            if (ck < 0x80 || ck > 0xBF) return i;
        }
        i += size;
    }
    return -1;
}

/* ---- base64: b64decode(mode=0) native/base64.c:659-817 ---- */
DGI int b64v(uint8_t c)
{
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
}

/* decode_block native/base64.c:539-657 over src[s0 + ...]; ipp/op relative;
 * output appended to o (op counts the decoded bytes). */
template <class S>
DGI int64_t decode_block(S &src, int64_t s0, int64_t ie, int64_t &ipp, Out &o, int64_t &op)
{
    int nb = 0;
    uint32_t v0 = 0;
    int64_t ip = ipp;
    while (nb < 4 && ip < ie) {
        uint8_t ch = src.raw(s0 + ip);
        if (ch == '\r' || ch == '\n') {
            ip++;
            continue;
        }
        int id = b64v(ch);
        if (id < 0) break;
        ip++;
        nb++;
        v0 = (v0 << 6) | (uint32_t)id;
    }
    if (nb == 1) return ip - ipp + 1;
    if (nb < 4) {
        if (ip == ie) return ip - ipp + 1;
        if (nb == 3) {
            if (src.raw(s0 + ip++) != '=') return ip - ipp;
        } else {
            if (ip >= ie - 1) return ip - ipp + 1;
            if (src.raw(s0 + ip++) != '=') return ip - ipp;
            if (src.raw(s0 + ip++) != '=') return ip - ipp;
        }
        if (ip < ie) return ip - ipp + 1;
        v0 <<= 6 * (4 - nb);
    }
    if (nb >= 2) {
        /* bytes (v0>>16, v0>>8, v0) of which nb-1 are kept */
        uint64_t le = ((v0 >> 16) & 0xff) | (((v0 >> 8) & 0xff) << 8) | ((uint64_t)(v0 & 0xff) << 16);
        o.wle(le, (uint32_t)(nb - 1));
    } else if (op > 0) {
        o.set_len(o.len - 1); /* nb == 0 ("==" alone): *opp = op - 1 */
    }
    ipp = ip;
    op = op + nb - 1;
    return 0;
}

/* Decodes src[s0, s0+nb), appending to o; returns the decoded length or
 * (ib - ip - dv) < 0 like the reference. */
template <class S>
DGI int64_t b64decode_from(Out &o, S &src, int64_t s0, int64_t nb, int64_t ip, int64_t op)
{
    /* whole 4-char quanta of alphabet characters: decode_block on such a
     * quantum consumes exactly it (the reference's 8/4-byte loops) */
    while (ip + 4 <= nb) {
        int a = b64v(src.raw(s0 + ip)), b = b64v(src.raw(s0 + ip + 1));
        int c = b64v(src.raw(s0 + ip + 2)), d = b64v(src.raw(s0 + ip + 3));
        if ((a | b | c | d) < 0) break;
        uint32_t v = ((uint32_t)a << 18) | ((uint32_t)b << 12) | ((uint32_t)c << 6) | (uint32_t)d;
        o.wle(((v >> 16) & 0xff) | (((v >> 8) & 0xff) << 8) | ((uint64_t)(v & 0xff) << 16), 3);
        ip += 4;
        op += 3;
    }
    while (ip < nb) {
        int64_t dv = decode_block(src, s0, nb, ip, o, op);
        if (dv != 0) return -ip - dv;
    }
    return op;
}
template <class S>
DGI int64_t b64decode(Out &o, S &src, int64_t s0, int64_t nb)
{
#ifdef DG_ABL_NOB64
    return (nb / 4) * 3;
#endif
    if (nb == 0) return 0;
    return b64decode_from(o, src, s0, nb, 0, 0);
}

/* ====================================================================== */
/* numbers                                                                 */
/* ====================================================================== */
__device__ __constant__ static const double P10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                                      1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                                      1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

DGI double with_sign(double v, int sgn)
{
    uint64_t b = __double_as_longlong(v);
    b |= ((uint64_t)(int64_t)sgn) >> 63 << 63;
    return __longlong_as_double(b);
}

/* is_atof_exact native/scanning.c:883-926 (IEEE mul/div, no FMA contraction) */
DGI bool is_atof_exact(uint64_t man, int exp, int sgn, double &val)
{
    val = (double)man;
    if (man >> 52 != 0) return false;
    val = with_sign(val, sgn);
    if (exp == 0 || man == 0) return true;
    if (exp > 0 && exp <= 15 + 22) {
        if (exp > 22) {
            val = __dmul_rn(val, P10[exp - 22]);
            exp = 22;
        }
        if (val > 1e15 || val < -1e15) return false;
        val = __dmul_rn(val, P10[exp]);
        return true;
    }
    if (exp < 0 && exp >= -22) {
        val = __ddiv_rn(val, P10[-exp]);
        return true;
    }
    return false;
}

/* atof_eisel_lemire64 native/atof_eisel_lemire.c:74-167; p_hi = the high
 * half of the 128-bit power (DG_POW10_M128[exp10 + 348][1]), supplied by the
 * caller (from the table, or from a window of it a kernel holds in LDS) */
DGI bool eisel_lemire_p(uint64_t mant, int exp10, int sgn, double &val, uint64_t p_hi)
{
    int clz = mant ? __clzll(mant) : 64;
    mant = clz < 64 ? mant << clz : mant;
    uint64_t ret_exp2 = ((uint64_t)(int64_t)((217706 * exp10) >> 16) + 64 + 1023) - (uint64_t)clz;
    uint64_t x_hi = __umul64hi(mant, p_hi), x_lo = mant * p_hi;
    if ((x_hi & 0x1FF) == 0x1FF && (x_lo + mant) < mant) {
        uint64_t p_lo = DG_POW10_M128[exp10 + 348][0];
        uint64_t y_hi = __umul64hi(mant, p_lo), y_lo = mant * p_lo;
        uint64_t merged_hi = x_hi, merged_lo = x_lo + y_hi;
        if (merged_lo < x_lo) merged_hi++;
        if ((merged_hi & 0x1FF) == 0x1FF && (merged_lo + 1) == 0 && (y_lo + mant) < mant) return false;
        x_hi = merged_hi;
        x_lo = merged_lo;
    }
    int msb = (int)(x_hi >> 63);
    uint64_t ret_man = x_hi >> (msb + 9);
    ret_exp2 -= 1 ^ msb;
    if ((x_lo == 0) && ((x_hi & 0x1FF) == 0) && ((ret_man & 3) == 1)) return false;
    ret_man += ret_man & 1;
    ret_man >>= 1;
    if ((ret_man >> 53) > 0) {
        ret_man >>= 1;
        ret_exp2 += 1;
    }
    if ((ret_exp2 - 1) >= (0x7FF - 1)) return false;
    uint64_t bits = (ret_exp2 << 52) | (ret_man & 0x000FFFFFFFFFFFFFull);
    if (sgn == -1) bits |= 1ull << 63;
    val = __longlong_as_double(bits);
    return true;
}
DGI bool eisel_lemire(uint64_t mant, int exp10, int sgn, double &val)
{
    if (exp10 < -348 || exp10 > 347) return false;
    return eisel_lemire_p(mant, exp10, sgn, val, DG_POW10_M128[exp10 + 348][1]);
}

/* ---- atof_native: big-decimal slow path native/atof_native.c:17-424 ---- */
constexpr int DCAP = 800;
struct Decimal {
    gu8 *d;
    int nd, dp, neg, trunc;
};
DGI void dtrim(Decimal &d)
{
    while (d.nd > 0 && d.d[d.nd - 1] == '0') d.nd--;
    if (d.nd == 0) d.dp = 0;
}
DGN void right_shift(Decimal &d, uint32_t k)
{
    int r = 0, w = 0;
    uint64_t n = 0;
    for (; n >> k == 0; r++) {
        if (r >= d.nd) {
            if (n == 0) {
                d.nd = 0;
                return;
            }
            while (n >> k == 0) {
                n *= 10;
                r++;
            }
            break;
        }
        n = n * 10 + d.d[r] - '0';
    }
    d.dp -= r - 1;
    uint64_t mask = (1ull << k) - 1;
    for (; r < d.nd; r++) {
        uint64_t dig = n >> k;
        n &= mask;
        d.d[w++] = (uint8_t)(dig + '0');
        n = n * 10 + d.d[r] - '0';
    }
    while (n > 0) {
        uint64_t dig = n >> k;
        n &= mask;
        if (w < DCAP) d.d[w++] = (uint8_t)(dig + '0');
        else if (dig > 0) d.trunc = 1;
        n *= 10;
    }
    d.nd = w;
    dtrim(d);
}
DGI bool prefix_is_less(const gu8 *b, const char *s, int bn)
{
    int i = 0;
    for (; i < bn; i++) {
        if (s[i] == '\0') return false;
        if (b[i] != (uint8_t)s[i]) return b[i] < (uint8_t)s[i];
    }
    return s[i] != '\0';
}
DGN void left_shift(Decimal &d, uint32_t k)
{
    int delta = DG_LSHIFT_DELTA[k];
    if (prefix_is_less(d.d, DG_LSHIFT_CUTOFF[k], d.nd)) delta--;
    int r = d.nd, w = d.nd + delta;
    uint64_t n = 0;
    for (r--; r >= 0; r--) {
        n += (uint64_t)(d.d[r] - '0') << k;
        uint64_t quo = n / 10, rem = n - 10 * quo;
        w--;
        if (w < DCAP) d.d[w] = (uint8_t)(rem + '0');
        else if (rem != 0) d.trunc = 1;
        n = quo;
    }
    while (n > 0) {
        uint64_t quo = n / 10, rem = n - 10 * quo;
        w--;
        if (w < DCAP) d.d[w] = (uint8_t)(rem + '0');
        else if (rem != 0) d.trunc = 1;
        n = quo;
    }
    d.nd += delta;
    if (d.nd >= DCAP) d.nd = DCAP;
    d.dp += delta;
    dtrim(d);
}
DGI void decimal_shift(Decimal &d, int k)
{
    if (d.nd == 0 || k == 0) return;
    if (k > 0) {
        while (k > 60) {
            left_shift(d, 60);
            k -= 60;
        }
        if (k) left_shift(d, k);
    }
    if (k < 0) {
        while (k < -60) {
            right_shift(d, 60);
            k += 60;
        }
        if (k) right_shift(d, -k);
    }
}
DGI int should_roundup(const Decimal &d, int nd)
{
    if (nd < 0 || nd >= d.nd) return 0;
    if (d.d[nd] == '5' && nd + 1 == d.nd) {
        if (d.trunc) return 1;
        return nd > 0 && (d.d[nd - 1] - '0') % 2 != 0;
    }
    return d.d[nd] >= '5';
}
__device__ __constant__ static const int POW_TAB[9] = {1, 3, 6, 9, 13, 16, 19, 23, 26};

/* decimal_set + decimal_to_f64 native/atof_native.c:71-416 */
template <class S>
DGN double atof_native(S src, int64_t s0, int64_t len, gu8 *dbuf)
{
    Decimal d;
    d.d = dbuf;
    for (int i = 0; i < DCAP; i++) dbuf[i] = 0;
    d.nd = d.dp = d.neg = d.trunc = 0;
    int64_t i = 0;
#define CH(k) src.at(s0 + (k))
    if (CH(i) == '-') {
        i++;
        d.neg = 1;
    }
    int saw_dot = 0;
    for (; i < len; i++) {
        uint8_t c = CH(i);
        if ('0' <= c && c <= '9') {
            if (c == '0' && d.nd == 0) {
                d.dp--;
                continue;
            }
            if (d.nd < DCAP) d.d[d.nd++] = c;
            else if (c != '0') d.trunc = 1;
        } else if (c == '.') {
            saw_dot = 1;
            d.dp = d.nd;
        } else
            break;
    }
    if (!saw_dot) d.dp = d.nd;
    if (i < len && (CH(i) == 'e' || CH(i) == 'E')) {
        int exp = 0, esgn = 1;
        i++;
        if (CH(i) == '+') i++;
        else if (CH(i) == '-') {
            i++;
            esgn = -1;
        }
        for (; i < len && ('0' <= CH(i) && CH(i) <= '9') && exp < 10000; i++) exp = exp * 10 + (CH(i) - '0');
        d.dp += exp * esgn;
    }
#undef CH
    int exp2 = 0;
    uint64_t mant = 0;
    int n;
    if (d.nd == 0) {
        exp2 = -1023;
        goto out;
    }
    if (d.dp > 310) goto overflow;
    if (d.dp < -330) {
        exp2 = -1023;
        goto out;
    }
    while (d.dp > 0) {
        n = d.dp >= 9 ? 27 : POW_TAB[d.dp];
        decimal_shift(d, -n);
        exp2 += n;
    }
    while ((d.dp < 0) || ((d.dp == 0) && (d.d[0] < '5'))) {
        n = -d.dp >= 9 ? 27 : POW_TAB[-d.dp];
        decimal_shift(d, n);
        exp2 -= n;
    }
    exp2--;
    if (exp2 < -1022) {
        n = -1022 - exp2;
        decimal_shift(d, -n);
        exp2 += n;
    }
    if ((exp2 + 1023) >= 0x7FF) goto overflow;
    decimal_shift(d, 53);
    {
        /* rounded_integer native/atof_native.c:302-319 */
        if (d.dp > 20) mant = 0xFFFFFFFFFFFFFFFFull;
        else {
            int j;
            mant = 0;
            for (j = 0; j < d.dp && j < d.nd; j++) mant = mant * 10 + (d.d[j] - '0');
            for (; j < d.dp; j++) mant *= 10;
            if (should_roundup(d, d.dp)) mant++;
        }
    }
    if (mant == (2ull << 52)) {
        mant >>= 1;
        exp2++;
        if ((exp2 + 1023) >= 0x7FF) goto overflow;
    }
    if ((mant & (1ull << 52)) == 0) exp2 = -1023;
    goto out;
overflow:
    mant = 0;
    exp2 = 0x7FF - 1023;
out:
    uint64_t bits = mant & 0x000FFFFFFFFFFFFFull;
    bits |= (uint64_t)((exp2 + 1023) & 0x7FF) << 52;
    if (d.neg) bits |= 1ull << 63;
    return __longlong_as_double(bits);
}

struct JState {
    int64_t vt;
    double dv;
    int64_t iv;
};

/* vnumber native/scanning.c:958-1083 */
template <class S>
DGI void vnumber(S &src, int64_t &p, JState &ret, gu8 *dbuf)
{
#ifdef DG_ABL_NONUM
    {
        int64_t i = p;
        uint64_t acc = 0;
        while (i < src.n) {
            uint8_t c = src.raw(i);
            if (!((c >= '0' && c <= '9') || c == '-' || c == '.' || c == 'e' || c == 'E' || c == '+')) break;
            acc = acc * 10 + c;
            i++;
        }
        p = i;
        ret.vt = V_INTEGER;
        ret.iv = (int64_t)acc;
        ret.dv = 0;
        return;
    }
#endif
    int sgn = 1;
    uint64_t man = 0;
    int man_nd = 0, exp10 = 0, trunc = 0;
    int64_t i = p, n = src.n;
    ret.vt = V_INTEGER;
    ret.dv = 0.0;
    ret.iv = 0;
    if (i >= n) {
        p = n;
        ret.vt = -(int64_t)E_EOF;
        return;
    }
    uint8_t c = src.raw(i);
    if (c == '-') {
        i++;
        sgn = -1;
        if (i >= n) {
            p = n;
            ret.vt = -(int64_t)E_EOF;
            return;
        }
        c = src.raw(i);
    }
    if (c < '0' || c > '9') {
        p = i;
        ret.vt = -(int64_t)E_INVAL;
        return;
    }
    if (c == '0') {
        uint8_t c1 = src.at(i + 1);
        if (c1 != '.' && c1 != 'e' && c1 != 'E') {
            p = ++i;
            return;
        }
    }
    while (i < n) {
        c = src.raw(i);
        if (c < '0' || c > '9') break;
        if (man_nd < 19) {
            man = man * 10 + (c - '0');
            man_nd++;
        } else
            exp10++;
        i++;
    }
    if (exp10 > 0) trunc = 1;
    if (i < n && src.raw(i) == '.') {
        i++;
        ret.vt = V_DOUBLE;
        if (i >= n) {
            p = n;
            ret.vt = -(int64_t)E_EOF;
            return;
        }
        c = src.raw(i);
        if (c < '0' || c > '9') {
            p = i;
            ret.vt = -(int64_t)E_INVAL;
            return;
        }
    }
    if (man == 0 && exp10 == 0) {
        while (i < n && src.raw(i) == '0') {
            i++;
            exp10--;
        }
        man = 0;
        man_nd = 0;
    }
    while (i < n && man_nd < 19) {
        c = src.raw(i);
        if (c < '0' || c > '9') break;
        man = man * 10 + (c - '0');
        man_nd++;
        exp10--;
        i++;
    }
    while (i < n) {
        c = src.raw(i);
        if (c < '0' || c > '9') break;
        trunc = 1;
        i++;
    }
    if (i < n && (src.raw(i) == 'e' || src.raw(i) == 'E')) {
        int esm = 1, exp = 0;
        i++;
        ret.vt = V_DOUBLE;
        if (i >= n) {
            p = n;
            ret.vt = -(int64_t)E_EOF;
            return;
        }
        c = src.raw(i);
        if (c == '+' || c == '-') {
            esm = c == '+' ? 1 : -1;
            i++;
            if (i >= n) {
                p = n;
                ret.vt = -(int64_t)E_EOF;
                return;
            }
            c = src.raw(i);
        }
        if (c < '0' || c > '9') {
            p = i;
            ret.vt = -(int64_t)E_INVAL;
            return;
        }
        while (i < n) {
            c = src.raw(i);
            if (c < '0' || c > '9') break;
            if (exp < 10000) exp = exp * 10 + (c - '0');
            i++;
        }
        exp10 += exp * esm;
    } else if (ret.vt == V_INTEGER) {
        /* is_overflow native/scanning.c:950-956 */
        bool ovf = exp10 != 0 || ((man >> 63) == 1 && (((uint64_t)(int64_t)sgn) & man) != (1ull << 63));
        if (!ovf) {
            ret.iv = (int64_t)(man * (uint64_t)(int64_t)sgn);
            ret.dv = with_sign((double)man, sgn);
            p = i;
            return;
        }
        ret.vt = V_DOUBLE;
    }
    /* atof_fast native/scanning.c:928-948 */
    double val = 0;
    bool ok = false;
    if (is_atof_exact(man, exp10, sgn, val)) ok = true;
    else if (eisel_lemire(man, exp10, sgn, val)) {
        double vu;
        if (!trunc || (eisel_lemire(man + 1, exp10, sgn, vu) && vu == val)) ok = true;
    }
    if (!ok) val = atof_native(src, p, i - p, dbuf);
    if ((__double_as_longlong(val) << 1) == 0xFFE0000000000000ull) ret.vt = -(int64_t)E_FLOAT_INF;
    ret.dv = val;
    p = i;
}

/* ====================================================================== */
/* skipping unknown values: skip_one/fsm_exec native/scanning.c:1134-1631  */
/* ====================================================================== */
DGI bool numch(uint8_t c)
{
    return (c >= '0' && c <= '9') || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-';
}

/* skip_number native/scanning.c:1317-1535 as the AVX2 build decomposes it:
 * 32-byte blocks while >= 32 bytes remain, then 16-byte blocks, then scalar. */
template <class S>
DGN int64_t skip_number(S src, int64_t base, int64_t nb)
{
    int64_t di = -1, ei = -1, si = -1;
    int64_t off = 0;
    if (nb == 0) return -1;
    if (src.raw(base) == '0' && (nb == 1 || (src.raw(base + 1) != '.' && src.raw(base + 1) != 'e' && src.raw(base + 1) != 'E'))) return 1;
    for (int W = 32; W >= 16; W -= 16) {
        while (nb >= W) {
            uint32_t md = 0, me = 0, ms = 0, v;
            int i = W;
            for (int k = 0; k < W; k++) {
                uint8_t c = src.raw(base + off + k);
                if (!numch(c)) {
                    i = k;
                    break;
                }
                if (c == '.') md |= 1u << k;
                else if (c == 'e' || c == 'E') me |= 1u << k;
                else if (c == '+' || c == '-') ms |= 1u << k;
            }
            if ((v = md & (md - 1)) != 0) return -(off + __builtin_ctz(v) + 1);
            if ((v = me & (me - 1)) != 0) return -(off + __builtin_ctz(v) + 1);
            if ((v = ms & (ms - 1)) != 0) return -(off + __builtin_ctz(v) + 1);
            if (md) {
                if (di == -1) di = off + __builtin_ctz(md);
                else return -(off + __builtin_ctz(md) + 1);
            }
            if (me) {
                if (ei == -1) ei = off + __builtin_ctz(me);
                else return -(off + __builtin_ctz(me) + 1);
            }
            if (ms) {
                if (si == -1) si = off + __builtin_ctz(ms);
                else return -(off + __builtin_ctz(ms) + 1);
            }
            if (i != W) {
                off += i;
                goto check_index;
            }
            off += W;
            nb -= W;
        }
    }
    while (nb-- > 0) {
        uint8_t c = src.raw(base + off++);
        if (c >= '0' && c <= '9') continue;
        int64_t *iv = c == '.' ? &di : (c == 'e' || c == 'E') ? &ei : (c == '+' || c == '-') ? &si : nullptr;
        if (!iv) {
            off--;
            goto check_index;
        }
        if (*iv == -1) *iv = off - 1;
        else return -off;
    }
check_index:
    if (di == 0 || si == 0 || ei == 0) return -1;
    if (di == off - 1 || si == off - 1 || ei == off - 1) return -off;
    if (si > 0 && ei != si - 1) return -si - 1;
    if (di >= 0 && ei >= 0 && di > ei - 1) return -di - 1;
    if (di >= 0 && ei >= 0 && di == ei - 1) return -ei - 1;
    return off;
}

template <class S>
DGI int64_t skip_string(S &s, int64_t &p)
{
    bool esc;
    int64_t q = p - 1;
    int64_t e = advance_string(s, p, esc);
    if (e >= 0) {
        p = e;
        return q;
    }
    p = s.n;
    return e;
}

/* skip-FSM states (native/scanning.h:22-28); frames below the top are
 * always ARR or OBJ, so the stack is a bit per level (1 = OBJ) plus the top
 * state. `bits` holds `cap` levels. Returns vi (>=0) or -errcode; returns
 * -0x7fff when the bit stack is exhausted (caller reports DG_ST_DEEP). */
enum { FV = 0, FARR = 1, FOBJ = 2, FKEY = 3, FELEM = 4, FARR0 = 5, FOBJ0 = 6 };
constexpr int64_t SKIP_DEEP = -0x7fff;

struct SkipRes {
    int64_t r; /* vi >= 0, -errcode, or SKIP_DEEP */
    int64_t p; /* position after the skip (or at the error) */
};

/* Levels 0..63 of the container bit-stack live in a register; deeper levels
 * in `bits` (device workspace, deep pass only). */
template <class S>
DGN SkipRes skip_one(S s, int64_t p, gu64 *bits, uint32_t cap)
{
    uint32_t sp = 1;
    int top = FV;
    int64_t vi = -1;
    uint64_t low = 0;
    auto below_kind = [&](uint32_t lvl) -> int {
        uint64_t w = lvl < 64 ? low : bits[(lvl >> 6) - 1];
        return ((w >> (lvl & 63)) & 1) ? FOBJ : FARR;
    };
    auto push = [&](int newtop) -> int64_t {
        /* the current top (ARR/OBJ) becomes level sp-1 */
        if (sp >= MAX_RECURSE) return -(int64_t)E_RECURSE_MAX;
        if (sp > cap) return SKIP_DEEP;
        uint32_t lvl = sp - 1;
        uint64_t m = 1ull << (lvl & 63);
        if (lvl < 64) {
            low = top == FOBJ ? (low | m) : (low & ~m);
        } else {
            gu64 *w = &bits[(lvl >> 6) - 1];
            *w = top == FOBJ ? (*w | m) : (*w & ~m);
        }
        sp++;
        top = newtop;
        return 0;
    };
    auto drop = [&]() {
        sp--;
        if (sp) top = below_kind(sp - 1);
    };
    while (sp) {
        uint8_t ch = advance_ns(s, p);
        if (vi == -1) vi = p - 1;
        switch (top) {
        default: /* FV */
            drop();
            break;
        case FARR:
            if (ch == ']') {
                drop();
                continue;
            }
            if (ch == ',') {
                int64_t r = push(FV);
                if (r) return SkipRes{r, p};
                continue;
            }
            return SkipRes{-(int64_t)E_INVAL, p};
        case FOBJ:
            if (ch == '}') {
                drop();
                continue;
            }
            if (ch == ',') {
                int64_t r = push(FKEY);
                if (r) return SkipRes{r, p};
                continue;
            }
            return SkipRes{-(int64_t)E_INVAL, p};
        case FKEY: {
            if (ch != '"') return SkipRes{-(int64_t)E_INVAL, p};
            top = FELEM;
            int64_t r = skip_string(s, p);
            if (r < 0) return SkipRes{r, p};
            continue;
        }
        case FELEM:
            if (ch != ':') return SkipRes{-(int64_t)E_INVAL, p};
            top = FV;
            continue;
        case FARR0:
            if (ch == ']') {
                drop();
                continue;
            }
            top = FARR;
            break;
        case FOBJ0:
            if (ch == '}') {
                drop();
                continue;
            }
            if (ch == '"') {
                top = FOBJ;
                int64_t r = skip_string(s, p);
                if (r < 0) return SkipRes{r, p};
                r = push(FELEM);
                if (r) return SkipRes{r, p};
                continue;
            }
            return SkipRes{-(int64_t)E_INVAL, p};
        }
        /* value, with `top` already replaced/dropped as the reference does */
        switch (ch) {
        case '0': case '1': case '2': case '3': case '4':
        case '5': case '6': case '7': case '8': case '9': {
            int64_t i = p - 1; /* skip_positive native/scanning.c:1616-1631 */
            int64_t r = skip_number(s, i, s.n - i);
            if (r < 0) {
                p -= r + 2;
                return SkipRes{-(int64_t)E_INVAL, p};
            }
            p += r - 1;
            break;
        }
        case '-': {
            int64_t i = p; /* skip_negative native/scanning.c:1599-1614 */
            int64_t r = skip_number(s, i, s.n - i);
            if (r < 0) {
                p -= r + 1;
                return SkipRes{-(int64_t)E_INVAL, p};
            }
            p += r;
            break;
        }
        case 'n': {
            int64_t r = advance_dword(s, p, 1, p - 1, VS_NULL);
            if (r < 0) return SkipRes{r, p};
            break;
        }
        case 't': {
            int64_t r = advance_dword(s, p, 1, p - 1, VS_TRUE);
            if (r < 0) return SkipRes{r, p};
            break;
        }
        case 'f': {
            int64_t r = advance_dword(s, p, 0, p - 1, VS_ALSE);
            if (r < 0) return SkipRes{r, p};
            break;
        }
        case '[': {
            if (sp == 0) { sp = 1; top = FARR0; break; }
            int64_t r = push(FARR0);
            if (r) return SkipRes{r, p};
            break;
        }
        case '{': {
            if (sp == 0) { sp = 1; top = FOBJ0; break; }
            int64_t r = push(FOBJ0);
            if (r) return SkipRes{r, p};
            break;
        }
        case '"': {
            int64_t r = skip_string(s, p);
            if (r < 0) return SkipRes{r, p};
            break;
        }
        case 0:
            return SkipRes{-(int64_t)E_EOF, p};
        default:
            return SkipRes{-(int64_t)E_INVAL, p};
        }
    }
    return SkipRes{vi, p};
}

}  // namespace dg
