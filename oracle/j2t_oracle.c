/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
 *
 * j2t_oracle.c: a plain-C (scalar, no SIMD) restatement of the reference's
 * JSON -> Thrift-binary path, conv/j2t BinaryConv.Do over native j2t_fsm_exec,
 * reading the flattened dg_desc v1 descriptor (include/dgj2t_desc.h).
 * Every function cites the reference file:line it restates. It is pinned
 * byte-for-byte against the reference engine itself (oracle/_ref, built by
 * oracle/Makefile from /root/reference/native) and against tests/golden/.
 *
 * Conventions shared with the GPU path:
 *  - reading src[i] for i >= len yields 0 (the reference reads one byte past
 *    the end in check_leading_zero; the harness pads with NUL);
 *  - output buffers never run out (the reference's OOM re-entry is a
 *    transparent retry in Go, conv/j2t/impl_amd64.go:199-226);
 *  - host callbacks ERR_HM and ERR_HM_END are returned as codes; ERR_VM_END
 *    is served like the Go host does for the test mappings (vm_host.h).
 */
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dgj2t_desc.h"
#include "../dynamicgo_amd/csrc/dg_tables.h"

/* ---- error codes native/native.h:47-70 ---- */
enum { E_EOF = 1, E_INVAL = 2, E_ESCAPE = 3, E_UNICODE = 4, E_OVERFLOW = 5, E_NUMBER_FMT = 6,
       E_RECURSE_MAX = 7, E_FLOAT_INF = 8, E_DISMATCH_TYPE = 9, E_NULL_REQUIRED = 10,
       E_UNSUPPORT_THRIFT_TYPE = 11, E_UNKNOWN_FIELD = 12, E_DISMATCH_TYPE2 = 13,
       E_DECODE_BASE64 = 14, E_HM = 19, E_UNSUPPORT_VM_TYPE = 20, E_HM_END = 21, E_VM_END = 24 };
enum { V_EOF = 1, V_DOUBLE = 8, V_INTEGER = 9 };
/* flags native/thrift.h:23-32 */
#define F_ALLOW_UNKNOWN 1ull
#define F_WRITE_DEFAULT (1ull << 1)
#define F_ENABLE_VM (1ull << 2)
#define F_ENABLE_HM (1ull << 3)
#define F_ENABLE_I2S (1ull << 4)
#define F_WRITE_REQUIRE (1ull << 5)
#define F_NO_BASE64 (1ull << 6)
#define F_WRITE_OPTIONAL (1ull << 7)
#define F_TRACE_BACK (1ull << 8)
#define F_NO_WRITE_BASE (1ull << 9)
#define F_VALIDATE_UTF8 (1ull << 16) /* extension, see utf8_check */
/* J2T states native/thrift.h:204-221 */
enum { J_VAL = 0, J_ARR = 1, J_OBJ = 2, J_KEY = 3, J_ELEM = 4, J_ARR_0 = 5, J_OBJ_0 = 6 };
#define ST_FIELD (1u << 16)
#define ST_SKIP (1u << 17)
#define ST_VM (1u << 18)
#define MAX_RECURSE 4096

/* WRAP_ERR_POS / WRAP_ERR0 native/thrift.h:226-242 (v, p already cast by caller) */
#include "vm_host.h"

#define PACK(e, v, p) ((((uint64_t)(v)) << 40) | (((uint64_t)(p)) << 8) | (uint8_t)(e))
#define PACK0(e, v) ((((uint64_t)(v)) << 8) | (uint8_t)(e))
/* WRAP_ERR2's value: ((uint32_t)(vh) << 8 | (uint8_t)(vl)) */
#define V2(vh, vl) ((uint32_t)(((uint32_t)(vh) << 8) | (uint8_t)(vl)))

typedef struct {
    const uint8_t *s;
    int64_t n;
} Src;
static inline uint8_t AT(const Src *s, int64_t i) { return (i >= 0 && i < s->n) ? s->s[i] : 0; }

typedef struct {
    uint8_t *b;
    size_t len, cap;
} Buf;
static void bgrow(Buf *b, size_t need)
{
    if (need <= b->cap)
        return;
    size_t c = b->cap ? b->cap : 256;
    while (c < need)
        c *= 2;
    b->b = (uint8_t *)realloc(b->b, c);
    b->cap = c;
}
/* buf_malloc native/thrift.c:25-38 (never OOM here) */
static size_t bmalloc(Buf *b, size_t n)
{
    size_t s = b->len;
    bgrow(b, b->len + n);
    b->len += n;
    return s;
}
/* tb_write_* native/thrift.c:40-104 */
static void w8(Buf *b, uint8_t v)
{
    size_t s = bmalloc(b, 1);
    b->b[s] = v;
}
static void w16(Buf *b, uint16_t v)
{
    size_t s = bmalloc(b, 2);
    b->b[s] = v >> 8;
    b->b[s + 1] = v;
}
static void w32(Buf *b, uint32_t v)
{
    size_t s = bmalloc(b, 4);
    for (int i = 0; i < 4; i++)
        b->b[s + i] = v >> (24 - 8 * i);
}
static void w64(Buf *b, uint64_t v)
{
    size_t s = bmalloc(b, 8);
    for (int i = 0; i < 8; i++)
        b->b[s + i] = v >> (56 - 8 * i);
}
static void put32(Buf *b, size_t at, uint32_t v)
{
    for (int i = 0; i < 4; i++)
        b->b[at + i] = v >> (24 - 8 * i);
}
static void wdouble(Buf *b, double d)
{
    uint64_t u;
    memcpy(&u, &d, 8);
    w64(b, u);
}
static void wstring(Buf *b, const uint8_t *p, size_t n)
{
    w32(b, (uint32_t)n);
    size_t s = bmalloc(b, n);
    if (n)
        memcpy(b->b + s, p, n);
}

/* ---- descriptor access ---- */
typedef struct {
    const uint8_t *blob;
    const dg_desc_hdr *h;
    const dg_type *T;
    const dg_struct *S;
    const dg_field *F;
    const dg_name *N;
    const uint64_t *R;
    const uint8_t *P;
} Desc;

/* x86 cvttsd2si: NaN / out of range -> the "integer indefinite" value */
static int32_t cvt32(double d)
{
    if (!(d > -2147483649.0 && d < 2147483648.0))
        return INT32_MIN;
    return (int32_t)d;
}
static int64_t cvt64(double d)
{
    if (!(d >= -9223372036854775808.0 && d < 9223372036854775808.0))
        return INT64_MIN;
    return (int64_t)d;
}

/* ====================================================================== */
/* scanning: native/scanning.c                                             */
/* ====================================================================== */
static inline bool isspace_(uint8_t c) { return c == ' ' || c == '\r' || c == '\n' || c == '\t'; }

/* advance_ns native/scanning.c:64-105 (+ lspace native/fastbytes.c:25-123) */
static uint8_t advance_ns(const Src *s, int64_t *p)
{
    int64_t vi = *p;
    for (int k = 0; k < 4; k++) {
        if (vi < s->n && !isspace_(s->s[vi]))
            goto nospace;
        vi++;
    }
    if (vi >= s->n) {
        *p = vi;
        return 0;
    }
    while (vi < s->n && isspace_(s->s[vi]))
        vi++;
    if (vi >= s->n)
        return 0;
nospace:
    *p = vi + 1;
    return s->s[vi];
}

/* advance_dword native/scanning.c:107-128 */
static int64_t advance_dword(const Src *s, int64_t *p, int64_t dec, int64_t ret, uint32_t val)
{
    /* the reference compares long against size_t: unsigned semantics */
    if ((uint64_t)*p > (uint64_t)(s->n + dec - 4)) {
        *p = s->n;
        return -E_EOF;
    }
    uint32_t w = (uint32_t)AT(s, *p - dec) | ((uint32_t)AT(s, *p - dec + 1) << 8) |
                 ((uint32_t)AT(s, *p - dec + 2) << 16) | ((uint32_t)AT(s, *p - dec + 3) << 24);
    if (w == val) {
        *p += 4 - dec;
        return ret;
    }
    *p -= dec;
    while (AT(s, *p) == (val & 0xff)) {
        val >>= 8;
        ++*p;
    }
    return -E_INVAL;
}
#define VS_NULL 0x6c6c756e
#define VS_TRUE 0x65757274
#define VS_ALSE 0x65736c61

/* advance_string native/scanning.c:130-375: index after the closing quote,
 * *ep = index of the first backslash (only the [p, e) part is ever used). */
static int64_t advance_string(const Src *s, int64_t p, int64_t *ep)
{
    *ep = -1;
    if (s->n == p)
        return -E_EOF;
    int64_t i = p;
    while (i < s->n) {
        uint8_t c = s->s[i++];
        if (c == '"')
            return i;
        if (c == '\\') {
            if (*ep == -1)
                *ep = i - 1;
            if (i >= s->n)
                return -E_EOF;
            i++;
        }
    }
    return -E_EOF;
}

/* ====================================================================== */
/* unquote native/parsing.c:702-945 (flags == 0)                          */
/* ====================================================================== */
static int hexv(uint8_t c)
{
    if (c >= '0' && c <= '9')
        return c - '0';
    if (c >= 'a' && c <= 'f')
        return c - 'a' + 10;
    if (c >= 'A' && c <= 'F')
        return c - 'A' + 10;
    return -1;
}
static bool hex4(const uint8_t *q, uint32_t *v)
{
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        int h = hexv(q[i]);
        if (h < 0)
            return false;
        r = (r << 4) | (uint32_t)h;
    }
    *v = r;
    return true;
}
/* returns output length or -errcode; writes to dp (room for nb bytes) */
static int64_t unquote(const uint8_t *sp, int64_t nb, uint8_t *dp)
{
    uint8_t *d0 = dp;
    while (nb > 0) {
        if (*sp != '\\') {
            *dp++ = *sp++;
            nb--;
            continue;
        }
        sp += 2;
        nb -= 2;
        if (nb < 0)
            return -E_EOF;
        uint8_t c = sp[-1];
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
        default: return -E_ESCAPE;
        }
        if (cc != 0xff) {
            *dp++ = cc;
            continue;
        }
        if (nb < 4)
            return -E_EOF;
        uint32_t r0, r1;
        if (!hex4(sp, &r0))
            return -E_INVAL;
        sp += 4;
        nb -= 4;
        if (r0 <= 0x7f) {
            *dp++ = (uint8_t)r0;
            continue;
        }
        if (r0 <= 0x7ff) {
            *dp++ = 0xc0 | (r0 >> 6);
            *dp++ = 0x80 | (r0 & 0x3f);
            continue;
        }
        if (r0 < 0xd800 || r0 > 0xdfff) {
            *dp++ = 0xe0 | (r0 >> 12);
            *dp++ = 0x80 | ((r0 >> 6) & 0x3f);
            *dp++ = 0x80 | (r0 & 0x3f);
            continue;
        }
        if (nb < 6 || r0 > 0xdbff || sp[0] != '\\' || sp[1] != 'u')
            return -E_UNICODE;
        if (!hex4(sp + 2, &r1))
            return -E_INVAL;
        sp += 6;
        nb -= 6;
        if (r1 < 0xdc00 || r1 > 0xdfff)
            return -E_UNICODE;
        r0 = ((r0 - 0xd800) << 10) + (r1 - 0xdc00) + 0x10000;
        *dp++ = 0xf0 | (r0 >> 18);
        *dp++ = 0x80 | ((r0 >> 12) & 0x3f);
        *dp++ = 0x80 | ((r0 >> 6) & 0x3f);
        *dp++ = 0x80 | (r0 & 0x3f);
    }
    return dp - d0;
}

/* ====================================================================== */
/* base64: b64decode(mode=0) native/base64.c:659-817, decode_block 539-657 */
/* ====================================================================== */
static int b64v(uint8_t c)
{
    if (c >= 'A' && c <= 'Z')
        return c - 'A';
    if (c >= 'a' && c <= 'z')
        return c - 'a' + 26;
    if (c >= '0' && c <= '9')
        return c - '0' + 52;
    if (c == '+')
        return 62;
    if (c == '/')
        return 63;
    return -1;
}
/* returns 0 or (error offset from block start + 1 style) like decode_block */
static int64_t decode_block(const uint8_t *ie, const uint8_t **ipp, uint8_t **opp)
{
    int nb = 0;
    uint32_t v0 = 0;
    uint8_t *op = *opp;
    const uint8_t *ip = *ipp;
    while (nb < 4 && ip < ie) {
        uint8_t ch = *ip;
        if (ch == '\r' || ch == '\n') {
            ip++;
            continue;
        }
        int id = b64v(ch);
        if (id < 0)
            break;
        ip++;
        nb++;
        v0 = (v0 << 6) | (uint32_t)id;
    }
    if (nb == 1)
        return ip - *ipp + 1;
    if (nb < 4) {
        if (ip == ie)
            return ip - *ipp + 1; /* R1, mode has no MODE_RAW */
        else if (nb == 3) {
            if (*ip++ != '=')
                return ip - *ipp;
        } else {
            if (ip >= ie - 1)
                return ip - *ipp + 1;
            if (*ip++ != '=')
                return ip - *ipp;
            if (*ip++ != '=')
                return ip - *ipp;
        }
        if (ip < ie)
            return ip - *ipp + 1;
        v0 <<= 6 * (4 - nb);
    }
    switch (nb) {
    case 4: op[2] = v0 & 0xff; /* fallthrough */
    case 3: op[1] = (v0 >> 8) & 0xff; /* fallthrough */
    case 2: op[0] = (v0 >> 16) & 0xff;
    }
    *ipp = ip;
    *opp = op + nb - 1;
    return 0;
}
static int64_t b64decode(uint8_t *out, const uint8_t *src, int64_t nb)
{
    if (nb == 0)
        return 0;
    uint8_t *op = out;
    const uint8_t *ib = src, *ip = src, *ie = src + nb;
    while (ip < ie) {
        int64_t dv = decode_block(ie, &ip, &op);
        if (dv != 0)
            return ib - ip - dv;
    }
    return op - out;
}

/* ====================================================================== */
/* numbers: vnumber native/scanning.c:958-1083 and helpers                 */
/* ====================================================================== */
static const double P10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

static double u2d_signed(uint64_t man, int sgn)
{
    double v = (double)man;
    uint64_t b;
    memcpy(&b, &v, 8);
    b |= ((uint64_t)(int64_t)sgn) >> 63 << 63;
    memcpy(&v, &b, 8);
    return v;
}

/* is_atof_exact native/scanning.c:883-926 */
static bool is_atof_exact(uint64_t man, int exp, int sgn, double *val)
{
    *val = (double)man;
    if (man >> 52 != 0)
        return false;
    *val = u2d_signed(man, sgn);
    if (exp == 0 || man == 0)
        return true;
    if (exp > 0 && exp <= 15 + 22) {
        if (exp > 22) {
            *val *= P10[exp - 22];
            exp = 22;
        }
        if (*val > 1e15 || *val < -1e15)
            return false;
        *val *= P10[exp];
        return true;
    }
    if (exp < 0 && exp >= -22) {
        *val /= P10[-exp];
        return true;
    }
    return false;
}

/* atof_eisel_lemire64 native/atof_eisel_lemire.c:74-167 */
static bool eisel_lemire(uint64_t mant, int exp10, int sgn, double *val)
{
    if (exp10 < -348 || exp10 > 347)
        return false;
    int clz = mant ? __builtin_clzll(mant) : 64;
    mant = clz < 64 ? mant << clz : mant;
    uint64_t ret_exp2 = ((uint64_t)(int64_t)((217706 * exp10) >> 16) + 64 + 1023) - (uint64_t)clz;
    unsigned __int128 x = (unsigned __int128)mant * DG_POW10_M128[exp10 + 348][1];
    uint64_t x_hi = (uint64_t)(x >> 64), x_lo = (uint64_t)x;
    if ((x_hi & 0x1FF) == 0x1FF && (x_lo + mant) < mant) {
        unsigned __int128 y = (unsigned __int128)mant * DG_POW10_M128[exp10 + 348][0];
        uint64_t y_hi = (uint64_t)(y >> 64), y_lo = (uint64_t)y;
        uint64_t merged_hi = x_hi, merged_lo = x_lo + y_hi;
        if (merged_lo < x_lo)
            merged_hi++;
        if ((merged_hi & 0x1FF) == 0x1FF && (merged_lo + 1) == 0 && (y_lo + mant) < mant)
            return false;
        x_hi = merged_hi;
        x_lo = merged_lo;
    }
    int msb = (int)(x_hi >> 63);
    uint64_t ret_man = x_hi >> (msb + 9);
    ret_exp2 -= 1 ^ msb;
    if ((x_lo == 0) && ((x_hi & 0x1FF) == 0) && ((ret_man & 3) == 1))
        return false;
    ret_man += ret_man & 1;
    ret_man >>= 1;
    if ((ret_man >> 53) > 0) {
        ret_man >>= 1;
        ret_exp2 += 1;
    }
    if ((ret_exp2 - 1) >= (0x7FF - 1))
        return false;
    uint64_t bits = (ret_exp2 << 52) | (ret_man & 0x000FFFFFFFFFFFFFull);
    if (sgn == -1)
        bits |= 1ull << 63;
    memcpy(val, &bits, 8);
    return true;
}

/* atof_native: Decimal slow path native/atof_native.c:17-424 (cap 800,
 * internal/types/types.go:268) */
#define DCAP 800
typedef struct {
    char d[DCAP];
    int nd, dp, neg, trunc;
} Decimal;

static void decimal_set(Decimal *d, const uint8_t *s, int64_t len)
{
    int64_t i = 0;
    memset(d, 0, sizeof(*d));
    if (s[i] == '-') {
        i++;
        d->neg = 1;
    }
    int saw_dot = 0;
    for (; i < len; i++) {
        if ('0' <= s[i] && s[i] <= '9') {
            if (s[i] == '0' && d->nd == 0) {
                d->dp--;
                continue;
            }
            if (d->nd < DCAP)
                d->d[d->nd++] = s[i];
            else if (s[i] != '0')
                d->trunc = 1;
        } else if (s[i] == '.') {
            saw_dot = 1;
            d->dp = d->nd;
        } else
            break;
    }
    if (!saw_dot)
        d->dp = d->nd;
    if (i < len && (s[i] == 'e' || s[i] == 'E')) {
        int exp = 0, esgn = 1;
        i++;
        if (s[i] == '+')
            i++;
        else if (s[i] == '-') {
            i++;
            esgn = -1;
        }
        for (; i < len && ('0' <= s[i] && s[i] <= '9') && exp < 10000; i++)
            exp = exp * 10 + (s[i] - '0');
        d->dp += exp * esgn;
    }
}
static void trim(Decimal *d)
{
    while (d->nd > 0 && d->d[d->nd - 1] == '0')
        d->nd--;
    if (d->nd == 0)
        d->dp = 0;
}
static void right_shift(Decimal *d, uint32_t k)
{
    int r = 0, w = 0;
    uint64_t n = 0;
    for (; n >> k == 0; r++) {
        if (r >= d->nd) {
            if (n == 0) {
                d->nd = 0;
                return;
            }
            while (n >> k == 0) {
                n *= 10;
                r++;
            }
            break;
        }
        n = n * 10 + d->d[r] - '0';
    }
    d->dp -= r - 1;
    uint64_t mask = (1ull << k) - 1;
    for (; r < d->nd; r++) {
        uint64_t dig = n >> k;
        n &= mask;
        d->d[w++] = (char)(dig + '0');
        n = n * 10 + d->d[r] - '0';
    }
    while (n > 0) {
        uint64_t dig = n >> k;
        n &= mask;
        if (w < DCAP)
            d->d[w++] = (char)(dig + '0');
        else if (dig > 0)
            d->trunc = 1;
        n *= 10;
    }
    d->nd = w;
    trim(d);
}
static bool prefix_is_less(const char *b, const char *s, int bn)
{
    int i = 0;
    for (; i < bn; i++) {
        if (s[i] == '\0')
            return false;
        if (b[i] != s[i])
            return b[i] < s[i];
    }
    return s[i] != '\0';
}
static void left_shift(Decimal *d, uint32_t k)
{
    int delta = DG_LSHIFT_DELTA[k];
    if (prefix_is_less(d->d, DG_LSHIFT_CUTOFF[k], d->nd))
        delta--;
    int r = d->nd, w = d->nd + delta;
    uint64_t n = 0;
    for (r--; r >= 0; r--) {
        n += (uint64_t)(d->d[r] - '0') << k;
        uint64_t quo = n / 10, rem = n - 10 * quo;
        w--;
        if (w < DCAP)
            d->d[w] = (char)(rem + '0');
        else if (rem != 0)
            d->trunc = 1;
        n = quo;
    }
    while (n > 0) {
        uint64_t quo = n / 10, rem = n - 10 * quo;
        w--;
        if (w < DCAP)
            d->d[w] = (char)(rem + '0');
        else if (rem != 0)
            d->trunc = 1;
        n = quo;
    }
    d->nd += delta;
    if (d->nd >= DCAP)
        d->nd = DCAP;
    d->dp += delta;
    trim(d);
}
static void decimal_shift(Decimal *d, int k)
{
    if (d->nd == 0 || k == 0)
        return;
    if (k > 0) {
        while (k > 60) {
            left_shift(d, 60);
            k -= 60;
        }
        if (k)
            left_shift(d, k);
    }
    if (k < 0) {
        while (k < -60) {
            right_shift(d, 60);
            k += 60;
        }
        if (k)
            right_shift(d, -k);
    }
}
static int should_roundup(Decimal *d, int nd)
{
    if (nd < 0 || nd >= d->nd)
        return 0;
    if (d->d[nd] == '5' && nd + 1 == d->nd) {
        if (d->trunc)
            return 1;
        return nd > 0 && (d->d[nd - 1] - '0') % 2 != 0;
    }
    return d->d[nd] >= '5';
}
static uint64_t rounded_integer(Decimal *d)
{
    if (d->dp > 20)
        return 0xFFFFFFFFFFFFFFFFull;
    int i;
    uint64_t n = 0;
    for (i = 0; i < d->dp && i < d->nd; i++)
        n = n * 10 + (d->d[i] - '0');
    for (; i < d->dp; i++)
        n *= 10;
    if (should_roundup(d, d->dp))
        n++;
    return n;
}
static const int POW_TAB[9] = {1, 3, 6, 9, 13, 16, 19, 23, 26};
static double decimal_to_f64(Decimal *d)
{
    int exp2 = 0;
    uint64_t mant = 0;
    if (d->nd == 0) {
        mant = 0;
        exp2 = -1023;
        goto out;
    }
    if (d->dp > 310)
        goto overflow;
    if (d->dp < -330) {
        mant = 0;
        exp2 = -1023;
        goto out;
    }
    int n;
    while (d->dp > 0) {
        n = d->dp >= 9 ? 27 : POW_TAB[d->dp];
        decimal_shift(d, -n);
        exp2 += n;
    }
    while ((d->dp < 0) || ((d->dp == 0) && (d->d[0] < '5'))) {
        n = -d->dp >= 9 ? 27 : POW_TAB[-d->dp];
        decimal_shift(d, n);
        exp2 -= n;
    }
    exp2--;
    if (exp2 < -1022) {
        n = -1022 - exp2;
        decimal_shift(d, -n);
        exp2 += n;
    }
    if ((exp2 + 1023) >= 0x7FF)
        goto overflow;
    decimal_shift(d, 53);
    mant = rounded_integer(d);
    if (mant == (2ull << 52)) {
        mant >>= 1;
        exp2++;
        if ((exp2 + 1023) >= 0x7FF)
            goto overflow;
    }
    if ((mant & (1ull << 52)) == 0)
        exp2 = -1023;
    goto out;
overflow:
    mant = 0;
    exp2 = 0x7FF - 1023;
out:;
    uint64_t bits = mant & 0x000FFFFFFFFFFFFFull;
    bits |= (uint64_t)((exp2 + 1023) & 0x7FF) << 52;
    if (d->neg)
        bits |= 1ull << 63;
    double v;
    memcpy(&v, &bits, 8);
    return v;
}
static double atof_native(const uint8_t *sp, int64_t nb)
{
    static __thread Decimal d;
    decimal_set(&d, sp, nb);
    return decimal_to_f64(&d);
}

typedef struct {
    int64_t vt;
    double dv;
    int64_t iv;
} JState;

/* vnumber native/scanning.c:958-1083 */
static void vnumber(const Src *src, int64_t *p, JState *ret)
{
    int sgn = 1;
    uint64_t man = 0;
    int man_nd = 0, exp10 = 0, trunc = 0;
    double val = 0;
    int64_t i = *p, n = src->n;
#define S(k) AT(src, (k))
    ret->vt = V_INTEGER;
    ret->dv = 0.0;
    ret->iv = 0;
    if (i >= n) {
        *p = n;
        ret->vt = -E_EOF;
        return;
    }
    if (S(i) == '-') {
        i++;
        sgn = -1;
        if (i >= n) {
            *p = n;
            ret->vt = -E_EOF;
            return;
        }
    }
    if (S(i) < '0' || S(i) > '9') {
        *p = i;
        ret->vt = -E_INVAL;
        return;
    }
    if (S(i) == '0' && (i >= n || (S(i + 1) != '.' && S(i + 1) != 'e' && S(i + 1) != 'E'))) {
        *p = ++i;
        return;
    }
    while (i < n && S(i) >= '0' && S(i) <= '9') {
        if (man_nd < 19) {
            man = man * 10 + (S(i) - '0');
            man_nd++;
        } else
            exp10++;
        i++;
    }
    if (exp10 > 0)
        trunc = 1;
    if (i < n && S(i) == '.') {
        i++;
        ret->vt = V_DOUBLE;
        if (i >= n) {
            *p = n;
            ret->vt = -E_EOF;
            return;
        }
        if (S(i) < '0' || S(i) > '9') {
            *p = i;
            ret->vt = -E_INVAL;
            return;
        }
    }
    if (man == 0 && exp10 == 0) {
        while (i < n && S(i) == '0') {
            i++;
            exp10--;
        }
        man = 0;
        man_nd = 0;
    }
    while (i < n && man_nd < 19 && S(i) >= '0' && S(i) <= '9') {
        man = man * 10 + (S(i) - '0');
        man_nd++;
        exp10--;
        i++;
    }
    while (i < n && S(i) >= '0' && S(i) <= '9') {
        trunc = 1;
        i++;
    }
    if (i < n && (S(i) == 'e' || S(i) == 'E')) {
        int esm = 1, exp = 0;
        i++;
        ret->vt = V_DOUBLE;
        if (i >= n) {
            *p = n;
            ret->vt = -E_EOF;
            return;
        }
        if (S(i) == '+' || S(i) == '-') {
            esm = S(i++) == '+' ? 1 : -1;
            if (i >= n) {
                *p = n;
                ret->vt = -E_EOF;
                return;
            }
        }
        if (S(i) < '0' || S(i) > '9') {
            *p = i;
            ret->vt = -E_INVAL;
            return;
        }
        while (i < n && S(i) >= '0' && S(i) <= '9') {
            if (exp < 10000)
                exp = exp * 10 + (S(i) - '0');
            i++;
        }
        exp10 += exp * esm;
        goto parse_float;
    }
    if (ret->vt == V_INTEGER) {
        /* is_overflow native/scanning.c:950-956 */
        bool ovf = exp10 != 0 || ((man >> 63) == 1 && (((uint64_t)(int64_t)sgn) & man) != (1ull << 63));
        if (!ovf) {
            ret->iv = (int64_t)(man * (uint64_t)(int64_t)sgn);
            ret->dv = u2d_signed(man, sgn);
            *p = i;
            return;
        }
        ret->vt = V_DOUBLE;
    }
parse_float:
    /* atof_fast native/scanning.c:928-948 */
    {
        bool ok = false;
        double vu = 0;
        if (is_atof_exact(man, exp10, sgn, &val))
            ok = true;
        else if (eisel_lemire(man, exp10, sgn, &val)) {
            if (!trunc || (eisel_lemire(man + 1, exp10, sgn, &vu) && vu == val))
                ok = true;
        }
        if (!ok)
            val = atof_native(src->s + *p, i - *p);
    }
    {
        uint64_t b;
        memcpy(&b, &val, 8);
        if ((b << 1) == 0xFFE0000000000000ull)
            ret->vt = -E_FLOAT_INF;
    }
    ret->dv = val;
    *p = i;
#undef S
}

/* ====================================================================== */
/* skipping: fsm_exec/skip_* native/scanning.c:1134-1631 (AVX2 build)      */
/* ====================================================================== */
static inline bool numch(uint8_t c)
{
    return (c >= '0' && c <= '9') || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-';
}
static int ctz32(uint32_t v) { return __builtin_ctz(v); }

/* skip_number native/scanning.c:1317-1535: 32-byte blocks, then 16-byte
 * blocks, then scalar (the AVX2 variant's block decomposition). */
static int64_t skip_number(const uint8_t *sp, int64_t nb)
{
    int64_t di = -1, ei = -1, si = -1;
    const uint8_t *ss = sp;
    if (nb == 0)
        return -1;
    if (*sp == '0' && (nb == 1 || (sp[1] != '.' && sp[1] != 'e' && sp[1] != 'E')))
        return 1;
    for (int W = 32; W >= 16; W -= 16) {
        while (nb >= W) {
            uint32_t md = 0, me = 0, ms = 0, v;
            int i = W;
            for (int k = 0; k < W; k++) {
                if (!numch(sp[k])) {
                    i = k;
                    break;
                }
            }
            for (int k = 0; k < i; k++) {
                uint8_t c = sp[k];
                if (c == '.')
                    md |= 1u << k;
                else if (c == 'e' || c == 'E')
                    me |= 1u << k;
                else if (c == '+' || c == '-')
                    ms |= 1u << k;
            }
            if ((v = md & (md - 1)) != 0)
                return -(sp - ss + ctz32(v) + 1);
            if ((v = me & (me - 1)) != 0)
                return -(sp - ss + ctz32(v) + 1);
            if ((v = ms & (ms - 1)) != 0)
                return -(sp - ss + ctz32(v) + 1);
            if (md) {
                if (di == -1)
                    di = sp - ss + ctz32(md);
                else
                    return -(sp - ss + ctz32(md) + 1);
            }
            if (me) {
                if (ei == -1)
                    ei = sp - ss + ctz32(me);
                else
                    return -(sp - ss + ctz32(me) + 1);
            }
            if (ms) {
                if (si == -1)
                    si = sp - ss + ctz32(ms);
                else
                    return -(sp - ss + ctz32(ms) + 1);
            }
            if (i != W) {
                sp += i;
                goto check_index;
            }
            sp += W;
            nb -= W;
        }
    }
    while (nb-- > 0) {
        uint8_t c = *sp++;
        if (c >= '0' && c <= '9')
            continue;
        int64_t *iv = c == '.' ? &di : (c == 'e' || c == 'E') ? &ei : (c == '+' || c == '-') ? &si : NULL;
        if (!iv) {
            sp--;
            goto check_index;
        }
        if (*iv == -1)
            *iv = sp - ss - 1;
        else
            return -(sp - ss);
    }
check_index:
    if (di == 0 || si == 0 || ei == 0)
        return -1;
    else if (di == sp - ss - 1 || si == sp - ss - 1 || ei == sp - ss - 1)
        return -(sp - ss);
    else if (si > 0 && ei != si - 1)
        return -si - 1;
    else if (di >= 0 && ei >= 0 && di > ei - 1)
        return -di - 1;
    else if (di >= 0 && ei >= 0 && di == ei - 1)
        return -ei - 1;
    return sp - ss;
}

enum { FV = 0, FARR = 1, FOBJ = 2, FKEY = 3, FELEM = 4, FARR0 = 5, FOBJ0 = 6 };

static int64_t skip_string(const Src *s, int64_t *p)
{
    int64_t v, q = *p - 1;
    int64_t e = advance_string(s, *p, &v);
    if (e >= 0) {
        *p = e;
        return q;
    }
    *p = s->n;
    return e;
}

/* skip_one = fsm_exec(VALID_DEFAULT) native/scanning.c:1134-1315,1537-1541 */
static int64_t skip_one(const Src *s, int64_t *p, int *stk)
{
    int sp = 1;
    stk[0] = FV;
    int64_t vi = -1;
    while (sp) {
        uint8_t ch = advance_ns(s, p);
        int vt = stk[sp - 1];
        if (vi == -1)
            vi = *p - 1;
        switch (vt) {
        default:
            sp--;
            break;
        case FARR:
            if (ch == ']') {
                sp--;
                continue;
            }
            if (ch == ',') {
                if (sp >= MAX_RECURSE)
                    return -E_RECURSE_MAX;
                stk[sp++] = FV;
                continue;
            }
            return -E_INVAL;
        case FOBJ:
            if (ch == '}') {
                sp--;
                continue;
            }
            if (ch == ',') {
                if (sp >= MAX_RECURSE)
                    return -E_RECURSE_MAX;
                stk[sp++] = FKEY;
                continue;
            }
            return -E_INVAL;
        case FKEY: {
            if (ch != '"')
                return -E_INVAL;
            stk[sp - 1] = FELEM;
            int64_t r = skip_string(s, p);
            if (r < 0)
                return r;
            continue;
        }
        case FELEM:
            if (ch != ':')
                return -E_INVAL;
            stk[sp - 1] = FV;
            continue;
        case FARR0:
            if (ch == ']') {
                sp--;
                continue;
            }
            stk[sp - 1] = FARR;
            break;
        case FOBJ0:
            if (ch == '}') {
                sp--;
                continue;
            }
            if (ch == '"') {
                stk[sp - 1] = FOBJ;
                int64_t r = skip_string(s, p);
                if (r < 0)
                    return r;
                if (sp >= MAX_RECURSE)
                    return -E_RECURSE_MAX;
                stk[sp++] = FELEM;
                continue;
            }
            return -E_INVAL;
        }
        switch (ch) {
        case '0': case '1': case '2': case '3': case '4':
        case '5': case '6': case '7': case '8': case '9': {
            int64_t i = *p - 1; /* skip_positive native/scanning.c:1616-1631 */
            int64_t r = skip_number(s->s + i, s->n - i);
            if (r < 0) {
                *p -= r + 2;
                return -E_INVAL;
            }
            *p += r - 1;
            break;
        }
        case '-': {
            int64_t i = *p; /* skip_negative native/scanning.c:1599-1614 */
            int64_t r = skip_number(s->s + i, s->n - i);
            if (r < 0) {
                *p -= r + 1;
                return -E_INVAL;
            }
            *p += r;
            break;
        }
        case 'n': {
            int64_t r = advance_dword(s, p, 1, *p - 1, VS_NULL);
            if (r < 0)
                return r;
            break;
        }
        case 't': {
            int64_t r = advance_dword(s, p, 1, *p - 1, VS_TRUE);
            if (r < 0)
                return r;
            break;
        }
        case 'f': {
            int64_t r = advance_dword(s, p, 0, *p - 1, VS_ALSE);
            if (r < 0)
                return r;
            break;
        }
        case '[':
            if (sp >= MAX_RECURSE)
                return -E_RECURSE_MAX;
            stk[sp++] = FARR0;
            break;
        case '{':
            if (sp >= MAX_RECURSE)
                return -E_RECURSE_MAX;
            stk[sp++] = FOBJ0;
            break;
        case '"': {
            int64_t r = skip_string(s, p);
            if (r < 0)
                return r;
            break;
        }
        case 0:
            return -E_EOF;
        default:
            return -E_INVAL;
        }
    }
    return vi;
}

/* ====================================================================== */
/* j2t: native/thrift.c                                                    */
/* ====================================================================== */
typedef struct {
    uint32_t st;      /* state | ST_* */
    uint32_t td;      /* type index */
    uint64_t bp, size;/* J2TExtra_Cont */
    uint32_t reqs;    /* J2TExtra_Struct: offset of this instance's bits in reqs pool */
    uint32_t f;       /* J2TExtra_Field */
} Frame;

typedef struct {
    Desc D;
    Buf *buf;
    const Src *src;
    uint64_t flag;
    Frame *vt;
    size_t sp;
    uint64_t *reqs; /* requires-bit pool (bm_malloc_reqs native/thrift.c:232-256) */
    size_t reqs_len, reqs_cap;
    size_t field_cache_len;
    JState jt;
    int *skipstk;
    uint8_t *keybuf;
} M;

static inline const dg_type *TY(M *m, uint32_t t) { return &m->D.T[t]; }

/* tb_write_empty native/thrift.c:171-203 */
static uint64_t tb_write_empty(M *m, uint32_t td, int64_t p)
{
    const dg_type *t = TY(m, td);
    Buf *b = m->buf;
    switch (t->ttype) {
    case DG_T_BOOL: w8(b, 0); return 0;
    case DG_T_BYTE: w8(b, 0); return 0;
    case DG_T_I16: w16(b, 0); return 0;
    case DG_T_I32: w32(b, 0); return 0;
    case DG_T_I64: w64(b, 0); return 0;
    case DG_T_DOUBLE: w64(b, 0); return 0;
    case DG_T_STRING: w32(b, 0); return 0;
    case DG_T_LIST:
    case DG_T_SET:
        w8(b, TY(m, t->elem)->ttype);
        w32(b, 0);
        return 0;
    case DG_T_MAP:
        w8(b, TY(m, t->key)->ttype);
        w8(b, TY(m, t->elem)->ttype);
        w32(b, 0);
        return 0;
    case DG_T_STRUCT: w8(b, 0); return 0;
    default: return PACK(E_UNSUPPORT_THRIFT_TYPE, (uint64_t)t->ttype, (uint64_t)p);
    }
}

/* tb_write_default_or_empty native/thrift.c:205-217 */
static uint64_t tb_write_default_or_empty(M *m, const dg_field *f, int64_t p)
{
    if (f->dflt_len != DG_NONE) {
        size_t s = bmalloc(m->buf, f->dflt_len);
        memcpy(m->buf->b + s, m->D.P + f->dflt_off, f->dflt_len);
        return 0;
    }
    return tb_write_empty(m, f->type, p);
}

/* j2t_write_unset_fields native/thrift.c:258-310 */
static uint64_t write_unset_fields(M *m, const dg_struct *st, uint32_t reqs, int64_t p)
{
    bool wr = m->flag & F_WRITE_REQUIRE, wd = m->flag & F_WRITE_DEFAULT;
    bool wo = m->flag & F_WRITE_OPTIONAL, tb = m->flag & F_TRACE_BACK;
    for (uint32_t k = 0; k < st->n_fields; k++) {
        if (!((m->reqs[reqs + k / 64] >> (k % 64)) & 1))
            continue;
        const dg_field *f = &m->D.F[st->field_begin + k];
        if (f->flags & DG_FF_REQUEST_BASE)
            continue;
        if (tb && (f->required == DG_REQ_REQUIRED || m->sp == 1))
            m->field_cache_len++;
        else if (!wr && f->required == DG_REQ_REQUIRED)
            return PACK(E_NULL_REQUIRED, (uint64_t)f->id, (uint64_t)p);
        else if ((wr && f->required == DG_REQ_REQUIRED) || (wd && f->required == DG_REQ_DEFAULT) ||
                 (wo && f->required == DG_REQ_OPTIONAL)) {
            w8(m->buf, TY(m, f->type)->ttype);
            w16(m->buf, f->id);
            uint64_t r = tb_write_default_or_empty(m, f, p);
            if (r)
                return r;
        }
    }
    return 0;
}

/* j2t_number native/thrift.c:312-365 */
static uint64_t j2t_number(M *m, uint32_t td, const Src *src, int64_t *p)
{
    int64_t s = *p;
    JState *r = &m->jt;
    vnumber(src, p, r);
    if (r->vt < 0)
        return PACK(-r->vt, (uint64_t)s, (uint64_t)*p);
    Buf *b = m->buf;
    switch (TY(m, td)->ttype) {
    case DG_T_BYTE:
        w8(b, r->vt == V_INTEGER ? (uint8_t)r->iv : (uint8_t)cvt32(r->dv));
        return 0;
    case DG_T_I16:
        w16(b, r->vt == V_INTEGER ? (uint16_t)r->iv : (uint16_t)cvt32(r->dv));
        return 0;
    case DG_T_I32:
        w32(b, r->vt == V_INTEGER ? (uint32_t)r->iv : (uint32_t)cvt32(r->dv));
        return 0;
    case DG_T_I64:
        w64(b, r->vt == V_INTEGER ? (uint64_t)r->iv : (uint64_t)cvt64(r->dv));
        return 0;
    case DG_T_DOUBLE:
        wdouble(b, r->dv);
        return 0;
    }
    return PACK(E_DISMATCH_TYPE, V2(TY(m, td)->ttype, V_INTEGER), (uint64_t)*p);
}

/* Extension F_VALIDATE_UTF8 (bit 16, no reference counterpart): the raw JSON
 * bytes of every string written as a Thrift STRING (string values and STRING
 * map keys) must be valid UTF-8 as utf8_validate (native/utf8.c:101-212)
 * defines it. Returns -1 if valid, else the offset of the first invalid
 * sequence; the caller reports ERR_INVAL, value = that byte, pos = its offset. */
static int64_t utf8_check(const uint8_t *s, int64_t n)
{
    int64_t i = 0;
    while (i < n) {
        uint8_t c = s[i];
        if (c < 0x80) {
            i++;
            continue;
        }
        int size;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF)
            size = 2;
        else if (c >= 0xE0 && c <= 0xEF) {
            size = 3;
            if (c == 0xE0)
                lo = 0xA0;
            else if (c == 0xED)
                hi = 0x9F;
        } else if (c >= 0xF0 && c <= 0xF4) {
            size = 4;
            if (c == 0xF0)
                lo = 0x90;
            else if (c == 0xF4)
                hi = 0x8F;
        } else
            return i;
        if (n - i < size)
            return i;
        if (s[i + 1] < lo || s[i + 1] > hi)
            return i;
        for (int k = 2; k < size; k++)
            if (s[i + k] < 0x80 || s[i + k] > 0xBF)
                return i;
        i += size;
    }
    return -1;
}

/* j2t_string native/thrift.c:367-399 */
static uint64_t j2t_string(M *m, int64_t *p)
{
    const Src *src = m->src;
    int64_t s = *p, ep;
    int64_t e = advance_string(src, s, &ep);
    if (e < 0)
        return PACK(-e, (uint64_t)s, (uint64_t)*p);
    *p = e;
    int64_t n = e - s - 1;
    if (m->flag & F_VALIDATE_UTF8) {
        int64_t r = utf8_check(src->s + s, n);
        if (r >= 0)
            return PACK(E_INVAL, (uint64_t)src->s[s + r], (uint64_t)(s + r));
    }
    if (ep >= s && ep < e) {
        size_t lp = bmalloc(m->buf, 4);
        size_t o = bmalloc(m->buf, n);
        int64_t l = unquote(src->s + s, n, m->buf->b + o);
        if (l < 0)
            return PACK(-l, (uint64_t)s, (uint64_t)*p);
        m->buf->len = o + l;
        put32(m->buf, lp, (uint32_t)l);
    } else {
        wstring(m->buf, src->s + s, n);
    }
    return 0;
}

/* j2t_binary native/thrift.c:401-420 */
static uint64_t j2t_binary(M *m, int64_t *p)
{
    const Src *src = m->src;
    int64_t s = *p, ep;
    int64_t e = advance_string(src, s, &ep);
    if (e < 0)
        return PACK(-e, (uint64_t)s, (uint64_t)*p);
    *p = e;
    int64_t n = e - s - 1;
    size_t back = bmalloc(m->buf, 4);
    bgrow(m->buf, m->buf->len + n + 8);
    int64_t l = b64decode(m->buf->b + m->buf->len, src->s + s, n);
    if (l < 0)
        return PACK(E_DECODE_BASE64, (uint64_t)(-l - 1), (uint64_t)*p);
    m->buf->len += l;
    put32(m->buf, back, (uint32_t)l);
    return 0;
}

/* j2t_map_key native/thrift.c:422-447 */
static uint64_t j2t_map_key(M *m, const uint8_t *sp, int64_t n, uint32_t kt, int64_t p)
{
    switch (TY(m, kt)->ttype) {
    case DG_T_STRING:
        wstring(m->buf, sp, n);
        return 0;
    case DG_T_BYTE:
    case DG_T_I16:
    case DG_T_I32:
    case DG_T_I64:
    case DG_T_DOUBLE: {
        Src tmp = {sp, n};
        int64_t q = 0;
        return j2t_number(m, kt, &tmp, &q);
    }
    default:
        return PACK(E_UNSUPPORT_THRIFT_TYPE, (uint64_t)TY(m, kt)->ttype, (uint64_t)p);
    }
}

/* field lookup: j2t_find_field_key native/thrift.c:449-468 (exact-match map) */
static const dg_field *find_field(M *m, const dg_struct *st, const uint8_t *k, int64_t kn)
{
    uint32_t h = DG_NAME_HASH_SEED;
    for (int64_t i = 0; i < kn; i++)
        h = DG_NAME_HASH_STEP(h, k[i]);
    uint32_t j = h & st->name_mask;
    for (;;) {
        const dg_name *nm = &m->D.N[st->name_begin + j];
        if (nm->field == DG_NONE)
            return NULL;
        if (nm->hash == h && nm->key_len == (uint32_t)kn && memcmp(m->D.P + nm->key_off, k, kn) == 0)
            return &m->D.F[nm->field];
        j = (j + 1) & st->name_mask;
    }
}

/* j2t_read_key native/thrift.c:470-504 */
static uint64_t j2t_read_key(M *m, int64_t *p, const uint8_t **spp, int64_t *knp)
{
    const Src *src = m->src;
    int64_t s = *p, ep;
    int64_t e = advance_string(src, s, &ep);
    if (e < 0)
        return PACK(-e, (uint64_t)s, (uint64_t)*p);
    *p = e;
    int64_t kn = e - s - 1;
    const uint8_t *sp = src->s + s;
    if (ep >= s && ep < e) {
        int64_t l = unquote(sp, kn, m->keybuf);
        if (l < 0)
            return PACK(-l, (uint64_t)s, (uint64_t)*p);
        sp = m->keybuf;
        kn = l;
    }
    *spp = sp;
    *knp = kn;
    return 0;
}

static inline bool bm_is_set(M *m, uint32_t reqs, uint32_t k) { return (m->reqs[reqs + k / 64] >> (k % 64)) & 1; }
/* bm_set_req native/map.c:140-154 */
static inline void bm_set_req(M *m, uint32_t reqs, uint32_t k, int req)
{
    uint64_t *w = &m->reqs[reqs + k / 64];
    if (req == DG_REQ_DEFAULT || req == DG_REQ_REQUIRED)
        *w |= 1ull << (k % 64);
    else if (req == DG_REQ_OPTIONAL)
        *w &= ~(1ull << (k % 64));
}

#define PUSH(M_, ST_, TD_)                                                        \
    do {                                                                          \
        if ((M_)->sp >= MAX_RECURSE)                                              \
            return PACK(E_RECURSE_MAX, (uint64_t)(M_)->sp, (uint64_t)*p);         \
        Frame *xp_ = &(M_)->vt[(M_)->sp++];                                       \
        xp_->st = (ST_);                                                          \
        xp_->td = (TD_);                                                          \
    } while (0)

/* j2t_key native/thrift.c:668-763 */
static uint64_t j2t_key(M *m, int64_t *p, uint32_t dc, bool obj0, size_t *unwindPos,
                        const dg_field **lastField, Frame *vt)
{
    const uint8_t *sp = NULL;
    int64_t kn = 0, ks = *p;
    uint64_t r = j2t_read_key(m, p, &sp, &kn);
    if (r)
        return r;
    const dg_type *t = TY(m, dc);
    if (t->ttype == DG_T_MAP) {
        if ((m->flag & F_VALIDATE_UTF8) && TY(m, t->key)->ttype == DG_T_STRING) {
            int64_t u = utf8_check(m->src->s + ks, *p - ks - 1);
            if (u >= 0)
                return PACK(E_INVAL, (uint64_t)m->src->s[ks + u], (uint64_t)(ks + u));
        }
        *unwindPos = m->buf->len;
        r = j2t_map_key(m, sp, kn, t->key, *p);
        if (r)
            return r;
        if (obj0) {
            vt->size = 0;
            PUSH(m, J_ELEM, t->elem);
        } else {
            Frame *x = &m->vt[m->sp - 1];
            x->st = J_ELEM;
            x->td = t->elem;
        }
        return 0;
    }
    Frame *pex = obj0 ? vt : &m->vt[m->sp - 2];
    const dg_struct *st = &m->D.S[t->st];
    const dg_field *f = find_field(m, st, sp, kn);
    if (f == NULL || ((f->flags & DG_FF_REQUEST_BASE) && (m->flag & F_NO_WRITE_BASE))) {
        if (f == NULL && (m->flag & F_ALLOW_UNKNOWN) == 0)
            return PACK(E_UNKNOWN_FIELD, (uint64_t)kn, (uint64_t)*p);
        if (obj0)
            PUSH(m, J_ELEM | ST_SKIP, DG_NONE);
        else {
            Frame *x = &m->vt[m->sp - 1];
            x->st = J_ELEM | ST_SKIP;
            x->td = DG_NONE;
        }
        return 0;
    }
    uint32_t k = (uint32_t)(f - m->D.F) - st->field_begin;
    if ((m->flag & F_ENABLE_HM) && (f->flags & DG_FF_HTTP_MAPPING) && !bm_is_set(m, pex->reqs, k)) {
        if (obj0)
            PUSH(m, J_ELEM | ST_SKIP, f->type);
        else {
            Frame *x = &m->vt[m->sp - 1];
            x->st = J_ELEM | ST_SKIP;
            x->td = f->type;
        }
        return 0;
    }
    uint32_t vm = ST_VM;
    if ((m->flag & F_ENABLE_VM) == 0 || f->vm == DG_VM_NONE) {
        vm = ST_FIELD;
        *unwindPos = m->buf->len;
        *lastField = f;
        w8(m->buf, TY(m, f->type)->ttype);
        w16(m->buf, f->id);
    }
    Frame *x;
    if (obj0) {
        PUSH(m, J_ELEM | vm, f->type);
        x = &m->vt[m->sp - 1];
    } else {
        x = &m->vt[m->sp - 1];
        x->st = J_ELEM | vm;
        x->td = f->type;
    }
    x->bp = 0;
    x->size = 0;
    x->reqs = 0;
    x->f = (uint32_t)(f - m->D.F);
    bm_set_req(m, pex->reqs, k, DG_REQ_OPTIONAL);
    return 0;
}

/* j2t_field_vm native/thrift.c:506-666 */
static uint64_t j2t_field_vm(M *m, int64_t *p, Frame *vt)
{
    const dg_field *f = &m->D.F[vt->f];
    const Src *src = m->src;
    Buf *b = m->buf;
    uint8_t ft = TY(m, f->type)->ttype;
    if (f->vm <= DG_VM_INLINE_MAX) {
        w8(b, ft);
        w16(b, f->id);
        if (f->vm != DG_VM_JSCONV)
            return PACK(E_UNSUPPORT_VM_TYPE, (uint64_t)f->vm, (uint64_t)*p);
        uint8_t ch = AT(src, *p - 1);
        if (ch == '"') {
            if (ft == DG_T_STRING)
                return j2t_string(m, p);
            if (AT(src, *p) == '"') {
                uint64_t r = tb_write_default_or_empty(m, f, *p);
                if (r)
                    return r;
                *p += 1;
                return 0;
            }
        } else {
            if (ch != '-' && (ch < '0' || ch > '9'))
                return PACK(E_INVAL, (uint64_t)(int64_t)(int8_t)ch, (uint64_t)*p);
            *p -= 1;
        }
        int64_t s = *p;
        vnumber(src, p, &m->jt);
        if (m->jt.vt != V_INTEGER && m->jt.vt != V_DOUBLE)
            return PACK(E_NUMBER_FMT, (uint64_t)m->jt.vt, (uint64_t)*p);
        bool isint = m->jt.vt == V_INTEGER;
        switch (ft) {
        case DG_T_STRING:
            wstring(b, src->s + s, *p - s);
            return 0;
        case DG_T_I64:
            w64(b, isint ? (uint64_t)m->jt.iv : (uint64_t)cvt64(m->jt.dv));
            break;
        case DG_T_I32:
            w32(b, isint ? (uint32_t)m->jt.iv : (uint32_t)cvt32(m->jt.dv));
            break;
        case DG_T_I16:
            w16(b, isint ? (uint16_t)m->jt.iv : (uint16_t)cvt32(m->jt.dv));
            /* fallthrough: the reference misses a break (native/thrift.c:590-603) */
        case DG_T_BYTE:
            w8(b, isint ? (uint8_t)m->jt.iv : (uint8_t)cvt32(m->jt.dv));
            break;
        case DG_T_DOUBLE:
            wdouble(b, m->jt.dv);
            break;
        default:
            return PACK(E_UNSUPPORT_THRIFT_TYPE, (uint64_t)ft, (uint64_t)*p);
        }
        if (ch == '"') {
            if (AT(src, *p) != '"')
                return PACK(E_INVAL, (uint64_t)(int64_t)(int8_t)AT(src, *p), (uint64_t)*p);
            *p += 1;
        }
        return 0;
    }
    /* non-inline value mapping: host callback (ERR_VM_END), served here the
     * way the Go host does and resumed (oracle/vm_host.h); a failing callback
     * returns the ERR_VM_END word */
    *p -= 1;
    int64_t s = *p;
    int64_t r = skip_one(src, p, m->skipstk);
    if (r < 0)
        return PACK(-r, (uint64_t)s, (uint64_t)*p);
    if (*p >= src->n) /* "invalid value-mapping position" (conv/j2t/impl_amd64.go:132-134) */
        return PACK0(E_VM_END, (uint64_t)*p);
    bgrow(b, b->len + (size_t)(*p - r) + 16);
    long k = vmh_write(f->vm, ft, f->id, src->s + r, (size_t)(*p - r), b->b + b->len);
    if (k < 0)
        return PACK0(E_VM_END, (uint64_t)*p);
    b->len += (size_t)k;
    return 0;
}

/* j2t_fsm_exec native/thrift.c:765-1187 */
static uint64_t fsm_exec(M *m)
{
    const Src *src = m->src;
    Buf *buf = m->buf;
    int64_t pv = 0, *p = &pv;
    bool null_val = false;
    size_t unwindPos = 0;
    const dg_field *lastField = NULL;
    uint64_t flag = m->flag;
    while (m->sp) {
        if (m->sp >= MAX_RECURSE)
            return PACK(E_RECURSE_MAX, (uint64_t)m->sp, (uint64_t)*p);
        Frame *vt = &m->vt[m->sp - 1];
        uint32_t dc = vt->td;
        uint32_t st = vt->st;
        uint8_t ch = advance_ns(src, p);
        switch (st & 0xffff) {
        default:
            m->sp--;
            break;
        case J_ARR_0:
            if (ch == ']') {
                put32(buf, vt->bp, 0);
                m->sp--;
                continue;
            }
            vt->size = 0;
            vt->st = J_ARR;
            *p -= 1;
            PUSH(m, J_VAL, TY(m, dc)->elem);
            continue;
        case J_ARR:
            if (ch == ']') {
                if (!null_val)
                    vt->size += 1;
                else
                    null_val = false;
                put32(buf, vt->bp, (uint32_t)vt->size);
                m->sp--;
                continue;
            }
            if (ch == ',') {
                if (!null_val)
                    vt->size += 1;
                else
                    null_val = false;
                PUSH(m, J_VAL, TY(m, dc)->elem);
                continue;
            }
            return PACK(E_INVAL, V2((int8_t)ch, J_ARR), (uint64_t)*p);
        case J_OBJ_0:
            if (ch == '}') {
                if (TY(m, dc)->ttype == DG_T_STRUCT) {
                    const dg_struct *sd = &m->D.S[TY(m, dc)->st];
                    uint64_t r = write_unset_fields(m, sd, vt->reqs, *p - 1);
                    if (r)
                        return r;
                    m->reqs_len -= sd->req_words;
                    if ((flag & F_ENABLE_HM) && m->field_cache_len > 0)
                        return PACK0(E_HM_END, (uint64_t)*p);
                    w8(buf, 0);
                } else {
                    put32(buf, vt->bp, 0);
                }
                m->sp--;
                continue;
            }
            if (ch == '"') {
                vt->st = J_OBJ;
                uint64_t r = j2t_key(m, p, dc, true, &unwindPos, &lastField, vt);
                if (r)
                    return r;
                continue;
            }
            return PACK(E_INVAL, V2((int8_t)ch, J_OBJ_0), (uint64_t)*p);
        case J_OBJ:
            if (ch == '}') {
                if (TY(m, dc)->ttype == DG_T_STRUCT) {
                    const dg_struct *sd = &m->D.S[TY(m, dc)->st];
                    if (null_val) {
                        null_val = false;
                        uint32_t k = (uint32_t)(lastField - m->D.F) - sd->field_begin;
                        bm_set_req(m, vt->reqs, k, lastField->required);
                        buf->len = unwindPos;
                    }
                    uint64_t r = write_unset_fields(m, sd, vt->reqs, *p - 1);
                    if (r)
                        return r;
                    m->reqs_len -= sd->req_words;
                    if ((flag & F_ENABLE_HM) && m->field_cache_len != 0)
                        return PACK0(E_HM_END, (uint64_t)*p);
                    w8(buf, 0);
                } else {
                    if (!null_val)
                        vt->size += 1;
                    else {
                        null_val = false;
                        buf->len = unwindPos;
                    }
                    put32(buf, vt->bp, (uint32_t)vt->size);
                }
                m->sp--;
                continue;
            }
            if (ch == ',') {
                if (TY(m, dc)->ttype == DG_T_MAP) {
                    if (!null_val)
                        vt->size += 1;
                    else {
                        null_val = false;
                        buf->len = unwindPos;
                    }
                } else if (null_val) {
                    null_val = false;
                    const dg_struct *sd = &m->D.S[TY(m, dc)->st];
                    uint32_t k = (uint32_t)(lastField - m->D.F) - sd->field_begin;
                    bm_set_req(m, vt->reqs, k, lastField->required);
                    buf->len = unwindPos;
                }
                PUSH(m, J_KEY, dc);
                continue;
            }
            return PACK(E_INVAL, V2((int8_t)ch, J_OBJ), (uint64_t)*p);
        case J_KEY: {
            if (ch != '"')
                return PACK(E_INVAL, V2('"', J_KEY), (uint64_t)*p);
            uint64_t r = j2t_key(m, p, dc, false, &unwindPos, &lastField, vt);
            if (r)
                return r;
            continue;
        }
        case J_ELEM:
            if (ch != ':')
                return PACK(E_INVAL, V2(':', J_ELEM), (uint64_t)*p);
            vt->st = J_VAL | (st & 0xffff0000u);
            continue;
        }
        /* J_VAL (already dropped) */
        if (st & ST_SKIP) {
            *p -= 1;
            int64_t s = *p;
            int64_t r = skip_one(src, p, m->skipstk);
            if (r < 0)
                return PACK(-r, (uint64_t)s, (uint64_t)*p);
            continue;
        }
        if ((flag & F_ENABLE_VM) && (st & ST_VM)) {
            uint64_t r = j2t_field_vm(m, p, vt);
            if (r)
                return r;
            continue;
        }
        const dg_type *t = TY(m, dc);
        switch (ch) {
        case '0': case '1': case '2': case '3': case '4':
        case '5': case '6': case '7': case '8': case '9': case '-': {
            *p -= 1;
            uint64_t r = j2t_number(m, dc, src, p);
            if (r)
                return r;
            break;
        }
        case 'n': {
            int64_t s = *p;
            int64_t r = advance_dword(src, p, 1, *p - 1, VS_NULL);
            if (r < 0)
                return PACK(-r, (uint64_t)s, (uint64_t)*p);
            null_val = true;
            break;
        }
        case 't':
        case 'f': {
            int64_t s = *p;
            int64_t r = ch == 't' ? advance_dword(src, p, 1, *p - 1, VS_TRUE)
                                  : advance_dword(src, p, 0, *p - 1, VS_ALSE);
            if (r < 0)
                return PACK(-r, (uint64_t)s, (uint64_t)*p);
            if (t->ttype != DG_T_BOOL)
                return PACK(E_DISMATCH_TYPE, V2(t->ttype, DG_T_BOOL), (uint64_t)*p);
            w8(buf, ch == 't' ? 1 : 0);
            break;
        }
        case '[': {
            if (t->ttype != DG_T_LIST && t->ttype != DG_T_SET)
                return PACK(E_DISMATCH_TYPE2,
                            (uint32_t)(((uint32_t)t->ttype << 16) | ((uint16_t)DG_T_SET << 8) | (uint8_t)DG_T_LIST),
                            (uint64_t)*p);
            w8(buf, TY(m, t->elem)->ttype);
            size_t bp = bmalloc(buf, 4);
            PUSH(m, J_ARR_0, dc);
            m->vt[m->sp - 1].bp = bp;
            m->vt[m->sp - 1].size = 0;
            break;
        }
        case '{': {
            if (t->ttype != DG_T_STRUCT && t->ttype != DG_T_MAP)
                return PACK(E_DISMATCH_TYPE2,
                            (uint32_t)(((uint32_t)t->ttype << 16) | ((uint16_t)DG_T_MAP << 8) | (uint8_t)DG_T_STRUCT),
                            (uint64_t)*p);
            if (t->ttype == DG_T_STRUCT) {
                const dg_struct *sd = &m->D.S[t->st];
                PUSH(m, J_OBJ_0, dc);
                Frame *x = &m->vt[m->sp - 1];
                /* bm_malloc_reqs native/thrift.c:232-250 */
                if (m->reqs_len + sd->req_words > m->reqs_cap) {
                    m->reqs_cap = (m->reqs_len + sd->req_words) * 2;
                    m->reqs = (uint64_t *)realloc(m->reqs, m->reqs_cap * 8);
                }
                x->reqs = (uint32_t)m->reqs_len;
                memcpy(&m->reqs[m->reqs_len], &m->D.R[sd->req_begin], sd->req_words * 8);
                m->reqs_len += sd->req_words;
                if ((flag & F_ENABLE_HM) && (sd->flags & DG_SF_HTTP_MAPPING))
                    return PACK0(E_HM, (uint64_t)(*p - 1));
            } else {
                w8(buf, TY(m, t->key)->ttype);
                w8(buf, TY(m, t->elem)->ttype);
                size_t bp = bmalloc(buf, 4);
                PUSH(m, J_OBJ_0, dc);
                m->vt[m->sp - 1].bp = bp;
                m->vt[m->sp - 1].size = 0;
            }
            break;
        }
        case '"': {
            uint64_t r;
            if (t->ttype == DG_T_STRING) {
                if ((flag & F_NO_BASE64) == 0 && (t->flags & DG_TF_BINARY))
                    r = j2t_binary(m, p);
                else
                    r = j2t_string(m, p);
                if (r)
                    return r;
            } else if ((flag & F_ENABLE_I2S) &&
                       (t->ttype == DG_T_I64 || t->ttype == DG_T_I32 || t->ttype == DG_T_I16 ||
                        t->ttype == DG_T_BYTE || t->ttype == DG_T_DOUBLE)) {
                if (AT(src, *p) == '"') {
                    r = tb_write_empty(m, dc, *p);
                    if (r)
                        return r;
                } else {
                    r = j2t_number(m, dc, src, p);
                    if (r)
                        return r;
                    int64_t x = *p;
                    if (x >= src->n)
                        return PACK(E_EOF, 0, (uint64_t)*p);
                    if (AT(src, x) != '"')
                        return PACK(E_INVAL, V2((int8_t)AT(src, x), J_VAL), (uint64_t)*p);
                }
                *p += 1;
            } else {
                return PACK(E_DISMATCH_TYPE, V2(t->ttype, DG_T_STRING), (uint64_t)*p);
            }
            break;
        }
        case 0:
            return PACK(E_EOF, 0, (uint64_t)*p);
        default:
            return PACK(E_INVAL, V2((int8_t)ch, J_VAL), (uint64_t)*p);
        }
    }
    return 0;
}

/* ====================================================================== */
/* C ABI (same shape as oracle/ref_harness.c)                              */
/* ====================================================================== */
void *dgo_desc_create(const uint8_t *blob, size_t len)
{
    const dg_desc_hdr *h = (const dg_desc_hdr *)blob;
    if (len < sizeof(*h) || h->magic != DG_DESC_MAGIC || h->total_len > len)
        return NULL;
    Desc *d = (Desc *)calloc(1, sizeof(Desc));
    uint8_t *b = (uint8_t *)malloc(len);
    memcpy(b, blob, len);
    d->blob = b;
    d->h = (const dg_desc_hdr *)b;
    d->T = (const dg_type *)(b + h->off_types);
    d->S = (const dg_struct *)(b + h->off_structs);
    d->F = (const dg_field *)(b + h->off_fields);
    d->N = (const dg_name *)(b + h->off_names);
    d->R = (const uint64_t *)(b + h->off_reqwords);
    d->P = b + h->off_pool;
    return d;
}

void dgo_desc_destroy(void *p)
{
    Desc *d = (Desc *)p;
    if (d) {
        free((void *)d->blob);
        free(d);
    }
}

typedef struct {
    Frame *vt;
    int *skipstk;
    uint64_t *reqs;
    size_t reqs_cap;
    uint8_t *keybuf;
    size_t keycap;
    uint8_t *src;
    size_t srccap;
    Buf buf;
} Ctx;

static Ctx *ctx_new(void)
{
    Ctx *c = (Ctx *)calloc(1, sizeof(Ctx));
    c->vt = (Frame *)calloc(MAX_RECURSE + 1, sizeof(Frame));
    c->skipstk = (int *)calloc(MAX_RECURSE + 1, sizeof(int));
    c->reqs_cap = 512;
    c->reqs = (uint64_t *)malloc(c->reqs_cap * 8);
    return c;
}
static void ctx_free(Ctx *c)
{
    free(c->vt);
    free(c->skipstk);
    free(c->reqs);
    free(c->keybuf);
    free(c->src);
    free(c->buf.b);
    free(c);
}

/* quote of an unquoted STRING root (conv/j2t/impl.go:85-88) followed by the
 * FSM's unquote is the identity on the raw bytes: json.EncodeString escapes
 * only '"', '\\' and control bytes (native/parsing.c:28-62), all of which
 * unquote restores byte-for-byte. */
static uint64_t do_one(Ctx *c, Desc *d, uint32_t root, const uint8_t *json, size_t n, uint64_t flags)
{
    c->buf.len = 0;
    if (n == 0) {
        w8(&c->buf, 0);
        return 0;
    }
    if (d->T[root].ttype == DG_T_STRING && json[0] != '"') {
        wstring(&c->buf, json, n);
        return 0;
    }
    if (c->srccap < n + 8) {
        free(c->src);
        c->srccap = n + 8;
        c->src = (uint8_t *)malloc(c->srccap);
    }
    memcpy(c->src, json, n);
    memset(c->src + n, 0, 8);
    if (c->keycap < n + 8) {
        free(c->keybuf);
        c->keycap = n + 8;
        c->keybuf = (uint8_t *)malloc(c->keycap);
    }
    Src src = {c->src, (int64_t)n};
    M m;
    memset(&m, 0, sizeof(m));
    m.D = *d;
    m.buf = &c->buf;
    m.src = &src;
    m.flag = flags;
    m.vt = c->vt;
    m.sp = 1;
    m.vt[0].st = J_VAL;
    m.vt[0].td = root;
    m.reqs = c->reqs;
    m.reqs_cap = c->reqs_cap;
    m.skipstk = c->skipstk;
    m.keybuf = c->keybuf;
    uint64_t r = fsm_exec(&m);
    c->reqs = m.reqs;
    c->reqs_cap = m.reqs_cap;
    return r;
}

static Ctx *g_ctx;

uint64_t dgo_j2t(void *desc, uint32_t root, const uint8_t *json, size_t n, uint64_t flags, uint8_t *out,
                 size_t out_cap, size_t *out_len)
{
    if (!g_ctx)
        g_ctx = ctx_new();
    uint64_t r = do_one(g_ctx, (Desc *)desc, root, json, n, flags);
    *out_len = 0;
    if (r)
        return r;
    *out_len = g_ctx->buf.len;
    if (g_ctx->buf.len <= out_cap)
        memcpy(out, g_ctx->buf.b, g_ctx->buf.len);
    return 0;
}

int dgo_j2t_batch(void *desc, uint32_t root, const uint8_t *json, const uint64_t *in_off, uint64_t n,
                  uint64_t flags, uint8_t *out, const uint64_t *out_off, uint32_t *out_len, uint64_t *ret,
                  int nthreads)
{
    (void)nthreads; /* scalar port: one thread */
    Ctx *c = ctx_new();
    for (uint64_t i = 0; i < n; i++) {
        uint64_t r = do_one(c, (Desc *)desc, root, json + in_off[i], in_off[i + 1] - in_off[i], flags);
        ret[i] = r;
        out_len[i] = r ? 0 : (uint32_t)c->buf.len;
        uint64_t cap = out_off[i + 1] - out_off[i];
        if (!r && c->buf.len <= cap)
            memcpy(out + out_off[i], c->buf.b, c->buf.len);
    }
    ctx_free(c);
    return 0;
}
