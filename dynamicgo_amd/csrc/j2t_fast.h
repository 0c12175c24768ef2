/*
 * j2t_fast.h — the fast path of the lane-per-message transcoder.
 *
 * The exact machine (j2t_kernel.hip, Machine<>) restates j2t_fsm_exec state by
 * state, error word by error word. Almost every production message takes only
 * a small, error-free part of that automaton, so the kernel first runs this
 * leaner converter, which accepts exactly the inputs on which it can produce
 * the reference's output and BAILS on everything else (any error, unusual
 * flags, escaped keys, deep nesting, >64-field structs, numbers needing the
 * big-decimal slow path, output-slot overflow). A bailed message is redone
 * from scratch by the exact machine, so results are bit-identical either way
 * and error words always come from the exact machine.
 *
 * What makes it faster than the state-by-state FSM:
 *  - the innermost container lives in registers (LDS holds only parents);
 *  - object keys are matched against a PREDICTED field (the one after the
 *    previous field, dg_field.key_off/key_len in descriptor v2) by 8-byte word
 *    compares; the hash table is only probed on a miss;
 *  - digits are scanned and accumulated 8 at a time (SWAR), base64 is decoded
 *    8 characters -> 6 bytes at a time, escaped strings are copied in runs
 *    between backslashes.
 *
 * Reference semantics reproduced here: j2t_fsm_exec native/thrift.c:765-1187
 * (container/null/unset handling), vnumber native/scanning.c:958-1083,
 * unquote native/parsing.c:702-945, b64decode native/base64.c:659-817.
 */
#pragma once
#include "j2t_device.h"

namespace dg {

/* -DDG_FPROF: wave-time breakdown of the fast path by region (cycles per
 * wave, s_memtime, summed in LDS by the first active lane of each mark) */
#ifdef DG_FPROF
DGI unsigned long long *fprof_slots()
{
    __shared__ unsigned long long s_fp[16][17]; /* [wave][0..15 regions, 16 = last mark] */
    return &s_fp[0][0];
}
DGI void fprof_mark(int k)
{
    const uint64_t now = __builtin_amdgcn_s_memtime();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t ex = __builtin_amdgcn_read_exec();
    if (lane == (uint32_t)__builtin_ctzll(ex)) {
        unsigned long long *f = fprof_slots() + w * 17;
        f[k] += now - f[16];
        f[16] = now;
    }
}
#define FP_MARK(k) fprof_mark(k)
#else
#define FP_MARK(k)
#endif

/* positions inside one message: the source's index type (32-bit for an
 * LDS-staged source, 64-bit for a global one) */
#define SI typename S::idx

constexpr uint32_t FK_STRUCT = 1, FK_MAP = 2, FK_LIST = 3;
constexpr uint32_t FAST_LDS_DEPTH = 8; /* parent frames per lane in LDS */

/* one parent container of the fast path (16 B) */
struct FFrame {
    uint32_t a; /* struct: struct index; map/list: element type */
    uint32_t b; /* kind | (hint or count) << 2 */
    uint64_t u; /* struct: requires bits; list: size position; map: size position | key type << 32 */
};
typedef __attribute__((address_space(3))) FFrame LFFrame;
typedef const __attribute__((address_space(3))) double lds_f64;

/* flags the fast path handles itself; any other flag bit -> bail at entry */
/* F_ENABLE_HM is in: its only effects are on structs with HTTP-mapped fields
 * (ERR_HM at entry native/thrift.c:1119-1123, mapped keys skipped
 * native/thrift.c:725), which the fast paths decline; ERR_HM_END needs
 * F_TRACE_BACK, which stays out. DG_F_HM_SPLIT only changes what the exact
 * machine does at such a struct (j2t_machine.h), so it is in too. */
constexpr uint64_t FAST_FLAGS = DG_F_ALLOW_UNKNOWN | DG_F_WRITE_DEFAULT | DG_F_ENABLE_VM | DG_F_ENABLE_I2S |
                                DG_F_WRITE_REQUIRE | DG_F_NO_BASE64 | DG_F_WRITE_OPTIONAL | DG_F_NO_WRITE_BASE |
                                DG_F_ENABLE_HM | DG_F_HM_SPLIT | DG_F_CB_COLLECT;

/* small power tables, copied to LDS by the kernel prologue */
/* DG_POW10_M128[e + 348][1] for e in [EL_WLO, EL_WLO + EL_WN): the decimal
 * exponents of ordinary JSON doubles, so Eisel-Lemire reads LDS, not the
 * 11 KiB table in global memory */
constexpr int EL_WLO = -40;
constexpr int EL_WN = 64;
struct FastTabs {
    const __attribute__((address_space(3))) uint64_t *p10u; /* 10^k, k = 0..19 */
    lds_f64 *p10d;                                          /* 1e0 .. 1e22 */
    const __attribute__((address_space(3))) uint64_t *pw = nullptr; /* the window above, or none */
};
/* fill a FastTabs window (lanes t < EL_WN of the block) */
DGI void el_window_fill(uint64_t *pw, uint32_t t)
{
    if (t < (uint32_t)EL_WN) pw[t] = DG_POW10_M128[EL_WLO + 348 + (int)t][1];
}
DGI bool eisel_lemire_t(uint64_t mant, int exp10, int sgn, double &val, const FastTabs &tb)
{
    if (exp10 < -348 || exp10 > 347) return false;
    const uint32_t wi = (uint32_t)(exp10 - EL_WLO);
    const uint64_t p_hi = tb.pw && wi < (uint32_t)EL_WN ? tb.pw[wi] : DG_POW10_M128[exp10 + 348][1];
    return eisel_lemire_p(mant, exp10, sgn, val, p_hi);
}

/* ---- SWAR helpers ---- */

/* leading ASCII digits among the 8 bytes at src[i..] (bytes at >= n excluded);
 * x = the bytes XOR '0' (digit values in the digit bytes) */
template <class S>
DGI uint32_t digits8(S &src, SI i, uint64_t &x)
{
    uint64_t w = src.get8(i);
    const uint32_t xl = (uint32_t)w ^ 0x30303030u, xh = (uint32_t)(w >> 32) ^ 0x30303030u;
    x = (uint64_t)xl | ((uint64_t)xh << 32);
    /* a byte is a digit iff (b ^ '0') < 10: adding 0x76 sets its top bit otherwise */
    uint32_t ndl = (((xl & 0x7F7F7F7Fu) + 0x76767676u) | xl) & 0x80808080u;
    uint32_t ndh = (((xh & 0x7F7F7F7Fu) + 0x76767676u) | xh) & 0x80808080u;
    SI lim = src.n - i;
    if (lim < 8) {
        if (lim <= 4) {
            ndh = 0x80808080u;
            if (lim < 4) ndl |= lim <= 0 ? 0x80808080u : (0x80808080u & (~0u << (lim << 3)));
        } else {
            ndh |= 0x80808080u & (~0u << ((lim - 4) << 3));
        }
    }
    if (ndl) return (uint32_t)__builtin_ctz(ndl) >> 3;
    return ndh ? 4u + ((uint32_t)__builtin_ctz(ndh) >> 3) : 8u;
}

/* value of the first k (0..4) digits of a 32-bit group (bytes XOR '0', first
 * digit lowest): shifts and 24-bit multiplies only */
DGI uint32_t swar_val4(uint32_t x, uint32_t k)
{
    uint32_t y = k >= 4 ? x : (k == 0 ? 0u : x << ((4 - k) << 3));
    y &= 0x0F0F0F0Fu;
    y = (((y << 3) + (y << 1)) + (y >> 8)) & 0x00FF00FFu; /* d0*10+d1 | d2*10+d3 << 16 */
    return __umul24(y & 0xFFu, 100u) + (y >> 16);
}
/* value of the first t (1..8) digits of x */
DGI uint64_t swar_val(uint64_t x, uint32_t t)
{
    const uint32_t t1 = t < 4 ? t : 4u, t2 = t - t1;
    const uint32_t v1 = swar_val4((uint32_t)x, t1);
    if (!t2) return v1;
    const uint32_t v2 = swar_val4((uint32_t)(x >> 32), t2);
    const uint32_t p = t2 == 1 ? 10u : t2 == 2 ? 100u : t2 == 3 ? 1000u : 10000u;
    return (uint64_t)v1 * p + v2; /* < 10^8 */
}

/* man = man * 10^t + (first t digits), t = min(k, 19 - nd) (the reference's
 * `if (man_nd < 19)` digit cap); returns t */
DGI uint32_t acc_digits(uint64_t &man, int &nd, uint64_t x, uint32_t k, const FastTabs &tb)
{
    (void)tb;
    uint32_t room = (uint32_t)(19 - nd);
    uint32_t t = k < room ? k : room;
    if (t) {
        /* 10^t (t <= 8) in registers: 32-bit, so man * p is one 64x32 product */
        uint32_t p = (t & 1) ? 10u : 1u;
        p = (t & 2) ? p * 100u : p;
        p = (t & 4) ? p * 10000u : p;
        p = (t & 8) ? 100000000u : p;
        man = man * (uint64_t)p + swar_val(x, t);
        nd += (int)t;
    }
    return t;
}

/* is_atof_exact (native/scanning.c:883-926) with the powers in LDS */
DGI bool atof_exact_l(uint64_t man, int exp, int sgn, double &val, const FastTabs &tb)
{
    val = (double)man;
    if (man >> 52 != 0) return false;
    val = with_sign(val, sgn);
    if (exp == 0 || man == 0) return true;
    if (exp > 0 && exp <= 15 + 22) {
        if (exp > 22) {
            val = __dmul_rn(val, tb.p10d[exp - 22]);
            exp = 22;
        }
        if (val > 1e15 || val < -1e15) return false;
        val = __dmul_rn(val, tb.p10d[exp]);
        return true;
    }
    if (exp < 0 && exp >= -22) {
        val = __ddiv_rn(val, tb.p10d[-exp]);
        return true;
    }
    return false;
}

/* A whole token that is a plain integer, -?(0|[1-9][0-9]{0,18}), from a
 * register source (RSrc / RSrcL: the token's first 24 bytes in registers,
 * src.n its exact length): its value in a fixed number of steps -- three
 * 8-digit SWAR chunks, no data-dependent loop -- so a wave whose lanes hold
 * integers of different lengths runs one path. Anything else (a '.', an
 * exponent, a sign without digits, a leading zero before digits, 20+ digits,
 * a 19-digit value past int64) returns false and takes fast_vnumber's
 * general loop, whose results these are (native/scanning.c:958-1083 on this
 * shape: is_overflow false, iv = man * sgn, dv = (double)man with the sign). */
template <class S>
DGI bool fast_int_regs(const S &src, int64_t &iv, double &dv, int32_t &end)
{
    const int32_t n = (int32_t)src.n;
    if (n < 1 || n > 20) return false;
    const uint64_t a0 = src.get8(0), a1 = src.get8(8), a2 = src.get8(16);
    const uint32_t neg = (uint8_t)a0 == '-' ? 1u : 0u;
    const uint32_t nd = (uint32_t)n - neg;
    /* the digits from byte 0 */
    const uint64_t d0 = neg ? (a0 >> 8) | (a1 << 56) : a0, d1 = neg ? (a1 >> 8) | (a2 << 56) : a1,
                   d2 = neg ? a2 >> 8 : a2;
    const uint64_t x0 = d0 ^ 0x3030303030303030ull, x1 = d1 ^ 0x3030303030303030ull, x2 = d2 ^ 0x3030303030303030ull;
    auto nondig = [](uint64_t x) { return (((x & 0x7F7F7F7F7F7F7F7Full) + 0x7676767676767676ull) | x) & 0x8080808080808080ull; };
    auto upto = [](uint32_t k) { return k >= 8 ? ~0ull : (1ull << (k << 3)) - 1; }; /* the first k bytes */
    const uint32_t t0 = nd < 8 ? nd : 8u, t1 = nd <= 8 ? 0u : nd - 8 < 8 ? nd - 8 : 8u, t2 = nd <= 16 ? 0u : nd - 16;
    const uint64_t bad = (nondig(x0) & upto(t0)) | (nondig(x1) & upto(t1)) | (nondig(x2) & upto(t2));
    const uint32_t f = (uint32_t)(x0 & 0xFF); /* first digit's value */
    if (nd < 1 || nd > 19 || bad || (f == 0 && nd > 1)) return false;
    auto p10 = [](uint32_t t) {
        uint32_t p = (t & 1) ? 10u : 1u;
        p = (t & 2) ? p * 100u : p;
        p = (t & 4) ? p * 10000u : p;
        return (t & 8) ? 100000000u : p;
    };
    uint64_t man = swar_val(x0, t0);
    man = man * (uint64_t)p10(t1) + swar_val(x1, t1);
    man = man * (uint64_t)p10(t2) + swar_val(x2, t2);
    if ((man >> 63) && !(neg && man == (1ull << 63))) return false; /* is_overflow: the double path */
    const int sgn = neg ? -1 : 1;
    iv = (int64_t)(man * (uint64_t)(int64_t)sgn);
    dv = man ? with_sign((double)man, sgn) : 0.0; /* "-0": the general path's +0.0 */
    end = n;
    return true;
}

/* A whole token that is a plain decimal, -?[0-9]+\.[0-9]+ with at most 19
 * digits in all, from a register source: its mantissa (every digit, the
 * point removed) and exponent (minus the fraction digits) in a fixed number
 * of steps, as fast_int_regs. These are exactly the (man, exp10) that
 * vnumber's digit loops (native/scanning.c:958-1083, fast_vnumber's general
 * path) build for such a token: leading zeros add nothing to man, and 19
 * digits never reach the 19-digit cap, so nothing is truncated. A leading
 * zero before more integer digits, an exponent, a second point or anything
 * else returns false and takes the general path. */
template <class S>
DGI bool fast_dec_regs(const S &src, uint64_t &man, int &exp10, int &sgn)
{
    const int32_t n = (int32_t)src.n;
    if (n < 3 || n > 21) return false;
    const uint64_t a0 = src.get8(0), a1 = src.get8(8), a2 = src.get8(16);
    const uint32_t neg = (uint8_t)a0 == '-' ? 1u : 0u;
    const uint32_t len = (uint32_t)n - neg; /* digits and the point */
    const uint64_t d0 = neg ? (a0 >> 8) | (a1 << 56) : a0, d1 = neg ? (a1 >> 8) | (a2 << 56) : a1,
                   d2 = neg ? a2 >> 8 : a2;
    auto upto = [](uint32_t k) { return k >= 8 ? ~0ull : (1ull << (k << 3)) - 1; }; /* the first k bytes */
    auto eqdot = [](uint64_t x) {
        const uint64_t y = x ^ 0x2E2E2E2E2E2E2E2Eull;
        return ~(((y & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | y | 0x7F7F7F7F7F7F7F7Full);
    };
    const uint32_t u0 = len < 8 ? len : 8u, u1 = len <= 8 ? 0u : len - 8 < 8 ? len - 8 : 8u,
                   u2 = len <= 16 ? 0u : len - 16;
    const uint64_t m0 = eqdot(d0) & upto(u0), m1 = eqdot(d1) & upto(u1), m2 = eqdot(d2) & upto(u2);
    if (__builtin_popcountll(m0) + __builtin_popcountll(m1) + __builtin_popcountll(m2) != 1) return false;
    const uint32_t pd = m0 ? (uint32_t)__builtin_ctzll(m0) >> 3
                       : m1 ? 8u + ((uint32_t)__builtin_ctzll(m1) >> 3) : 16u + ((uint32_t)__builtin_ctzll(m2) >> 3);
    if (pd < 1 || pd + 2 > len) return false; /* a digit on both sides */
    /* the point removed: bytes above it move down one */
    const uint64_t s0 = (d0 >> 8) | (d1 << 56), s1 = (d1 >> 8) | (d2 << 56), s2 = d2 >> 8;
    const uint64_t k0 = upto(pd), k1 = pd <= 8 ? 0ull : upto(pd - 8), k2 = pd <= 16 ? 0ull : upto(pd - 16);
    const uint64_t r0 = (d0 & k0) | (s0 & ~k0), r1 = (d1 & k1) | (s1 & ~k1), r2 = (d2 & k2) | (s2 & ~k2);
    const uint32_t nd = len - 1;
    const uint64_t x0 = r0 ^ 0x3030303030303030ull, x1 = r1 ^ 0x3030303030303030ull, x2 = r2 ^ 0x3030303030303030ull;
    auto nondig = [](uint64_t x) { return (((x & 0x7F7F7F7F7F7F7F7Full) + 0x7676767676767676ull) | x) & 0x8080808080808080ull; };
    const uint32_t t0 = nd < 8 ? nd : 8u, t1 = nd <= 8 ? 0u : nd - 8 < 8 ? nd - 8 : 8u, t2 = nd <= 16 ? 0u : nd - 16;
    const uint64_t bad = (nondig(x0) & upto(t0)) | (nondig(x1) & upto(t1)) | (nondig(x2) & upto(t2));
    if (nd > 19 || bad || ((x0 & 0xFF) == 0 && pd > 1)) return false;
    auto p10 = [](uint32_t t) {
        uint32_t p = (t & 1) ? 10u : 1u;
        p = (t & 2) ? p * 100u : p;
        p = (t & 4) ? p * 10000u : p;
        return (t & 8) ? 100000000u : p;
    };
    uint64_t m = swar_val(x0, t0);
    m = m * (uint64_t)p10(t1) + swar_val(x1, t1);
    m = m * (uint64_t)p10(t2) + swar_val(x2, t2);
    man = m;
    exp10 = -(int)(nd - pd);
    sgn = neg ? -1 : 1;
    return true;
}

/* register sources (RSrc, RSrcL: kRegs) take fast_int_regs first */
template <class S, class = void>
struct is_regsrc {
    static constexpr bool value = false;
};
template <class S>
struct is_regsrc<S, decltype((void)S::kRegs)> {
    static constexpr bool value = S::kRegs;
};

/* vnumber (native/scanning.c:958-1083) on the success paths; false = the
 * reference would error or need atof_native -> bail. */
template <class S>
DGI bool fast_vnumber(S &src, SI &p, const FastTabs &tb, int64_t &iv, double &dv, bool &isint)
{
    SI i = p;
    uint64_t man = 0;
    int exp10 = 0, sgn = 1;
    bool trunc = false, regdec = false;
    if constexpr (is_regsrc<S>::value) {
        int32_t e;
        if (p == 0 && fast_int_regs(src, iv, dv, e)) {
            isint = true;
            p = (SI)e;
            return true;
        }
        if (p == 0 && fast_dec_regs(src, man, exp10, sgn)) {
            regdec = true;
            i = (SI)src.n;
        }
    }
    if (!regdec) {
    uint8_t c = src.at(i);
    if (c == '-') {
        sgn = -1;
        c = src.at(++i);
    }
    if ((uint8_t)(c - '0') > 9) return false;
    isint = true;
    iv = 0;
    dv = 0.0;
    if (c == '0') {
        uint8_t c1 = src.at(i + 1);
        if (c1 != '.' && c1 != 'e' && c1 != 'E') {
            p = i + 1;
            return true;
        }
    }
    int nd = 0;
    bool dbl = false;
    uint64_t x;
    for (;;) { /* integer digits */
        uint32_t k = digits8(src, i, x);
        uint32_t t = acc_digits(man, nd, x, k, tb);
        exp10 += (int)(k - t);
        i += k;
        if (k < 8) break;
    }
    if (exp10 > 0) trunc = true;
    if (src.at(i) == '.') {
        i++;
        dbl = true;
        if ((uint8_t)(src.at(i) - '0') > 9) return false;
    }
    if (man == 0 && exp10 == 0) {
        while (src.at(i) == '0') {
            i++;
            exp10--;
        }
        nd = 0;
    }
    /* without a '.', the integer loop stopped at a non-digit: the two loops
     * below would read no digit */
    while (dbl && nd < 19) { /* fraction digits up to the cap */
        uint32_t k = digits8(src, i, x);
        uint32_t t = acc_digits(man, nd, x, k, tb);
        exp10 -= (int)t;
        i += t;
        if (t < 8) break;
    }
    while (dbl) { /* digits beyond the cap */
        uint32_t k = digits8(src, i, x);
        if (k) trunc = true;
        i += k;
        if (k < 8) break;
    }
    c = src.at(i);
    if (c == 'e' || c == 'E') {
        int esm = 1, e = 0;
        dbl = true;
        c = src.at(++i);
        if (c == '+' || c == '-') {
            esm = c == '+' ? 1 : -1;
            c = src.at(++i);
        }
        if ((uint8_t)(c - '0') > 9) return false;
        while ((uint8_t)(c - '0') <= 9) {
            if (e < 10000) e = e * 10 + (c - '0');
            c = src.at(++i);
        }
        exp10 += e * esm;
    } else if (!dbl) {
        /* is_overflow native/scanning.c:950-956 */
        bool ovf = exp10 != 0 || ((man >> 63) == 1 && (((uint64_t)(int64_t)sgn) & man) != (1ull << 63));
        if (!ovf) {
            iv = (int64_t)(man * (uint64_t)(int64_t)sgn);
            dv = with_sign((double)man, sgn);
            p = i;
            return true;
        }
    }
    } /* !regdec */
    /* atof_fast native/scanning.c:928-948; atof_native -> bail */
    double val;
    if (!atof_exact_l(man, exp10, sgn, val, tb)) {
        if (!eisel_lemire_t(man, exp10, sgn, val, tb)) return false;
        if (trunc) {
            double vu;
            if (!eisel_lemire_t(man + 1, exp10, sgn, vu, tb) || vu != val) return false;
        }
    }
    if ((__double_as_longlong(val) << 1) == 0xFFE0000000000000ull) return false; /* ERR_FLOAT_INF */
    isint = false;
    dv = val;
    p = i;
    return true;
}

/* j2t_number's writes (native/thrift.c:312-365); O = any byte writer */
template <class O>
DGI bool emit_number(O &out, uint8_t tt, bool isint, int64_t iv, double dv)
{
    switch (tt) {
    case DG_T_BYTE: out.w8(isint ? (uint8_t)iv : (uint8_t)cvt32(dv)); return true;
    case DG_T_I16: out.w16(isint ? (uint16_t)iv : (uint16_t)cvt32(dv)); return true;
    case DG_T_I32: out.w32(isint ? (uint32_t)iv : (uint32_t)cvt32(dv)); return true;
    case DG_T_I64: out.w64(isint ? (uint64_t)iv : (uint64_t)cvt64(dv)); return true;
    case DG_T_DOUBLE: out.w64((uint64_t)__double_as_longlong(dv)); return true;
    }
    return false;
}

/* copy src[s0, s0+n) to the output, 8 bytes per step */
template <class S, class O>
DGI void fast_copy(S &src, SI s0, SI n, O &out)
{
    SI i = 0;
    for (; i + 8 <= n; i += 8) out.wle(src.get8(s0 + i), 8);
    if (i < n) out.wle(src.get8(s0 + i), (uint32_t)(n - i));
}

/* 4 hex digits at src[i..i+4) */
template <class S>
DGI bool hex4w(S &src, SI i, uint32_t &v)
{
    uint32_t w = (uint32_t)src.get8(i);
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int h = hexv((uint8_t)(w >> (8 * k)));
        if (h < 0) return false;
        r = (r << 4) | (uint32_t)h;
    }
    v = r;
    return true;
}

/* unquote (native/parsing.c:702-945, flags 0) of src[s0, s0+nb) appended to
 * out: runs between backslashes are copied as words. false = error. */
template <class S, class O>
DGI bool fast_unquote(S &src, SI s0, SI nb, O &out)
{
    SI i = s0, end = s0 + nb;
    while (i < end) {
        uint64_t w = src.get8(i);
        SI rem = end - i;
        uint64_t m = eqbytes(w, '\\');
        if (rem < 8) m &= (1ull << (rem << 3)) - 1;
        if (m == 0) {
            uint32_t k = rem < 8 ? (uint32_t)rem : 8u;
            out.wle(w, k);
            i += k;
            continue;
        }
        uint32_t j = (uint32_t)__builtin_ctzll(m) >> 3;
        if (j) out.wle(w, j);
        i += j;
        if (end - i < 2) return false;
        uint8_t c = src.at(i + 1);
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
        case 'u': cc = 0; break;
        default: return false;
        }
        if (c != 'u') {
            out.w8(cc);
            i += 2;
            continue;
        }
        if (end - i < 6) return false;
        uint32_t r0, r1;
        if (!hex4w(src, i + 2, r0)) return false;
        i += 6;
        if (r0 <= 0x7f) {
            out.w8((uint8_t)r0);
        } else if (r0 <= 0x7ff) {
            out.wle((0xc0 | (r0 >> 6)) | ((0x80 | (r0 & 0x3f)) << 8), 2);
        } else if (r0 < 0xd800 || r0 > 0xdfff) {
            out.wle((0xe0 | (r0 >> 12)) | ((0x80 | ((r0 >> 6) & 0x3f)) << 8) | ((0x80 | (r0 & 0x3f)) << 16), 3);
        } else {
            if (end - i < 6 || r0 > 0xdbff || src.at(i) != '\\' || src.at(i + 1) != 'u') return false;
            if (!hex4w(src, i + 2, r1)) return false;
            if (r1 < 0xdc00 || r1 > 0xdfff) return false;
            i += 6;
            r0 = ((r0 - 0xd800) << 10) + (r1 - 0xdc00) + 0x10000;
            out.wle((0xf0 | (r0 >> 18)) | ((0x80 | ((r0 >> 12) & 0x3f)) << 8) | ((0x80 | ((r0 >> 6) & 0x3f)) << 16) |
                        ((uint64_t)(0x80 | (r0 & 0x3f)) << 24),
                    4);
        }
    }
    return true;
}

/* j2t_string (native/thrift.c:367-399); p is just past the opening quote */
template <class S>
DGI bool fast_string(S &src, SI &p, Out &out)
{
    SI s0 = p;
    bool esc;
    SI e = advance_string(src, s0, esc);
    if (e < 0) return false;
    p = e;
    SI nb = e - 1 - s0;
    if (!esc) {
        out.w32((uint32_t)nb);
        fast_copy(src, s0, nb, out);
        return true;
    }
    uint64_t lp = out.alloc(4);
    uint64_t st = out.len;
    if (!fast_unquote(src, s0, nb, out)) return false;
    out.put32(lp, (uint32_t)(out.len - st));
    return true;
}

/* 8 base64 characters -> 6 bytes (little-endian in *o); false if any is not
 * in the standard alphabet */
/* 4 base64 characters (little-endian in w) -> 3 bytes in output order in the
 * low 24 bits of o; false if any is not in the standard alphabet */
DGI bool b64_4(uint32_t w, uint32_t &o)
{
    const uint32_t H = 0x80808080u;
    if (w & H) return false;
#define DG_GE(lo) ((w + (uint32_t)(0x80 - (lo)) * 0x01010101u) & H)
    const uint32_t up = DG_GE('A') & ~DG_GE('Z' + 1);
    const uint32_t lw = DG_GE('a') & ~DG_GE('z' + 1);
    const uint32_t dg = DG_GE('0') & ~DG_GE('9' + 1);
#undef DG_GE
    const uint32_t pl = zb32(w ^ 0x2B2B2B2Bu), sl = zb32(w ^ 0x2F2F2F2Fu);
    if ((up | lw | dg | pl | sl) != H) return false;
    /* per-byte offsets: 'A'->0 (-65), 'a'->26 (-71), '0'->52 (+4), '+'->62 (+19), '/'->63 (+16) */
    const uint32_t off = (ff32(up) & 0xBFBFBFBFu) | (ff32(lw) & 0xB9B9B9B9u) | (ff32(dg) & 0x04040404u) |
                         (ff32(pl) & 0x13131313u) | (ff32(sl) & 0x10101010u);
    const uint32_t v = ((w & 0x7F7F7F7Fu) + (off & 0x7F7F7F7Fu)) ^ ((w ^ off) & H); /* bytewise add mod 256 */
    const uint32_t t = ((v & 0x3Fu) << 18) | (((v >> 8) & 0x3Fu) << 12) | (((v >> 16) & 0x3Fu) << 6) | (v >> 24);
    o = (t >> 16) | (t & 0xFF00u) | ((t & 0xFFu) << 16);
    return true;
}
/* 8 base64 characters -> 6 bytes (little-endian in *o); false if any is not
 * in the standard alphabet */
DGI bool b64_8(uint64_t w, uint64_t &o)
{
    uint32_t lo, hi;
    const bool a = b64_4((uint32_t)w, lo), b = b64_4((uint32_t)(w >> 32), hi);
    o = (uint64_t)lo | ((uint64_t)hi << 24);
    return a && b;
}

/* j2t_binary (native/thrift.c:401-420) */
template <class S>
DGI bool fast_binary(S &src, SI &p, Out &out)
{
    SI s0 = p;
    bool esc;
    SI e = advance_string(src, s0, esc);
    if (e < 0 || esc) return false; /* '\\' is outside the alphabet: decode error */
    p = e;
    SI nb = e - 1 - s0;
    /* a canonical padded body decodes to nb/4*3 - pad bytes: write that length
     * up front (no back-patch); any other shape (\r \n, bad padding) is
     * decoded behind a reserved length as before */
    int64_t want = -1;
    if ((nb & 3) == 0) {
        const uint8_t c2 = nb ? src.raw(s0 + nb - 2) : 0, c3 = nb ? src.raw(s0 + nb - 1) : 0;
        want = (int64_t)(nb / 4 * 3) - (c3 == '=' ? (c2 == '=' ? 2 : 1) : 0);
    }
    uint64_t lp = 0;
    if (want >= 0) out.w32((uint32_t)want);
    else lp = out.alloc(4);
    SI ip = 0;
    int64_t op = 0;
    while (ip + 8 <= nb) {
        uint64_t o;
        if (!b64_8(src.get8(s0 + ip), o)) break;
        out.wle(o, 6);
        ip += 8;
        op += 6;
    }
    if (ip < nb) {
        op = b64decode_from(out, src, s0, nb, ip, op);
        if (op < 0) return false;
    }
    if (want >= 0) return op == want;
    out.put32(lp, (uint32_t)op);
    return true;
}

/* key bytes src[k0, k0+kn) == the zero-padded 8-aligned pool key at pk */
template <class S, int AS>
DGI bool key_eq(S &src, SI k0, uint32_t kn, const __attribute__((address_space(AS))) uint64_t *pk)
{
    for (uint32_t j = 0; j < kn; j += 8) {
        uint64_t a = src.get8(k0 + j);
        uint32_t rem = kn - j;
        if (rem < 8) a &= (1ull << (rem << 3)) - 1;
        if (a != pk[j >> 3]) return false;
    }
    return true;
}

/* the fast converter over one message; true = out holds the reference's
 * output, false = bail to the exact machine.
 * LEAN (the small kernel): also bail on unknown-field skips, non-string map
 * keys and default/empty writes for unset fields. Those need skip_one, a
 * second vnumber and the tb_write_empty switch; leaving them to the list
 * pass (which runs the full fast path, then the exact machine) cuts the
 * small kernel's registers and SGPR spills (C2: 93 -> 83 us/launch). */
template <bool LEAN = false, class S, class DV>
DGI bool fast_convert(const DV &D, S &src, Out &out, uint64_t flag, uint32_t root, LFFrame *fr, uint32_t fstride,
                      const FastTabs &tb)
{
    /* empty body and unquoted STRING roots are the prelude's business (convert_one) */
    if (src.n == 0 || ldrec(&D.T[root]).ttype == DG_T_STRING) return false;
    SI p = 0;
    uint32_t sp = 0;                  /* open containers */
    uint32_t ca = 0, ck = 0, cb = 0;  /* innermost: a, kind, hint/count */
    uint64_t cu = 0;                  /* innermost: reqs or size position */
    bool null_val = false;
    uint64_t unwind = 0;
    uint32_t lastf = 0;
    uint32_t td = root;
    bool vmv = false;                 /* the value is an api.js_conv field's (VM_JSCONV) */
    uint8_t c;

#define FAST_PUSH(na, nk, nu)                                             \
    do {                                                                  \
        if (sp) {                                                         \
            if (sp > FAST_LDS_DEPTH) return false;                        \
            LFFrame &f_ = fr[(sp - 1) * fstride];                         \
            f_.a = ca;                                                    \
            f_.b = ck | (cb << 2);                                        \
            f_.u = cu;                                                    \
        }                                                                 \
        sp++;                                                             \
        ca = (na);                                                        \
        ck = (nk);                                                        \
        cb = 0;                                                           \
        cu = (nu);                                                        \
    } while (0)
#define FAST_POP()                                                        \
    do {                                                                  \
        if (--sp) {                                                       \
            const LFFrame &f_ = fr[(sp - 1) * fstride];                   \
            ca = f_.a;                                                    \
            ck = f_.b & 3;                                                \
            cb = f_.b >> 2;                                               \
            cu = f_.u;                                                    \
        }                                                                 \
    } while (0)

    for (;;) {
        /* ---------------- a value of type td ---------------- */
        FP_MARK(0);
        c = src.at(p++);
        while (c <= ' ') {
            if (!isspace_(c)) return false;
            c = src.at(p++);
        }
        const dg_type t = ldrec(&D.T[td]);
        bool opened = false; /* a container was opened: look for its first key/element */
        FP_MARK(1);
        if (vmv) {
            /* j2t_field_vm VM_JSCONV (native/thrift.c:514-634): the field
             * header is already written; a quoted or bare number into an
             * int/double/string field, "" -> default or empty */
            vmv = false;
            const bool quoted = c == '"';
            bool number = true;
            if (quoted) {
                if (t.ttype == DG_T_STRING) {
                    if (!fast_string(src, p, out)) return false;
                    number = false;
                } else if (src.at(p) == '"') {
                    if constexpr (LEAN) return false; /* tb_write_default_or_empty: the list pass */
                    const dg_field f = ldrec(&D.F[lastf]);
                    if (f.dflt_len != DG_NONE) {
                        for (uint32_t j = 0; j < f.dflt_len; j++) out.w8(D.P[f.dflt_off + j]);
                    } else {
                        switch (t.ttype) { /* tb_write_empty native/thrift.c:171-203 */
                        case DG_T_BOOL:
                        case DG_T_BYTE: out.w8(0); break;
                        case DG_T_I16: out.w16(0); break;
                        case DG_T_I32: out.w32(0); break;
                        case DG_T_I64:
                        case DG_T_DOUBLE: out.w64(0); break;
                        default: return false;
                        }
                    }
                    p += 1;
                    number = false;
                }
            } else {
                if (c != '-' && (uint8_t)(c - '0') > 9) return false; /* ERR_INVAL */
                p -= 1;
            }
            if (number) {
                const SI s0 = p;
                int64_t iv;
                double dv;
                bool isint;
                if (!fast_vnumber(src, p, tb, iv, dv, isint)) return false;
                if (t.ttype == DG_T_STRING) {
                    out.w32((uint32_t)(p - s0));
                    fast_copy(src, s0, p - s0, out);
                } else if (t.ttype == DG_T_I16) { /* the reference's missing break: i16 then i8 */
                    emit_number(out, DG_T_I16, isint, iv, dv);
                    emit_number(out, DG_T_BYTE, isint, iv, dv);
                } else if (t.ttype == DG_T_BOOL || !emit_number(out, t.ttype, isint, iv, dv)) {
                    return false; /* ERR_UNSUPPORT_THRIFT_TYPE */
                }
                if (quoted) {
                    if (src.at(p) != '"') return false;
                    p += 1;
                }
            }
            goto after_value;
        }
        switch (c) {
        case '"':
            if (t.ttype != DG_T_STRING) return false;
            if ((flag & DG_F_NO_BASE64) == 0 && (t.flags & DG_TF_BINARY)) {
                if (!fast_binary(src, p, out)) return false;
                FP_MARK(2);
            } else {
                if (!fast_string(src, p, out)) return false;
                FP_MARK(3);
            }
            break;
        case '0': case '1': case '2': case '3': case '4':
        case '5': case '6': case '7': case '8': case '9': case '-': {
            p -= 1;
            int64_t iv;
            double dv;
            bool isint;
            if (!fast_vnumber(src, p, tb, iv, dv, isint)) return false;
            FP_MARK(4);
            if (!emit_number(out, t.ttype, isint, iv, dv)) return false;
            FP_MARK(5);
            break;
        }
        case 't':
            if (p + 3 > src.n || (uint32_t)src.get8(p - 1) != VS_TRUE || t.ttype != DG_T_BOOL) return false;
            p += 3;
            out.w8(1);
            break;
        case 'f':
            if (p + 4 > src.n || (uint32_t)src.get8(p) != VS_ALSE || t.ttype != DG_T_BOOL) return false;
            p += 4;
            out.w8(0);
            break;
        case 'n':
            if (p + 3 > src.n || (uint32_t)src.get8(p - 1) != VS_NULL || sp == 0) return false;
            p += 3;
            null_val = true;
            break;
        case '[': {
            if (t.ttype != DG_T_LIST && t.ttype != DG_T_SET) return false;
            out.w8(ldrec(&D.T[t.elem]).ttype);
            uint64_t bp = out.alloc(4);
            FAST_PUSH(t.elem, FK_LIST, bp);
            opened = true;
            break;
        }
        case '{':
            if (t.ttype == DG_T_STRUCT) {
                const dg_struct sd = ldrec(&D.S[t.st]);
                if (sd.req_words != 1) return false;
                if ((flag & DG_F_ENABLE_HM) && (sd.flags & DG_SF_HTTP_MAPPING)) return false; /* ERR_HM callback */
                FAST_PUSH(t.st, FK_STRUCT, D.R[sd.req_begin]);
            } else if (t.ttype == DG_T_MAP) {
                out.wle(ldrec(&D.T[t.key]).ttype | ((uint32_t)ldrec(&D.T[t.elem]).ttype << 8), 2);
                uint64_t bp = out.alloc(4);
                FAST_PUSH(t.elem, FK_MAP, bp | ((uint64_t)t.key << 32));
            } else {
                return false;
            }
            opened = true;
            break;
        default:
            return false;
        }

        after_value:
        /* ------------- after a value / an opening bracket ------------- */
        FP_MARK(6);
        bool first = opened;
        for (;;) {
            if (sp == 0) {
                out.finish();
                return out.len <= out.cap;
            }
            c = src.at(p++);
            while (c <= ' ') {
                if (!isspace_(c)) return false;
                c = src.at(p++);
            }
            if (ck == FK_LIST) {
                if (first) {
                    first = false;
                    if (c == ']') { /* size 0 already written */
                        FAST_POP();
                        continue;
                    }
                    p -= 1;
                    td = ca;
                    break;
                }
                if (null_val) null_val = false;
                else cb++;
                if (c == ',') {
                    td = ca;
                    break;
                }
                if (c != ']') return false;
                out.put32(cu, cb);
                FAST_POP();
                continue;
            }
            /* objects: struct or map */
            if (first) {
                first = false;
                if (c == '}') {
                    if (ck == FK_MAP) {
                        FAST_POP();
                        continue;
                    }
                    goto close_struct;
                }
            } else if (ck == FK_MAP) {
                if (null_val) {
                    null_val = false;
                    out.set_len(unwind);
                } else {
                    cb++;
                }
                if (c == '}') {
                    out.put32((uint32_t)cu, cb);
                    FAST_POP();
                    continue;
                }
                if (c != ',') return false;
                c = src.at(p++);
                while (c <= ' ') {
                    if (!isspace_(c)) return false;
                    c = src.at(p++);
                }
            } else {
                if (null_val) { /* native/thrift.c:1016-1032 */
                    null_val = false;
                    const dg_field f = ldrec(&D.F[lastf]);
                    const dg_struct sd = ldrec(&D.S[ca]);
                    uint64_t m = 1ull << (lastf - sd.field_begin);
                    if (f.required == DG_REQ_DEFAULT || f.required == DG_REQ_REQUIRED) cu |= m;
                    else if (f.required == DG_REQ_OPTIONAL) cu &= ~m;
                    out.set_len(unwind);
                }
                if (c == '}') goto close_struct;
                if (c != ',') return false;
                c = src.at(p++);
                while (c <= ' ') {
                    if (!isspace_(c)) return false;
                    c = src.at(p++);
                }
            }
            /* a key */
            FP_MARK(7);
            if (c != '"') return false;
            {
                SI k0 = p;
                uint32_t kn;
                int32_t fi = -1;
                dg_field f;
                /* the predicted field (the one after the previous): its plain
                 * alias followed by the closing quote IS the key advance_string
                 * would find, so one compare replaces the scan and the lookup */
                if (ck == FK_STRUCT) {
                    const dg_struct sdp = ldrec(&D.S[ca]);
                    if (cb < sdp.n_fields) {
                        f = ldrec(&D.F[sdp.field_begin + cb]);
                        kn = f.key_len;
                        if ((f.flags & (DG_FF_ALIAS_SELF | DG_FF_KEY_PLAIN)) == (DG_FF_ALIAS_SELF | DG_FF_KEY_PLAIN) &&
                            k0 + (SI)kn < src.n && key_eq(src, k0, kn, (decltype(&D.R[0]))(&D.P[f.key_off])) &&
                            src.raw(k0 + (SI)kn) == '"') {
                            fi = (int32_t)(sdp.field_begin + cb);
                            p = k0 + (SI)kn + 1;
                        }
                    }
                }
                if (fi < 0) {
                    bool esc;
                    SI e = advance_string(src, k0, esc);
                    if (e < 0 || esc) return false;
                    p = e;
                    kn = (uint32_t)(e - 1 - k0);
                }
                c = src.at(p++);
                while (c <= ' ') {
                    if (!isspace_(c)) return false;
                    c = src.at(p++);
                }
                if (c != ':') return false;
                FP_MARK(8);
                if (ck == FK_MAP) { /* j2t_map_key native/thrift.c:422-447 */
                    unwind = out.len;
                    const uint8_t kt = ldrec(&D.T[(uint32_t)(cu >> 32)]).ttype;
                    if (kt == DG_T_STRING) {
                        out.w32(kn);
                        fast_copy(src, k0, kn, out);
                    } else {
                        if constexpr (LEAN) return false;
                        S ks = src.sub(k0, kn);
                        SI q = 0;
                        int64_t iv;
                        double dv;
                        bool isint;
                        if (!fast_vnumber(ks, q, tb, iv, dv, isint)) return false;
                        if (!emit_number(out, kt, isint, iv, dv)) return false;
                    }
                    td = ca;
                    break;
                }
                /* struct field: predicted, then hashed (j2t_key native/thrift.c:668-763) */
                const dg_struct sd = ldrec(&D.S[ca]);
                if (fi < 0 && cb < sd.n_fields) {
                    f = ldrec(&D.F[sd.field_begin + cb]);
                    if ((f.flags & DG_FF_ALIAS_SELF) && f.key_len == kn &&
                        key_eq(src, k0, kn, (decltype(&D.R[0]))(&D.P[f.key_off])))
                        fi = (int32_t)(sd.field_begin + cb);
                }
                if (fi < 0) {
                    uint32_t h = DG_NAME_HASH_SEED;
                    for (uint32_t j = 0; j < kn; j += 8) { /* a word per 8 key bytes (16 readable bytes past the end) */
                        const uint64_t w = src.get8(k0 + (SI)j);
                        const uint32_t r = kn - j < 8 ? kn - j : 8u;
#pragma unroll
                        for (uint32_t b = 0; b < 8; b++)
                            if (b < r) h = DG_NAME_HASH_STEP(h, (uint8_t)(w >> (8 * b)));
                    }
                    for (uint32_t s = h & sd.name_mask;; s = (s + 1) & sd.name_mask) {
                        const dg_name nm = ldrec(&D.N[sd.name_begin + s]);
                        if (nm.field == DG_NONE) break;
                        if (nm.hash == h && nm.key_len == kn &&
                            key_eq(src, k0, kn, (decltype(&D.R[0]))(&D.P[nm.key_off]))) {
                            fi = (int32_t)nm.field;
                            break;
                        }
                    }
                    if (fi >= 0) f = ldrec(&D.F[fi]);
                }
                if (fi < 0 || ((f.flags & DG_FF_REQUEST_BASE) && (flag & DG_F_NO_WRITE_BASE))) {
                    if (fi < 0 && (flag & DG_F_ALLOW_UNKNOWN) == 0) return false;
                    /* skip the value (skip_one native/scanning.c:1134-1631) */
                    c = src.at(p++);
                    while (c <= ' ') {
                        if (!isspace_(c)) return false;
                        c = src.at(p++);
                    }
                    p -= 1;
                    if constexpr (LEAN) return false; /* the list pass skips it */
                    SkipRes sr = skip_one(src, p, nullptr, 64);
                    if (sr.r < 0) return false;
                    p = sr.p;
                    continue; /* back to "after a value" */
                }
                uint32_t k = (uint32_t)fi - sd.field_begin;
                const dg_type ft = ldrec(&D.T[f.type]);
                if ((flag & DG_F_ENABLE_VM) && f.vm != DG_VM_NONE) {
                    /* value mapping (native/thrift.c:739-757): the header is
                     * written here by j2t_field_vm's tb_write_field_begin, and
                     * unwindPos/lastField are NOT updated (a null value is an
                     * error there anyway); only inline js_conv is handled */
                    if (f.vm != DG_VM_JSCONV) return false; /* ERR_VM_END / ERR_UNSUPPORT_VM_TYPE */
                    vmv = true;
                    lastf = (uint32_t)fi; /* read back only for the "" default (same field) */
                } else {
                    unwind = out.len;
                    lastf = (uint32_t)fi;
                }
                out.wle((uint32_t)ft.ttype | ((uint32_t)__builtin_bswap16(f.id) << 8), 3);
                cu &= ~(1ull << k);
                cb = k + 1;
                td = f.type;
                FP_MARK(9);
                break;
            }
        close_struct: { /* j2t_write_unset_fields native/thrift.c:258-310, then STOP */
            FP_MARK(10);
            const dg_struct sd = ldrec(&D.S[ca]);
            uint64_t bits = cu;
            bool wr = flag & DG_F_WRITE_REQUIRE, wd = flag & DG_F_WRITE_DEFAULT, wo = flag & DG_F_WRITE_OPTIONAL;
            while (bits) {
                uint32_t k = __builtin_ctzll(bits);
                bits &= bits - 1;
                const dg_field f = ldrec(&D.F[sd.field_begin + k]);
                if (f.flags & DG_FF_REQUEST_BASE) continue;
                if (!wr && f.required == DG_REQ_REQUIRED) return false; /* ERR_NULL_REQUIRED */
                if ((wr && f.required == DG_REQ_REQUIRED) || (wd && f.required == DG_REQ_DEFAULT) ||
                    (wo && f.required == DG_REQ_OPTIONAL)) {
                    if constexpr (LEAN) return false;
                    const dg_type ft = ldrec(&D.T[f.type]);
                    out.wle((uint32_t)ft.ttype | ((uint32_t)__builtin_bswap16(f.id) << 8), 3);
                    if (f.dflt_len != DG_NONE) {
                        for (uint32_t j = 0; j < f.dflt_len; j++) out.w8(D.P[f.dflt_off + j]);
                        continue;
                    }
                    switch (ft.ttype) { /* tb_write_empty native/thrift.c:171-203 */
                    case DG_T_BOOL:
                    case DG_T_BYTE: out.w8(0); break;
                    case DG_T_I16: out.w16(0); break;
                    case DG_T_I32:
                    case DG_T_STRING: out.w32(0); break;
                    case DG_T_I64:
                    case DG_T_DOUBLE: out.w64(0); break;
                    case DG_T_LIST:
                    case DG_T_SET:
                        out.w8(ldrec(&D.T[ft.elem]).ttype);
                        out.w32(0);
                        break;
                    case DG_T_MAP:
                        out.w8(ldrec(&D.T[ft.key]).ttype);
                        out.w8(ldrec(&D.T[ft.elem]).ttype);
                        out.w32(0);
                        break;
                    case DG_T_STRUCT: out.w8(0); break;
                    default: return false;
                    }
                }
            }
            out.w8(0);
            FAST_POP();
            FP_MARK(11);
            continue;
        }
        }
    }
#undef FAST_PUSH
#undef FAST_POP
}
#undef SI

}  // namespace dg
