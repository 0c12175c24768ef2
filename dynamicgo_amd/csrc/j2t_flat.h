/*
 * j2t_flat.h — the flat-struct kernel: one GROUP of FL_G lanes per message,
 * one lane per FIELD.
 *
 * For a root struct whose fields are all scalars or strings (C2's
 * baseline.Simple, conv/j2t/conv_test.go's Simple), a message is
 *     ws '{' ws "key" ws ':' ws value ws (',' ...)* '}' ws
 * and every field can be converted on its own once its span is known. The
 * lane-per-message kernel (j2t_small.h) walks the message byte-serially in
 * one lane; here the group first finds the top-level commas in parallel
 * (each lane classifies 64 bytes: quote parity with a prefix XOR carried
 * across the group, commas and brackets outside strings), then lane k
 * converts field k -- key lookup, value parse, Thrift size -- the group
 * prefix-sums the sizes, and every lane writes its field at its offset.
 * JSON fields are written in input order, exactly as j2t_fsm_exec writes them
 * (native/thrift.c:765-1187, one tb_write_field_begin + value per key).
 *
 * Anything outside that shape -- nesting, null values, escaped keys, a
 * backslash before '"' or '\\', unset fields that need writing, errors --
 * is declined to the bail list, whose list pass (lane kernel fast path, then
 * the exact machine) produces the reference's bytes or error. Messages
 * longer than big_max go to the wave kernel's list as in the small kernel.
 */
#pragma once
#include "j2t_small.h"

namespace dg {

constexpr uint32_t FL_G = 8;                      /* lanes per message */
#ifndef DG_FL_WAVES
#define DG_FL_WAVES 4
#endif
#ifndef DG_FL_WPE
#define DG_FL_WPE 4 /* waves per SIMD the register budget is cut for (LDS allows 4) */
#endif
constexpr uint32_t FL_WAVES = DG_FL_WAVES;        /* waves per block */
constexpr uint32_t FL_MPW = 64 / FL_G;            /* messages per wave */
constexpr uint32_t FL_MPB = FL_WAVES * FL_MPW;    /* messages per block */
constexpr uint32_t FL_MAXLEN = 64 * FL_G;         /* bytes a group classifies (64 per lane) */
constexpr uint32_t FL_IN_WORDS = FL_MAXLEN / 8 + 3;
constexpr uint32_t FL_MAXSEP = 48;                /* top-level commas per message */
constexpr uint32_t FL_OUTW = 64;                  /* output stage per message (words): 512 B */
constexpr uint32_t FL_DESC = 16 * 1024;           /* descriptor bytes in LDS (dynamic) */
constexpr uint32_t FL_FPR = 64 * FL_WAVES / FL_MPB; /* fields per message per round (phase 2) */

/* group (FL_G lanes) collectives on 32-bit values */
DGI uint32_t grp_incl_sum(uint32_t v, uint32_t g)
{
#pragma unroll
    for (uint32_t d = 1; d < FL_G; d <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, d, FL_G);
        if (g >= d) v += u;
    }
    return v;
}
DGI uint32_t grp_sum(uint32_t v)
{
#pragma unroll
    for (uint32_t d = 1; d < FL_G; d <<= 1) v += (uint32_t)__shfl_xor((int)v, d, FL_G);
    return v;
}
DGI uint32_t grp_or(uint32_t v)
{
#pragma unroll
    for (uint32_t d = 1; d < FL_G; d <<= 1) v |= (uint32_t)__shfl_xor((int)v, d, FL_G);
    return v;
}

/* 0x80 in each byte of w (32-bit half) equal to c */
DGI uint32_t eq32(uint32_t w, uint32_t cc) { return zb32(w ^ cc); }

/* A byte writer into an 8-aligned buffer (global: the output slot; LDS: a
 * message's output stage) starting at an arbitrary byte offset; several
 * lanes write disjoint ranges of the same buffer. Whole words inside the
 * range are stored as words, the partial words at its two ends byte by byte
 * (those bytes' neighbours belong to other lanes). */
template <int AS>
struct BOut {
    typedef __attribute__((address_space(AS))) uint8_t B8;
    typedef __attribute__((address_space(AS))) uint64_t B64;
    B8 *b;       /* buffer base (8-aligned) */
    uint64_t len;/* absolute position in the buffer */
    uint64_t wbuf;
    uint32_t lo; /* first byte of the current word that is ours */
    DGI void init(B8 *base, uint64_t start)
    {
        b = base;
        len = start;
        wbuf = 0;
        lo = (uint32_t)(start & 7);
    }
    DGI void put_word(uint64_t wi, uint64_t v)
    {
        if (lo == 0) {
            *(B64 *)(b + (wi << 3)) = v;
        } else {
            for (uint32_t k = lo; k < 8; k++) b[(wi << 3) + k] = (uint8_t)(v >> (8 * k));
            lo = 0;
        }
    }
    DGI void wle(uint64_t v, uint32_t n)
    {
        const uint32_t used = (uint32_t)(len & 7), sh = used << 3;
        if (n < 8) v &= (1ull << (n << 3)) - 1;
        const uint64_t low = (wbuf & ((1ull << sh) - 1)) | (v << sh);
        const uint64_t high = used ? (v >> (64 - sh)) : 0;
        const uint64_t wi = len >> 3;
        len += n;
        if (used + n >= 8) {
            put_word(wi, low);
            wbuf = high;
        } else {
            wbuf = low;
        }
    }
    DGI void w8(uint8_t v) { wle(v, 1); }
    DGI void w16(uint16_t v) { wle(__builtin_bswap16(v), 2); }
    DGI void w32(uint32_t v) { wle(__builtin_bswap32(v), 4); }
    DGI void w64(uint64_t v) { wle(__builtin_bswap64(v), 8); }
    DGI void finish()
    {
        const uint32_t e = (uint32_t)(len & 7);
        const uint64_t wi = len >> 3;
        for (uint32_t k = lo; k < e; k++) b[(wi << 3) + k] = (uint8_t)(wbuf >> (8 * k));
    }
};
typedef BOut<1> GOut;
typedef BOut<3> LOut;

/* counts bytes only (string sizes with escapes) */
struct CountW {
    uint64_t len = 0;
    DGI void wle(uint64_t, uint32_t n) { len += n; }
    DGI void w8(uint8_t) { len += 1; }
};

/* one parsed field */
enum : uint32_t { FV_NONE = 0, FV_NUM, FV_STR, FV_BIN, FV_BOOL, FV_NUMSTR };
struct FField {
    int32_t fi;       /* global field index, -1 = unknown key (skipped) */
    uint32_t kind;    /* FV_* */
    uint32_t s0, nb;  /* string / binary / number-text span */
    bool esc;         /* string has escapes */
    bool isint;
    int64_t iv;
    double dv;
    uint32_t size;    /* Thrift bytes of this field */
    uint8_t tt;       /* field type */
    uint16_t id;
    bool i16q;        /* js_conv i16 quirk: i16 then i8 */
};

template <class S>
DGI uint32_t skip_ws(S &s, uint32_t p)
{
    while (p < (uint32_t)s.n && isspace_(s.raw((int32_t)p))) p++;
    return p;
}

/* field k's span [sk, ek): parse and size it; false = decline the message */
template <class S, class DV>
DGI bool flat_parse(const DV &D, const dg_struct &sd, S &src, uint32_t sk, uint32_t ek, uint32_t k, uint64_t flag,
                    const FastTabs &tb, FField &F)
{
    typedef typename S::idx SI;
    uint32_t p = skip_ws(src, sk);
    if (p >= ek || src.raw((SI)p) != '"') return false;
    const uint32_t k0 = p + 1;
    bool esc;
    int64_t e = advance_string(src, k0, esc);
    if (e < 0 || esc || (uint64_t)e > ek) return false;
    const uint32_t kn = (uint32_t)e - 1 - k0;
    p = skip_ws(src, (uint32_t)e);
    if (p >= ek || src.raw((SI)p) != ':') return false;
    p = skip_ws(src, p + 1);
    if (p >= ek) return false;
    /* the key: predicted (field k in IDL order), else the name table */
    int32_t fi = -1;
    dg_field f;
    if (k < sd.n_fields) {
        f = ldrec(&D.F[sd.field_begin + k]);
        if ((f.flags & DG_FF_ALIAS_SELF) && f.key_len == kn && key_eq(src, (SI)k0, kn, (decltype(&D.R[0]))(&D.P[f.key_off])))
            fi = (int32_t)(sd.field_begin + k);
    }
    if (fi < 0) {
        uint32_t h = DG_NAME_HASH_SEED;
        for (uint32_t j = 0; j < kn; j += 8) {
            const uint64_t w = src.get8((SI)(k0 + j));
            const uint32_t r = kn - j < 8 ? kn - j : 8u;
#pragma unroll
            for (uint32_t bb = 0; bb < 8; bb++)
                if (bb < r) h = DG_NAME_HASH_STEP(h, (uint8_t)(w >> (8 * bb)));
        }
        for (uint32_t s = h & sd.name_mask;; s = (s + 1) & sd.name_mask) {
            const dg_name nm = ldrec(&D.N[sd.name_begin + s]);
            if (nm.field == DG_NONE) break;
            if (nm.hash == h && nm.key_len == kn && key_eq(src, (SI)k0, kn, (decltype(&D.R[0]))(&D.P[nm.key_off]))) {
                fi = (int32_t)nm.field;
                break;
            }
        }
        if (fi >= 0) f = ldrec(&D.F[fi]);
    }
    /* the value */
    const uint8_t c = src.raw((SI)p);
    uint32_t vk;
    uint32_t vs0 = 0, vnb = 0;
    bool vesc = false, isint = false, bv = false;
    int64_t iv = 0;
    double dv = 0.0;
    if (c == '"') {
        vs0 = p + 1;
        e = advance_string(src, vs0, vesc);
        if (e < 0 || (uint64_t)e > ek) return false;
        vnb = (uint32_t)e - 1 - vs0;
        p = (uint32_t)e;
        vk = FV_STR;
    } else if (c == '-' || (uint8_t)(c - '0') <= 9) {
        SI q = (SI)p;
        vs0 = p;
        if (!fast_vnumber(src, q, tb, iv, dv, isint)) return false;
        p = (uint32_t)q;
        vnb = p - vs0;
        vk = FV_NUM;
    } else if (c == 't') {
        if (p + 4 > ek || (uint32_t)src.get8((SI)p) != VS_TRUE) return false;
        p += 4;
        bv = true;
        vk = FV_BOOL;
    } else if (c == 'f') {
        if (p + 5 > ek || (uint32_t)src.get8((SI)(p + 1)) != VS_ALSE) return false;
        p += 5;
        vk = FV_BOOL;
    } else {
        return false; /* null, containers, garbage: the list pass */
    }
    if (skip_ws(src, p) != ek) return false;
    F.fi = fi;
    if (fi < 0 || ((f.flags & DG_FF_REQUEST_BASE) && (flag & DG_F_NO_WRITE_BASE))) {
        if (fi < 0 && !(flag & DG_F_ALLOW_UNKNOWN)) return false; /* ERR_UNKNOWN_FIELD */
        if (fi >= 0) return false;
        F.kind = FV_NONE; /* an unknown key with a scalar value: skipped */
        F.size = 0;
        return true;
    }
    const uint8_t tt = ldrec(&D.T[f.type]).ttype;
    const bool bin = (ldrec(&D.T[f.type]).flags & DG_TF_BINARY) && !(flag & DG_F_NO_BASE64);
    F.tt = tt;
    F.id = f.id;
    F.i16q = false;
    uint32_t vsize;
    if ((flag & DG_F_ENABLE_VM) && f.vm != DG_VM_NONE) {
        /* j2t_field_vm VM_JSCONV (native/thrift.c:514-634) */
        if (f.vm != DG_VM_JSCONV) return false;
        if (vk == FV_STR && tt != DG_T_STRING) {
            if (vnb == 0 || vesc) return false; /* "" -> default write: the list pass */
            S sub = src.sub((SI)vs0, (SI)vnb);
            SI q = 0;
            if (!fast_vnumber(sub, q, tb, iv, dv, isint) || (uint32_t)q != vnb) return false;
            vk = FV_NUM;
        } else if (vk == FV_NUM && tt == DG_T_STRING) {
            vk = FV_NUMSTR; /* the number's text as the string */
        } else if (vk == FV_BOOL) {
            return false;
        }
        if (vk == FV_NUM && tt == DG_T_I16) F.i16q = true;
    }
    switch (vk) {
    case FV_STR:
        if (tt != DG_T_STRING) return false;
        if (bin) {
            if (vesc || (vnb & 3)) return false; /* non-canonical base64: the list pass */
            const uint8_t c2 = vnb ? src.raw((SI)(vs0 + vnb - 2)) : 0, c3 = vnb ? src.raw((SI)(vs0 + vnb - 1)) : 0;
            vsize = 4 + vnb / 4 * 3 - (c3 == '=' ? (c2 == '=' ? 2 : 1) : 0);
            vk = FV_BIN;
        } else if (vesc) {
            CountW cw;
            if (!fast_unquote(src, (SI)vs0, (SI)vnb, cw)) return false;
            vsize = 4 + (uint32_t)cw.len;
        } else {
            vsize = 4 + vnb;
        }
        break;
    case FV_NUMSTR:
        vsize = 4 + vnb;
        break;
    case FV_NUM:
        switch (tt) {
        case DG_T_BYTE: vsize = 1; break;
        case DG_T_I16: vsize = F.i16q ? 3 : 2; break;
        case DG_T_I32: vsize = 4; break;
        case DG_T_I64: case DG_T_DOUBLE: vsize = 8; break;
        default: return false; /* ERR_DISMATCH_TYPE etc.: the list pass */
        }
        break;
    default: /* FV_BOOL */
        if (tt != DG_T_BOOL) return false;
        vsize = 1;
        break;
    }
    F.kind = vk;
    F.s0 = vs0;
    F.nb = vnb;
    F.esc = vesc;
    F.isint = isint;
    F.iv = vk == FV_BOOL ? (int64_t)bv : iv;
    F.dv = dv;
    F.size = 3 + vsize;
    return true;
}

/* write a parsed field (header + value) */
template <class S, class O>
DGI bool flat_write(S &src, const FField &F, O &o)
{
    typedef typename S::idx SI;
    if (F.kind == FV_NONE) return true;
    o.wle((uint32_t)F.tt | ((uint32_t)__builtin_bswap16(F.id) << 8), 3);
    switch (F.kind) {
    case FV_BOOL: o.w8((uint8_t)F.iv); return true;
    case FV_NUM:
        if (F.i16q) {
            emit_number(o, DG_T_I16, F.isint, F.iv, F.dv);
            emit_number(o, DG_T_BYTE, F.isint, F.iv, F.dv);
            return true;
        }
        return emit_number(o, F.tt, F.isint, F.iv, F.dv);
    case FV_NUMSTR:
        o.w32(F.nb);
        fast_copy(src, (SI)F.s0, (SI)F.nb, o);
        return true;
    case FV_STR:
        o.w32(F.size - 7);
        if (F.esc) return fast_unquote(src, (SI)F.s0, (SI)F.nb, o);
        fast_copy(src, (SI)F.s0, (SI)F.nb, o);
        return true;
    default: { /* FV_BIN: canonical padded base64 */
        o.w32(F.size - 7);
        uint32_t ip = 0;
        const uint32_t full = F.nb >= 4 ? F.nb - 4 : 0; /* the last quantum may hold '=' */
        for (; ip + 8 <= full; ip += 8) {
            uint64_t v;
            if (!b64_8(src.get8((SI)(F.s0 + ip)), v)) return false;
            o.wle(v, 6);
        }
        for (; ip < full; ip += 4) {
            uint32_t v;
            if (!b64_4((uint32_t)src.get8((SI)(F.s0 + ip)), v)) return false;
            o.wle(v, 3);
        }
        if (F.nb >= 4) {
            uint32_t w = (uint32_t)src.get8((SI)(F.s0 + ip));
            const uint32_t c2 = (w >> 16) & 0xFF, c3 = w >> 24;
            const uint32_t keep = c3 == '=' ? (c2 == '=' ? 1u : 2u) : 3u;
            if (c3 == '=') w = (w & 0x00FFFFFFu) | ((uint32_t)'A' << 24);
            if (c2 == '=') w = (w & 0xFF00FFFFu) | ((uint32_t)'A' << 16);
            uint32_t v;
            if (!b64_4(w, v)) return false;
            o.wle(v, keep); /* decode_block keeps nb-1 bytes; the padding bits are not checked */
        }
        return true;
    }
    }
}

struct FlatParams {
    const uint8_t *blob;
    dg_desc_hdr hdr;
    uint32_t *bail_count;
    uint32_t *bail_list;
};

/* -DDG_FLPROF: cycles per wave by phase (s_memtime at the marks, summed
 * into P.stats[2..] by each wave's first lane) */
#ifdef DG_FLPROF
#define FLP_DECL uint64_t flp_t = __builtin_amdgcn_s_memtime(); uint64_t flp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define FLP(k)                                              \
    do {                                                    \
        const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
        flp[k] += now_ - flp_t;                             \
        flp_t = now_;                                       \
    } while (0)
#define FLP_END()                                                                        \
    do {                                                                                 \
        if ((threadIdx.x & 63) == 0 && (blockIdx.x & 31) == 0) /* sampled: 1 block in 32 */ \
            for (int k_ = 0; k_ < 8; k_++) atomicAdd(&P.stats[2 + k_], (unsigned long long)flp[k_]); \
    } while (0)
#else
#define FLP_DECL
#define FLP(k)
#define FLP_END()
#endif

/* per message of the block, between the phases */
struct FlatMsg {
    uint32_t ok;      /* still on the flat path */
    uint32_t open, close, nf;
    uint32_t base;    /* output bytes written by the previous rounds */
    uint32_t plo, phi;/* present fields (struct field-index bits) */
    uint32_t a7n;     /* message start & 7 | length << 3 (0 when not staged) */
    uint64_t oa, cap; /* output slot */
};

template <int V>
__global__ __launch_bounds__(64 * FL_WAVES) __attribute__((amdgpu_waves_per_eu(DG_FL_WPE))) void j2t_flat_kernel(
    Params P, FlatParams S)
{
    __shared__ __attribute__((aligned(16))) uint64_t s_in[FL_MPB * FL_IN_WORDS];
    __shared__ uint16_t s_sep[FL_MPB * FL_MAXSEP];
    __shared__ FlatMsg s_msg[FL_MPB];
    __shared__ uint32_t s_size[FL_FPR * FL_MPB];
    __shared__ __attribute__((aligned(16))) uint64_t s_out[FL_MPB * FL_OUTW];
    __shared__ uint32_t s_rounds;
    __shared__ uint64_t s_p10u[20];
    __shared__ double s_p10d[23];
    extern __shared__ __attribute__((aligned(16))) uint64_t s_fdesc[];
    FLP_DECL
    const uint32_t tid = threadIdx.x, lane = tid & 63, g = lane & (FL_G - 1);
    const uint32_t m = tid / FL_G; /* phase 1: the message of this lane's group */
    {
        const uint4 *gd = (const uint4 *)S.blob;
        uint4 *ld = (uint4 *)s_fdesc;
        for (uint32_t k = tid; k < (S.hdr.total_len + 15) / 16; k += 64 * FL_WAVES) ld[k] = gd[k];
    }
    if (tid < 20) {
        uint64_t v = 1;
        for (uint32_t k = 0; k < tid; k++) v *= 10;
        s_p10u[tid] = v;
    }
    if (tid < 23) s_p10d[tid] = P10[tid];
    if (tid == 0) s_rounds = 0;
    const uint64_t b0 = (uint64_t)blockIdx.x * FL_MPB;
    const uint64_t i = b0 + m;
    const bool have = i < P.n;
    uint64_t a = 0, b = 0;
    if (have) {
        a = P.in_off[i];
        b = P.in_off[i + 1];
    }
    const uint64_t n64 = b - a;
    const bool big = have && P.big_list && n64 > P.big_max;
    bool ok = have && !big && n64 > 0 && n64 <= FL_MAXLEN;
    /* stage the message's aligned words (a slack word past the end) */
    if (ok) {
        const uint32_t nw = (uint32_t)(((b + 7) >> 3) - (a >> 3)) + 1;
        const glb_u64 *gsrc = (const glb_u64 *)(const void *)P.json + (a >> 3); /* arena: 16 readable bytes past the end */
        for (uint32_t w = g; w < nw; w += FL_G) s_in[m * FL_IN_WORDS + w] = gsrc[w];
    }
    if (big && g == 0) {
        const uint32_t q = __hip_atomic_fetch_add(P.big_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        P.big_list[q] = (uint32_t)i;
    }
    __syncthreads();
    FLP(0);
    const auto D = desc_view<3>((const __attribute__((address_space(3))) uint8_t *)(void *)s_fdesc, S.hdr);
    const FastTabs tb{(const __attribute__((address_space(3))) uint64_t *)(void *)s_p10u, (lds_f64 *)(void *)s_p10d};
    const dg_type rt = ldrec(&D.T[P.root]);
    const dg_struct sd = ldrec(&D.S[rt.st]);

    /* ---- 1. structure (a group of FL_G lanes per message): this lane's 64
     *      bytes [64g, 64g+64) -> the top-level commas ---- */
    {
        const uint32_t n = ok ? (uint32_t)n64 : 0;
        SrcT<lds_u64, int32_t> src;
        src.init((lds_u64 *)(void *)&s_in[m * FL_IN_WORDS], (int32_t)(a & 7), (int32_t)n);
        uint32_t nsep = 0, nbrk = 0, bad = 0;
        uint64_t cm[8]; /* commas outside strings (0x80 per byte), per word */
        uint32_t lane_q = 0;
        {
            uint64_t qm[8], sm[8], bm[8];
            const uint32_t base = 64 * g;
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) {
                const uint32_t at = base + 8 * j;
                uint64_t w = at < n ? src.get8((int32_t)at) : 0;
                if (at < n && at + 8 > n) w &= (1ull << ((n - at) << 3)) - 1; /* bytes past the end: 0 */
                const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
                const uint32_t l20 = lo | 0x20202020u, h20 = hi | 0x20202020u;
                qm[j] = (uint64_t)eq32(lo, 0x22222222u) | ((uint64_t)eq32(hi, 0x22222222u) << 32);
                bm[j] = (uint64_t)eq32(lo, 0x5C5C5C5Cu) | ((uint64_t)eq32(hi, 0x5C5C5C5Cu) << 32);
                cm[j] = (uint64_t)eq32(lo, 0x2C2C2C2Cu) | ((uint64_t)eq32(hi, 0x2C2C2C2Cu) << 32);
                sm[j] = (uint64_t)(eq32(l20, 0x7B7B7B7Bu) | eq32(l20, 0x7D7D7D7Du)) |
                        ((uint64_t)(eq32(h20, 0x7B7B7B7Bu) | eq32(h20, 0x7D7D7D7Du)) << 32); /* { } [ ] */
                lane_q += (uint32_t)__builtin_popcountll(qm[j]);
            }
            /* a backslash before '"' or '\\' (escaped quote or backslash) -> decline */
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) {
                const uint64_t nxt = ((qm[j] | bm[j]) >> 8) | (j < 7 ? (qm[j + 1] | bm[j + 1]) << 56 : 0);
                if (bm[j] & nxt) bad = 1;
            }
            const uint32_t next_first = (uint32_t)__shfl_down((int)(uint32_t)((qm[0] | bm[0]) & 0x80), 1, FL_G);
            if (g + 1 < FL_G && (bm[7] >> 63) && next_first) bad = 1;
            /* quote parity: prefix XOR over the bytes, carried across words and lanes */
            const uint32_t incl = grp_incl_sum(lane_q, g);
            uint32_t inside = (incl - lane_q) & 1;
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) {
                uint64_t x = qm[j] >> 7; /* 1 per quote byte */
                x ^= x << 8;
                x ^= x << 16;
                x ^= x << 32;
                x = (x << 8) - x; /* 0xFF in each byte where the parity is odd */
                const uint64_t ins = x ^ (inside ? ~0ull : 0ull); /* inside a string, opening quote included */
                inside ^= (uint32_t)(__builtin_popcountll(qm[j]) & 1);
                cm[j] &= ~ins;
                nsep += (uint32_t)__builtin_popcountll(cm[j]);
                nbrk += (uint32_t)__builtin_popcountll(sm[j] & ~ins);
            }
            bad |= (uint32_t)__shfl(incl, FL_G - 1, FL_G) & 1; /* an unterminated string */
        }
        const uint32_t sep_incl = grp_incl_sum(nsep, g);
        const uint32_t sep_tot = (uint32_t)__shfl(sep_incl, FL_G - 1, FL_G);
        const uint32_t brk_tot = grp_sum(nbrk);
        bad = grp_or(bad);
        ok = ok && !bad && brk_tot == 2 && sep_tot < FL_MAXSEP;
        if (ok) {
            __attribute__((address_space(3))) uint16_t *sep =
                (__attribute__((address_space(3))) uint16_t *)(void *)&s_sep[m * FL_MAXSEP];
            uint32_t idx = sep_incl - nsep;
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) {
                uint64_t c = cm[j];
                while (c) {
                    const uint32_t bit = (uint32_t)__builtin_ctzll(c);
                    c &= c - 1;
                    sep[idx++] = (uint16_t)(64 * g + 8 * j + (bit >> 3));
                }
            }
        }
        if (g == 0) {
            /* the braces: the first and last non-space bytes */
            uint32_t open = 0, close = 0, nf = 0;
            if (ok) {
                open = skip_ws(src, 0);
                close = n - 1;
                while (close > open && isspace_(src.raw((int32_t)close))) close--;
                ok = open < close && src.raw((int32_t)open) == '{' && src.raw((int32_t)close) == '}';
                nf = sep_tot + 1;
                if (ok && sep_tot == 0 && skip_ws(src, open + 1) == close) nf = 0; /* {} */
            }
            FlatMsg fm;
            fm.ok = ok ? 1u : 0u;
            fm.open = open;
            fm.close = close;
            fm.nf = nf;
            fm.base = 0;
            fm.plo = fm.phi = 0;
            fm.a7n = (uint32_t)(a & 7) | (n << 3);
            fm.oa = have ? P.out_off[i] : 0;
            fm.cap = have ? P.out_off[i + 1] - fm.oa : 0;
            s_msg[m] = fm;
            if (ok) atomicMax(&s_rounds, (nf + FL_FPR - 1) / FL_FPR);
        }
    }
    FLP(1);
    __syncthreads();
    FLP(2);

    /* ---- 2. fields, field-major: lane (fs, mm) converts field r*FL_FPR + fs
     *      of message mm, so a wave's lanes hold the same field of many
     *      messages (same type, same path) ---- */
    const uint32_t mm = tid % FL_MPB, fs = tid / FL_MPB;
    const uint32_t a7n = s_msg[mm].a7n;
    const uint64_t oa = s_msg[mm].oa;
    SrcT<lds_u64, int32_t> src;
    src.init((lds_u64 *)(void *)&s_in[mm * FL_IN_WORDS], (int32_t)(a7n & 7), (int32_t)(a7n >> 3));
    const uint32_t rounds = s_rounds;
    for (uint32_t r = 0; r < rounds; r++) {
        const FlatMsg fm = s_msg[mm];
        const uint32_t k = r * FL_FPR + fs;
        FField F;
        F.size = 0;
        F.kind = FV_NONE;
        const bool mine = fm.ok && k < fm.nf;
        if (mine) {
            const __attribute__((address_space(3))) uint16_t *sep =
                (const __attribute__((address_space(3))) uint16_t *)(void *)&s_sep[mm * FL_MAXSEP];
            const uint32_t sk = k == 0 ? fm.open + 1 : (uint32_t)sep[k - 1] + 1;
            const uint32_t ek = k == fm.nf - 1 ? fm.close : (uint32_t)sep[k];
            if (!flat_parse(D, sd, src, sk, ek, k, P.flag, tb, F)) {
                s_msg[mm].ok = 0; /* any lane may clear it */
                F.size = 0;
            } else if (F.fi >= 0) {
                const uint32_t bit = (uint32_t)F.fi - sd.field_begin;
                if (bit < 32) atomicOr(&s_msg[mm].plo, 1u << bit);
                else atomicOr(&s_msg[mm].phi, 1u << (bit - 32));
            }
        }
        s_size[fs * FL_MPB + mm] = F.size;
        FLP(3);
        __syncthreads();
        FLP(4);
        /* offsets: one lane per message adds up the round's sizes in field order */
        if (tid < FL_MPB) {
            FlatMsg &q = s_msg[tid];
            uint32_t off = q.base;
#pragma unroll
            for (uint32_t f = 0; f < FL_FPR; f++) {
                const uint32_t sz = s_size[f * FL_MPB + tid];
                s_size[f * FL_MPB + tid] = off;
                off += sz;
            }
            /* room for STOP in the stage and (word-rounded) in the slot; else the list pass */
            if (off + 1 > FL_OUTW * 8 || (((uint64_t)off + 8) & ~7ull) > q.cap) q.ok = 0;
            q.base = off;
        }
        __syncthreads();
        FLP(5);
        if (mine && s_msg[mm].ok && F.size) {
            LOut o;
            o.init((LOut::B8 *)(void *)&s_out[mm * FL_OUTW], s_size[fs * FL_MPB + mm]);
            const bool wok = flat_write(src, F, o);
            o.finish();
            if (!wok) s_msg[mm].ok = 0;
        }
        FLP(6);
        __syncthreads();
        FLP(7);
    }
    /* ---- 3. per message: requires and STOP (one lane per message), then the
     *      staged output to the slot (a group per message, word stores) ---- */
    if (tid < FL_MPB && b0 + tid < P.n) {
        const uint64_t ii = b0 + tid;
        FlatMsg &q = s_msg[tid];
        bool good = q.ok != 0;
        if (good) {
            const uint64_t present = (uint64_t)q.plo | ((uint64_t)q.phi << 32);
            uint64_t bits = D.R[sd.req_begin] & ~present;
            const uint64_t flag = P.flag;
            while (bits) { /* unset fields that error or need a default write -> the list pass */
                const uint32_t kk = (uint32_t)__builtin_ctzll(bits);
                bits &= bits - 1;
                const dg_field f = ldrec(&D.F[sd.field_begin + kk]);
                if (f.flags & DG_FF_REQUEST_BASE) continue;
                if (f.required == DG_REQ_REQUIRED || ((flag & DG_F_WRITE_DEFAULT) && f.required == DG_REQ_DEFAULT) ||
                    ((flag & DG_F_WRITE_OPTIONAL) && f.required == DG_REQ_OPTIONAL)) {
                    good = false;
                    break;
                }
            }
        }
        if (good) {
            ((__attribute__((address_space(3))) uint8_t *)(void *)&s_out[tid * FL_OUTW])[q.base] = 0; /* STOP */
        } else {
            q.ok = 0;
            const uint64_t lo8 = P.in_off[ii], hi8 = P.in_off[ii + 1];
            if (!(P.big_list && hi8 - lo8 > P.big_max)) { /* not the wave kernel's */
                const uint32_t qq = atomicAdd(S.bail_count, 1u);
                S.bail_list[qq] = (uint32_t)ii;
            }
        }
    }
    __syncthreads();
    if (!have || !s_msg[m].ok) return;
    {
        const uint32_t len = s_msg[m].base + 1;
        const uint64_t oa1 = s_msg[m].oa;
        gu64 *dst = (gu64 *)(void *)(P.out + oa1);
        const __attribute__((address_space(3))) uint64_t *st = (const __attribute__((address_space(3))) uint64_t *)(void *)&s_out[m * FL_OUTW];
        for (uint32_t w = g; w < (len + 7) / 8; w += FL_G) dst[w] = st[w];
        if (g == 0) {
            P.ret[i] = 0;
            P.out_len[i] = len;
        }
    }
    FLP_END();
}

void launch_flat_kernel(dim3 grid, hipStream_t s, const Params &P, const FlatParams &S); /* LDS: + the blob */

}  // namespace dg
