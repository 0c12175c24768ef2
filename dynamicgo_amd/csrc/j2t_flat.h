/*
 * j2t_flat.h — the flat-struct kernel: field-major conversion of small
 * messages whose root struct has only scalar and string fields (C2's
 * baseline.Simple, conv/j2t/conv_test.go's Simple).
 *
 * A message is   ws '{' ws "key" ws ':' ws value ws (',' ...)* '}' ws
 * and once the top-level commas and colons are known every field converts on
 * its own. The lane-per-message kernel (j2t_small.h) walks a message
 * byte-serially in one lane, so a 64K batch is one wave per SIMD and every
 * latency is exposed. Here a block of 4 waves takes 64 messages:
 *
 *  1. structure: 4 lanes per message, each classifies 64 bytes of the
 *     staged message into bit masks (quote, comma, colon; backslash only
 *     when the message has one), bit b = byte b; the in-string mask is a
 *     prefix XOR of the quote bits carried across the 4 lanes with DPP
 *     scans; commas and colons outside strings are recorded (with the count
 *     of quotes before each comma).
 *  2. fields, field-major: wave w converts field w (+4r) of all 64
 *     messages, so the lanes of a wave hold the same field of 64 messages --
 *     the same type, the same code path. Key lookup (the predicted IDL-order
 *     field, else the name table), value parse and Thrift size.
 *  3. every lane reads the sizes of the fields before its own (one barrier)
 *     and writes its field straight into the message's slot, byte-exact at
 *     the partial words it shares with its neighbours; string/base64 bodies
 *     over 16 B are left to chunk tasks the whole block takes after a
 *     barrier; a lane per message then checks unset fields and writes STOP.
 *
 * No output stage in LDS: ~36 KiB per block with a small descriptor, so 4
 * blocks (16 waves) fit a CU and a 64K-message batch (1024 blocks) is
 * resident in one round instead of 1.33.
 *
 * JSON fields are written in input order, exactly as j2t_fsm_exec writes them
 * (native/thrift.c:765-1187: tb_write_field_begin + value per key,
 * native/thrift.c:312-420 for the values). Anything outside that shape --
 * nesting, null values, escaped keys, a backslash before '"' or '\\', unset
 * fields that need writing, any error -- goes to the bail list, whose list
 * pass (lane kernel fast path, then the exact machine) produces the
 * reference's bytes or error. Messages longer than big_max go to the wave
 * kernel's list as in the small kernel.
 */
#pragma once
#include "j2t_small.h"

namespace dg {

constexpr uint32_t FL_G = 4;                     /* lanes per message in the structure phase */
#ifndef DG_FL_WAVES
#define DG_FL_WAVES 4
#endif
constexpr uint32_t FL_WAVES = DG_FL_WAVES;       /* waves per block (the structure phase uses the first 4) */
#ifndef DG_FL_FPW
#define DG_FL_FPW 2
#endif
constexpr uint32_t FL_FPW = DG_FL_FPW;           /* fields per wave per round (each one more inlined parser) */
constexpr uint32_t FL_SLOTS = FL_FPW * FL_WAVES; /* fields per round */
constexpr uint32_t FL_MPB = 64;                  /* messages per block (= lanes of a wave in phase 2) */
constexpr uint32_t FL_LW = 9;                    /* aligned words a structure lane reads: 64 bytes at any alignment */
constexpr uint32_t FL_MAXLEN = 256;              /* longest message on this kernel */
constexpr uint32_t FL_SLOTW = FL_MAXLEN / 8;     /* words per message when the block's span is not staged */
constexpr uint32_t FL_STAGEW = FL_MPB * FL_SLOTW;/* 16 KiB */
constexpr uint32_t FL_SLACKW = FL_G * FL_LW + 2; /* reads past the last message stay in the array */
constexpr uint32_t FL_MAXF = 24;                 /* fields per message (top-level commas + 1) */
constexpr uint32_t FL_DESC = 16 * 1024;          /* descriptor bytes in LDS (dynamic) */
#ifndef DG_FL_INLINE
#define DG_FL_INLINE 8 /* r7p: 8 vs 16 bytes, the flat kernel 2 % faster on C2, c2s, c2x; C1 even */
#endif
#ifndef DG_FL_CHUNK
#define DG_FL_CHUNK 32
#endif
constexpr uint32_t FL_INLINE = DG_FL_INLINE;     /* longer string / base64 bodies are written as chunk tasks */
constexpr uint32_t FL_CHUNK = DG_FL_CHUNK;       /* input bytes per chunk task (a multiple of 8) */
constexpr uint32_t FL_MAXTASK = 320;             /* chunk tasks per block (more: the message declines; C2 ~160) */
constexpr uint32_t FL_KEYS = 32;                  /* name-table slots of the flat struct kept as a key table (larger: name table) */
constexpr uint32_t FL_NESC = 8;                  /* escapes per message (more: the message declines; C1's string has 8) */
#ifndef DG_FL_WPE
#define DG_FL_WPE 4 /* waves per SIMD the register budget is cut for: 128 VGPRs; LDS allows 4 blocks (16 waves) per CU */
#endif

#ifndef DG_FL_DEFER_NUM
#define DG_FL_DEFER_NUM 0 /* 1: numbers of known fields parsed in the write phase (measured 51.6 vs 50.2 us/step: off) */
#endif
#ifndef DG_FL_PERM
#define DG_FL_PERM 0
#endif
#ifndef DG_FL_REMAP
#define DG_FL_REMAP 1 /* the field remap (phase 2a) */
#endif

/* -DDG_FLPROF_G: cycles per wave in the stages of a field's parse, summed
 * over the fields (P.stats[2 + stage]): 0 separators from LDS, 1 delimiter
 * bytes, 2 key, 3 value, 4 sizes, 5 bookkeeping after fl_field */
#ifdef DG_FLPROF_G
#define FLG_ARG , uint64_t *flg
#define FLG_PASS , flg
#define FLG(k)                                             \
    do {                                                   \
        const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
        flg[k] += now_ - flg[7];                           \
        flg[7] = now_;                                     \
    } while (0)
#else
#define FLG_ARG
#define FLG_PASS
#define FLG(k)
#endif
/* the field (within a round) wave w converts as its h-th: w + 4h, or with
 * DG_FL_PERM 1 a snake (w, then 7 - w) that pairs early with late fields */
DGI uint32_t fl_slot(uint32_t w, uint32_t h)
{
    return DG_FL_PERM == 1 ? (h & 1 ? (h + 1) * FL_WAVES - 1 - w : h * FL_WAVES + w) : w + h * FL_WAVES;
}

/* ---- group (4 lanes, a DPP quad) collectives; converged code only ---- */
#define DG_DPP(v, ctrl) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(v), (ctrl), 0xF, 0xF, false))
DGI uint32_t g4_incl_sum(uint32_t v, uint32_t g)
{
    uint32_t t = DG_DPP(v, 0x111); /* row_shr:1 */
    v += g >= 1 ? t : 0u;
    t = DG_DPP(v, 0x112); /* row_shr:2 */
    v += g >= 2 ? t : 0u;
    return v;
}
DGI uint32_t g4_sum(uint32_t v)
{
    v += DG_DPP(v, 0xB1); /* quad_perm [1,0,3,2] */
    v += DG_DPP(v, 0x4E); /* quad_perm [2,3,0,1] */
    return v;
}
/* the value of the next lane of the group (0 for the last lane) */
DGI uint32_t g4_next(uint32_t v, uint32_t g)
{
    const uint32_t t = DG_DPP(v, 0x101); /* row_shl:1 */
    return g < 3 ? t : 0u;
}

/* 0x80 in each byte of w (32-bit half) equal to c */
DGI uint32_t eq32(uint32_t w, uint32_t cc) { return zb32(w ^ cc); }

/* The staged message in LDS, the SrcT interface without SrcT's one-word
 * cache: every access is its own LDS read, so independent reads overlap
 * instead of chaining through the cache tag (and no per-lane branch). */
struct LSrc {
    typedef int32_t idx;
    const __attribute__((address_space(3))) uint64_t *w8;
    int32_t off0;
    int32_t n;
    DGI void init(const __attribute__((address_space(3))) uint64_t *words, int32_t off, int32_t len)
    {
        w8 = words;
        off0 = off;
        n = len;
    }
    DGI uint8_t raw(int32_t i) const
    {
        return ((const __attribute__((address_space(3))) uint8_t *)w8)[off0 + i];
    }
    DGI uint8_t at(int32_t i) const { return (uint32_t)i < (uint32_t)n ? raw(i) : 0; }
    /* 8 bytes at [i, i+8), first byte lowest (the stage has slack words past the end) */
    DGI uint64_t get8(int32_t i) const
    {
        const uint32_t b = (uint32_t)(off0 + i), k = b >> 3, sh = (b & 7) << 3;
        const uint64_t lo = w8[k], hi = w8[k + 1];
        return (lo >> sh) | ((hi << 1) << (63 - sh));
    }
    DGI LSrc sub(int32_t s0, int32_t len) const
    {
        LSrc r;
        r.init(w8, off0 + s0, len);
        return r;
    }
};

/* A number's bytes in registers: the 5 aligned staged words covering
 * [p, p + 32) of the message, read together (one LDS round trip) instead of
 * the parse loops' dependent word-at-a-time reads. Numbers up to RSL_MAX
 * bytes use it (digits8 reads 8 bytes at i <= n: word index <= 4); longer
 * ones parse from LDS. The stage has slack words past every message. */
constexpr int32_t RSL_MAX = 24;
struct RSrcL {
    typedef int32_t idx;
    static constexpr bool kRegs = true; /* fast_vnumber: the fixed-step integer path */
    uint64_t w0, w1, w2, w3, w4;
    uint32_t sh; /* byte offset of the number's first byte in w0 */
    int32_t n;
    DGI void load(const LSrc &src, int32_t p, int32_t len)
    {
        const uint32_t b = (uint32_t)(src.off0 + p);
        const __attribute__((address_space(3))) uint64_t *q = src.w8 + (b >> 3);
        sh = b & 7;
        n = len;
        w0 = q[0];
        w1 = q[1];
        w2 = q[2];
        w3 = q[3];
        w4 = q[4];
    }
    DGI uint64_t word(uint32_t j) const { return j == 0 ? w0 : j == 1 ? w1 : j == 2 ? w2 : j == 3 ? w3 : w4; }
    DGI uint8_t raw(int32_t i) const
    {
        const uint32_t b = sh + (uint32_t)i;
        return (uint8_t)(word(b >> 3) >> ((b & 7) << 3));
    }
    DGI uint8_t at(int32_t i) const { return (uint32_t)i < (uint32_t)n ? raw(i) : 0; }
    DGI uint64_t get8(int32_t i) const
    {
        const uint32_t b = sh + (uint32_t)i, j = b >> 3, s8 = (b & 7) << 3;
        return (word(j) >> s8) | ((word(j + 1) << 1) << (63 - s8));
    }
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
    bool defer;       /* FV_NUM: the text [s0, s0+nb) is parsed by flat_write */
};

template <class S>
DGI uint32_t skip_ws(S &s, uint32_t p)
{
    while (p < (uint32_t)s.n && isspace_(s.raw((int32_t)p))) p++;
    return p;
}

/* the name table of struct sd (native/thrift.c:449-468 j2t_find_field_key):
 * the global field index of key src[k0, k0+kn), or -1 */
template <class S, class DV>
DGI int32_t fl_lookup(const DV &D, const dg_struct &sd, S &src, uint32_t k0, uint32_t kn)
{
    typedef typename S::idx SI;
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
        if (nm.field == DG_NONE) return -1;
        if (nm.hash == h && nm.key_len == kn && key_eq(src, (SI)k0, kn, (decltype(&D.R[0]))(&D.P[nm.key_off])))
            return (int32_t)nm.field;
    }
}

/* ---- escapes: decoded once, in the structure phase ----
 * Every backslash of a flat message starts an escape (one before '"' or '\\'
 * declines the message), so the structure phase decodes each one where it
 * finds it (4 lanes per message, in parallel) into the message's escape
 * table: position, JSON bytes (2 or 6), UTF-8 bytes (1..3) and their value.
 * A string's Thrift size is then its length minus what its escapes shrink,
 * and its body is written as runs copied around the escapes -- no serial
 * unquote loop over the string on the field's wave, twice (size and write).
 * unquote's semantics (native/parsing.c:702-945, flags 0) for everything
 * the flat path keeps; a surrogate, an invalid escape or more than FL_NESC
 * escapes decline the message to the list pass. */
typedef const __attribute__((address_space(3))) uint32_t lds_esc;
/* an entry: bit 31 set | position (12 bits) | \u form << 12 | code point << 13 */
DGI uint32_t esc_pos(uint32_t x) { return x & 0xFFF; }
DGI uint32_t esc_in(uint32_t x) { return (x >> 12) & 1 ? 6u : 2u; }           /* JSON bytes */
DGI uint32_t esc_cp(uint32_t x) { return (x >> 13) & 0xFFFF; }
DGI uint32_t esc_out(uint32_t x) { const uint32_t cp = esc_cp(x); return cp <= 0x7f ? 1u : cp <= 0x7ff ? 2u : 3u; }
DGI uint32_t esc_utf8(uint32_t x) /* its UTF-8 bytes, first byte lowest */
{
    const uint32_t cp = esc_cp(x);
    return cp <= 0x7f ? cp
           : cp <= 0x7ff ? (0xc0 | (cp >> 6)) | ((0x80 | (cp & 0x3f)) << 8)
                         : (0xe0 | (cp >> 12)) | ((0x80 | ((cp >> 6) & 0x3f)) << 8) | ((0x80 | (cp & 0x3f)) << 16);
}
DGI bool fl_hex4(uint32_t w, uint32_t &v)
{
    uint32_t r = 0, ok = 1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t b = (w >> (8 * k)) & 0xFF, d = b - '0', l = (b | 0x20) - 'a';
        ok &= (uint32_t)(d < 10) | (uint32_t)(l < 6);
        r = (r << 4) | (d < 10 ? d : (l + 10) & 0xF);
    }
    v = r;
    return ok != 0;
}
/* the escape at message position p (e0: the 8 bytes from its backslash) ->
 * its table entry, or 0 if the flat path leaves it to the exact machine */
DGI uint32_t fl_escape(uint32_t p, uint64_t e0)
{
    const uint32_t c = (uint32_t)(e0 >> 8) & 0xFF;
    if (c == 'u') {
        uint32_t cp;
        if (!fl_hex4((uint32_t)(e0 >> 16), cp) || (cp >= 0xd800 && cp <= 0xdfff)) return 0;
        return 0x80000000u | p | (1u << 12) | (cp << 13);
    }
    /* _UnquoteTab native/parsing.c:565-575 */
    const uint32_t cc = c == 'b' ? 8u : c == 'f' ? 12u : c == 'n' ? 10u : c == 'r' ? 13u : c == 't' ? 9u : c;
    const bool ok = (c == '"') | (c == '\\') | (c == '/') | (c == 'b') | (c == 'f') | (c == 'n') | (c == 'r') | (c == 't');
    return ok ? 0x80000000u | p | (cc << 13) : 0u;
}
/* escapes in [a, b): any, and the bytes they shrink the body by */
DGI bool fl_esc_in(lds_esc *E, uint32_t ne, uint32_t a, uint32_t b, uint32_t &shrink)
{
    bool any = false;
    shrink = 0;
    for (uint32_t e = 0; e < ne; e++) {
        const uint32_t x = E[e];
        const uint32_t p = esc_pos(x);
        const bool in = p >= a && p < b;
        any |= in;
        shrink += in ? esc_in(x) - esc_out(x) : 0u;
    }
    return any;
}

/* Field k: bytes (sk, ek) between its separators, its colon at ck, nq quotes
 * inside. Key lookup, value parse and Thrift size; false = decline the
 * message. Every quote of the message is a delimiter (phase 1 declined \" and
 * \\), so a field holds exactly the key's two quotes, plus two when the value
 * is a string: the key and a string value are delimited without scanning. */
template <bool KO = false, class S, class DV>
DGI bool fl_field(const DV &D, const dg_struct &sd, S &src, uint32_t sk, uint32_t ck, uint32_t ek, uint32_t nq,
                  bool hasbs, lds_esc *E, uint32_t ne, const __attribute__((address_space(3))) uint64_t *KW,
                  const __attribute__((address_space(3))) uint32_t *KM, uint32_t nk, uint32_t k, uint64_t flag,
                  const FastTabs &tb, FField &F FLG_ARG)
{
    typedef typename S::idx SI;
    /* Round 1 of LDS reads: the four delimiting bytes and the predicted
     * field's record (field k in IDL order), issued together; every test is
     * written without short-circuit branches, so the loads are not sunk into
     * branches and chained one after another. Spaces around the delimiters
     * take the loops. */
    const uint8_t d_s = src.raw((SI)sk), d_q = src.raw((SI)(ck - 1)), d_v = src.raw((SI)(ck + 1)),
                  d_e = src.raw((SI)(ek - 1));
    const bool pred = k < sd.n_fields;
    dg_field f = ldrec(&D.F[sd.field_begin + (pred ? k : 0u)]);
    uint32_t p = sk, q = ck, v0 = ck + 1, ve = ek;
    uint8_t cs = d_s, cq = d_q, c = d_v, ce = d_e;
    if (isspace_(d_s) | isspace_(d_q) | isspace_(d_v) | isspace_(d_e) | (ck + 1 >= ek)) {
        p = skip_ws(src, sk);
        while (q > p && isspace_(src.raw((SI)(q - 1)))) q--;
        v0 = skip_ws(src, ck + 1);
        while (ve > v0 && isspace_(src.raw((SI)(ve - 1)))) ve--;
        if (v0 >= ve) return false;
        cs = src.raw((SI)p);
        cq = src.raw((SI)(q - 1));
        c = src.raw((SI)v0);
        ce = src.raw((SI)(ve - 1));
    }
    if ((q < p + 2) | (cs != '"') | (cq != '"') | (nq != (c == '"' ? 4u : 2u))) return false;
    const uint32_t k0 = p + 1, kn = q - 1 - k0;
    FLG(1);
    uint32_t shrink = 0;
    if (hasbs && fl_esc_in(E, ne, k0, k0 + kn, shrink)) return false; /* escaped key: unquoted before lookup -> the list pass */
    /* the key (native/thrift.c:668-763): predicted (field k in IDL order),
     * else the name table. Round 2: a key of up to 16 bytes and the
     * predicted key's pool words, compared in one step (the pool keys are
     * zero-padded to 8 bytes, key_eq's semantics) */
    int32_t fi = -1;
    uint64_t a0m = 0, a1m = 0; /* a key of up to 16 bytes, zero-padded like the pool's */
    {
        const __attribute__((address_space(3))) uint64_t *pk = (decltype(&D.R[0]))(&D.P[f.key_off]);
        bool hit;
        if (kn <= 16) {
            const uint64_t a0 = src.get8((SI)k0), a1 = src.get8((SI)(k0 + 8)), b0 = pk[0], b1 = pk[1];
            const uint64_t m0 = kn >= 8 ? ~0ull : (1ull << (kn << 3)) - 1;
            const uint64_t m1 = kn >= 16 ? ~0ull : kn <= 8 ? 0ull : (1ull << ((kn - 8) << 3)) - 1;
            a0m = a0 & m0;
            a1m = a1 & m1;
            hit = (a0m == b0) & ((kn <= 8) | (a1m == b1));
        } else {
            hit = key_eq(src, (SI)k0, kn, pk);
        }
        if (pred & ((f.flags & DG_FF_ALIAS_SELF) != 0) & (f.key_len == kn) & hit) fi = (int32_t)(sd.field_begin + k);
    }
    if (fi < 0) {
        if (nk && kn <= 16) {
            /* the struct's names from the key table (phase 1): every lane
             * scans the same entries (uniform addresses, broadcast reads),
             * no byte-serial hash and no probe chain -- the shuffled-key
             * case (c2s) misses the predicted field on most fields */
#pragma unroll 4
            for (uint32_t e = 0; e < nk; e++) {
                const uint32_t mt = KM[e];
                if (((mt >> 24) == kn) & (KW[2 * e] == a0m) & (KW[2 * e + 1] == a1m)) fi = (int32_t)(mt & 0xFFFFFFu);
            }
        } else {
            fi = fl_lookup(D, sd, src, k0, kn);
        }
        if (fi >= 0) f = ldrec(&D.F[fi]);
    }
    if constexpr (KO) { /* the key pass (field remap): the field only */
        F.fi = fi;
        return true;
    }
    FLG(2);
    /* the value, [v0, ve) */
    F.defer = false;
    uint32_t vk;
    uint32_t vs0 = 0, vnb = 0;
    bool vesc = false, isint = false, bv = false;
    int64_t iv = 0;
    double dv = 0.0;
    if (c == '"') {
        if ((ve - v0 < 2) | (ce != '"')) return false;
        vs0 = v0 + 1;
        vnb = ve - 1 - vs0;
        vesc = hasbs && fl_esc_in(E, ne, vs0, vs0 + vnb, shrink); /* shrink: what its escapes take off */
        vk = FV_STR;
    } else if (c == '-' || (uint8_t)(c - '0') <= 9) {
        /* a known field without a value mapping: a number's Thrift size
         * follows from the field type alone, so its text is parsed by
         * flat_write after the size barrier (the wave holding a double no
         * longer holds the others back); skipped and mapped fields parse it
         * here, as the reference validates them before anything else */
        const bool later = DG_FL_DEFER_NUM && fi >= 0 && !((flag & DG_F_ENABLE_VM) && f.vm != DG_VM_NONE);
        if (!later) {
            const int32_t nl = (int32_t)(ve - v0);
            bool okn;
            if (nl <= RSL_MAX) { /* the number's words in registers: one LDS round trip */
                RSrcL rs;
                rs.load(src, (int32_t)v0, nl);
                int32_t qq = 0;
                okn = fast_vnumber(rs, qq, tb, iv, dv, isint) && qq == nl;
            } else {
                SI qq = (SI)v0;
                okn = fast_vnumber(src, qq, tb, iv, dv, isint) && (uint32_t)qq == ve;
            }
            if (!okn) return false;
        }
        F.defer = later;
        vs0 = v0;
        vnb = ve - v0;
        vk = FV_NUM;
    } else if (c == 't') {
        if (ve - v0 != 4 || (uint32_t)src.get8((SI)v0) != VS_TRUE) return false;
        bv = true;
        vk = FV_BOOL;
    } else if (c == 'f') {
        if (ve - v0 != 5 || (uint32_t)src.get8((SI)(v0 + 1)) != VS_ALSE) return false;
        vk = FV_BOOL;
    } else {
        return false; /* null, containers, garbage: the list pass */
    }
    FLG(3);
    F.fi = fi;
    if (fi < 0 || ((f.flags & DG_FF_REQUEST_BASE) && (flag & DG_F_NO_WRITE_BASE))) {
        if (fi < 0 && !(flag & DG_F_ALLOW_UNKNOWN)) return false; /* ERR_UNKNOWN_FIELD */
        if (fi >= 0) return false;
        F.kind = FV_NONE; /* an unknown key with a scalar value: skipped */
        F.size = 0;
        return true;
    }
    const dg_type ft = ldrec(&D.T[f.type]);
    const uint8_t tt = ft.ttype;
    const bool bin = (ft.flags & DG_TF_BINARY) && !(flag & DG_F_NO_BASE64);
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
            SI qq = 0;
            if (!fast_vnumber(sub, qq, tb, iv, dv, isint) || (uint32_t)qq != vnb) return false;
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
            vsize = 4 + vnb - shrink;
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
    FLG(4);
    return true;
}

/* a piece of a string body: src[s0, s0+n) copied */
template <class S, class O>
DGI void body_copy(S &src, uint32_t s0, uint32_t n, O &o)
{
    fast_copy(src, (typename S::idx)s0, (typename S::idx)n, o);
}
/* a piece of a canonical padded base64 body, src[s0, s0+n) (n % 4 == 0);
 * `last`: the piece holds the final quantum, which may carry '=' */
template <class S, class O>
DGI bool body_b64(S &src, uint32_t s0, uint32_t n, bool last, O &o)
{
    typedef typename S::idx SI;
    uint32_t ip = 0;
    const uint32_t full = last && n >= 4 ? n - 4 : n;
    for (; ip + 8 <= full; ip += 8) {
        uint64_t v;
        if (!b64_8(src.get8((SI)(s0 + ip)), v)) return false;
        o.wle(v, 6);
    }
    for (; ip < full; ip += 4) {
        uint32_t v;
        if (!b64_4((uint32_t)src.get8((SI)(s0 + ip)), v)) return false;
        o.wle(v, 3);
    }
    if (last && n >= 4) {
        uint32_t w = (uint32_t)src.get8((SI)(s0 + ip));
        const uint32_t c2 = (w >> 16) & 0xFF, c3 = w >> 24;
        if (c2 == '=' && c3 != '=') return false; /* "xx=y": a decode error in the reference */
        const uint32_t keep = c3 == '=' ? (c2 == '=' ? 1u : 2u) : 3u;
        if (c3 == '=') w = (w & 0x00FFFFFFu) | ((uint32_t)'A' << 24);
        if (c2 == '=') w = (w & 0xFF00FFFFu) | ((uint32_t)'A' << 16);
        uint32_t v;
        if (!b64_4(w, v)) return false;
        o.wle(v, keep); /* decode_block keeps nb-1 bytes; the padding bits are not checked */
    }
    return true;
}

/* write a parsed field: header, then the value (j2t_number/j2t_string/
 * j2t_binary, native/thrift.c:312-420). Returns 0 = error, 1 = written,
 * 2 = header and length written, the body (> FL_INLINE bytes of a string
 * without escapes or of canonical base64) is left to chunk tasks. */
template <class S, class O>
DGI uint32_t flat_write(S &src, const FField &F, const FastTabs &tb, O &o, lds_esc *E, uint32_t ne)
{
    typedef typename S::idx SI;
    if (F.kind == FV_NONE) return 1;
    bool isint = F.isint;
    int64_t iv = F.iv;
    double dv = F.dv;
    if (F.kind == FV_NUM && F.defer) { /* the number's text, parsed now (native/scanning.c vnumber) */
        SI qq = (SI)F.s0;
        if (!fast_vnumber(src, qq, tb, iv, dv, isint) || (uint32_t)qq != F.s0 + F.nb) return 0;
    }
    o.wle((uint32_t)F.tt | ((uint32_t)__builtin_bswap16(F.id) << 8), 3);
    switch (F.kind) {
    case FV_BOOL: o.w8((uint8_t)iv); return 1;
    case FV_NUM:
        if (F.i16q) {
            emit_number(o, DG_T_I16, isint, iv, dv);
            emit_number(o, DG_T_BYTE, isint, iv, dv);
            return 1;
        }
        return emit_number(o, F.tt, isint, iv, dv) ? 1u : 0u;
    case FV_NUMSTR:
    case FV_STR:
        o.w32(F.kind == FV_NUMSTR ? F.nb : F.size - 7);
        if (F.esc) { /* runs copied around the escapes (decoded in the structure phase), in position order */
            uint32_t cur = F.s0;
            const uint32_t end = F.s0 + F.nb;
            for (uint32_t it = 0; it < FL_NESC; it++) {
                uint32_t best = 0xFFFFFFFFu; /* position 0xFFF: none */
                for (uint32_t e = 0; e < ne; e++) {
                    const uint32_t x = E[e], p = esc_pos(x);
                    if (p >= cur && p < end && p < esc_pos(best)) best = x;
                }
                if (best == 0xFFFFFFFFu) break;
                const uint32_t p = esc_pos(best);
                body_copy(src, cur, p - cur, o);
                o.wle(esc_utf8(best), esc_out(best));
                cur = p + esc_in(best);
            }
            body_copy(src, cur, end - cur, o);
            return 1;
        }
        if (F.nb > FL_INLINE) return 2;
        body_copy(src, F.s0, F.nb, o);
        return 1;
    default: /* FV_BIN: canonical padded base64 */
        o.w32(F.size - 7);
        if (F.nb > FL_INLINE) return 2;
        return body_b64(src, F.s0, F.nb, true, o) ? 1u : 0u;
    }
}

struct FlatParams {
    const uint8_t *blob;
    dg_desc_hdr hdr;
    uint32_t *bail_count;
    uint32_t *bail_list;
    /* wrapped mode: the batch root R (P.root) is not flat, but a message
     * {"key":{...}} whose one member is a field of R with the flat struct
     * type wrap_inner converts as that field's header, the inner object on
     * this kernel, STOP, STOP. wrap_ok: the fields of R (bit = index in R)
     * allowed as that member: type wrap_inner, no value mapping or base
     * skip in play, and R's other fields need nothing at '}' under the
     * batch's flags (j2t_write_unset_fields, native/thrift.c:258-310).
     * Anything else declines to the list pass. */
    uint32_t wrap;
    uint32_t wrap_inner;
    uint64_t wrap_ok;
};

/* -DDG_FLPROF: cycles per wave by phase (s_memtime at the marks, summed
 * into P.stats[2..] by each wave's first lane, 1 block in 32 sampled) */
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
        if ((threadIdx.x & 63) == 0 && (blockIdx.x & 31) == 0)                           \
            for (int k_ = 0; k_ < 8; k_++) atomicAdd(&P.stats[2 + k_], (unsigned long long)flp[k_]); \
    } while (0)
#else
#define FLP_DECL
#define FLP(k)
#define FLP_END()
#endif
/* -DDG_FLPROF_F: cycles per wave spent in each field slot's parse
 * (P.stats[2 + slot]) and write (P.stats[8 + slot]), slots 0..5, 1 block in
 * 32 sampled (tools/flprof.py --fields) */
#ifdef DG_FLPROF_F
#define FLF_DECL uint64_t flf[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define FLF_T0() const uint64_t flf_t0 = __builtin_amdgcn_s_memtime()
#define FLF_ADD(k) do { if ((k) < 12) flf[k] += __builtin_amdgcn_s_memtime() - flf_t0; } while (0)
#define FLF_END()                                                                         \
    do {                                                                                  \
        if ((threadIdx.x & 63) == 0 && (blockIdx.x & 31) == 0)                            \
            for (int k_ = 0; k_ < 12; k_++) atomicAdd(&P.stats[2 + k_], (unsigned long long)flf[k_]); \
    } while (0)
#else
#define FLF_DECL
#define FLF_T0()
#define FLF_ADD(k)
#define FLF_END()
#endif

/* per-message state of the block, one array per member (lane = message:
 * consecutive banks). ~36 KiB with a small descriptor: 4 blocks (16 waves)
 * per CU, so a 64K-message batch (1024 blocks) is resident in one round. */
struct FlatLds {
    uint64_t in[FL_STAGEW + FL_SLACKW];     /* the staged JSON */
    uint64_t task[FL_MAXTASK];              /* chunk tasks */
    uint64_t oa[FL_MPB];                    /* output slot */
    uint32_t cap[FL_MPB];
    uint32_t ok[FL_MPB];                    /* still on the flat path (any lane may clear it) */
    uint32_t n[FL_MPB];                     /* JSON length */
    uint32_t lw[FL_MPB];                    /* LDS word of the first aligned word << 3 | arena offset & 7 */
    uint32_t oc[FL_MPB];                    /* open | close << 16 */
    uint32_t nfq[FL_MPB];                   /* fields | quotes << 8 | backslash seen << 31 */
    uint32_t plo[FL_MPB], phi[FL_MPB];      /* present fields (struct field-index bits) */
    uint32_t big[FL_MPB];                   /* listed for the wave kernel */
    uint32_t nbytes[FL_MPB];                /* Thrift bytes before STOP */
    uint32_t wid[FL_MPB];                   /* wrapped mode: 0x10000 | the outer field's id, 0 = not wrapped */
    uint32_t nesc[FL_MPB];                  /* escapes found in the message (phase 1) */
    uint32_t esc[FL_MPB * FL_NESC];         /* [m][e]: fl_escape's entries */
    uint64_t kw[2 * FL_KEYS];               /* key table: the flat struct's names up to 16 bytes, zero-padded */
    uint32_t km[FL_KEYS];                   /* ... field | key_len << 24 (0xFF << 24: empty slot, longer key) */
    uint32_t fkm[FL_SLOTS];                 /* field j's own key length (the order check; 0xFF: not predictable) */
    uint32_t sep[FL_MAXF * FL_MPB];         /* [k][m]: comma position | quotes before it << 16 */
    uint16_t col[FL_MAXF * FL_MPB];         /* [k][m]: colon position */
    uint16_t size[2 * FL_SLOTS * FL_MPB];   /* [round & 1][slot][m] */
    uint32_t fseen[FL_MPB];                 /* key pass: the fields found in the message (bit = field index) */
    uint32_t rounds, ntask, tgrab, noremap;
    /* kernel arguments used only by the writes and the finish, read from
     * here where they are needed instead of held in SGPRs through the parse
     * (the kernel is at the SGPR limit: uniform values spill to VGPR lanes) */
    uint8_t *a_out;
    uint64_t *a_ret;
    uint32_t *a_out_len, *a_bail_count, *a_bail_list;
    uint32_t a_nb, a_wrap; /* messages in the block; S.wrap */
    uint64_t p10u[20];
    double p10d[23];
    uint64_t pw[EL_WN];                     /* Eisel-Lemire powers window (j2t_fast.h) */
};

template <int V>
__global__ __launch_bounds__(64 * FL_WAVES) __attribute__((amdgpu_waves_per_eu(DG_FL_WPE))) void j2t_flat_kernel(
    Params P, FlatParams S)
{
    __shared__ __attribute__((aligned(16))) FlatLds L;
    extern __shared__ __attribute__((aligned(16))) uint64_t s_fdesc[];
    FLP_DECL
    FLF_DECL
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t b0 = (uint64_t)blockIdx.x * FL_MPB;
    const uint64_t b1 = b0 + FL_MPB < P.n ? b0 + FL_MPB : P.n;

    /* ---- 0. the block's JSON span to LDS (16-byte coalesced), the descriptor,
     *      per-message offsets ---- */
    const uint64_t lo = P.in_off[b0], hi = P.in_off[b1];
    const uint64_t base = lo & ~15ull;
    const bool staged = hi - base <= (uint64_t)FL_STAGEW * 8;
    if (staged) {
        /* every thread's (up to 4) 16-byte loads issued before any is
         * stored: one HBM round trip for the block's span, not one per
         * loop trip */
        const uint4 *gs = (const uint4 *)(P.json + base); /* arena: 16 readable bytes past the end */
        uint4 *ls = (uint4 *)L.in;
        const uint32_t nw = (uint32_t)((hi - base + 15) >> 4);
        constexpr uint32_t NT = 64 * FL_WAVES;
        static_assert(FL_STAGEW * 8 / 16 <= 4 * NT, "four 16-byte loads per thread cover the stage");
        if (nw) { /* unconditional loads (clamped index), conditional stores: no branch between the loads */
            const uint32_t l = nw - 1;
            const uint4 v0 = gs[min(tid, l)], v1 = gs[min(tid + NT, l)], v2 = gs[min(tid + 2 * NT, l)],
                        v3 = gs[min(tid + 3 * NT, l)];
            if (tid < nw) ls[tid] = v0;
            if (tid + NT < nw) ls[tid + NT] = v1;
            if (tid + 2 * NT < nw) ls[tid + 2 * NT] = v2;
            if (tid + 3 * NT < nw) ls[tid + 3 * NT] = v3;
        }
    }
    {
        const uint4 *gd = (const uint4 *)S.blob;
        uint4 *ld = (uint4 *)s_fdesc;
        for (uint32_t k = tid; k < (S.hdr.total_len + 15) / 16; k += 64 * FL_WAVES) ld[k] = gd[k];
    }
    if (tid < 20) {
        uint64_t v = 1;
        for (uint32_t k = 0; k < tid; k++) v *= 10;
        L.p10u[tid] = v;
    }
    if (tid < 23) L.p10d[tid] = P10[tid];
    el_window_fill(L.pw, tid);
    if (tid == 0) {
        L.rounds = 0;
        L.ntask = 0;
        L.tgrab = 0;
        L.noremap = 0;
        L.a_out = P.out;
        L.a_ret = P.ret;
        L.a_out_len = P.out_len;
        L.a_bail_count = S.bail_count;
        L.a_bail_list = S.bail_list;
        L.a_nb = (uint32_t)(b1 - b0);
        L.a_wrap = S.wrap;
    }
    if (tid < FL_MPB) {
        uint32_t ok = 0, n = 0, lw = 0, big = 0, cap = 0;
        uint64_t oa = 0;
        const uint64_t i = b0 + tid;
        if (i < b1) {
            const uint64_t a = P.in_off[i], b = P.in_off[i + 1];
            const uint64_t n64 = b - a;
            oa = P.out_off[i];
            cap = (uint32_t)min(P.out_off[i + 1] - oa, (uint64_t)0xFFFFFFFFu);
            const bool tobig = P.big_list && (n64 > P.big_max || n64 > FL_MAXLEN);
            list_big_w(P, tobig, i, n64); /* the wave kernel */
            if (tobig) {
                big = 1;
            } else if (n64 > 0 && n64 <= FL_MAXLEN) {
                n = (uint32_t)n64;
                if (staged) {
                    ok = 1;
                    lw = (uint32_t)(((a - base) >> 3) << 3) | (uint32_t)(a & 7);
                } else {
                    ok = 1; /* its own 256-byte slot, realigned to byte 0 */
                    lw = (tid * FL_SLOTW) << 3;
                }
            }
        }
        L.ok[tid] = ok;
        L.n[tid] = n;
        L.lw[tid] = lw;
        L.big[tid] = big;
        L.oa[tid] = oa;
        L.cap[tid] = cap;
        L.plo[tid] = 0;
        L.phi[tid] = 0;
        L.oc[tid] = 0;
        L.nfq[tid] = 0;
        L.nesc[tid] = 0;
        L.fseen[tid] = 0;
    }
    if (tid < FL_SLOTS * FL_MPB / 4) ((uint32_t *)(void *)L.task)[tid] = 0xFFFFFFFFu; /* the field map (in the task area): none */
    __syncthreads();
    const uint32_t g = tid & 3, m1 = tid >> 2; /* phase 1: 4 lanes per message */
    if (!staged) {
        /* a span too long for the stage (large messages in between, as in a
         * mixed batch): each message is copied to its own 256-byte slot,
         * shifted to start at byte 0 (two aligned global words per word; the
         * arena has 16 readable bytes past its end) */
        if (tid < FL_G * FL_MPB && L.ok[m1]) {
            const uint64_t a = P.in_off[b0 + m1];
            const uint32_t nw = (L.n[m1] + 7) >> 3, sh = (uint32_t)(a & 7) << 3;
            const glb_u64 *gsrc = (const glb_u64 *)(const void *)P.json + (a >> 3);
            /* lane g: words g, g + 4, ... (<= 8 of them, 256 bytes); all its
             * loads issued before the first use (indices clamped to the word
             * past the message, inside the arena's 16 readable bytes) */
            constexpr uint32_t NWL = FL_MAXLEN / 8 / FL_G;
            uint64_t lo[NWL], hi[NWL];
#pragma unroll
            for (uint32_t j = 0; j < NWL; j++) {
                const uint32_t w = g + FL_G * j;
                lo[j] = gsrc[min(w, nw)];
                hi[j] = gsrc[min(w + 1, nw)];
            }
#pragma unroll
            for (uint32_t j = 0; j < NWL; j++) {
                const uint32_t w = g + FL_G * j;
                if (w < nw) L.in[(L.lw[m1] >> 3) + w] = sh ? (lo[j] >> sh) | (hi[j] << (64 - sh)) : lo[j];
            }
        }
        __syncthreads();
    }
    FLP(0);
#if defined(DG_FL_STOP) && DG_FL_STOP == 9
    return; /* ablation: launch, staging and the block's tables only */
#endif
    const auto D = desc_view<3>((const __attribute__((address_space(3))) uint8_t *)(void *)s_fdesc, S.hdr);
    const FastTabs tb{(const __attribute__((address_space(3))) uint64_t *)(void *)L.p10u, (lds_f64 *)(void *)L.p10d,
                      (const __attribute__((address_space(3))) uint64_t *)(void *)L.pw};
    const dg_type rt = ldrec(&D.T[S.wrap ? S.wrap_inner : P.root]);
    const dg_struct sd = ldrec(&D.S[rt.st]);
    /* the key table: the name table's slots (read by phase 2, after phase 1's barrier) */
    const uint32_t nk = sd.name_mask + 1 <= FL_KEYS ? sd.name_mask + 1 : 0u;
    if (tid < nk) {
        const dg_name nm = ldrec(&D.N[sd.name_begin + tid]);
        uint32_t mt = 0xFF000000u;
        uint64_t w0 = 0, w1 = 0;
        if (nm.field != DG_NONE && nm.key_len <= 16) {
            const __attribute__((address_space(3))) uint64_t *pk = (decltype(&D.R[0]))(&D.P[nm.key_off]);
            w0 = nm.key_len ? pk[0] : 0ull; /* the pool pads keys with zeros to 8 bytes */
            w1 = nm.key_len > 8 ? pk[1] : 0ull;
            mt = nm.field | (nm.key_len << 24);
        }
        L.km[tid] = mt;
        L.kw[2 * tid] = w0;
        L.kw[2 * tid + 1] = w1;
    }
    if (tid >= 64 && tid < 64 + FL_SLOTS) { /* the predicted keys' lengths, for the order check */
        const uint32_t j = tid - 64;
        uint32_t len = 0xFF;
        if (j < sd.n_fields) {
            const dg_field f = ldrec(&D.F[sd.field_begin + j]);
            if (f.flags & DG_FF_ALIAS_SELF) len = f.key_len;
        }
        L.fkm[j] = len;
    }
    if (S.wrap) {
        /* ---- 0b. wrapped mode: ws '{' ws "key" ws ':' ws {inner} ws '}' ws
         *      with the key a wrap_ok field of R: the inner object becomes
         *      the message (its bytes, slot +3 for the outer header) ---- */
        if (tid < FL_MPB) {
            uint32_t wid = 0;
            if (L.ok[tid]) {
                const uint32_t n = L.n[tid], lwa = L.lw[tid];
                LSrc src;
                src.init((const __attribute__((address_space(3))) uint64_t *)(void *)&L.in[lwa >> 3], (int32_t)(lwa & 7),
                         (int32_t)n);
                uint32_t p = skip_ws(src, 0);
                bool ok = p < n && src.raw((int32_t)p) == '{';
                p = ok ? skip_ws(src, p + 1) : p;
                ok = ok && p < n && src.raw((int32_t)p) == '"';
                const uint32_t k0 = p + 1;
                uint32_t q = k0;
                while (ok && q < n && src.raw((int32_t)q) != '"') {
                    if (src.raw((int32_t)q) == '\\') ok = false; /* an escaped key: the list pass unquotes it */
                    q++;
                }
                ok = ok && q < n;
                const uint32_t kn = q - k0;
                p = ok ? skip_ws(src, q + 1) : p;
                ok = ok && p < n && src.raw((int32_t)p) == ':';
                p = ok ? skip_ws(src, p + 1) : p;
                ok = ok && p < n && src.raw((int32_t)p) == '{';
                uint32_t e = n;
                while (ok && e > p && isspace_(src.raw((int32_t)(e - 1)))) e--;
                ok = ok && e > p + 1 && src.raw((int32_t)(e - 1)) == '}';
                uint32_t ic = e - 1;
                while (ok && ic > p && isspace_(src.raw((int32_t)(ic - 1)))) ic--;
                ok = ok && ic > p + 1 && src.raw((int32_t)(ic - 1)) == '}';
                if (ok) {
                    const dg_struct rs = ldrec(&D.S[ldrec(&D.T[P.root]).st]);
                    const int32_t fi = fl_lookup(D, rs, src, k0, kn);
                    const uint32_t k = (uint32_t)fi - rs.field_begin;
                    ok = fi >= 0 && k < 64 && ((S.wrap_ok >> k) & 1);
                    if (ok) {
                        wid = 0x10000u | ldrec(&D.F[fi]).id;
                        L.lw[tid] = lwa + p;
                        L.n[tid] = ic - p;
                        L.oa[tid] += 3;
                        L.cap[tid] = L.cap[tid] > 4 ? L.cap[tid] - 4 : 0u;
                    }
                }
                if (!ok) L.ok[tid] = 0;
            }
            L.wid[tid] = wid;
        }
        __syncthreads();
    }

    /* ---- 1. structure: lane g of a message holds message bytes
     *      [64g, 64g+64) as 64-bit masks, bit b = byte 64g + b (quotes,
     *      commas, colons; backslashes only when the message has one) ---- */
    if (tid < FL_G * FL_MPB) {
        const bool on = L.ok[m1] != 0;
        const uint32_t n = L.n[m1], lwa = L.lw[m1], a7 = lwa & 7, lw = lwa >> 3;
        const int32_t nv0 = on ? (int32_t)n - 64 * (int32_t)g : 0;
        const uint32_t nv = nv0 <= 0 ? 0u : nv0 >= 64 ? 64u : (uint32_t)nv0; /* message bytes in this lane */
        const uint64_t vmask = nv >= 64 ? ~0ull : (1ull << nv) - 1;
        /* the lane's 64 bytes start a7 bytes into aligned word lw + 8g: nine
         * words read (the stage has slack past every message), re-aligned
         * to the message with byte funnel shifts */
        uint32_t d[18];
#pragma unroll
        for (uint32_t j = 0; j < 9; j++) {
            const uint64_t w = L.in[lw + 8 * g + j];
            d[2 * j] = (uint32_t)w;
            d[2 * j + 1] = (uint32_t)(w >> 32);
        }
        const bool hi4 = a7 >= 4;
        const uint32_t sh = a7 & 3;
        uint32_t x[16];
#pragma unroll
        for (uint32_t i = 0; i < 16; i++) {
            const uint32_t lo_ = hi4 ? d[i + 1] : d[i], hi_ = hi4 ? d[i + 2] : d[i + 1];
            x[i] = __builtin_amdgcn_alignbyte(hi_, lo_, sh);
        }
        /* 0x80-per-byte flags of two dwords -> 8 bits (byte i of the pair at bit i) */
        auto pack8 = [](uint32_t m0, uint32_t m1_) -> uint32_t {
            return (((m0 >> 7) | (m1_ >> 3)) * 0x01020408u) >> 24;
        };
        uint32_t ql = 0, qh = 0, cl = 0, ch = 0, kl = 0, kh = 0, anybs = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t x0 = x[2 * j], x1 = x[2 * j + 1];
            const uint32_t q8 = pack8(eq32(x0, 0x22222222u), eq32(x1, 0x22222222u));
            const uint32_t c8 = pack8(eq32(x0, 0x2C2C2C2Cu), eq32(x1, 0x2C2C2C2Cu));
            const uint32_t k8 = pack8(eq32(x0, 0x3A3A3A3Au), eq32(x1, 0x3A3A3A3Au));
            anybs |= eq32(x0, 0x5C5C5C5Cu) | eq32(x1, 0x5C5C5C5Cu);
            if (j < 4) {
                ql |= q8 << (8 * j);
                cl |= c8 << (8 * j);
                kl |= k8 << (8 * j);
            } else {
                qh |= q8 << (8 * (j - 4));
                ch |= c8 << (8 * (j - 4));
                kh |= k8 << (8 * (j - 4));
            }
        }
        uint64_t Q = ((uint64_t)qh << 32 | ql) & vmask, C = ((uint64_t)ch << 32 | cl) & vmask,
                 K = ((uint64_t)kh << 32 | kl) & vmask;
        const uint32_t nq = (uint32_t)__builtin_popcountll(Q);
        const uint32_t qx = g4_incl_sum(nq, g) - nq; /* quotes in the lanes before */
        /* in-string bytes: inclusive prefix XOR of the quotes (opening quote
         * inside, closing quote outside), carried across the group */
        uint64_t S = Q;
        S ^= S << 1;
        S ^= S << 2;
        S ^= S << 4;
        S ^= S << 8;
        S ^= S << 16;
        S ^= S << 32;
        if (qx & 1) S = ~S;
        C &= ~S;
        K &= ~S;
        const uint32_t nc = (uint32_t)__builtin_popcountll(C), nk = (uint32_t)__builtin_popcountll(K);
        const uint32_t pk = nc | (nk << 10) | (nq << 20);
        const uint32_t pin = g4_incl_sum(pk, g);
        const uint32_t ptot = g4_sum(pk);
        const uint32_t hasbs = g4_sum((anybs & 0x80808080u) && nv ? 1u : 0u);
        FLP(1);
        uint32_t bad = 0;
        if (hasbs) {
            /* a backslash before '"' or '\\' (an escaped quote or backslash) -> decline,
             * so every quote is a delimiter */
            uint32_t bl = 0, bh = 0;
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) {
                const uint32_t b8 = pack8(eq32(x[2 * j], 0x5C5C5C5Cu), eq32(x[2 * j + 1], 0x5C5C5C5Cu));
                if (j < 4) bl |= b8 << (8 * j);
                else bh |= b8 << (8 * (j - 4));
            }
            const uint64_t B = ((uint64_t)bh << 32 | bl) & vmask, QB = Q | B;
            const uint32_t nxt = g4_next((uint32_t)(QB & 1), g); /* the next lane's first byte */
            const uint64_t bb = B & ((QB >> 1) | ((uint64_t)nxt << 63));
            /* decode this lane's escapes into the message's table (an escape
             * may run into the next lane's bytes: read from the stage) */
            uint32_t ebad = 0;
            if (on && !bb && B) {
                LSrc es;
                es.init((const __attribute__((address_space(3))) uint64_t *)(void *)&L.in[lw], (int32_t)a7, (int32_t)n);
                for (uint64_t eb = B; eb; eb &= eb - 1) {
                    const uint32_t p = 64 * g + (uint32_t)__builtin_ctzll(eb);
                    const uint32_t x = fl_escape(p, es.get8((int32_t)p));
                    const uint32_t idx = atomicAdd(&L.nesc[m1], 1u);
                    if (!x || p + esc_in(x) > n) ebad = 1;
                    else if (idx < FL_NESC) L.esc[m1 * FL_NESC + idx] = x;
                    else ebad = 1;
                }
            }
            bad = g4_sum((bb ? 1u : 0u) | ebad);
        }
        if (on) {
            uint32_t ci = (pin & 0x3FF) - nc, ki = ((pin >> 10) & 0x3FF) - nk;
            const uint32_t pos0 = 64 * g;
            uint64_t c = C, k = K;
            while (c) {
                const uint32_t bit = (uint32_t)__builtin_ctzll(c);
                c &= c - 1;
                if (ci < FL_MAXF)
                    L.sep[ci * FL_MPB + m1] =
                        (pos0 + bit) | ((qx + (uint32_t)__builtin_popcountll(Q & ((1ull << bit) - 1))) << 16);
                ci++;
            }
            while (k) {
                const uint32_t bit = (uint32_t)__builtin_ctzll(k);
                k &= k - 1;
                if (ki < FL_MAXF) L.col[ki * FL_MPB + m1] = (uint16_t)(pos0 + bit);
                ki++;
            }
        }
        FLP(2);
        if (g == 0 && on) {
            LSrc src;
            src.init((const __attribute__((address_space(3))) uint64_t *)(void *)&L.in[lw], (int32_t)a7, (int32_t)n);
            const uint32_t open = skip_ws(src, 0);
            uint32_t close = n - 1;
            while (close > open && isspace_(src.raw((int32_t)close))) close--;
            const uint32_t nsep = ptot & 0x3FF, ncol = (ptot >> 10) & 0x3FF, qtot = ptot >> 20;
            bool ok = !bad && open < close && src.raw((int32_t)open) == '{' && src.raw((int32_t)close) == '}' &&
                      !(qtot & 1) && nsep + 1 < FL_MAXF;
            uint32_t nf = nsep + 1;
            if (ok && nsep == 0 && ncol == 0 && skip_ws(src, open + 1) == close) nf = 0; /* {} */
            ok = ok && ncol == nf;
            L.ok[m1] = ok ? 1u : 0u;
            L.oc[m1] = open | (close << 16);
            L.nfq[m1] = nf | (qtot << 8) | (hasbs ? 1u << 31 : 0u);
            if (ok) atomicMax(&L.rounds, (nf + FL_SLOTS - 1) / FL_SLOTS);
        }
    }
    __syncthreads();
    FLP(3);
#if defined(DG_FL_STOP) && DG_FL_STOP == 1
    return;
#endif

    /* ---- 2./3. fields, field-major: wave w converts field 4r + w of the
     *      block's messages (lane = message) and writes it
     *      straight into the slots, byte-exact at the shared edge words ---- */
    {
        const uint32_t mm = lane;
        /* the field slots wave w converts rotate with the block: the waves
         * of one SIMD (wave w of each resident block) then hold different
         * fields -- a double beside a byte -- instead of the same heavy or
         * light one in every block, so no SIMD carries all the heavy slots */
#ifndef DG_FL_ROT
#define DG_FL_ROT 1
#endif
        const uint32_t fwave = DG_FL_ROT ? (wave + blockIdx.x) % FL_WAVES : wave;
        const uint32_t ok0 = L.ok[mm], lwa = L.lw[mm], oc = L.oc[mm], nfq = L.nfq[mm];
        const uint32_t nf = nfq & 0xFF, qtot = (nfq >> 8) & 0x3FF;
        const bool hasbs = (nfq >> 31) != 0;
        const uint32_t cap = L.cap[mm];
        gu8 *const slot = (gu8 *)(void *)(L.a_out + L.oa[mm]);
        LSrc src;
        src.init((const __attribute__((address_space(3))) uint64_t *)(void *)&L.in[lwa >> 3], (int32_t)(lwa & 7), (int32_t)L.n[mm]);
        const uint32_t rounds = L.rounds;
        uint32_t nbytes = 0;
        lds_esc *E = (lds_esc *)(void *)&L.esc[mm * FL_NESC];
        const __attribute__((address_space(3))) uint64_t *KW = (const __attribute__((address_space(3))) uint64_t *)(void *)L.kw;
        const __attribute__((address_space(3))) uint32_t *KM = (const __attribute__((address_space(3))) uint32_t *)(void *)L.km;
        const uint32_t ne = min(L.nesc[mm], FL_NESC);
#ifdef DG_FLPROF_G
        uint64_t flg[8] = {0, 0, 0, 0, 0, 0, 0, __builtin_amdgcn_s_memtime()};
#endif
        auto parse = [&](uint32_t k, FField &F) {
            F.size = 0;
            F.kind = FV_NONE;
            if (ok0 && k < nf) {
                const uint32_t e0 = k ? L.sep[(k - 1) * FL_MPB + mm] : 0;
                const uint32_t sk = k ? (e0 & 0xFFFF) + 1 : (oc & 0xFFFF) + 1, q0 = e0 >> 16;
                uint32_t ek = oc >> 16, q1 = qtot;
                if (k + 1 < nf) {
                    const uint32_t e1 = L.sep[k * FL_MPB + mm];
                    ek = e1 & 0xFFFF;
                    q1 = e1 >> 16;
                }
                const uint32_t ck = L.col[k * FL_MPB + mm];
                FLG(0);
                if (!(ck >= sk && ck < ek && fl_field(D, sd, src, sk, ck, ek, q1 - q0, hasbs, E, ne, KW, KM, nk, k, P.flag, tb, F FLG_PASS))) {
                    L.ok[mm] = 0;
                    F.size = 0;
                    F.kind = FV_NONE;
                } else if (F.fi >= 0) {
                    const uint32_t bit = (uint32_t)F.fi - sd.field_begin;
                    atomicOr(&L.plo[mm], bit < 32 ? 1u << (bit & 31) : 0u);
                    atomicOr(&L.phi[mm], bit >= 32 ? 1u << (bit & 31) : 0u);
                }
                FLG(5);
            }
        };
        /* 0 = error, 1 = written, 2 = the body is left to chunk tasks */
        auto write = [&](const FField &F, uint32_t off) -> uint32_t {
            if (!F.size) return 1;
            if (off + F.size >= cap) return 0; /* the slot holds the field and STOP */
            WOut o;
            o.init(slot + off);
#ifdef DG_FL_ABL_NOSTORE
            o.dry = true; /* ablation (timing only): the field stores are not issued */
#endif
            const uint32_t wr = flat_write(src, F, tb, o, E, ne);
            o.finish();
            return wr;
        };
        /* ---- 2a. field remap: a wave converts the same FIELD of its 64
         *      messages, not the same position. With the keys in IDL order
         *      (C2) that is the same thing; with shuffled keys (c2s) a
         *      position holds a different field, type and code path in every
         *      lane, and the wave ran the union of all of them (VALU 4.8 K vs
         *      2.9 K per wave, r6c). A key pass finds each position's field
         *      (fmap[field][message] = position, in the task area, unused
         *      until the tasks); the block remaps only when every message
         *      fits one round and every key is a known field once. ---- */
        uint8_t *fmap = (uint8_t *)(void *)L.task;
        bool remap_try = DG_FL_REMAP && rounds == 1 && sd.n_fields <= FL_SLOTS && nk != 0;
        if (remap_try) {
            /* the order check: a key's length at every position equals the
             * predicted (IDL-order) field's. Keys in IDL order (C2) pass and
             * skip the key pass (a key pass on every block cost C2 4 %, r6f);
             * a false pass only keeps the positional assignment, which is
             * always correct */
            uint32_t mis = 0;
#pragma unroll
            for (uint32_t h = 0; h < FL_FPW; h++) {
                const uint32_t k = fl_slot(fwave, h);
                if (ok0 && k < nf) {
                    const uint32_t sk = k ? (L.sep[(k - 1) * FL_MPB + mm] & 0xFFFF) + 1 : (oc & 0xFFFF) + 1;
                    const uint32_t ck = L.col[k * FL_MPB + mm];
                    mis |= (k >= sd.n_fields || L.fkm[k] != ck - sk - 2) ? 1u : 0u;
                }
            }
            if (ballot(mis != 0) && lane == 0) atomicOr(&L.noremap, 2u);
            __syncthreads();
            remap_try = (L.noremap & 2u) != 0;
        }
        if (remap_try) {
            uint32_t fail = 0;
#pragma unroll
            for (uint32_t h = 0; h < FL_FPW; h++) {
                const uint32_t k = fl_slot(fwave, h);
                if (ok0 && k < nf) {
                    const uint32_t e0 = k ? L.sep[(k - 1) * FL_MPB + mm] : 0;
                    const uint32_t sk = k ? (e0 & 0xFFFF) + 1 : (oc & 0xFFFF) + 1, q0 = e0 >> 16;
                    uint32_t ek = oc >> 16, q1 = qtot;
                    if (k + 1 < nf) {
                        const uint32_t e1 = L.sep[k * FL_MPB + mm];
                        ek = e1 & 0xFFFF;
                        q1 = e1 >> 16;
                    }
                    const uint32_t ck = L.col[k * FL_MPB + mm];
                    FField G;
                    G.fi = -1;
                    if (!(ck >= sk && ck < ek &&
                          fl_field<true>(D, sd, src, sk, ck, ek, q1 - q0, hasbs, E, ne, KW, KM, nk, k, P.flag, tb, G FLG_PASS)) ||
                        G.fi < 0) {
                        fail = 1;
                    } else {
                        const uint32_t j = (uint32_t)G.fi - sd.field_begin;
                        if (atomicOr(&L.fseen[mm], 1u << j) & (1u << j)) fail = 1; /* a duplicate key */
                        else fmap[j * FL_MPB + mm] = (uint8_t)k;
                    }
                }
            }
            if (ballot(fail != 0) && lane == 0) atomicOr(&L.noremap, 1u);
            __syncthreads();
        }
        const bool remap = remap_try && (L.noremap & 1u) == 0; /* block-uniform */
        for (uint32_t r = 0; r < rounds; r++) {
            FField F[FL_FPW];
            uint32_t kslot[FL_FPW]; /* the position of F[h] in the message */
            uint16_t *sz = &L.size[(r & 1) * FL_SLOTS * FL_MPB];
#pragma unroll
            for (uint32_t h = 0; h < FL_FPW; h++) {
                FLF_T0();
                const uint32_t j = fl_slot(fwave, h);
                const uint32_t k = remap ? (uint32_t)fmap[j * FL_MPB + mm] : r * FL_SLOTS + j; /* 0xFF: no such field */
                const uint32_t si = remap ? k : j; /* its position within the round */
                kslot[h] = si;
                parse(k, F[h]);
                if (si < FL_SLOTS) sz[si * FL_MPB + mm] = (uint16_t)F[h].size;
                if (remap && j >= nf) sz[j * FL_MPB + mm] = 0; /* positions past the message's fields */
                FLF_ADD(r * FL_SLOTS + fl_slot(fwave, h));
            }
            FLP(4);
            __syncthreads();
            FLP(5);
#if defined(DG_FL_STOP) && DG_FL_STOP == 2
            continue;
#endif
            uint32_t off[FL_FPW], tot = 0;
#pragma unroll
            for (uint32_t h = 0; h < FL_FPW; h++) off[h] = nbytes;
#pragma unroll
            for (uint32_t f = 0; f < FL_SLOTS; f++) {
                const uint32_t v = sz[f * FL_MPB + mm];
#pragma unroll
                for (uint32_t h = 0; h < FL_FPW; h++) off[h] += f < kslot[h] ? v : 0u;
                tot += v;
            }
            nbytes += tot;
            /* bodies of more than FL_INLINE bytes (a string without escapes,
             * canonical base64) are left to chunk tasks of FL_CHUNK input
             * bytes: reserved before the writes (one LDS atomic per wave,
             * lane 63 reserves the wave's total), so that after the last
             * round's barrier every wave takes tasks as soon as its own
             * writes are done -- no barrier between the writes and the
             * tasks (a task owns its body bytes, the header's wave the rest) */
            uint32_t nch[FL_FPW], nsum = 0, good = 1;
#pragma unroll
            for (uint32_t h = 0; h < FL_FPW; h++) {
                const FField &G = F[h];
                const bool body = G.kind == FV_BIN || ((G.kind == FV_STR || G.kind == FV_NUMSTR) && !G.esc);
                nch[h] = body && G.nb > FL_INLINE && off[h] + G.size < cap ? (G.nb + FL_CHUNK - 1) / FL_CHUNK : 0u;
                nsum += nch[h];
            }
            {
                const uint32_t incl = wave_incl_sum(nsum, lane);
                const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                if (wtot) {
                    uint32_t tb0 = 0;
                    if (lane == 63) tb0 = atomicAdd(&L.ntask, wtot);
                    tb0 = (uint32_t)__builtin_amdgcn_readlane((int)tb0, 63);
                    uint32_t t0 = tb0 + incl - nsum;
                    if (nsum && t0 + nsum <= FL_MAXTASK) {
#pragma unroll
                        for (uint32_t h = 0; h < FL_FPW; h++) {
                            const bool b64 = F[h].kind == FV_BIN;
                            for (uint32_t c = 0; c < nch[h]; c++) {
                                const uint32_t cs = c * FL_CHUNK, cn = min(FL_CHUNK, F[h].nb - cs);
                                const uint32_t dst = off[h] + 7 + (b64 ? c * (FL_CHUNK / 4 * 3) : cs);
                                L.task[t0 + c] = (uint64_t)mm | ((uint64_t)b64 << 6) |
                                                 ((uint64_t)(c + 1 == nch[h]) << 7) | ((uint64_t)(F[h].s0 + cs) << 8) |
                                                 ((uint64_t)cn << 20) | ((uint64_t)dst << 32);
                            }
                            t0 += nch[h];
                        }
                    } else if (nsum) {
                        /* past the cap: the message declines, and its slots
                         * below the cap are marked empty (the task pass reads
                         * every slot up to min(ntask, cap)) */
                        good = 0;
                        for (uint32_t c = t0; c < t0 + nsum && c < FL_MAXTASK; c++) L.task[c] = ~0ull;
                    }
                }
            }
            if (r + 1 == rounds) __syncthreads(); /* the task list is complete */
#pragma unroll
            for (uint32_t h = 0; h < FL_FPW; h++) {
                FLF_T0();
                const uint32_t wr = write(F[h], off[h]);
                FLF_ADD(6 + r * FL_SLOTS + fl_slot(fwave, h));
                good &= wr != 0;
            }
            if (!good) L.ok[mm] = 0;
            FLP(6);
        }
        if (wave == 0) L.nbytes[mm] = nbytes;
#ifdef DG_FLPROF_G
        if (lane == 0 && (blockIdx.x & 31) == 0)
            for (int k_ = 0; k_ < 6; k_++) atomicAdd(&P.stats[2 + k_], (unsigned long long)flg[k_]);
#endif
    }
    FLP(6);
    /* ---- 3b. chunk tasks: long string / base64 bodies, taken 64 at a time
     *      by the waves as they finish their writes ---- */
    {
        const uint32_t nt = min(L.ntask, FL_MAXTASK);
        for (;;) {
            uint32_t t0 = 0;
            if (lane == 0) t0 = atomicAdd(&L.tgrab, 64u);
            t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)t0);
            if (t0 >= nt) break;
            const uint32_t t = t0 + lane;
            const uint64_t tk = t < nt ? L.task[t] : ~0ull;
            if (tk == ~0ull) continue; /* past the list, or a declined message's slot */
            const uint32_t m = (uint32_t)tk & 63, s0 = (uint32_t)(tk >> 8) & 0xFFF, cn = (uint32_t)(tk >> 20) & 0xFFF;
            const uint32_t lwa = L.lw[m];
            LSrc src;
            src.init((const __attribute__((address_space(3))) uint64_t *)(void *)&L.in[lwa >> 3], (int32_t)(lwa & 7), (int32_t)L.n[m]);
            WOut o;
            o.init((gu8 *)(void *)(L.a_out + L.oa[m] + (uint32_t)(tk >> 32)));
#ifdef DG_FL_ABL_NOSTORE
            o.dry = true;
#endif
            bool cok = true;
            if ((tk >> 6) & 1) cok = body_b64(src, s0, cn, ((tk >> 7) & 1) != 0, o);
            else body_copy(src, s0, cn, o);
            o.finish();
            if (!cok) L.ok[m] = 0;
        }
    }
    __syncthreads();
    FLP(7);

    /* ---- 4. per message (a lane): unset fields, then STOP and the result ---- */
    if (tid < FL_MPB) {
        const uint32_t m = tid;
        const uint64_t i = (uint64_t)blockIdx.x * FL_MPB + m;
        if (m < L.a_nb) {
            const uint32_t len = L.nbytes[m] + 1;
            const uint32_t wid = L.a_wrap ? L.wid[m] : 0u;
            bool good = L.ok[m] && len <= L.cap[m];
            if (good) {
                const uint64_t present = (uint64_t)L.plo[m] | ((uint64_t)L.phi[m] << 32);
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
            if (good && wid) {
                /* the outer field header, the inner STOP, the outer STOP */
                gu8 *o = (gu8 *)(void *)L.a_out + L.oa[m];
                o[-3] = DG_T_STRUCT;
                o[-2] = (uint8_t)(wid >> 8);
                o[-1] = (uint8_t)wid;
                o[len - 1] = 0;
                o[len] = 0;
                L.a_ret[i] = 0;
                L.a_out_len[i] = len + 4;
            } else if (good) {
                ((gu8 *)(void *)L.a_out)[L.oa[m] + len - 1] = 0; /* STOP */
                L.a_ret[i] = 0;
                L.a_out_len[i] = len;
            } else if (!L.big[m]) {
                const uint32_t qq = atomicAdd(L.a_bail_count, 1u);
                L.a_bail_list[qq] = (uint32_t)i;
            }
        }
    }
    FLP_END();
    FLF_END();
}

void launch_flat_kernel(dim3 grid, hipStream_t s, const Params &P, const FlatParams &S); /* LDS: + the blob */

}  // namespace dg
