/*
 * j2t_wave.h — the wave-per-message, token-parallel transcoder (gfx950).
 *
 * Why: one lane per message gives 65 536 lanes = one wave per SIMD for a 64K
 * batch (and 64 waves in total for 4K large messages), so the lane kernel is
 * latency-bound by construction. Here a whole wavefront converts ONE message,
 * and the work inside the message is spread over the 64 lanes:
 *
 *  1. Structural scan (simdjson's stage 1 mapped onto a wavefront): 64 lanes
 *     x 4 bytes are classified per step through a 256-entry class table in
 *     LDS; backslash escapes, the in-string mask and scalar runs are carried
 *     across lanes with ballots and popcounts. Tokens ({ } [ ] : , string,
 *     scalar) are compacted into a per-wave token ring in LDS (kind | pos),
 *     and the terminator of every string/scalar writes the token's end.
 *  2. Pages of 64 tokens, one token per lane:
 *     - depth by ballot prefix counts, parent = the last opener one level up
 *       (per-level ballots; parents from earlier pages come from a level
 *       stack), grammar checked against the neighbouring tokens;
 *     - Thrift types resolved level by level (keys are hashed and looked up
 *       in parallel), output length of every token (field headers, container
 *       headers, scalars, strings, unset fields + STOP at '}');
 *     - one wave prefix sum gives every token its output offset, and all
 *       tokens write their bytes at once (byte-exact stores); list/map sizes
 *       are LDS atomic counters written by the closing bracket.
 *
 * Scope: the error-free common grammar, exactly like the lane fast path
 * (j2t_fast.h). Anything else (every error, escaped keys, duplicate keys,
 * >64-field structs, nesting beyond WV_MAXD, big-decimal numbers, non-canonical
 * base64, flags outside FAST_FLAGS, non-container roots) BAILS: the message is
 * appended to a list that the lane kernel's exact machine (Machine<S>::run,
 * the restatement of j2t_fsm_exec native/thrift.c:765-1187) converts from
 * scratch. Results are therefore bit-identical to the reference either way;
 * the wave path decides speed, never output.
 *
 * Reference semantics reproduced (cited where used): container headers and
 * back-patched sizes native/thrift.c:132-162, 810-875, 1093-1133; null
 * handling native/thrift.c:942-947, 996-1032; unset fields
 * native/thrift.c:258-310 + 171-217; key lookup native/thrift.c:668-763;
 * numbers native/scanning.c:958-1083 + native/thrift.c:312-365; strings
 * native/thrift.c:367-399 + native/parsing.c:702-945; binary
 * native/thrift.c:401-420 + native/base64.c:539-817; skipping
 * native/scanning.c:1134-1572.
 */
#pragma once
#include "j2t_machine.h"

namespace dg {

/* Occupancy (measured, C3 65536 x 2.2 KB): 2 waves/SIMD (ring 512, 4 KiB
 * staging, 191 VGPRs) 4.18 ms; 3 waves (168 VGPRs) 3.34 ms; 4 waves (ring
 * 256, 2 KiB staging, 128 VGPRs + 24 spilled, 4 blocks/CU) 2.88 ms. The
 * kernel is latency-bound (dependent ballot/LDS chains), so waves per SIMD
 * beat per-wave efficiency.
 *
 * Two instances are built: this default (4 waves/SIMD, j2t_kern_wave.hip)
 * and a 5-waves/SIMD one (j2t_kern_wave5.hip: 96 VGPRs, 128 B staging, so
 * that 5 blocks fit the CU's LDS). With machine LICM off (build.py) the
 * 5-wave instance runs C3 in 2.14 ms against 2.30 ms, but a message longer
 * than WV_HUGE_MIN keeps one wave busy for about 1 ms, and sharing its SIMD
 * with a fifth wave lengthens that tail (C5 5.94 -> 6.14 ms). The host picks
 * the 5-wave instance when the caller's max_len rules huge messages out. */
#ifndef DG_WV_RING
#define DG_WV_RING 256
#endif
#ifndef DG_WV_MSG
#define DG_WV_MSG 2048
#endif
#ifndef DG_WV_BPC
#define DG_WV_BPC 4
#endif
#ifndef DG_WV_WPE
#define DG_WV_WPE 4
#endif
constexpr uint32_t WV_WAVES = 4;               /* waves (= messages in flight) per block */
constexpr uint32_t WV_RING = DG_WV_RING;       /* token ring per wave (a scan step that would overrun it bails) */
constexpr uint32_t WV_RMASK = WV_RING - 1;
constexpr uint32_t WV_CHUNK = 256;             /* bytes classified per scan step: 64 lanes x 4 */
constexpr uint32_t WV_MAXD = 16;               /* container levels handled on the wave path */
#ifndef DG_WV_FILL
#define DG_WV_FILL 120
#endif
constexpr uint32_t WV_FILL = DG_WV_FILL;       /* entries scanned ahead before a page is converted */
constexpr uint32_t WV_NOEND = 0xFFFFFFFFu;     /* string not closed (yet) */
constexpr uint32_t WV_POSMASK = (1u << 29) - 1;
constexpr uint32_t WV_MSG = DG_WV_MSG;         /* messages up to this (minus 16) are staged in LDS */
constexpr uint32_t WV_DESC = 16384;            /* the wave path needs the descriptor in LDS (dynamic, sized to it) */
constexpr uint32_t WV_BLOCKS_PER_CU = DG_WV_BPC; /* persistent grid: blocks of 4 waves per CU */
constexpr uint32_t WV5_BLOCKS_PER_CU = 5;      /* the 5-waves/SIMD instance (j2t_kern_wave5.hip) */
constexpr uint32_t WV_MIN_DEFAULT = 512;       /* messages longer than this go to the wave kernel (DG_WAVE_MIN) */
constexpr uint64_t WV_HUGE_MIN = 16384;        /* ... and longer than this are queued first */
constexpr uint32_t WV_REQMASKS = 64;           /* per-struct REQUIRED-field masks kept in LDS */

/* token kinds (3 bits, stored above the 29-bit position) */
enum : uint32_t {
    K_LBRACE = 0, K_RBRACE = 1, K_LBRACK = 2, K_RBRACK = 3, K_COLON = 4, K_COMMA = 5, K_STRING = 6, K_SCALAR = 7,
    K_NONE = 8
};
/* byte classes (LDS table); the low 3 bits give a structural byte's kind */
constexpr uint8_t C_STRUCT = 0x08, C_WS = 0x10, C_QUOTE = 0x20, C_BS = 0x40;

/* one open container (32 B): in-page openers at crec[lane], earlier pages'
 * openers at crec[64 + level] */
struct CRec {
    uint32_t type;   /* dg type index */
    uint32_t flags;  /* CF_* */
    uint32_t outpos; /* output offset of its header (relative to the slot) */
    uint32_t count;  /* list/map: elements written (LDS atomic) */
    uint64_t seen;   /* struct: fields that occurred (by index; LDS atomic) */
    uint64_t nulldr; /* struct: DEFAULT/REQUIRED fields that occurred as null */
};
constexpr uint32_t CF_SKIP = 1, CF_OBJ = 2, CF_STRUCT = 4, CF_MAP = 8, CF_LIST = 16;
constexpr uint32_t CF_ST_SHIFT = 8; /* struct: its dg_struct index above the CF_* bits (no dg_type read per round) */

struct WaveLds {
    uint32_t tpos[WV_RING]; /* kind << 29 | position */
    uint32_t tend[WV_RING]; /* string: closing quote position; scalar: one past its last byte */
    uint32_t tsep[WV_RING]; /* separators after the entry: colons (bits 0-7) + commas << 8 */
    uint8_t tbs[WV_RING];   /* string: a backslash inside (set by the scan) */
    uint8_t pg[64];         /* the page: lane -> entry offset from `consumed` */
    CRec crec[64 + WV_MAXD + 1];
    /* the page's string / base64 bodies as chunk tasks, per token lane */
    uint32_t cinc[64];      /* inclusive prefix of chunk counts */
    uint32_t cbs[64];       /* body source position */
    uint32_t cbd[64];       /* body output offset in the slot */
    uint32_t cbn[64];       /* body length | base64 << 31 */
};
#ifndef DG_WV_CH
#define DG_WV_CH 8
#endif
constexpr uint32_t WV_CH = DG_WV_CH; /* input bytes per string-copy chunk task (a multiple of 8) */
#ifndef DG_WV_CHB
#define DG_WV_CHB 16
#endif
constexpr uint32_t WV_CHB = DG_WV_CHB; /* base64 characters per chunk task of a body longer than WV_CHB_MIN (a multiple
                                        * of 8; r6i: C4's 48 KiB bodies 0.828 ms at 16 vs 0.863 at 8; C3's short ones
                                        * prefer 8: 1.313 vs 1.329 ms) */
constexpr uint32_t WV_CHB_MIN = 256;
DGI uint32_t wv_task_bytes(bool bin, uint32_t n) { return bin && n > WV_CHB_MIN ? WV_CHB : WV_CH; }

struct WaveParams {
    const uint8_t *blob; /* descriptor blob (device) */
    dg_desc_hdr hdr;
    uint32_t *bail_count; /* out: messages left to the exact machine */
    uint32_t *bail_list;
    const uint32_t *list; /* in: the messages to convert (the lane kernel's large ones) */
    const uint32_t *list_count;
    const uint32_t *huge_count; /* huge messages listed from the end of `list` (taken first) */
    uint64_t list_cap;          /* the list's length (the batch size) */
    uint8_t *ws;          /* DCAP bytes of big-decimal digits per wave of the grid */
    uint32_t *queue;      /* next list entry to take (zero at launch; reset by the list-mode lane kernel) */
};

#ifdef DG_WPROF
/* phase timers (cycles, summed over waves) -> P.stats[2 + k] */
#define WP_DECL uint64_t wp_t = __builtin_readcyclecounter(); uint64_t wp_acc[10] = {0};
#define WP(k) do { uint64_t t_ = __builtin_readcyclecounter(); wp_acc[k] += t_ - wp_t; wp_t = t_; } while (0)
#define WP_FLUSH() do { if (lane == 0) for (int k_ = 0; k_ < 10; k_++) atomicAdd(&P.stats[2 + k_], (unsigned long long)wp_acc[k_]); } while (0)
#else
#define WP_DECL
#define WP(k)
#define WP_FLUSH()
#endif

/* ---------------- wavefront helpers ---------------- */
DGI uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
DGI uint32_t popc(uint64_t x) { return (uint32_t)__builtin_popcountll(x); }
DGI uint32_t msb(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }
DGI uint32_t wave_or(uint32_t v)
{
#pragma unroll
    for (int d = 32; d; d >>= 1) v |= (uint32_t)__shfl_xor((int)v, d);
    return v;
}
/* inclusive prefix sum over the 64 lanes */
DGI uint32_t wave_incl_sum(uint32_t v, uint32_t lane)
{
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        uint32_t u = (uint32_t)__shfl_up((int)v, d);
        if (lane >= d) v += u;
    }
    return v;
}
template <class T>
DGI T uni(T v) /* wave-uniform value -> SGPR */
{
    return (T)__builtin_amdgcn_readfirstlane((int)v);
}

/* ---------------- byte-exact output ---------------- */
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint16_t gu16;

/* store bytes [lo, hi) of the little-endian word v at the 8-aligned w:
 * at most 6 naturally aligned stores, straight-line (no divergent loop).
 * AS: the address space written (1 = global, 3 = LDS) */
template <int AS>
DGI void store_part_as(__attribute__((address_space(AS))) uint8_t *w, uint64_t v, uint32_t lo, uint32_t hi)
{
    typedef __attribute__((address_space(AS))) uint16_t u16p;
    typedef __attribute__((address_space(AS))) uint32_t u32p;
    typedef __attribute__((address_space(AS))) uint64_t u64p;
    if (lo == 0 && hi == 8) {
        *(u64p *)w = v;
        return;
    }
    uint32_t i = lo;
    if ((i & 1) && i < hi) { w[i] = (uint8_t)(v >> (i * 8)); i += 1; }
    if ((i & 2) && i + 2 <= hi) { *(u16p *)(w + i) = (uint16_t)(v >> (i * 8)); i += 2; }
    if ((i & 4) && i + 4 <= hi) { *(u32p *)(w + i) = (uint32_t)(v >> (i * 8)); i += 4; }
    if (i + 4 <= hi) { *(u32p *)(w + i) = (uint32_t)(v >> (i * 8)); i += 4; }
    if (i + 2 <= hi) { *(u16p *)(w + i) = (uint16_t)(v >> (i * 8)); i += 2; }
    if (i < hi) w[i] = (uint8_t)(v >> (i * 8));
}
DGI void store_part(gu8 *w, uint64_t v, uint32_t lo, uint32_t hi) { store_part_as<1>(w, v, lo, hi); }

#ifndef DG_UNALIGNED_OUT
#define DG_UNALIGNED_OUT 1
#endif
#if DG_UNALIGNED_OUT
/* A writer that owns exactly [start, start + written): every 8 bytes as one
 * unaligned 8-byte store (the HSA code object runs the memory pipeline in
 * unaligned mode: a dwordx2 store at any byte address writes exactly those
 * 8 bytes), the last 1..7 as 4/2/1-byte stores. No aligned-word edge
 * bookkeeping, and neighbouring tokens written by other lanes or waves are
 * never touched, so they can write concurrently. AS: the address space. */
typedef uint64_t __attribute__((aligned(1))) u64_a1;
typedef uint32_t __attribute__((aligned(1))) u32_a1;
typedef uint16_t __attribute__((aligned(1))) u16_a1;
template <int AS>
DGI void store_tail_as(__attribute__((address_space(AS))) uint8_t *p, uint64_t v, uint32_t n) /* n < 8 bytes */
{
    if (n & 4) {
        *(__attribute__((address_space(AS))) u32_a1 *)p = (uint32_t)v;
        p += 4;
        v >>= 32;
    }
    if (n & 2) {
        *(__attribute__((address_space(AS))) u16_a1 *)p = (uint16_t)v;
        p += 2;
        v >>= 16;
    }
    if (n & 1) *p = (uint8_t)v;
}
template <int AS>
struct WOutT {
    typedef __attribute__((address_space(AS))) uint8_t b8;
    typedef __attribute__((address_space(AS))) u64_a1 b64u;
    b8 *p;         /* the next byte stored */
    uint32_t used; /* bytes held in wbuf */
    uint64_t wbuf;
    uint64_t len;  /* bytes written */
    bool dry;      /* count only (lengths before the offsets are known) */
    DGI void init(b8 *q)
    {
        p = q;
        used = 0;
        wbuf = 0;
        len = 0;
        dry = false;
    }
    DGI void init_dry()
    {
        p = nullptr;
        used = 0;
        wbuf = 0;
        len = 0;
        dry = true;
    }
    DGI void wle(uint64_t v, uint32_t n)
    {
        if (dry) {
            len += n;
            return;
        }
        if (n < 8) v &= (1ull << (n << 3)) - 1;
        const uint32_t sh = used << 3;
        const uint64_t lo_w = wbuf | (v << sh);
        const uint64_t hi_w = used ? (v >> (64 - sh)) : 0;
        len += n;
        if (used + n >= 8) {
            *(b64u *)p = lo_w;
            p += 8;
            wbuf = hi_w;
            used = used + n - 8;
        } else {
            wbuf = lo_w;
            used += n;
        }
    }
    DGI void w8(uint8_t v) { wle(v, 1); }
    DGI void w16(uint16_t v) { wle(__builtin_bswap16(v), 2); }
    DGI void w32(uint32_t v) { wle(__builtin_bswap32(v), 4); }
    DGI void w64(uint64_t v) { wle(__builtin_bswap64(v), 8); }
    DGI void finish()
    {
        if (!dry && used) store_tail_as<AS>(p, wbuf, used);
    }
};
#else
/* A writer that owns exactly [start, start + written): whole aligned words
 * inside the range are stored as 8-byte words, the partial words at both
 * ends byte-exactly, so neighbouring tokens can write concurrently. AS: the
 * address space written (WOut = global; the flat kernel also stages
 * messages in LDS). */
template <int AS>
struct WOutT {
    typedef __attribute__((address_space(AS))) uint8_t b8;
    typedef __attribute__((address_space(AS))) uint64_t b64;
    b8 *wa;        /* 8-aligned address of the current word */
    uint32_t lo;   /* first owned byte of the current word (first word only) */
    uint32_t used; /* bytes of the current word filled */
    uint64_t wbuf;
    uint64_t len;  /* bytes written */
    bool dry;      /* count only (lengths before the offsets are known) */
    DGI void init(b8 *p)
    {
        const uintptr_t a = (uintptr_t)p;
        wa = (b8 *)(a & ~(uintptr_t)7);
        lo = used = (uint32_t)(a & 7);
        wbuf = 0;
        len = 0;
        dry = false;
    }
    DGI void init_dry()
    {
        wa = nullptr;
        lo = used = 0;
        wbuf = 0;
        len = 0;
        dry = true;
    }
    DGI void wle(uint64_t v, uint32_t n)
    {
        if (dry) {
            len += n;
            return;
        }
        if (n < 8) v &= (1ull << (n << 3)) - 1;
        uint32_t sh = used << 3;
        uint64_t lo_w = wbuf | (used ? (v << sh) : v);
        uint64_t hi_w = used ? (v >> (64 - sh)) : 0;
        len += n;
        if (used + n >= 8) {
            if (lo == 0) *(b64 *)wa = lo_w;
            else store_part_as<AS>(wa, lo_w, lo, 8);
            wa += 8;
            lo = 0;
            wbuf = hi_w;
            used = used + n - 8;
        } else {
            wbuf = lo_w;
            used += n;
        }
    }
    DGI void w8(uint8_t v) { wle(v, 1); }
    DGI void w16(uint16_t v) { wle(__builtin_bswap16(v), 2); }
    DGI void w32(uint32_t v) { wle(__builtin_bswap32(v), 4); }
    DGI void w64(uint64_t v) { wle(__builtin_bswap64(v), 8); }
    DGI void finish()
    {
        if (!dry && used > lo) store_part_as<AS>(wa, wbuf, lo, used);
    }
};
#endif
typedef WOutT<1> WOut;

/* big-endian u32 at an arbitrary byte address, byte-exact */
DGI void put_be32(gu8 *p, uint32_t v)
{
    WOut w;
    w.init(p);
    w.w32(v);
    w.finish();
}

DGI uint32_t num_size(uint8_t tt)
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

/* decoded length of a standard-padded base64 body of nb chars (nb % 4 == 0),
 * or -1 for a shape the wave path leaves to the exact machine */
template <class S>
DGI int64_t b64_len(S &src, int64_t s0, int64_t nb)
{
    if (nb == 0) return 0;
    if (nb & 3) return -1;
    uint8_t c2 = src.raw(s0 + nb - 2), c3 = src.raw(s0 + nb - 1);
    int64_t pad = c3 == '=' ? (c2 == '=' ? 2 : 1) : 0;
    return nb / 4 * 3 - pad;
}


/* j2t_write_unset_fields (native/thrift.c:258-310) for one struct instance
 * whose remaining requires bits are `bits`: false = ERR_NULL_REQUIRED (bail) */
template <class DV, class O>
DGI bool unset_fields(const DV &D, const dg_struct &sd, uint64_t bits, uint64_t flag, O &out)
{
    bool wr = flag & DG_F_WRITE_REQUIRE, wd = flag & DG_F_WRITE_DEFAULT, wo = flag & DG_F_WRITE_OPTIONAL;
    while (bits) {
        uint32_t k = __builtin_ctzll(bits);
        bits &= bits - 1;
        const dg_field f = ldrec(&D.F[sd.field_begin + k]);
        if (f.flags & DG_FF_REQUEST_BASE) continue;
        if (!wr && f.required == DG_REQ_REQUIRED) return false;
        if ((wr && f.required == DG_REQ_REQUIRED) || (wd && f.required == DG_REQ_DEFAULT) ||
            (wo && f.required == DG_REQ_OPTIONAL)) {
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
    return true;
}

/* field lookup j2t_key (native/thrift.c:668-763) by the struct's name table:
 * global field index or -1 */
template <class S, class DV>
DGI int32_t wv_lookup(const DV &D, const dg_struct &sd, S &src, int64_t k0, uint32_t kn, uint32_t h)
{
    for (uint32_t s = h & sd.name_mask;; s = (s + 1) & sd.name_mask) {
        const dg_name nm = ldrec(&D.N[sd.name_begin + s]);
        if (nm.field == DG_NONE) return -1;
        if (nm.hash == h && nm.key_len == kn && key_eq(src, k0, kn, (decltype(&D.R[0]))(&D.P[nm.key_off])))
            return (int32_t)nm.field;
    }
}

/* src[s0, s0+nb) -> dst, by the 64 lanes of the wave: lane l stores the
 * destination bytes [8l, 8l+8), [8l+512, ...) (unaligned 8-byte stores, the
 * last partial one byte-exactly) */
template <class S>
DGI void coop_copy(S &src, int64_t s0, int64_t nb, gu8 *dst, uint32_t lane)
{
#if DG_UNALIGNED_OUT
    const int64_t nw = (nb + 7) >> 3;
    for (int64_t k = lane; k < nw; k += 64) {
        const int64_t off = k * 8, rem = nb - off;
        const uint64_t v = src.get8(s0 + off);
        gu8 *w = dst + off;
        if (rem >= 8) *(__attribute__((address_space(1))) u64_a1 *)w = v;
        else store_tail_as<1>(w, v, (uint32_t)rem);
    }
#else
    const uintptr_t da = (uintptr_t)(void *)dst, wb = da & ~(uintptr_t)7;
    const uint32_t lead = (uint32_t)(da - wb);
    const int64_t nw = (int64_t)(lead + nb + 7) >> 3;
    for (int64_t k = lane; k < nw; k += 64) {
        int64_t off = k * 8 - (int64_t)lead; /* string offset of the word's first byte */
        uint32_t lo = off < 0 ? (uint32_t)-off : 0u;
        int64_t rem = nb - off;
        uint32_t hi = rem < 8 ? (uint32_t)rem : 8u;
        uint64_t v = off < 0 ? src.get8(s0) << (lo * 8) : src.get8(s0 + off);
        gu8 *w = (gu8 *)(void *)(wb + (uintptr_t)k * 8);
        if (lo == 0 && hi == 8) *(gu64 *)w = v;
        else store_part(w, v, lo, hi);
    }
#endif
}


/* a chunk of a canonical padded base64 body: src[s0, s0+n) (n % 4 == 0);
 * `last`: the chunk holds the final quantum, "xx==" / "xxx=" keeping 1 / 2
 * bytes like decode_block (native/base64.c:600-631). false = a character
 * outside the alphabet or '=' anywhere else: the exact machine reports it. */
template <class S, class O>
DGI bool chunk_b64(S &src, int64_t s0, int64_t n, bool last, O &o)
{
    int64_t ip = 0;
    const int64_t full = last && n >= 4 ? n - 4 : n;
    for (; ip + 8 <= full; ip += 8) {
        uint64_t v;
        if (!b64_8(src.get8(s0 + ip), v)) return false;
        o.wle(v, 6);
    }
    for (; ip < full; ip += 4) {
        uint32_t v;
        if (!b64_4((uint32_t)src.get8(s0 + ip), v)) return false;
        o.wle(v, 3);
    }
    if (last && n >= 4) {
        uint32_t w = (uint32_t)src.get8(s0 + ip);
        const uint32_t c2 = (w >> 16) & 0xFF, c3 = w >> 24;
        if (c2 == '=' && c3 != '=') return false;
        const uint32_t keep = c3 == '=' ? (c2 == '=' ? 1u : 2u) : 3u;
        if (c3 == '=') w = (w & 0x00FFFFFFu) | ((uint32_t)'A' << 24);
        if (c2 == '=') w = (w & 0xFF00FFFFu) | ((uint32_t)'A' << 16);
        uint32_t v;
        if (!b64_4(w, v)) return false;
        o.wle(v, keep);
    }
    return true;
}

/* A number token's bytes held in registers: the 5 aligned words covering
 * [p, p + 32) of the message, loaded together (one wait) instead of the
 * dependent word-at-a-time loads of the parse loops. Tokens up to RS_MAX
 * bytes use it; longer ones take the exact parser. */
constexpr int64_t RS_MAX = 24;
struct RSrc {
    typedef int64_t idx;
    static constexpr bool kRegs = true; /* fast_vnumber: the fixed-step integer path */
    uint64_t w0, w1, w2, w3, w4;
    uint32_t sh; /* byte offset of the token's first byte in w0 */
    int64_t n;
    template <class S>
    DGI void load(const S &src, int64_t p, int64_t len)
    {
        const int64_t b = src.off0 + p;
        const uint64_t *q = src.w8 + (b >> 3);
        sh = (uint32_t)(b & 7);
        n = len;
        const uint32_t need = (sh + (uint32_t)len + 8 + 7) >> 3; /* words up to get8(n) */
        w0 = q[0];
        w1 = need > 1 ? q[1] : 0;
        w2 = need > 2 ? q[2] : 0;
        w3 = need > 3 ? q[3] : 0;
        w4 = need > 4 ? q[4] : 0;
    }
    DGI uint64_t word(uint32_t j) const { return j == 0 ? w0 : j == 1 ? w1 : j == 2 ? w2 : j == 3 ? w3 : w4; }
    DGI uint8_t raw(int64_t i) const
    {
        const uint32_t b = sh + (uint32_t)i;
        return (uint8_t)(word(b >> 3) >> ((b & 7) << 3));
    }
    DGI uint8_t at(int64_t i) const { return (uint64_t)i < (uint64_t)n ? raw(i) : 0; }
    DGI uint64_t get8(int64_t i) const
    {
        const uint32_t b = sh + (uint32_t)i, j = b >> 3, s8 = (b & 7) << 3;
        return (word(j) >> s8) | ((word(j + 1) << 1) << (63 - s8));
    }
};

/* the exact number parser, out of line (rare: keeps the kernel small) */
__device__ __noinline__ void vnumber_slow(SrcT<const uint64_t> src, int64_t &p, JState &js, gu8 *dbuf)
{
    vnumber(src, p, js, dbuf);
}

/* ---------------- stage 1: structural scan of one chunk ---------------- */
struct ScanState {
    uint32_t produced;   /* entries appended to the ring so far */
    uint32_t esc_carry;  /* an escape is pending at the chunk boundary */
    uint32_t str_carry;  /* inside a string at the chunk boundary */
    uint32_t scal_carry; /* the chunk's last byte was a scalar byte */
    uint32_t bad;        /* a separator before the first entry */
};

/* this lane's 4 bytes of chunk `chunk` (spaces past the end) */
template <class WP>
DGI uint32_t chunk_word(WP wbase, int64_t head, int64_t len, uint32_t chunk, uint32_t lane)
{
    int64_t wi = (int64_t)chunk * 64 + lane;
    return wi * 4 - head < len ? wbase[wi] : 0x20202020u;
}

/* One 256-byte chunk. Entries are the brackets, strings and scalars; the
 * separators ':' and ',' are NOT entries: each one adds to the separator
 * word of the entry before it (colon +1, comma +256), so that a string
 * followed by a colon is a key and grammar is checked on entry pairs.
 * Returns false, with no side effect, when the chunk's entries would not fit
 * the ring's free space `room` (the caller converts a page first). */
template <class LW>
DGI bool scan_chunk(uint32_t x, int64_t head, int64_t len, uint32_t chunk, ScanState &st, LW &L,
                    const __attribute__((address_space(3))) uint8_t *cls, uint32_t lane, uint64_t lt, uint32_t room)
{
    int64_t wi = (int64_t)chunk * 64 + lane;
    int64_t p0 = wi * 4 - head; /* message position of this lane's byte 0 */
    /* string interior without a quote or backslash anywhere in the chunk
     * (long strings, base64 blobs): no entries, carries unchanged */
    if (st.str_carry) {
        const uint32_t M = 0x7F7F7F7Fu;
        uint32_t vq = x ^ 0x22222222u, vb = x ^ 0x5C5C5C5Cu;
        uint32_t z = ~(((vq & M) + M) | vq | M) | ~(((vb & M) + M) | vb | M);
        if (!ballot(z != 0)) {
            st.esc_carry = 0;
            return true;
        }
    }
    uint32_t q = 0, bs = 0, sm = 0, ws = 0, knib = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        int64_t p = p0 + j;
        uint8_t c = cls[(x >> (8 * j)) & 0xff];
        if (p < 0 || p >= len) c = C_WS;
        q |= (uint32_t)((c >> 5) & 1) << j;
        bs |= (uint32_t)((c >> 6) & 1) << j;
        sm |= (uint32_t)((c >> 3) & 1) << j;
        ws |= (uint32_t)((c >> 4) & 1) << j;
        knib |= (uint32_t)(c & 7) << (3 * j);
    }
    /* escapes: byte j is escaped when an odd backslash run precedes it. The
     * carry into a lane comes from the nearest lane below that is not all
     * backslashes (a 4-backslash lane passes its carry through unchanged). */
    uint32_t e0 = 0, e1 = 1, m0 = 0, m1 = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        uint32_t b = (bs >> j) & 1;
        if (e0) { m0 |= 1u << j; e0 = 0; } else e0 = b;
        if (e1) { m1 |= 1u << j; e1 = 0; } else e1 = b;
    }
    uint64_t nab = ballot(bs != 0xF);
    uint64_t c0b = ballot(e0 != 0);
    uint64_t below = nab & lt;
    uint32_t cin = below ? (uint32_t)(c0b >> msb(below)) & 1 : st.esc_carry;
    uint32_t escaped = cin ? m1 : m0;
    uint32_t cout = cin ? e1 : e0;
    /* in-string mask: prefix xor of unescaped quotes, carried by popcounts */
    uint32_t uq = q & ~escaped;
    uint32_t px = (uq ^ (uq << 1) ^ (uq << 2) ^ (uq << 3)) & 0xF;
    uint64_t pb = ballot(__builtin_popcount(uq) & 1);
    uint32_t sin = (popc(pb & lt) + st.str_carry) & 1;
    uint32_t instr = sin ? (px ^ 0xF) : px; /* bit j: inside a string after byte j */
    uint32_t openq = uq & instr, closeq = uq & ~instr & 0xF;
    uint32_t outside = ~(instr | uq) & 0xF;
    uint32_t stm = sm & outside;
    /* separators: ':' (kind 4) and ',' (kind 5) */
    uint32_t sepc = 0, sepm = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t k = (knib >> (3 * j)) & 7;
        if (k == K_COLON) sepc |= 1u << j;
        if (k == K_COMMA) sepm |= 1u << j;
    }
    sepc &= stm;
    sepm &= stm;
    const uint32_t seps = sepc | sepm;
    uint32_t scal = outside & ~ws & ~sm;
    uint64_t sb3 = ballot(scal & 8);
    uint32_t prevs = lane ? (uint32_t)(sb3 >> (lane - 1)) & 1 : st.scal_carry;
    uint32_t sprev = ((scal << 1) | prevs) & 0xF;
    uint32_t sstart = scal & ~sprev;
    uint32_t send = ~scal & sprev & 0xF;
    uint32_t tok = (stm & ~seps) | openq | sstart;
    uint32_t term = closeq | send;
    uint32_t cnt = (uint32_t)__builtin_popcount(tok);
    uint64_t b0 = ballot(cnt & 1), b1 = ballot(cnt & 2), b2 = ballot(cnt & 4);
    uint32_t total = popc(b0) + 2 * popc(b1) + 4 * popc(b2);
    if (total > room) return false; /* nothing written: the ring first drains a page */
    uint32_t pre = popc(b0 & lt) + 2 * popc(b1 & lt) + 4 * popc(b2 & lt);
    uint32_t k = st.produced + pre;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        if ((tok >> j) & 1) {
            uint32_t kind = ((stm >> j) & 1) ? (knib >> (3 * j)) & 7 : ((openq >> j) & 1) ? K_STRING : K_SCALAR;
            L.tpos[k & WV_RMASK] = (kind << 29) | (uint32_t)(p0 + j);
            L.tend[k & WV_RMASK] = WV_NOEND;
            L.tsep[k & WV_RMASK] = 0;
            L.tbs[k & WV_RMASK] = 0;
            k++;
        }
    }
    /* backslashes inside a string mark the open string: the last entry
     * started before them (after every entry write of the chunk; a wave's
     * LDS operations complete in order). An escape's backslash (one not
     * itself escaped) also counts what the escape takes off the string's
     * unquoted length in bits 16+ of the string's separator word: 1 for
     * \" \\ \/ \b \f \n \r \t; anything else (\u, an invalid escape, an
     * escape whose letter is in the next chunk) sets bit 31 and the page
     * sizes that string with unquote (native/parsing.c:702-945) */
    const uint32_t bsi = bs & instr;
    const uint32_t xn = (uint32_t)__shfl_down((int)x, 1); /* the next lane's bytes (converged) */
    if (bsi) {
        const uint32_t ei = bsi & ~escaped;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            if ((bsi >> j) & 1) {
                uint32_t kb = st.produced + pre + (uint32_t)__builtin_popcount(tok & ((1u << j) - 1));
                L.tbs[(kb - 1) & WV_RMASK] = 1;
                if ((ei >> j) & 1) {
                    const uint32_t c = j < 3 ? (x >> (8 * (j + 1))) & 0xFF : lane < 63 ? xn & 0xFF : 0u;
                    const bool simple = c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' ||
                                        c == 'r' || c == 't';
                    if (simple) atomicAdd(&L.tsep[(kb - 1) & WV_RMASK], 1u << 16);
                    else atomicOr(&L.tsep[(kb - 1) & WV_RMASK], 1u << 31);
                }
            }
        }
    }
    /* terminators and separators: the entry a terminator ends, or a
     * separator follows, is the last entry strictly before it */
    bool badsep = false;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t kb = st.produced + pre + (uint32_t)__builtin_popcount(tok & ((1u << j) - 1));
        if ((term >> j) & 1) L.tend[(kb - 1) & WV_RMASK] = (uint32_t)(p0 + j);
        if ((seps >> j) & 1) {
            if (kb == 0) badsep = true;
            /* a second separator after one entry is always a grammar error
             * (the exact machine reports it): every separator word then holds
             * at most one colon or comma, and no count carries into the next
             * field (256 colons read as one comma, 256 commas as escapes) */
            else if (atomicAdd(&L.tsep[(kb - 1) & WV_RMASK], ((sepc >> j) & 1) ? 1u : 256u) & 0xFFFFu) badsep = true;
        }
    }
    if (ballot(badsep)) st.bad = 1;
    st.produced += total;
    st.esc_carry = (uint32_t)__builtin_amdgcn_readlane((int)cout, 63);
    st.str_carry = (st.str_carry + popc(pb)) & 1;
    st.scal_carry = (uint32_t)(sb3 >> 63) & 1;
    return true;
}

/* the Thrift bytes of a parsed number (j2t_number's writes,
 * native/thrift.c:312-365) as a little-endian word of n bytes, for WOut::wle */
DGI void num_le(uint8_t tt, bool isint, int64_t iv, double dv, uint64_t &v, uint32_t &n)
{
    switch (tt) {
    case DG_T_BYTE: v = isint ? (uint8_t)iv : (uint8_t)cvt32(dv); n = 1; return;
    case DG_T_I16: v = __builtin_bswap16(isint ? (uint16_t)iv : (uint16_t)cvt32(dv)); n = 2; return;
    case DG_T_I32: v = __builtin_bswap32(isint ? (uint32_t)iv : (uint32_t)cvt32(dv)); n = 4; return;
    case DG_T_I64: v = __builtin_bswap64(isint ? (uint64_t)iv : (uint64_t)cvt64(dv)); n = 8; return;
    case DG_T_DOUBLE: v = __builtin_bswap64((uint64_t)__double_as_longlong(dv)); n = 8; return;
    }
    v = 0;
    n = 0;
}

/* ---------------- one message ---------------- */
typedef const __attribute__((address_space(3))) uint32_t lds_u32;

template <class S, class WP, class DV, class LW>
DGI bool wave_run(const Params &P, const DV &D, uint32_t D_nf, uint64_t m, LW &L, S src, WP wbase, int64_t head,
                  int64_t len, const __attribute__((address_space(3))) uint8_t *cls, const FastTabs &tb, uint32_t lane,
                  gu8 *dbuf, const __attribute__((address_space(3))) uint64_t *reqmask)
{
    const uint64_t flag = P.flag;
    uint64_t oa = P.out_off[m];
    uint64_t cap = P.out_off[m + 1] - oa;
    gu8 *ob = (gu8 *)(void *)(P.out + oa);
    uint32_t nchunks = (uint32_t)((len + head + WV_CHUNK - 1) / WV_CHUNK);
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t le = lt | (1ull << lane);

    WP_DECL
    ScanState ss{0, 0, 0, 0, 0};
    uint32_t scanned = 0, consumed = 0;
    int32_t depth = 0;
    uint64_t O = 0;
    bool rootdone = false;

    uint32_t xcur = chunk_word(wbase, head, len, 0, lane);
    for (;;) {
        /* scan ahead until WV_FILL entries wait (or the message is scanned):
         * the live window is [consumed - 2, produced) */
        while (scanned < nchunks && ss.produced - consumed < WV_FILL) {
            const uint32_t xnext = scanned + 1 < nchunks ? chunk_word(wbase, head, len, scanned + 1, lane) : 0u;
            if (!scan_chunk(xcur, head, len, scanned, ss, L, cls, lane, lt, WV_RING - 2 - (ss.produced - consumed)))
                break;
            scanned++;
            xcur = xnext;
            if (scanned == nchunks && ss.scal_carry) {
                if (lane == 0) L.tend[(ss.produced - 1) & WV_RMASK] = (uint32_t)len;
            }
        }
        if (ss.bad) return false;
        WP(0);
        /* entries whose separators and ends are final: all but the last one
         * while the scan goes on */
        const uint32_t lim = ss.produced - (scanned < nchunks ? 1u : 0u);
        if (lim <= consumed) {
            if (scanned < nchunks) return false; /* a chunk denser than the ring (pathological): exact machine */
            break;
        }
        /* ---------- a page: up to 64 VALUE entries (values and closing
         * brackets), one per lane; the key before a value (a string followed
         * by a colon) rides in the value's lane ---------- */
        uint32_t np, off;
        {
            const uint32_t win = lim - consumed < 128u ? lim - consumed : 128u;
            bool vA = false, vB = false;
            if (lane < win) {
                const uint32_t e = (consumed + lane) & WV_RMASK;
                vA = !((L.tpos[e] >> 29) == K_STRING && (L.tsep[e] & 0xFFu));
            }
            if (lane + 64 < win) {
                const uint32_t e = (consumed + 64 + lane) & WV_RMASK;
                vB = !((L.tpos[e] >> 29) == K_STRING && (L.tsep[e] & 0xFFu));
            }
            const uint64_t bA = ballot(vA), bB = ballot(vB);
            const uint32_t nA = popc(bA), ntot = nA + popc(bB);
            np = ntot < 64 ? ntot : 64u;
            if (np == 0) return false; /* only keys left: truncated input */
            if (vA) L.pg[popc(bA & lt)] = (uint8_t)lane;
            const uint32_t iB = nA + popc(bB & lt);
            if (vB && iB < 64) L.pg[iB] = (uint8_t)(64 + lane);
            __builtin_amdgcn_wave_barrier();
            off = lane < np ? (uint32_t)L.pg[lane] : 0u;
        }
        const uint32_t lastoff = (uint32_t)__builtin_amdgcn_readlane((int)off, (int)(np - 1));
        const uint32_t t = consumed + off;
        const bool act = lane < np;
        const uint32_t tp = act ? L.tpos[t & WV_RMASK] : 0;
        const uint32_t kind = act ? tp >> 29 : K_NONE;
        const int32_t pos = (int32_t)(tp & WV_POSMASK);
        const bool op = kind == K_LBRACE || kind == K_LBRACK;
        const bool cl = kind == K_RBRACE || kind == K_RBRACK;
        const uint64_t bo = ballot(op), bc = ballot(cl);
        const int32_t dafter = depth + (int32_t)popc(bo & le) - (int32_t)popc(bc & le);
        const uint64_t bend = ballot(cl && dafter == 0);
        const bool alive = act && (bend == 0 || lane <= (uint32_t)__builtin_ctzll(bend));
        const int32_t level = op ? dafter - 1 : dafter;
        const int32_t plev = cl ? level : level - 1; /* level of the parent opener */
        bool bad = alive && level >= (int32_t)WV_MAXD;
        if (consumed == 0 && lane == 0 && (t != 0 || !op)) bad = true; /* the root: entry 0, an object or array */
        if (ballot(bad)) return false;

        WP(1);
        /* parent: the last opener at level plev before t (in this page), else
         * the level stack */
        int32_t par = -1;
        {
            uint32_t need = wave_or(alive && plev >= 0 ? 1u << plev : 0u);
            uint32_t have = wave_or(alive && op ? 1u << level : 0u);
            for (uint32_t lm = uni(need & have); lm; lm &= lm - 1) {
                int32_t Lv = __builtin_ctz(lm);
                uint64_t mo = ballot(alive && op && level == Lv) & lt;
                if (plev == Lv && mo) par = (int32_t)msb(mo);
            }
        }
        const uint32_t ci = par >= 0 ? (uint32_t)par : 64u + (uint32_t)(plev < 0 ? 0 : plev);
        const uint32_t pkind = (uint32_t)__shfl((int)kind, par >= 0 ? par : 0);
        bool pobj = false;
        if (alive && plev >= 0) pobj = par >= 0 ? pkind == K_LBRACE : (L.crec[ci].flags & CF_OBJ) != 0;

        /* my key (the entry before me, when it is a string followed by a
         * colon) and the entry before me-or-my-key: grammar on entry pairs
         * and the separator counts between them */
        bool haskey = false, kesc = false;
        int32_t kpos = 0;
        uint32_t kend = 0, ksep = 0, kq = K_NONE, sq = 0;
        bool qkey = false;
        if (alive && t >= 1) {
            const uint32_t a = L.tpos[(t - 1) & WV_RMASK], sa = L.tsep[(t - 1) & WV_RMASK] & 0xFFFFu;
            if ((a >> 29) == K_STRING && (sa & 0xFFu)) {
                haskey = true;
                ksep = sa;
                kpos = (int32_t)(a & WV_POSMASK);
                kend = L.tend[(t - 1) & WV_RMASK];
                kesc = L.tbs[(t - 1) & WV_RMASK] != 0;
                if (t >= 2) {
                    const uint32_t b = L.tpos[(t - 2) & WV_RMASK];
                    kq = b >> 29;
                    sq = L.tsep[(t - 2) & WV_RMASK] & 0xFFFFu;
                    qkey = kq == K_STRING && (sq & 0xFFu);
                }
            } else {
                kq = a >> 29;
                sq = sa;
            }
        }
        const bool isval = kind == K_STRING || kind == K_SCALAR || op;
        const uint32_t te = (alive && (kind == K_STRING || kind == K_SCALAR)) ? L.tend[t & WV_RMASK] : 0;
        if (alive && t != 0) {
            const bool qvend = kq == K_SCALAR || kq == K_RBRACE || kq == K_RBRACK || (kq == K_STRING && !qkey);
            bool ok;
            if (isval) {
                if (pobj) ok = haskey && ksep == 1u && ((kq == K_LBRACE && sq == 0) || (qvend && sq == 256u));
                else ok = !haskey && ((kq == K_LBRACK && sq == 0) || (qvend && sq == 256u));
            } else if (kind == K_RBRACE) {
                ok = pobj && !haskey && ((kq == K_LBRACE && sq == 0) || (qvend && sq == 0));
            } else { /* K_RBRACK */
                ok = !pobj && !haskey && ((kq == K_LBRACK && sq == 0) || (qvend && sq == 0));
            }
            bad |= !ok;
        }
        if (alive && kind == K_STRING && te == WV_NOEND) bad = true; /* EOF inside a string */
        if (alive && haskey && kend == WV_NOEND) bad = true;
        if (ballot(bad)) return false;

        WP(2);
        /* key hashes, once (the level rounds below only probe) */
        uint32_t khash = DG_NAME_HASH_SEED;
        if (alive && haskey) {
            const int64_t k0 = kpos + 1, kl = (int64_t)kend - k0;
            for (int64_t j = 0; j < kl; j += 8) {
                uint64_t w = src.get8(k0 + j);
                const int64_t r = kl - j < 8 ? kl - j : 8;
#pragma unroll
                for (int b = 0; b < 8; b++)
                    if (b < r) khash = DG_NAME_HASH_STEP(khash, (uint8_t)(w >> (8 * b)));
            }
        }
        /* types, level by level (a value needs its container's type; an
         * opener's record feeds the next level) */
        uint32_t ty = DG_NONE; /* value type index */
        uint32_t fi = DG_NONE; /* struct parent: the key's field (global index) */
        uint32_t fbit = 0;     /* ... and its index within the struct */
        uint32_t pflags = 0, ptype = 0;
        bool skip = false;
        {
            uint32_t lv = wave_or(alive ? 1u << level : 0u);
            for (lv = uni(lv); lv; lv &= lv - 1) {
                const int32_t Lv = __builtin_ctz(lv);
                const bool me = alive && level == Lv;
                if (me && t != 0 && !cl) { /* a closer's opener may be written in this very round: below */
                    pflags = L.crec[ci].flags;
                    ptype = L.crec[ci].type;
                }
                if (me && isval) {
                    if (t == 0) {
                        ty = P.root;
                    } else if (pflags & CF_SKIP) {
                        skip = true;
                    } else if (pflags & CF_STRUCT) { /* j2t_key native/thrift.c:668-763 */
                        const dg_struct sd = ldrec(&D.S[pflags >> CF_ST_SHIFT]);
                        const int32_t f = kesc ? -2 : wv_lookup(D, sd, src, kpos + 1, kend - (uint32_t)kpos - 1, khash);
                        if (f == -2) {
                            bad = true; /* escaped key: exact machine */
                        } else if (f < 0) {
                            if ((flag & DG_F_ALLOW_UNKNOWN) == 0) bad = true;
                            skip = true;
                        } else {
                            const dg_field fd = ldrec(&D.F[f]);
                            if ((flag & DG_F_ENABLE_VM) && fd.vm != DG_VM_NONE) bad = true;
                            if ((fd.flags & DG_FF_REQUEST_BASE) && (flag & DG_F_NO_WRITE_BASE)) {
                                skip = true;
                            } else {
                                fi = (uint32_t)f;
                                fbit = (uint32_t)f - sd.field_begin;
                                ty = fd.type;
                            }
                        }
                    } else {
                        ty = ldrec(&D.T[ptype]).elem; /* list element, map value */
                    }
                    if (op) {
                        CRec c;
                        c.type = ty;
                        c.flags = (kind == K_LBRACE ? CF_OBJ : 0u) | (skip ? CF_SKIP : 0u);
                        c.outpos = 0;
                        c.count = 0;
                        c.seen = 0;
                        c.nulldr = 0;
                        if (!skip) {
                            const dg_type ct = ldrec(&D.T[ty]);
                            if (kind == K_LBRACE) {
                                if (ct.ttype == DG_T_STRUCT) {
                                    c.flags |= CF_STRUCT | (ct.st << CF_ST_SHIFT);
                                    /* bit 0: more than 64 fields, bit 1: HTTP-mapped fields
                                     * (the block's struct table; the record past it) */
                                    uint32_t sf;
                                    if (ct.st < WV_REQMASKS) {
                                        sf = ((const __attribute__((address_space(3))) uint8_t *)(reqmask + WV_REQMASKS))[ct.st];
                                    } else {
                                        const dg_struct csd = ldrec(&D.S[ct.st]);
                                        sf = (csd.req_words != 1 ? 1u : 0u) | ((csd.flags & DG_SF_HTTP_MAPPING) ? 2u : 0u);
                                    }
                                    if (sf & 1u) bad = true;
                                    if ((flag & DG_F_ENABLE_HM) && (sf & 2u)) bad = true;
                                } else if (ct.ttype == DG_T_MAP) {
                                    c.flags |= CF_MAP;
                                } else {
                                    bad = true;
                                }
                            } else {
                                if (ct.ttype == DG_T_LIST || ct.ttype == DG_T_SET) c.flags |= CF_LIST;
                                else bad = true;
                            }
                        }
                        L.crec[lane] = c;
                    }
                }
                /* a mistyped container must not feed the next level */
                if (ballot(bad)) return false;
            }
        }

        if (alive && cl) {
            pflags = L.crec[ci].flags;
            ptype = L.crec[ci].type;
        }
        WP(3);
        /* lengths, part A: the key part (field header, or map key) and the
         * value part, with the LDS atomics that count elements and record
         * struct fields. Every heavy helper has ONE call site below (I-cache:
         * the kernel must stay small). */
        bool isnull = alive && kind == K_SCALAR && src.at(pos) == 'n';
        bool esc = false, isbin = false;
        uint8_t tt = 0, ktt = 0;
        uint64_t kb = 0, vb = 0; /* key / value part bytes (little-endian) */
        uint32_t kbn = 0, vbn = 0;
        int32_t ks = 0, kn = 0;   /* string map key body */
        int32_t cs = 0, cn = 0;   /* string value body (copy / unquote / base64) */
        uint32_t vln = 0;         /* value bytes after vb: string body, or a container's 4-byte count */
        int32_t kns = -1, knn = 0; /* number map key text (trailing text ignored) */
        int32_t ns = -1, nn = 0;   /* number value text (all of it) */
        if (alive && !skip && isval) {
            tt = ldrec(&D.T[ty]).ttype;
            if (haskey) {
                if (pflags & CF_STRUCT) { /* native/thrift.c:668-763 + null unwinding 1016-1032 */
                    const dg_field f = ldrec(&D.F[fi]);
                    const uint64_t bit = 1ull << fbit;
                    const uint64_t old =
                        __hip_atomic_fetch_or(&L.crec[ci].seen, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (old & bit) bad = true; /* duplicate key: exact machine keeps the order semantics */
                    if (isnull && f.required != DG_REQ_OPTIONAL)
                        __hip_atomic_fetch_or(&L.crec[ci].nulldr, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    kb = (uint32_t)tt | ((uint32_t)__builtin_bswap16(f.id) << 8);
                    kbn = 3;
                } else { /* map key, j2t_map_key native/thrift.c:422-447: parsed even when the
                          * value turns out null (a bad key errors first) */
                    if (!isnull) atomicAdd(&L.crec[ci].count, 1u);
                    ktt = ldrec(&D.T[ldrec(&D.T[ptype]).key]).ttype;
                    if (kesc) bad = true;
                    if (ktt == DG_T_STRING) {
                        ks = kpos + 1;
                        kn = (int32_t)kend - ks;
                        kb = __builtin_bswap32((uint32_t)kn);
                        kbn = 4;
                    } else {
                        kns = kpos + 1;
                        knn = (int32_t)kend - kns;
                        if (!num_size(ktt)) bad = true; /* ERR_UNSUPPORT_THRIFT_TYPE */
                    }
                }
            }
            if (kind == K_SCALAR) {
                ns = pos;
                nn = (int32_t)te - pos;
            } else if (kind == K_STRING) {
                cs = pos + 1;
                cn = (int32_t)te - cs;
                if (tt != DG_T_STRING) bad = true;
                isbin = (flag & DG_F_NO_BASE64) == 0 && (ldrec(&D.T[ty]).flags & DG_TF_BINARY);
                if (!isbin) esc = L.tbs[t & WV_RMASK] != 0; /* a backslash inside (the scan marked it) */
                vbn = 4;
            } else if (kind == K_LBRACE) {
                if (L.crec[lane].flags & CF_MAP) {
                    const dg_type vt = ldrec(&D.T[ty]);
                    vb = ldrec(&D.T[vt.key]).ttype | ((uint32_t)ldrec(&D.T[vt.elem]).ttype << 8);
                    vbn = 2;
                    vln = 4; /* + size, written by the '}' */
                }
            } else { /* K_LBRACK */
                vb = ldrec(&D.T[ldrec(&D.T[ty]).elem]).ttype;
                vbn = 1;
                vln = 4;
            }
            /* a null list element is not counted; checked on the text here */
            if (t != 0 && (pflags & CF_LIST) && !isnull) atomicAdd(&L.crec[ci].count, 1u);
        } else if (alive && skip && kind == K_SCALAR) {
            ns = pos; /* skip_one validates skipped scalars (native/scanning.c:1134-1330) */
            nn = (int32_t)te - pos;
        }
        /* literals inline */
        if (ns >= 0) {
            const uint8_t c0 = src.at(ns);
            if (c0 == 'n' || c0 == 't' || c0 == 'f') {
                const uint32_t w4 = (uint32_t)src.get8(ns + (c0 == 'f'));
                const uint32_t want = c0 == 'n' ? VS_NULL : c0 == 't' ? VS_TRUE : VS_ALSE;
                if (nn != 4 + (c0 == 'f') || w4 != want) bad = true;
                if (c0 != 'n' && !skip) {
                    if (tt != DG_T_BOOL) bad = true;
                    vb = c0 == 't';
                    vbn = 1;
                }
                ns = -1;
            } else if (!skip && !num_size(tt)) {
                bad = true;
            }
        }
        /* numbers: the map key's, then the value's, through ONE parser call
         * site; each becomes its Thrift bytes at once (fewer live VGPRs) */
        /* round 0 parses each lane's key if it has a numeric one, else its
         * value; round 1 only the values of lanes that had both (a numeric
         * map key AND a numeric value): a page whose keys and values are
         * numbers in different lanes (map<i64,struct> keys beside struct
         * fields) pays ONE parser round, not two */
        bool kslow = false, vslow = false;
        for (uint32_t it = 0; it < 2; it++) {
            const bool isk = it == 0 && kns >= 0;
            const bool want = it == 0 ? (kns >= 0 || ns >= 0) : (kns >= 0 && ns >= 0);
            if (!ballot(want)) continue;
            if (want) {
                const int32_t s0 = isk ? kns : ns, n0 = isk ? knn : nn;
                int64_t q = 0, iv = 0;
                double dv = 0.0;
                bool isint = false;
#if defined(DG_WV_ABL) && (DG_WV_ABL & 16)
                q = n0; iv = n0; isint = true; /* ablation: no number parse */
                if (0) {
#else
                bool okn = false;
                if (n0 <= RS_MAX) {
                    RSrc rs;
                    rs.load(src, s0, n0);
                    okn = fast_vnumber(rs, q, tb, iv, dv, isint);
                }
                if (!okn) { /* long numbers (big decimals, long map keys), errors: the exact parser */
#endif
                    if (isk) kslow = true;
                    else vslow = true;
                } else if (isk) {
                    num_le(ktt, isint, iv, dv, kb, kbn);
                } else {
                    if (q != n0) bad = true;
                    if (!skip) num_le(tt, isint, iv, dv, vb, vbn);
                }
            }
        }
        /* numbers the fast parser declines (errors, big-decimal cases): the
         * reference's vnumber (native/scanning.c:958-1083, atof_native
         * native/atof_native.c:418-424), one lane at a time with the wave's
         * 800-byte digit buffer */
        for (uint64_t sm = ballot((kslow || vslow) && !bad); sm; sm &= sm - 1) {
            if (lane == (uint32_t)__builtin_ctzll(sm)) {
                for (uint32_t it = 0; it < 2; it++) {
                    if (!(it == 0 ? kslow : vslow)) continue;
                    const int32_t s0 = it == 0 ? kns : ns, n0 = it == 0 ? knn : nn;
                    JState js;
                    int64_t q = 0;
                    vnumber_slow(src.sub(s0, n0), q, js, dbuf);
                    if (js.vt < 0 || (it == 1 && q != n0)) {
                        bad = true;
                    } else if (it == 0) {
                        num_le(ktt, js.vt == V_INTEGER, js.iv, js.dv, kb, kbn);
                    } else if (!skip) {
                        num_le(tt, js.vt == V_INTEGER, js.iv, js.dv, vb, vbn);
                    }
                }
            }
        }
        /* strings: length of the body */
        if (alive && !skip && kind == K_STRING) {
            if (isbin) {
                int64_t bl = b64_len(src, cs, cn);
                if (bl < 0) bad = true;
                vln = (uint32_t)bl;
            } else if (esc) {
                /* the escapes the scan counted (bits 16+ of the separator
                 * word), else unquote without output */
                const uint32_t shr = L.tsep[t & WV_RMASK] >> 16;
                if (!(shr & 0x8000u) && cn < 32768) {
                    vln = (uint32_t)cn - shr;
                } else {
                    WOut co;
                    co.init_dry();
                    if (!fast_unquote(src, cs, cn, co)) bad = true;
                    vln = (uint32_t)co.len;
                }
            } else {
                vln = (uint32_t)cn;
            }
            vb = __builtin_bswap32(vln);
        }
        if (isnull) { /* a null value writes nothing, its key included */
            kbn = 0;
            kn = 0;
            vbn = 0;
            vln = 0;
        }
        WP(4);
        /* part B: closing brackets, once every atomic of the page is in */
        uint64_t reqs = 0;
        uint32_t sidx = 0; /* the closed struct (its dg_struct is reloaded at the emit) */
        uint32_t uln = 0;  /* bytes of the unset fields */
        if (alive && cl) {
            if (!(pflags & CF_SKIP) && (pflags & CF_STRUCT)) {
                sidx = pflags >> CF_ST_SHIFT;
                const dg_struct csd = ldrec(&D.S[sidx]);
                reqs = (D.R[csd.req_begin] & ~L.crec[ci].seen) | L.crec[ci].nulldr;
                if (!(flag & (DG_F_WRITE_REQUIRE | DG_F_WRITE_DEFAULT | DG_F_WRITE_OPTIONAL)) && sidx < WV_REQMASKS) {
                    /* nothing is written for unset fields: only a missing
                     * REQUIRED one matters (ERR_NULL_REQUIRED, native/thrift.c:286-290) */
                    if (reqs & reqmask[sidx]) bad = true;
                    reqs = 0;
                }
                if (reqs) {
                    WOut co;
                    co.init_dry();
                    if (!unset_fields(D, csd, reqs, flag, co)) bad = true;
                    uln = (uint32_t)co.len;
                }
                vb = 0; /* STOP after the unset fields */
                vbn = 1;
            }
        }
        if (ballot(bad)) return false;
        const uint32_t khead = kbn + (uint32_t)kn; /* bytes before the value part */
        const uint32_t ln = khead + uln + vbn + vln;

        WP(5);
        /* output offsets */
        const uint32_t incl = wave_incl_sum(ln, lane);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t opos = (uint32_t)(O + incl - ln); /* slot offsets are 32-bit (outpos, cbd) */
        if (O + tot > cap) return false; /* slot overflow: the exact machine reports it */
        if (alive && op) L.crec[lane].outpos = opos + khead;

        /* emit: key part, value header / number / literal, then the body;
         * string and base64 bodies go to chunk tasks below */
        const bool live = alive && !skip && !isnull;
        const bool chunked = live && kind == K_STRING && cn > 0 && (isbin || !esc);
        {
            WOut w;
            w.init(ob + opos);
#if defined(DG_WV_ABL) && (DG_WV_ABL & 4)
            w.dry = true; /* ablation: no header/number stores */
#endif
            if (live && kbn) w.wle(kb, kbn);
            if (live && kn > 0) fast_copy(src, ks, kn, w); /* string map key (no escapes) */
            if (live && cl && vbn == 1 && reqs) unset_fields(D, ldrec(&D.S[sidx]), reqs, flag, w); /* before the STOP */
            if (live && vbn) w.wle(vb, vbn);
#if defined(DG_WV_ABL) && (DG_WV_ABL & 64)
            if (0) /* ablation: escaped strings not written */
#endif
            if (live && !chunked && esc && kind == K_STRING) fast_unquote(src, cs, cn, w);
            w.finish();
#if defined(DG_WV_ABL) && (DG_WV_ABL & 96)
            if (live && !op && !chunked && !esc && w.len != ln) bad = true;
#else
            if (live && !op && !chunked && w.len != ln) bad = true;
#endif
        }
        if (alive && cl) {
            if (!(pflags & CF_SKIP) && !(pflags & CF_STRUCT))
                put_be32(ob + L.crec[ci].outpos + ((pflags & CF_MAP) ? 2 : 1), L.crec[ci].count);
        }
        WP(6);
        /* string / base64 bodies: WV_CH-byte chunk tasks over the 64 lanes
         * (task c belongs to the first lane whose inclusive chunk count
         * exceeds c), so the page's longest string does not set the time */
        {
            const uint32_t csz = wv_task_bytes(isbin, (uint32_t)cn);
            const uint32_t nch = chunked ? (uint32_t)((cn + csz - 1) / csz) : 0u;
            const uint32_t cinc = wave_incl_sum(nch, lane);
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)cinc, 63);
            if (T) {
                L.cinc[lane] = cinc;
                L.cbs[lane] = (uint32_t)cs;
                L.cbd[lane] = opos + khead + 4;
                L.cbn[lane] = (uint32_t)cn | (isbin ? 0x80000000u : 0u);
                __builtin_amdgcn_wave_barrier();
                uint32_t l = 0, lend = 0; /* the owner of this lane's previous task, its inclusive count */
#if defined(DG_WV_ABL) && (DG_WV_ABL & 8)
                for (uint32_t c = lane; c < 0; c += 64) { /* ablation: no body tasks */
#else
                for (uint32_t c = lane; c < T; c += 64) {
#endif
                    /* c only grows: a body longer than 64 tasks (C4's base64)
                     * keeps its owner, checked with one LDS read instead of a
                     * 6-read binary search per task */
                    if (c >= lend) {
                        l = 0;
#pragma unroll
                        for (uint32_t step = 32; step; step >>= 1)
                            if (L.cinc[l + step - 1] <= c) l += step;
                        lend = L.cinc[l];
                    }
                    const uint32_t bn = L.cbn[l], blen = bn & 0x7FFFFFFFu;
                    const uint32_t tsz = wv_task_bytes((bn >> 31) != 0, blen);
                    const uint32_t lch = (blen + tsz - 1) / tsz;
                    const uint32_t k = c - (lend - lch);
                    const int64_t s0 = (int64_t)L.cbs[l] + (int64_t)k * tsz;
                    const int64_t n = (int64_t)min(tsz, blen - k * tsz);
                    WOut w;
                    if (bn >> 31) {
                        w.init(ob + L.cbd[l] + (uint64_t)k * (tsz / 4 * 3));
                        if (!chunk_b64(src, s0, n, k + 1 == lch, w)) bad = true;
                    } else {
                        w.init(ob + L.cbd[l] + (uint64_t)k * WV_CH);
                        fast_copy(src, s0, n, w);
                    }
                    w.finish();
                }
            }
        }
        if (ballot(bad)) return false;
        O += tot;

        WP(7);
        /* carry the last opener of every level into the level stack */
        {
            uint32_t have = uni(wave_or(alive && op ? 1u << level : 0u));
            for (; have; have &= have - 1) {
                int32_t Lv = __builtin_ctz(have);
                uint64_t mo = ballot(alive && op && level == Lv);
                uint32_t last = msb(mo);
                if (lane < 8) {
                    const __attribute__((address_space(3))) uint32_t *s =
                        (const __attribute__((address_space(3))) uint32_t *)&L.crec[last];
                    __attribute__((address_space(3))) uint32_t *d =
                        (__attribute__((address_space(3))) uint32_t *)&L.crec[64 + Lv];
                    d[lane] = s[lane];
                }
            }
        }
        WP(8);
        depth = __builtin_amdgcn_readlane(dafter, (int)np - 1);
        consumed += lastoff + 1;
        if (bend) {
            rootdone = true;
            break;
        }
    }
    WP_FLUSH();
    if (!rootdone) return false;
    if (lane == 0) {
        P.ret[m] = 0;
        P.out_len[m] = (uint32_t)O;
    }
    return true;
}

/* one message: staged in the wave's LDS buffer when it fits, else read from
 * global memory through the same code */
template <class DV, class LW>
DGI bool wave_convert(const Params &P, const DV &D, uint32_t D_nf, uint64_t m, LW &L,
                      __attribute__((address_space(3))) uint64_t *mbuf,
                      const __attribute__((address_space(3))) uint8_t *cls, const FastTabs &tb, uint32_t lane, gu8 *dbuf,
                      const __attribute__((address_space(3))) uint64_t *reqmask)
{
    uint64_t a = P.in_off[m], b = P.in_off[m + 1];
    int64_t len = (int64_t)(b - a);
    if (len <= 0 || len > (int64_t)WV_POSMASK) return false;
    const dg_type rt = ldrec(&D.T[P.root]);
    if (rt.ttype != DG_T_STRUCT && rt.ttype != DG_T_MAP && rt.ttype != DG_T_LIST && rt.ttype != DG_T_SET) return false;
    const int64_t head = (int64_t)(a & 7);
    const uint64_t words = (uint64_t)(len + head + 7) >> 3;
    /* one instantiation for both cases (I-cache): generic (flat) pointers */
    const uint64_t *base;
    if (words + 2 <= WV_MSG / 8) {
        const glb_u64 *g = (const glb_u64 *)(const void *)(P.json + (a & ~7ull));
        for (uint64_t k = lane; k < words; k += 64) mbuf[k] = g[k];
        if (lane < 2) mbuf[words + lane] = 0;
        base = (const uint64_t *)(void *)mbuf;
    } else {
        base = (const uint64_t *)(const void *)(P.json + (a & ~7ull));
    }
    SrcT<const uint64_t> s;
    s.init(base, head, len);
    return wave_run(P, D, D_nf, m, L, s, (const uint32_t *)base, head, len, cls, tb, lane, dbuf, reqmask);
}

/* Persistent grid, one wavefront per message at a time. The messages are
 * the lane kernel's large ones (W.list) or, without a list, all of them.
 * The descriptor is copied to LDS once per block; messages that fit are
 * staged in the wave's LDS buffer. Bailed messages are listed for the exact
 * machine (j2t_lane_kernel in list mode). */
template <int V> /* <0> in j2t_kern_wave.hip, <5> in j2t_kern_wave5.hip */
#ifdef DG_WV_NUMVGPR
#define DG_WV_VGPR_ATTR __attribute__((amdgpu_num_vgpr(DG_WV_NUMVGPR)))
#else
#define DG_WV_VGPR_ATTR
#endif
__global__ __launch_bounds__(64 * WV_WAVES) __attribute__((amdgpu_waves_per_eu(DG_WV_WPE))) DG_WV_VGPR_ATTR void j2t_wave_kernel(
    Params P, WaveParams W)
{
    __shared__ __attribute__((aligned(16))) WaveLds wl[WV_WAVES];
    __shared__ __attribute__((aligned(16))) uint64_t s_msg[WV_WAVES][WV_MSG / 8];
    extern __shared__ __attribute__((aligned(16))) uint64_t s_desc[]; /* the blob, rounded to 16 B (launch size) */
    __shared__ uint8_t s_cls[256];
    __shared__ uint64_t s_reqmask[WV_REQMASKS + WV_REQMASKS / 8]; /* REQUIRED-field masks, then a flags byte per struct */
    __shared__ uint64_t s_p10u[20];
    __shared__ double s_p10d[23];
    __shared__ uint64_t s_pw[EL_WN]; /* Eisel-Lemire powers of ordinary doubles: LDS, not the global table */
    const uint32_t tid = threadIdx.x;
    const uint64_t nh = W.list && W.huge_count
                            ? (uint64_t)__hip_atomic_load((uint32_t *)W.huge_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : 0;
    const uint64_t total =
        W.list ? (uint64_t)__hip_atomic_load((uint32_t *)W.list_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + nh
               : P.n;
    if ((uint64_t)blockIdx.x * WV_WAVES >= total) return;
    {
        const uint4 *g = (const uint4 *)W.blob;
        uint4 *l = (uint4 *)s_desc;
        for (uint32_t k = tid; k < (W.hdr.total_len + 15) / 16; k += 64 * WV_WAVES) l[k] = g[k];
    }
    {
        uint32_t c = tid;
        uint8_t k = 0;
        switch (c) {
        case '{': k = C_STRUCT | K_LBRACE; break;
        case '}': k = C_STRUCT | K_RBRACE; break;
        case '[': k = C_STRUCT | K_LBRACK; break;
        case ']': k = C_STRUCT | K_RBRACK; break;
        case ':': k = C_STRUCT | K_COLON; break;
        case ',': k = C_STRUCT | K_COMMA; break;
        case ' ': case '\t': case '\n': case '\r': k = C_WS; break;
        case '"': k = C_QUOTE; break;
        case '\\': k = C_BS; break;
        }
        if (c < 256) s_cls[c] = k;
    }
    if (tid < 20) {
        uint64_t v = 1;
        for (uint32_t k = 0; k < tid; k++) v *= 10;
        s_p10u[tid] = v;
    }
    if (tid < 23) s_p10d[tid] = P10[tid];
    el_window_fill(s_pw, tid);
    __syncthreads();
    const auto dv = desc_view<3>((const __attribute__((address_space(3))) uint8_t *)(void *)s_desc, W.hdr);
    if (tid < WV_REQMASKS && tid < W.hdr.n_structs) {
        /* REQUIRED fields per struct (request-base fields are never written
         * nor checked, native/thrift.c:270-272) */
        const dg_struct sd = ldrec(&dv.S[tid]);
        uint64_t mk = 0;
        for (uint32_t k = 0; k < sd.n_fields && k < 64; k++) {
            const dg_field f = ldrec(&dv.F[sd.field_begin + k]);
            if (f.required == DG_REQ_REQUIRED && !(f.flags & DG_FF_REQUEST_BASE)) mk |= 1ull << k;
        }
        s_reqmask[tid] = mk;
        ((uint8_t *)(s_reqmask + WV_REQMASKS))[tid] =
            (uint8_t)((sd.req_words != 1 ? 1u : 0u) | ((sd.flags & DG_SF_HTTP_MAPPING) ? 2u : 0u));
    }
    __syncthreads();
    const uint32_t wave = tid >> 6, lane = tid & 63;
    FastTabs tb{(const __attribute__((address_space(3))) uint64_t *)(void *)s_p10u, (lds_f64 *)(void *)s_p10d,
                (const __attribute__((address_space(3))) uint64_t *)(void *)s_pw};
    const __attribute__((address_space(3))) uint8_t *cls = (const __attribute__((address_space(3))) uint8_t *)(void *)s_cls;
    __attribute__((address_space(3))) uint64_t *mbuf = (__attribute__((address_space(3))) uint64_t *)(void *)s_msg[wave];
    gu8 *dbuf = (gu8 *)(void *)(W.ws + ((uint64_t)blockIdx.x * WV_WAVES + wave) * DCAP);
    /* dynamic work queue: message sizes vary by 100x (C5), so waves take the
     * next message when they finish one instead of a fixed stride */
    for (;;) {
        uint32_t kq = 0;
        if (lane == 0) kq = __hip_atomic_fetch_add(W.queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)kq);
        if (k >= total) break;
        const uint64_t m = W.list ? (uint64_t)(k < nh ? W.list[W.list_cap - 1 - k] : W.list[k - nh]) : k;
        bool ok = wave_convert(P, dv, W.hdr.n_fields, m, wl[wave], mbuf, cls, tb, lane, dbuf,
                               (const __attribute__((address_space(3))) uint64_t *)(void *)s_reqmask);
        if (!ok && lane == 0) {
            uint32_t q = atomicAdd(W.bail_count, 1u);
            W.bail_list[q] = (uint32_t)m;
        }
    }
}

/* Output packing for the device->host copy: message i's out_len[i] bytes
 * move from its slot (out + out_off[i], 8-aligned) to dst + dst_off[i]
 * (dst_off = exclusive prefix sum of out_len), one wavefront per message,
 * byte-exact at the shared edge words. */
template <int V>
__global__ __launch_bounds__(256) void dg_pack_kernel(const uint8_t *out, const uint64_t *out_off,
                                                      const uint32_t *out_len, uint64_t n, uint8_t *dst,
                                                      const uint64_t *dst_off)
{
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (uint64_t)gridDim.x * 4) {
        const uint32_t nb = out_len[i];
        if (!nb) continue;
        SrcT<const uint64_t> s;
        s.init((const uint64_t *)(const void *)(out + out_off[i]), 0, nb);
        coop_copy(s, 0, nb, (gu8 *)(void *)(dst + dst_off[i]), lane);
    }
}

/* Prefix sum of out_len + packing in ONE launch (the e2e path's D2H staging).
 * A grid of G <= #CU blocks (all co-resident): block b owns messages
 * [b*per, (b+1)*per); it publishes its byte total, waits until every block
 * has (agent-scope release/acquire on sync[0]), adds the totals of the blocks
 * before it, then scans its range tile by tile (256 messages per tile),
 * writes dst_off[i] and copies message i's bytes with one wavefront.
 * dst_off[n] = the grand total. The last block to leave resets sync[]. */
DGI uint64_t block_sum_u64(uint64_t v, uint64_t *red)
{
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d);
    if (lane == 0) red[w] = v;
    __syncthreads();
    v = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return v;
}

/* Framing (HTTPConv.Do, conv/j2t/http_conv.go:68-94): with fr.hdr set, a
 * message that converted (ret 0) is packed as hdr + body + ftr. With fr.ret
 * set, a message that failed packs as nothing (its out_len may carry the
 * bytes an overflowed slot needs). */
struct MsgFrame {
    const uint8_t *hdr; /* device; 16 readable bytes past the end */
    uint32_t hdr_len;
    const uint8_t *ftr;
    uint32_t ftr_len;
    const uint64_t *ret;
    /* chained packing (dg_j2t_pipeline_host): positions start at *base_in
     * (the previous chunk's end, written by its pack), and bytes that would
     * end past dst_cap are not written (0: no limit). dst and dst_off may be
     * pinned host memory: the kernel's stores are then the download. */
    const uint64_t *base_in;
    uint64_t dst_cap;
    /* with base_mod16, positions start at (*base_in) & 15 instead: the
     * packed bytes keep the 16-byte phase they will have at their final
     * host address (dst + *base_in, dst & 15 given as phase_add), for an
     * aligned copy-out (dg_j2t_pipeline_host) */
    uint32_t base_mod16;
    uint32_t phase_add; /* base_mod16: added before the mod (the destination's own address phase) */
    uint64_t *ret_dst;  /* optional: a copy of ret (e.g. pinned host memory: the aggregator's download) */
    uint64_t *cur_out;  /* optional (device): the end position, dst_off[n] -- the next chunk's base_in */
    uint64_t *ovf_out;  /* optional (ret set): the count of DG_ST_OUT_OVERFLOW messages (plain store) */
};

template <int V>
__global__ __launch_bounds__(256) void dg_pack_scan_kernel(const uint8_t *out, const uint64_t *out_off,
                                                           const uint32_t *out_len, uint64_t n, uint8_t *dst,
                                                           uint64_t *dst_off, uint64_t *sums, uint32_t *sync, MsgFrame fr)
{
    __shared__ uint64_t red[4];
    __shared__ uint64_t s_pos[256];
    __shared__ uint32_t s_len[256];
    __shared__ uint64_t s_end;
    const uint32_t G = gridDim.x, b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t per = (n + G - 1) / G;
    const uint64_t lo = (uint64_t)b * per < n ? (uint64_t)b * per : n;
    const uint64_t hi = lo + per < n ? lo + per : n;
    const uint32_t fx = fr.hdr ? fr.hdr_len + fr.ftr_len : 0u;
    auto msg_len = [&](uint64_t i) -> uint32_t {
        if (!fr.ret) return out_len[i];
        if (fr.ret[i] == 0) return out_len[i] + fx;
        /* failed messages pack as nothing; an unframed DG_ST_HM_END keeps its
         * partial output and an ERR_VM_END its record for the host (dgj2t_defs.h) */
        const uint8_t c = (uint8_t)fr.ret[i];
        return !fr.hdr && (c == DG_ST_HM_END || c == 24u || c == DG_ST_HM_END_AT || c == DG_ST_CB_LIST) ? out_len[i]
                                                                                                         : 0u;
    };
    /* bytes, and (ovf_out) overflowed slots in bits 44+ of the same sum */
    constexpr uint32_t OVF_SH = 44;
    uint64_t s = 0;
    for (uint64_t i = lo + tid; i < hi; i += 256) {
        s += msg_len(i);
        if (fr.ovf_out && (uint8_t)fr.ret[i] == DG_ST_OUT_OVERFLOW) s += 1ull << OVF_SH;
    }
    s = block_sum_u64(s, red);
    const uint32_t n_ovf = (uint32_t)(s >> OVF_SH);
    s &= (1ull << OVF_SH) - 1;
    if (tid == 0) {
        __hip_atomic_store(&sums[b], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n_ovf) __hip_atomic_fetch_add(&sync[6], n_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&sync[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(&sync[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < G)
            __builtin_amdgcn_s_sleep(4);
    }
    __syncthreads();
    uint64_t base = 0;
    for (uint32_t k = tid; k < b; k += 256) base += __hip_atomic_load(&sums[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    base = block_sum_u64(base, red);
    if (fr.base_in) { /* one read per block (it may be pinned host memory) */
        if (tid == 0) s_pos[0] = *(volatile const uint64_t *)fr.base_in;
        __syncthreads();
        const uint64_t b0 = s_pos[0];
        __syncthreads();
        base += fr.base_mod16 ? ((b0 + fr.phase_add) & 15) : b0;
    }
    const uint64_t cap = fr.dst_cap ? fr.dst_cap : ~0ull;
    for (uint64_t t0 = lo; t0 < hi; t0 += 256) {
        const uint64_t i = t0 + tid;
        const uint32_t len = i < hi ? msg_len(i) : 0u;
        /* block exclusive scan of len */
        uint32_t incl = wave_incl_sum(len, lane);
        if (lane == 63) red[w] = incl;
        __syncthreads();
        uint64_t wpre = 0;
        for (uint32_t k = 0; k < w; k++) wpre += red[k];
        const uint64_t tile = red[0] + red[1] + red[2] + red[3];
        const uint64_t pos = base + wpre + incl - len;
        if (i < hi) dst_off[i] = pos;
        if (fr.ret_dst && i < hi) fr.ret_dst[i] = fr.ret[i];
        s_pos[tid] = pos;
        s_len[tid] = len;
        __syncthreads();
        const uint32_t nt = hi - t0 < 256 ? (uint32_t)(hi - t0) : 256u;
        if (!fr.hdr) {
            /* Unframed: the tile's output is one contiguous byte range, so
             * the block writes it word by word in address order -- every
             * thread a destination word, a wave 512 contiguous bytes per
             * store (coalesced; over the link when dst is pinned host
             * memory) -- each word gathered from the message(s) it holds
             * (binary search of the tile's positions in LDS). The words at
             * both ends, shared with the neighbouring tiles, are written
             * byte-exact. Messages that would end past cap form a suffix
             * (positions rise): the range stops at the last that fits. */
            if (tid == 0) s_end = s_pos[0];
            __syncthreads();
            if (tid < nt && s_pos[tid] + s_len[tid] <= cap &&
                (tid + 1 == nt || s_pos[tid + 1] + s_len[tid + 1] > cap))
                s_end = s_pos[tid] + s_len[tid];
            __syncthreads();
            const uint64_t P0 = s_pos[0], P1 = s_end;
            const uintptr_t D = (uintptr_t)dst, A0 = D + P0, A1 = D + P1;
            const uintptr_t wa = A0 & ~(uintptr_t)7, wb = (A1 + 7) & ~(uintptr_t)7;
            const uint64_t nw = P1 > P0 ? (uint64_t)((wb - wa) >> 3) : 0;
            for (uint64_t j = tid; j < nw; j += 256) {
                const uintptr_t W = wa + 8 * j, lo = W < A0 ? A0 : W, hi2 = W + 8 > A1 ? A1 : W + 8;
                const uint64_t p = (uint64_t)(lo - D);
                uint32_t l = 0, h = nt; /* the last message starting at or before p */
                while (h - l > 1) {
                    const uint32_t m = (l + h) >> 1;
                    if (s_pos[m] <= p) l = m;
                    else h = m;
                }
                uint32_t k = l;
                if (lo == W && hi2 == W + 8 && p + 8 <= s_pos[k] + s_len[k]) {
                    /* inside one message: an unaligned 8-byte read of its
                     * slot (8-aligned), as two words when it straddles; the
                     * second holds a byte of the message, so it is in bounds */
                    const uint64_t o = p - s_pos[k];
                    const uint64_t *sw = (const uint64_t *)(const void *)(out + out_off[t0 + k] + (o & ~7ull));
                    const uint32_t sh = (uint32_t)(o & 7) * 8;
                    uint64_t v = sw[0];
                    if (sh) v = (v >> sh) | (sw[1] << (64 - sh));
                    *(gu64 *)(void *)W = v;
                } else {
                    for (uintptr_t q = lo; q < hi2; q++) {
                        const uint64_t pq = (uint64_t)(q - D);
                        while (pq >= s_pos[k] + s_len[k]) k++; /* pq < P1: stays in the tile */
                        *(gu8 *)(void *)q = out[out_off[t0 + k] + (pq - s_pos[k])];
                    }
                }
            }
            base += tile;
            __syncthreads();
            continue;
        }
        for (uint32_t k = w; k < nt; k += 4) {
            uint32_t nb = s_len[k];
            if (!nb || s_pos[k] + nb > cap) continue;
            gu8 *d = (gu8 *)(void *)(dst + s_pos[k]);
            if (fr.hdr) { /* header, body, footer: byte-exact edges, in program order */
                SrcT<const uint64_t> h;
                h.init((const uint64_t *)(const void *)fr.hdr, 0, fr.hdr_len);
                coop_copy(h, 0, fr.hdr_len, d, lane);
                d += fr.hdr_len;
                nb -= fx;
            }
            SrcT<const uint64_t> src;
            src.init((const uint64_t *)(const void *)(out + out_off[t0 + k]), 0, nb);
            coop_copy(src, 0, nb, d, lane);
            if (fr.hdr && fr.ftr_len) {
                SrcT<const uint64_t> f;
                f.init((const uint64_t *)(const void *)fr.ftr, 0, fr.ftr_len);
                coop_copy(f, 0, fr.ftr_len, d + nb, lane);
            }
        }
        base += tile;
        __syncthreads();
    }
    if (tid == 0) {
        if (b == G - 1) { /* the last range ends at the grand total */
            dst_off[n] = base;
            if (fr.cur_out) *fr.cur_out = base;
            if (fr.ovf_out) *fr.ovf_out = __hip_atomic_load(&sync[6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint32_t prev = __hip_atomic_fetch_add(&sync[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == G - 1) { /* every block is past its wait: reset for the next launch */
            __hip_atomic_store(&sync[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&sync[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&sync[6], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

void launch_pack_scan_kernel(dim3 grid, hipStream_t s, const uint8_t *out, const uint64_t *out_off,
                             const uint32_t *out_len, uint64_t n, uint8_t *dst, uint64_t *dst_off, uint64_t *sums,
                             uint32_t *sync, const MsgFrame &fr);
void launch_wave_kernel(dim3 grid, hipStream_t s, const Params &P, const WaveParams &W); /* LDS: + the blob */
void launch_wave_kernel5(dim3 grid, hipStream_t s, const Params &P, const WaveParams &W); /* 5 waves/SIMD */
void launch_pack_kernel(dim3 grid, hipStream_t s, const uint8_t *out, const uint64_t *out_off, const uint32_t *out_len,
                        uint64_t n, uint8_t *dst, const uint64_t *dst_off);

}  // namespace dg
