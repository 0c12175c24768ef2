/*
 * j2t_small.h — the small-message kernel: one LANE per message, fast path only.
 *
 * The lane kernel (j2t_machine.h) carries the exact machine in the same
 * launch, which costs 328 VGPRs and ~145 KiB of LDS: one wave per SIMD, so
 * every LDS/HBM latency of the byte-serial fast path is exposed. Here the
 * exact machine is NOT in the kernel: a message the fast path declines is
 * appended to the bail list, which the lane kernel's list mode converts
 * exactly afterwards (so results stay bit-identical, j2t_fast.h). Without it
 * the kernel is small enough to run several waves per SIMD, and MPW (messages
 * per wave) < 64 trades lane utilisation for more resident waves: a 64K batch
 * is 1024 waves at MPW 64 (one per SIMD) but 2048 at MPW 32.
 *
 * Messages longer than big_max are listed for the wave kernel (j2t_wave.h).
 */
#pragma once
#include "j2t_wave.h"

namespace dg {

constexpr uint32_t SM_WAVES = 4;
constexpr uint32_t SM_DESC = 12 * 1024; /* descriptor copied to LDS (larger: lane kernel path) */

template <int MPW>
struct SmallCfg {
    static constexpr uint32_t MPB = SM_WAVES * MPW;       /* messages per block */
    static constexpr uint32_t STAGE = MPB * 256;           /* LDS staging of the block's JSON span */
};

struct SmallParams {
    const uint8_t *blob;
    dg_desc_hdr hdr;
    uint32_t *bail_count; /* fast-path declines -> exact machine (list mode) */
    uint32_t *bail_list;
};

#ifndef DG_SMALL_WPE
#define DG_SMALL_WPE 2 /* waves per SIMD the register budget is cut for */
#endif
template <int MPW, bool LEAN = true>
__global__ __launch_bounds__(64 * SM_WAVES) __attribute__((amdgpu_waves_per_eu(DG_SMALL_WPE))) void j2t_small_kernel(
    Params P, SmallParams S)
{
    typedef SmallCfg<MPW> C;
    __shared__ __attribute__((aligned(16))) uint64_t stage[C::STAGE / 8 + 2];
    __shared__ __attribute__((aligned(16))) FFrame lframes[FAST_LDS_DEPTH * C::MPB];
    __shared__ __attribute__((aligned(16))) uint64_t ldesc[SM_DESC / 8];
    __shared__ uint64_t s_p10u[20];
    __shared__ double s_p10d[23];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint64_t b0 = (uint64_t)blockIdx.x * C::MPB;
    const uint64_t b1 = b0 + C::MPB < P.n ? b0 + C::MPB : P.n;
    const uint64_t lo = P.in_off[b0], hi = P.in_off[b1];
    const uint64_t base = lo & ~15ull;
    const uint64_t words = (hi - base + 15) >> 4;
    const bool staged = words * 16 <= C::STAGE;
    if (staged) {
        const uint4 *g = (const uint4 *)(P.json + base);
        uint4 *l = (uint4 *)stage;
        for (uint64_t k = tid; k < words; k += 64 * SM_WAVES) l[k] = g[k];
    }
    {
        const uint4 *g = (const uint4 *)S.blob;
        uint4 *l = (uint4 *)ldesc;
        for (uint32_t k = tid; k < (S.hdr.total_len + 15) / 16; k += 64 * SM_WAVES) l[k] = g[k];
    }
    if (tid < 20) {
        uint64_t v = 1;
        for (uint32_t k = 0; k < tid; k++) v *= 10;
        s_p10u[tid] = v;
    }
    if (tid < 23) s_p10d[tid] = P10[tid];
#ifdef DG_FPROF
    if (lane < 17) fprof_slots()[wave * 17 + lane] = lane == 16 ? __builtin_amdgcn_s_memtime() : 0;
    FP_MARK(12);
#endif
    __syncthreads();
    const uint32_t j = wave * MPW + lane; /* message slot within the block */
    const uint64_t i = b0 + j;
    const bool mine = lane < (uint32_t)MPW && i < b1;
    uint64_t a = 0, b = 0;
    if (mine) {
        a = P.in_off[i];
        b = P.in_off[i + 1];
    }
    const bool big = mine && P.big_list && b - a > P.big_max;
    /* The block's span did not fit the stage (a mixed batch: large messages
     * sit between the small ones). Stage per WAVE instead: each lane copies
     * the aligned words of its own small message to a packed position in
     * the wave's quarter of the stage (wave prefix sum of word counts). A
     * lane only ever reads back what it wrote itself, so no barrier. */
    constexpr uint32_t WSTAGE = C::STAGE / 8 / SM_WAVES; /* words per wave */
    bool wst = false;
    uint32_t wbase = 0;
    if (!staged) {
        uint64_t wc64 = mine && !big ? ((b + 7) >> 3) - (a >> 3) + 1 : 0; /* +1: the window may read one word past */
        const uint32_t wc = wc64 > WSTAGE ? WSTAGE + 1 : (uint32_t)wc64;
        const uint32_t incl = wave_incl_sum(wc, lane);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (tot <= WSTAGE) {
            wst = true;
            wbase = wave * WSTAGE + incl - wc;
            const glb_u64 *g = (const glb_u64 *)(const void *)P.json + (a >> 3); /* arena: 16 readable bytes past the end */
            for (uint32_t k = 0; k < wc; k++) stage[wbase + k] = g[k];
        }
    }
    list_big_w(P, big, i, b - a);
    if (!mine || big) return;
    const auto dv = desc_view<3>((const __attribute__((address_space(3))) uint8_t *)(void *)ldesc, S.hdr);
    const uint64_t oa = P.out_off[i], ob = P.out_off[i + 1];
    Out out;
    out.init(P.out + oa, ob - oa);
    FastTabs tb{(const __attribute__((address_space(3))) uint64_t *)(void *)s_p10u, (lds_f64 *)(void *)s_p10d};
    LFFrame *ff = (LFFrame *)(void *)&lframes[j];
    bool done;
    if (staged || wst) {
        SrcT<lds_u64, int32_t> s; /* the stage is < 2 GiB: 32-bit positions */
        if (staged) s.init((lds_u64 *)(void *)stage, (int32_t)(a - base), (int32_t)(b - a));
        else s.init((lds_u64 *)(void *)stage + wbase, (int32_t)(a & 7), (int32_t)(b - a));
        done = fast_convert<LEAN>(dv, s, out, P.flag, P.root, ff, C::MPB, tb);
    } else {
        SrcT<glb_u64> s = global_src(P, i);
        done = fast_convert<LEAN>(dv, s, out, P.flag, P.root, ff, C::MPB, tb);
    }
    if (done) {
        P.ret[i] = 0;
        P.out_len[i] = (uint32_t)out.len;
    } else {
        uint32_t q = atomicAdd(S.bail_count, 1u);
        S.bail_list[q] = (uint32_t)i;
    }
#ifdef DG_FPROF
    FP_MARK(13);
    if (lane < 14) atomicAdd(&P.stats[2 + lane], fprof_slots()[wave * 17 + lane]);
#endif
}

void launch_small_kernel(int mpw, dim3 grid, hipStream_t s, const Params &P, const SmallParams &S);

}  // namespace dg
