/* t2j kernels (Thrift binary -> JSON): the LDS-frame pass and the deep pass. */
#include "t2j_device.h"

namespace dg {

/* one lane per message, frames in LDS; messages that need more frames are
 * queued for t2j_deep_kernel. Every SP-th lane takes a message: the per-lane
 * walk is a chain of dependent loads, so sparser waves, more of them per
 * SIMD, hide more of it. The best spread depends on the message size
 * (measured, LICM off): t2j-c2 (~100 B) 0.0705 / 0.0739 / 0.0977 ms at spread
 * 1 / 2 / 4; t2j-c3 (~1.2 KB) 5.59 / 3.95 / 3.76 ms. The host picks it from
 * the batch's longest message (t2j_spread). */
template <uint32_t SP>
__global__ __launch_bounds__(T2J_BLOCK) void t2j_kernel(T2JParams P)
{
    constexpr uint32_t MPB = T2J_BLOCK / SP; /* messages per block */
    __shared__ __attribute__((aligned(16))) T2JFrame lf[T2J_LDS_DEPTH * MPB];
    if (threadIdx.x % SP) return;
    const uint32_t slot = threadIdx.x / SP;
    const uint64_t i = (uint64_t)blockIdx.x * MPB + slot;
    if (i >= P.n) return;
    const auto D = desc_view<1>((const __attribute__((address_space(1))) uint8_t *)(const void *)P.blob, P.hdr);
    const T2JSide X = t2j_side(P.side);
    const uint64_t a = P.in_off[i], b = P.in_off[i + 1];
    SrcT<glb_u64> s;
    s.init((glb_u64 *)(const void *)(P.src + (a & ~7ull)), (int64_t)(a & 7), (int64_t)(b - a));
    Out o;
    o.init(P.out + P.out_off[i], P.out_off[i + 1] - P.out_off[i]);
    const uint64_t r = t2j_convert(D, X, s, P.root, P.opts, o,
                                   (__attribute__((address_space(3))) T2JFrame *)(void *)&lf[slot], MPB,
                                   T2J_LDS_DEPTH);
    if ((uint8_t)r == DG_ST_DEEP) {
        P.deep_list[atomicAdd(P.deep_count, 1u)] = (uint32_t)i;
        return;
    }
    t2j_store(P, i, r, o);
}

/* the queued deep messages (nested beyond the LDS frames, or holding a
 * struct of more than 64 fields), rerun from the start with T2J_DEEP_DEPTH
 * frames and T2J_WIDE_WORDS requires words per lane in device memory; a grid-stride loop over the queue (the grid is
 * small: deep messages are rare) */
__global__ __launch_bounds__(T2J_BLOCK) void t2j_deep_kernel(T2JParams P)
{
    const uint32_t cnt = *(volatile uint32_t *)P.deep_count;
    const uint32_t lane = blockIdx.x * T2J_BLOCK + threadIdx.x;
    const auto D = desc_view<1>((const __attribute__((address_space(1))) uint8_t *)(const void *)P.blob, P.hdr);
    const T2JSide X = t2j_side(P.side);
    T2JFrame *fr = (T2JFrame *)(void *)(P.ws + (uint64_t)lane * T2J_DEEP_DEPTH * sizeof(T2JFrame));
    /* after every lane's frames: the requires words of wide structs */
    gu64 *wide = (gu64 *)(void *)(P.ws + (uint64_t)T2J_DEEP_BLOCKS * T2J_BLOCK * T2J_DEEP_DEPTH * sizeof(T2JFrame) +
                                  (uint64_t)lane * T2J_WIDE_WORDS * 8);
    for (uint32_t g = lane; g < cnt; g += gridDim.x * T2J_BLOCK) {
        const uint64_t i = P.deep_list[g];
        const uint64_t a = P.in_off[i], b = P.in_off[i + 1];
        SrcT<glb_u64> s;
        s.init((glb_u64 *)(const void *)(P.src + (a & ~7ull)), (int64_t)(a & 7), (int64_t)(b - a));
        Out o;
        o.init(P.out + P.out_off[i], P.out_off[i + 1] - P.out_off[i]);
        uint64_t r = t2j_convert(D, X, s, P.root, P.opts, o, fr, 1, T2J_DEEP_DEPTH, wide, T2J_WIDE_WORDS);
        if ((uint8_t)r == DG_ST_DEEP) r = t2j_err(DG_T2J_E_DEPTH, 0, T2J_DEEP_DEPTH);
        t2j_store(P, i, r, o);
    }
}

void launch_t2j_pass(uint64_t n, hipStream_t s, const T2JParams &P, uint32_t spread)
{
    const uint32_t mpb = T2J_BLOCK / spread, blocks = (uint32_t)((n + mpb - 1) / mpb);
    if (spread == 1) hipLaunchKernelGGL(t2j_kernel<1>, dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
    else if (spread == 4) hipLaunchKernelGGL(t2j_kernel<4>, dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
    else hipLaunchKernelGGL(t2j_kernel<2>, dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
}

void launch_t2j_deep(hipStream_t s, const T2JParams &P)
{
    hipLaunchKernelGGL(t2j_deep_kernel, dim3(T2J_DEEP_BLOCKS), dim3(T2J_BLOCK), 0, s, P);
}
}  // namespace dg
