/* t2j kernels (Thrift binary -> JSON): the LDS-frame pass and the deep pass. */
#include "t2j_wave.h"

namespace dg {

/* one lane per message, frames in LDS; messages that need more frames are
 * queued for t2j_deep_kernel. Every SP-th lane takes a message: the per-lane
 * walk is a chain of dependent loads, so sparser waves, more of them per
 * SIMD, hide more of it. The best spread depends on the message size
 * (measured, LICM off): t2j-c2 (~100 B) 0.0705 / 0.0739 / 0.0977 ms at spread
 * 1 / 2 / 4; t2j-c3 (~1.2 KB) 5.59 / 3.95 / 3.76 ms. The host picks it from
 * the batch's longest message (t2j_spread). */
template <uint32_t SP, bool GO>
__global__ __launch_bounds__(T2J_BLOCK) void t2j_kernel(T2JParams P)
{
    constexpr uint32_t MPB = T2J_BLOCK / SP; /* messages per block */
    __shared__ __attribute__((aligned(16))) T2JFrame lf[T2J_LDS_DEPTH * MPB];
    if (threadIdx.x % SP) return;
    const uint32_t slot = threadIdx.x / SP;
    const auto D = desc_view<1>((const __attribute__((address_space(1))) uint8_t *)(const void *)P.blob, P.hdr);
    const T2JSide X = t2j_side(P.side);
    /* all n messages, or (list mode) the wave kernel's bails, grid-strided */
    const uint64_t cnt = P.list ? (uint64_t)*(volatile const uint32_t *)P.list_count : P.n;
    for (uint64_t k = (uint64_t)blockIdx.x * MPB + slot; k < cnt; k += (uint64_t)gridDim.x * MPB) {
        const uint64_t i = P.list ? (uint64_t)P.list[k] : k;
        const uint64_t a = P.in_off[i], b = P.in_off[i + 1];
        const bool big = (P.big_list || P.skip_big) && b - a > P.big_min;
        if (!P.skip_big) wave_push(P.big_list, P.big_count, big, (uint32_t)i); /* the wave kernel takes it */
        if (big) continue;
        SrcT<glb_u64> s;
        s.init((glb_u64 *)(const void *)(P.src + (a & ~7ull)), (int64_t)(a & 7), (int64_t)(b - a));
        JOut o;
        o.init(P.out + P.out_off[i], P.out_off[i + 1] - P.out_off[i]);
        const uint64_t r = t2j_convert<GO>(D, X, s, P.root, P.opts, o,
                                       (__attribute__((address_space(3))) T2JFrame *)(void *)&lf[slot], MPB,
                                       T2J_LDS_DEPTH, nullptr, 0, P.aux ? P.aux + i : nullptr,
                                       P.ans_tab ? P.ans_tab + i : nullptr, P.ans_bytes);
        if ((uint8_t)r == DG_ST_DEEP) {
            P.deep_list[atomicAdd(P.deep_count, 1u)] = (uint32_t)i;
            continue;
        }
        t2j_store(P, i, r, o);
    }
}

/* the long messages listed by length alone (the wave kernel's list, ahead
 * of the lane pass, which then skips them: t2j_launch's overlapped form) */
__global__ __launch_bounds__(256) void t2j_route_kernel(T2JParams P)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool big = i < P.n && P.in_off[i + 1] - P.in_off[i] > P.big_min;
    wave_push(P.big_list, P.big_count, big, (uint32_t)i);
}

/* the long messages (t2j_wave.h): a persistent grid; each wave takes
 * T2W_MPT of them at a time, every lane walks one into the wave's token
 * region, then the wave formats them one by one; bails are listed for the
 * lane kernel's list mode */
__global__ __launch_bounds__(64 * T2W_WAVES) __attribute__((amdgpu_waves_per_eu(4))) void t2j_wave_kernel(T2JParams P, T2WParams W)
{
    __shared__ __attribute__((aligned(16))) T2WLds wl[T2W_WAVES];
    __shared__ __attribute__((aligned(16))) T2WFrame s_fr[T2W_WAVES][T2W_BD * T2W_MPT];
    __shared__ uint64_t s_fx[T2W_FX];
    __shared__ __attribute__((aligned(16))) uint64_t s_msg[T2W_WAVES][T2W_MSG / 8];
    extern __shared__ __attribute__((aligned(16))) uint64_t s_desc[]; /* the blob, rounded to 16 B */
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint64_t total = *(volatile const uint32_t *)W.count;
    if ((uint64_t)blockIdx.x * T2W_WAVES * T2W_MPT >= total) return;
    /* the descriptor, then the side table (its keys are read 8 bytes at a
     * time: 16 zero bytes after it) */
    const uint32_t dlen = (P.hdr.total_len + 15) & ~15u, slen = (W.side_len + 15) & ~15u;
    {
        const uint4 *g = (const uint4 *)P.blob;
        uint4 *l = (uint4 *)s_desc;
        for (uint32_t k = tid; k < dlen / 16; k += 64 * T2W_WAVES) l[k] = g[k];
        const uint4 *gs = (const uint4 *)P.side;
        uint4 *ls = (uint4 *)((uint8_t *)s_desc + dlen);
        for (uint32_t k = tid; k < slen / 16 + 1; k += 64 * T2W_WAVES) ls[k] = k < slen / 16 ? gs[k] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const auto dv = desc_view<3>((const __attribute__((address_space(3))) uint8_t *)(void *)s_desc, P.hdr);
    T2WSide X;
    {
        const __attribute__((address_space(3))) uint8_t *sb =
            (const __attribute__((address_space(3))) uint8_t *)(void *)((uint8_t *)s_desc + dlen);
        const dg_t2j_hdr xh = *(const dg_t2j_hdr *)(const void *)((uint8_t *)s_desc + dlen);
        X.X = (const __attribute__((address_space(3))) dg_t2j_field *)(sb + xh.off_fields);
        X.P = sb + xh.off_pool;
    }
    /* the walker's per-field table: id, ttype, type flags, type index */
    for (uint32_t f = tid; f < P.hdr.n_fields && f < T2W_FX; f += 64 * T2W_WAVES) {
        const dg_field fd = ldrec(&dv.F[f]);
        const dg_type t = ldrec(&dv.T[fd.type]);
        s_fx[f] = (uint64_t)fd.id | ((uint64_t)t.ttype << 16) |
                  ((uint64_t)(t.flags | (fd.vm != DG_VM_NONE ? 0x80u : 0u)) << 24) | ((uint64_t)fd.type << 32);
    }
    __syncthreads();
    const __attribute__((address_space(3))) uint64_t *fx = (const __attribute__((address_space(3))) uint64_t *)(void *)s_fx;
    T2WTok *tokw = (T2WTok *)(void *)(W.tok + ((uint64_t)blockIdx.x * T2W_WAVES + wave) * T2W_MPT * T2W_TOKCAP *
                                                  sizeof(T2WTok));
    T2WFrame *frs = s_fr[wave];
    for (;;) {
        uint32_t kq = 0;
        if (lane == 0) kq = __hip_atomic_fetch_add(W.queue, T2W_MPT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)kq);
        if (k0 >= total) break;
        const uint32_t nm = (uint32_t)(total - k0 < T2W_MPT ? total - k0 : T2W_MPT);
        const uint64_t mine = lane < nm ? (uint64_t)W.list[k0 + lane] : 0ull;
        t2w_batch(P, W, dv, fx, X, mine, nm, wl[wave], frs, tokw,
                  (__attribute__((address_space(3))) uint64_t *)(void *)s_msg[wave], lane);
    }
}

/* the queued deep messages (nested beyond the LDS frames, or holding a
 * struct of more than 64 fields), rerun from the start with T2J_DEEP_DEPTH
 * frames and T2J_WIDE_WORDS requires words per lane in device memory; a grid-stride loop over the queue (the grid is
 * small: deep messages are rare) */
template <bool GO>
__global__ __launch_bounds__(T2J_BLOCK) void t2j_deep_kernel(T2JParams P)
{
    const uint32_t cnt = *(volatile uint32_t *)P.deep_count;
    const uint32_t lane = blockIdx.x * T2J_BLOCK + threadIdx.x;
    if (lane < 4 && P.reset_counts) P.reset_counts[lane] = 0; /* the next launch's counters */
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
        JOut o;
        o.init(P.out + P.out_off[i], P.out_off[i + 1] - P.out_off[i]);
        uint64_t r = t2j_convert<GO>(D, X, s, P.root, P.opts, o, fr, 1, T2J_DEEP_DEPTH, wide, T2J_WIDE_WORDS,
                                 P.aux ? P.aux + i : nullptr, P.ans_tab ? P.ans_tab + i : nullptr, P.ans_bytes);
        if ((uint8_t)r == DG_ST_DEEP) r = t2j_err(DG_T2J_E_DEPTH, 0, T2J_DEEP_DEPTH);
        t2j_store(P, i, r, o);
    }
}

/* the Go-side options (the lane kernel only: t2j_launch keeps them off
 * the wave kernel) take the GO instances, spread 1 */
static inline bool t2j_go(const T2JParams &P)
{
    return (P.opts & (DG_T2J_CONVERT_EXC | DG_T2J_SKIP_RESP_BASE | DG_T2J_HM)) != 0;
}

void launch_t2j_pass(uint64_t n, hipStream_t s, const T2JParams &P, uint32_t spread)
{
    if (t2j_go(P)) spread = 1;
    const uint32_t mpb = T2J_BLOCK / spread, blocks = (uint32_t)((n + mpb - 1) / mpb);
    if (t2j_go(P)) hipLaunchKernelGGL((t2j_kernel<1, true>), dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
    else if (spread == 1) hipLaunchKernelGGL((t2j_kernel<1, false>), dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
    else if (spread == 4) hipLaunchKernelGGL((t2j_kernel<4, false>), dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
    else hipLaunchKernelGGL((t2j_kernel<2, false>), dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
}

void launch_t2j_route(uint64_t n, hipStream_t s, const T2JParams &P)
{
    hipLaunchKernelGGL(t2j_route_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, P);
}

void launch_t2j_list(uint32_t blocks, hipStream_t s, const T2JParams &P)
{
    if (t2j_go(P)) hipLaunchKernelGGL((t2j_kernel<1, true>), dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
    else hipLaunchKernelGGL((t2j_kernel<1, false>), dim3(blocks), dim3(T2J_BLOCK), 0, s, P);
}

void launch_t2j_wave(uint32_t blocks, hipStream_t s, const T2JParams &P, const T2WParams &W)
/* W.tok: blocks * T2W_WAVES * T2W_MPT * T2W_TOKCAP tokens (t2j_wave_ws_bytes) */
{
    const size_t dyn = (P.hdr.total_len + 15) / 16 * 16 + (W.side_len + 15) / 16 * 16 + 16;
    hipLaunchKernelGGL(t2j_wave_kernel, dim3(blocks), dim3(64 * T2W_WAVES), dyn, s, P, W);
}

uint64_t t2j_wave_ws_bytes(uint32_t blocks) { return (uint64_t)blocks * T2W_WAVES * T2W_MPT * T2W_TOKCAP * sizeof(T2WTok); }

void launch_t2j_deep(hipStream_t s, const T2JParams &P)
{
    if (t2j_go(P)) hipLaunchKernelGGL(t2j_deep_kernel<true>, dim3(T2J_DEEP_BLOCKS), dim3(T2J_BLOCK), 0, s, P);
    else hipLaunchKernelGGL(t2j_deep_kernel<false>, dim3(T2J_DEEP_BLOCKS), dim3(T2J_BLOCK), 0, s, P);
}
}  // namespace dg
