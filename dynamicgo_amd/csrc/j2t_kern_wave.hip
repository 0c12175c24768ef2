/* j2t_wave_kernel instantiation (wave-per-message token-parallel path). */
#include "j2t_wave.h"

namespace dg {
void launch_wave_kernel(dim3 grid, hipStream_t s, const Params &P, const WaveParams &W)
{
    hipLaunchKernelGGL(j2t_wave_kernel<0>, grid, dim3(64 * WV_WAVES), (W.hdr.total_len + 15) & ~15u, s, P, W);
}
void launch_pack_kernel(dim3 grid, hipStream_t s, const uint8_t *out, const uint64_t *out_off, const uint32_t *out_len,
                        uint64_t n, uint8_t *dst, const uint64_t *dst_off)
{
    hipLaunchKernelGGL(dg_pack_kernel<0>, grid, dim3(256), 0, s, out, out_off, out_len, n, dst, dst_off);
}
void launch_pack_scan_kernel(dim3 grid, hipStream_t s, const uint8_t *out, const uint64_t *out_off,
                             const uint32_t *out_len, uint64_t n, uint8_t *dst, uint64_t *dst_off, uint64_t *sums,
                             uint32_t *sync, const MsgFrame &fr)
{
    hipLaunchKernelGGL(dg_pack_scan_kernel<0>, grid, dim3(256), 0, s, out, out_off, out_len, n, dst, dst_off, sums,
                       sync, fr);
}
}  // namespace dg
