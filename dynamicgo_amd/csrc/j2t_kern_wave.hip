/* j2t_wave_kernel instantiation (wave-per-message token-parallel path). */
#include "j2t_wave.h"

namespace dg {
void launch_wave_kernel(dim3 grid, hipStream_t s, const Params &P, const WaveParams &W)
{
    hipLaunchKernelGGL(j2t_wave_kernel<0>, grid, dim3(64 * WV_WAVES), 0, s, P, W);
}
}  // namespace dg
