/* j2t_small_kernel instantiations (lane-per-message fast path, exact machine out of line). */
#include "j2t_small.h"

namespace dg {
void launch_small_kernel(int mpw, dim3 grid, hipStream_t s, const Params &P, const SmallParams &S)
{
    if (mpw == 64) hipLaunchKernelGGL(j2t_small_kernel<64>, grid, dim3(64 * SM_WAVES), 0, s, P, S);
    else if (mpw == 65) /* experiment: the full (non-lean) fast path, 64 messages per wave */
        hipLaunchKernelGGL((j2t_small_kernel<64, false>), grid, dim3(64 * SM_WAVES), 0, s, P, S);
    else if (mpw == 16) hipLaunchKernelGGL(j2t_small_kernel<16>, grid, dim3(64 * SM_WAVES), 0, s, P, S);
    else hipLaunchKernelGGL(j2t_small_kernel<32>, grid, dim3(64 * SM_WAVES), 0, s, P, S);
}
}  // namespace dg
