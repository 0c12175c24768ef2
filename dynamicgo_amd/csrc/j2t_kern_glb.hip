/* j2t_lane_kernel instantiation: descriptor tables read from global memory. */
#include "j2t_machine.h"

namespace dg {
void launch_lane_kernel_glb(dim3 grid, hipStream_t s, const Params &P, const DeepParams &DP)
{
    hipLaunchKernelGGL(j2t_lane_kernel<false>, grid, dim3(LANE_BLOCK), 0, s, P, DP);
}
}  // namespace dg
