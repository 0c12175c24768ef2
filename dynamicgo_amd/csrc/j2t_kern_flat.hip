/* j2t_flat_kernel instantiation (a group of lanes per message, a lane per field). */
#include "j2t_flat.h"

namespace dg {
void launch_flat_kernel(dim3 grid, hipStream_t s, const Params &P, const FlatParams &S)
{
    const uint32_t shmem = (S.hdr.total_len + 15) & ~15u;
    hipLaunchKernelGGL(j2t_flat_kernel<0>, grid, dim3(64 * FL_WAVES), shmem, s, P, S);
}
}  // namespace dg
