/* j2t_wave_kernel at 5 waves/SIMD (see the occupancy note in j2t_wave.h):
 * 96 VGPRs, 128 B message staging and the full 256-token ring, so that five
 * 4-wave blocks (plus the descriptor) fit the CU's 160 KiB of LDS. */
#define DG_WV_WPE 5
#define DG_WV_NUMVGPR 102
#define DG_WV_RING 256
#define DG_WV_MSG 128
#define DG_WV_BPC 5
#include "j2t_wave.h"

namespace dg {
static_assert(WV_BLOCKS_PER_CU == WV5_BLOCKS_PER_CU, "grid and workspace are sized by WV5_BLOCKS_PER_CU");
void launch_wave_kernel5(dim3 grid, hipStream_t s, const Params &P, const WaveParams &W)
{
    hipLaunchKernelGGL(j2t_wave_kernel<5>, grid, dim3(64 * WV_WAVES), (W.hdr.total_len + 15) & ~15u, s, P, W);
}
}  // namespace dg
