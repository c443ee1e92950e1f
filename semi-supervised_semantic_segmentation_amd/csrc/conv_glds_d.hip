// LDS-DMA implicit-GEMM conv configs, group d (split from conv.hip for parallel compilation).
#include "conv_kernels.h"

template <typename TO>
int launch_glds_grp_d(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2,
                      unsigned x2b) {
  switch (cfg) {
    case 4: return launch_glds<TO, 128, 64, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 6: return launch_glds<TO, 256, 128, 4, 2, 8, 3>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    // 8-wave, 2-deep ring configs (round 3): more waves per CU at the LDS of the 4-wave 2-slot tiles
    case 18: return launch_glds<TO, 128, 64, 4, 2, 8, 2>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 19: return launch_glds<TO, 128, 128, 2, 4, 8, 2>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 20: return launch_glds<TO, 256, 64, 4, 2, 8, 2>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    default: return -1;
  }
}

template int launch_glds_grp_d<bf16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&,
                                        unsigned, unsigned, hipStream_t, float*, const PhaseTab*,
                                        const void*, unsigned);
template int launch_glds_grp_d<f16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&,
                                       unsigned, unsigned, hipStream_t, float*, const PhaseTab*,
                                        const void*, unsigned);
