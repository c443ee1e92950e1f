// LDS-DMA implicit-GEMM conv configs, group e: large 8-wave tiles (split from conv.hip for parallel compilation).
#include "conv_kernels.h"

template <typename TO>
int launch_glds_grp_e(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2,
                      unsigned x2b) {
  switch (cfg) {
    // large 8-wave tiles (64x64 or 128x64 per wave): fewer LDS-DMA bytes per flop
    case 21: return launch_glds<TO, 256, 128, 4, 2, 8, 2>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 22: return launch_glds<TO, 256, 256, 2, 4, 8, 2>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 23: return launch_glds<TO, 128, 256, 2, 4, 8, 2>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    default: return -1;
  }
}

template int launch_glds_grp_e<bf16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&,
                                        unsigned, unsigned, hipStream_t, float*, const PhaseTab*,
                                        const void*, unsigned);
template int launch_glds_grp_e<f16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&,
                                       unsigned, unsigned, hipStream_t, float*, const PhaseTab*,
                                        const void*, unsigned);
