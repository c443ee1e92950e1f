// LDS-DMA implicit-GEMM conv configs, group b (split from conv.hip for parallel compilation).
#include "conv_kernels.h"

template <typename TO>
int launch_glds_grp_b(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2,
                      unsigned x2b) {
  switch (cfg) {
    case 5: return launch_glds<TO, 64, 64, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 7: return launch_glds<TO, 256, 64, 4, 2, 8, 3>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 8: return launch_glds<TO, 128, 128, 2, 2, 4, 4>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 9: return launch_glds<TO, 128, 64, 2, 2, 4, 4>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 12: return launch_glds<TO, 128, 128, 2, 2, 4, 2>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    default: return -1;
  }
}

template int launch_glds_grp_b<bf16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&,
                                        unsigned, unsigned, hipStream_t, float*, const PhaseTab*,
                                        const void*, unsigned);
template int launch_glds_grp_b<f16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&,
                                       unsigned, unsigned, hipStream_t, float*, const PhaseTab*,
                                        const void*, unsigned);
