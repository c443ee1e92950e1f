// LDS-DMA implicit-GEMM conv configs, group a (split from conv.hip for parallel compilation).
#include "conv_kernels.h"

template <typename TO>
int launch_glds_grp_a(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2,
                      unsigned x2b) {
  switch (cfg) {
    case 1: return launch_glds<TO, 256, 128, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 2: return launch_glds<TO, 256, 64, 4, 1, 4, 3>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 3: return launch_glds<TO, 128, 128, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    default: return -1;
  }
}

template int launch_glds_grp_a<bf16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&,
                                        unsigned, unsigned, hipStream_t, float*, const PhaseTab*,
                                        const void*, unsigned);
template int launch_glds_grp_a<f16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&,
                                       unsigned, unsigned, hipStream_t, float*, const PhaseTab*,
                                        const void*, unsigned);
