// LDS-DMA implicit-GEMM conv configs, group d (split from conv.hip for parallel compilation).
#include "conv_kernels.h"

template <typename TO>
int launch_glds_grp_d(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph) {
  switch (cfg) {
    case 4: return launch_glds<TO, 128, 64, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s, ws, ph);
    case 6: return launch_glds<TO, 256, 128, 4, 2, 8, 3>(x, w, y, g, ep, xb, wb, s, ws, ph);
    default: return -1;
  }
}

template int launch_glds_grp_d<bf16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&,
                                        unsigned, unsigned, hipStream_t, float*, const PhaseTab*);
template int launch_glds_grp_d<f16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&,
                                       unsigned, unsigned, hipStream_t, float*, const PhaseTab*);
