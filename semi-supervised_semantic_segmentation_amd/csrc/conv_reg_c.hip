// Register-staged implicit-GEMM launches, group c (fp16) (split from conv.hip for parallel compilation).
#include "conv_kernels.h"

namespace {

template <typename T, typename TO, int BM, int BN, int WM, int WN>
int launch_igemm(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, float* ws, int splits,
                 hipStream_t s) {
  const long long tiles = ((g.M + BM - 1) / BM) * ((g.K + BN - 1) / BN);
  const dim3 grid((unsigned)tiles, (unsigned)splits);
  if (splits > 1) (void)hipMemsetAsync(ws, 0, sizeof(float) * g.M * g.K, s);
  if (ep.stats) {
    if constexpr (sizeof(T) == sizeof(TO))
      hipLaunchKernelGGL((igemm_kernel<T, TO, BM, BN, WM, WN, false, true>), grid, dim3(256), 0, s, (const T*)x,
                         (const T*)w, (TO*)y, g, ep, splits, ws);
    else
      return -1;   // statistics of a compute-dtype activation only
  } else if (g_knobs[0] == 0)
    hipLaunchKernelGGL((igemm_kernel<T, TO, BM, BN, WM, WN, false>), grid, dim3(256), 0, s, (const T*)x, (const T*)w,
                       (TO*)y, g, ep, splits, ws);
  else
    hipLaunchKernelGGL((igemm_kernel<T, TO, BM, BN, WM, WN, true>), grid, dim3(256), 0, s, (const T*)x, (const T*)w,
                       (TO*)y, g, ep, splits, ws);
  if (splits > 1)
    hipLaunchKernelGGL(splitk_finalize_kernel<TO>, dim3(ssseg_grid(g.M * g.K, 256)), dim3(256), 0, s, ws, (TO*)y, g,
                       ep);
  return BM;
}

}  // namespace

template <typename T, typename TO>
int dispatch_regstaged(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, float* ws,
                       hipStream_t s) {
  const long long t128 = ((g.M + 127) / 128) * ((g.K + 127) / 128);
  const bool small = g_knobs[2] == 0 ? (t128 < 512) : (g_knobs[2] > 0);
  if (g.K <= 16)
    return launch_igemm<T, TO, 256, 16, 4, 1>(x, w, y, g, ep, ws, ws ? plan_splits<T, 256, 16>(g) : 1, s);
  if (g.K <= 64 && !small)
    return launch_igemm<T, TO, 256, 64, 4, 1>(x, w, y, g, ep, ws, ws ? plan_splits<T, 256, 64>(g) : 1, s);
  if (small)
    return launch_igemm<T, TO, 64, 64, 2, 2>(x, w, y, g, ep, ws, ws ? plan_splits<T, 64, 64>(g) : 1, s);
  return launch_igemm<T, TO, 128, 128, 2, 2>(x, w, y, g, ep, ws, ws ? plan_splits<T, 128, 128>(g) : 1, s);
}

template int dispatch_regstaged<f16_t, f16_t>(const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&, float*,
                                               hipStream_t);
template int dispatch_regstaged<f16_t, float>(const void*, const void*, void*, const ConvGeom&, const Epi<float>&, float*,
                                              hipStream_t);
