// BatchNorm2d (training + eval) over NHWC activations, with fused ReLU and residual add, gfx950.
// Reference call sites: every ConvBlock (unet.py:9, simple_unet.py:116), the ResNet-50 encoder and
// SyncBatchNorm (distributed_trainer.py:36).  Training statistics are produced as fp64 (sum, sumsq)
// per channel so that SyncBN can all-reduce them (RCCL) before ssseg_bn_finalize.
//
//   stats:    sums[c] = sum_p x, sums[C+c] = sum_p x^2                    (2-stage, deterministic)
//   finalize: mean, invstd = 1/sqrt(var_biased + eps); running = (1-m)*running + m*{mean, var_unbiased}
//   apply:    y = act(gamma*(x-mean)*invstd + beta [+ residual])
//   bwd:      reduce  sums[c] = sum dyr, sums[C+c] = sum dyr*xhat,  dyr = dy*[y>0] (y recomputed)
//             apply   dx = gamma*invstd*(dyr - (sum_dyr + xhat*sum_dyr_xhat)/count)   (train)
//                     dx = gamma*invstd*dyr                                            (eval)
//             dres = dyr (residual branch gradient)
#include "common.h"

namespace {

constexpr int CH = 4;   // channels per thread chunk

template <typename T> struct V4;
template <> struct V4<float> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[4]) {
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[4]) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
};
template <> struct V4<bf16_t> {
  __device__ __forceinline__ static void ld(const bf16_t* p, float (&v)[4]) {
    const uint2 q = *(const uint2*)p;
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  }
  __device__ __forceinline__ static void st(bf16_t* p, const float (&v)[4]) {
    uint2 u;
    u.x = (unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16);
    u.y = (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16);
    *(uint2*)p = u;
  }
};

struct Layout {
  int cpb;        // chunks per block row (<= 256)
  int ppb;        // pixels per block iteration
  int cblocks;    // blocks along channels
};

static Layout layout_for(int64_t C) {
  Layout l;
  const int nch = (int)(C / CH);
  l.cpb = nch < 256 ? nch : 256;
  l.ppb = 256 / l.cpb;
  l.cblocks = (nch + l.cpb - 1) / l.cpb;
  return l;
}

constexpr int MAXG = 256;   // partial blocks along pixels

// per-block partial sums of 2 per-channel quantities; mode 0: (x, x^2); mode 1: (dyr, dyr*xhat)
template <typename T, int MODE>
__global__ void __launch_bounds__(256) bn_partial_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         const T* __restrict__ res, int64_t P, int C, int64_t ldx,
                                                         int64_t lddy, int64_t ldr, Layout L, const float* mean,
                                                         const float* invstd, const float* gamma, const float* beta,
                                                         int relu, double* part) {
  __shared__ double red[2][256][CH];
  const int t = threadIdx.x;
  const int cl = t % L.cpb, pl = t / L.cpb;
  const int chunk = blockIdx.y * L.cpb + cl;
  const int c0 = chunk * CH;
  const bool active = pl < L.ppb && c0 < C;
  double s1[CH] = {0, 0, 0, 0}, s2[CH] = {0, 0, 0, 0};
  if (active) {
    float mu[CH], is[CH], ga[CH], be[CH];
    if (MODE == 1) {
#pragma unroll
      for (int e = 0; e < CH; ++e) {
        mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e];
        ga[e] = gamma ? gamma[c0 + e] : 1.f; be[e] = beta ? beta[c0 + e] : 0.f;
      }
    }
    for (int64_t p = (int64_t)blockIdx.x * L.ppb + pl; p < P; p += (int64_t)gridDim.x * L.ppb) {
      float v[CH];
      V4<T>::ld(x + p * ldx + c0, v);
      if (MODE == 0) {
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          s1[e] += (double)v[e];
          s2[e] += (double)v[e] * (double)v[e];
        }
      } else {
        float g[CH];
        V4<T>::ld(dy + p * lddy + c0, g);
        float r[CH] = {0, 0, 0, 0};
        if (res && relu) V4<T>::ld(res + p * ldr + c0, r);
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          const float xh = (v[e] - mu[e]) * is[e];
          float gr = g[e];
          if (relu) {
            const float yv = fmaf(ga[e], xh, be[e]) + r[e];
            gr = yv > 0.f ? gr : 0.f;
          }
          s1[e] += (double)gr;
          s2[e] += (double)gr * (double)xh;
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < CH; ++e) {
    red[0][t][e] = s1[e];
    red[1][t][e] = s2[e];
  }
  __syncthreads();
  if (t < L.cpb && c0 < C) {
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      double a = 0, b = 0;
      for (int k = 0; k < L.ppb; ++k) {
        a += red[0][k * L.cpb + t][e];
        b += red[1][k * L.cpb + t][e];
      }
      part[((int64_t)blockIdx.x * 2) * C + c0 + e] = a;
      part[((int64_t)blockIdx.x * 2 + 1) * C + c0 + e] = b;
    }
  }
}

// sums over the per-block partials: block = 32 channels x 8 partial lanes
__global__ void __launch_bounds__(256) bn_partial_final_kernel(const double* part, int nparts, int C, double* sums) {
  __shared__ double red[2][8][32];
  const int cl = threadIdx.x & 31, pl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double a = 0, b = 0;
  if (c < C) {
    for (int i = pl; i < nparts; i += 8) {
      a += part[(int64_t)(2 * i) * C + c];
      b += part[(int64_t)(2 * i + 1) * C + c];
    }
  }
  red[0][pl][cl] = a;
  red[1][pl][cl] = b;
  __syncthreads();
  if (pl == 0 && c < C) {
    for (int k = 1; k < 8; ++k) {
      a += red[0][k][cl];
      b += red[1][k][cl];
    }
    sums[c] = a;
    sums[C + c] = b;
  }
}

__global__ void bn_finalize_kernel(const double* sums, int C, double count, float eps, float momentum, float* mean_out,
                                   float* invstd_out, float* rmean, float* rvar, int64_t* nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) *nbt += 1;
  if (c >= C) return;
  const double mean = sums[c] / count;
  double var = sums[C + c] / count - mean * mean;
  var = var < 0 ? 0 : var;
  mean_out[c] = (float)mean;
  invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
  }
}

__global__ void bn_eval_params_kernel(const float* rmean, const float* rvar, float eps, int C, float* mean_out,
                                      float* invstd_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean_out[c] = rmean[c];
  invstd_out[c] = 1.f / sqrtf(rvar[c] + eps);
}

template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y, int64_t P, int C,
                                int64_t ldx, int64_t ldr, int64_t ldy, const float* mean, const float* invstd,
                                const float* gamma, const float* beta, int relu) {
  const int nch = C / CH;
  const int64_t total = P * nch;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % nch) * CH;
    const int64_t p = i / nch;
    float v[CH], r[CH] = {0, 0, 0, 0};
    V4<T>::ld(x + p * ldx + c0, v);
    if (res) V4<T>::ld(res + p * ldr + c0, r);
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const float xh = (v[e] - mean[c0 + e]) * invstd[c0 + e];
      float o = fmaf(gamma ? gamma[c0 + e] : 1.f, xh, beta ? beta[c0 + e] : 0.f) + r[e];
      if (relu) o = fmaxf(o, 0.f);
      v[e] = o;
    }
    V4<T>::st(y + p * ldy + c0, v);
  }
}

template <typename T>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ res,
                                    T* __restrict__ dx, T* __restrict__ dres, int64_t P, int C, int64_t ldx,
                                    int64_t ldr, int64_t lddy, int64_t lddx, const float* mean, const float* invstd,
                                    const float* gamma, const float* beta, int relu, int train, const double* sums,
                                    double count) {
  const int nch = C / CH;
  const int64_t total = P * nch;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % nch) * CH;
    const int64_t p = i / nch;
    float v[CH], g[CH], r[CH] = {0, 0, 0, 0}, o[CH], od[CH];
    V4<T>::ld(x + p * ldx + c0, v);
    V4<T>::ld(dy + p * lddy + c0, g);
    if (res && relu) V4<T>::ld(res + p * ldr + c0, r);
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int c = c0 + e;
      const float is = invstd[c], ga = gamma ? gamma[c] : 1.f;
      const float xh = (v[e] - mean[c]) * is;
      float gr = g[e];
      if (relu) gr = (fmaf(ga, xh, beta ? beta[c] : 0.f) + r[e]) > 0.f ? gr : 0.f;
      od[e] = gr;
      float d = gr;
      if (train) {
        const float mdy = (float)(sums[c] / count), mdyx = (float)(sums[C + c] / count);
        d = gr - mdy - xh * mdyx;
      }
      o[e] = ga * is * d;
    }
    V4<T>::st(dx + p * lddx + c0, o);
    if (dres) V4<T>::st(dres + p * lddx + c0, od);
  }
}

__global__ void bn_param_grad_kernel(const double* sums, int C, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dbeta) dbeta[c] += (float)sums[c];
  if (dgamma) dgamma[c] += (float)sums[C + c];
}

template <typename T, int MODE>
int run_partials(const T* x, const T* dy, const T* res, int64_t P, int64_t C, int64_t ldx, int64_t lddy, int64_t ldr,
                 const float* mean, const float* invstd, const float* gamma, const float* beta, int relu,
                 double* sums, void* ws, hipStream_t s) {
  const Layout L = layout_for(C);
  int64_t gx = (P + (int64_t)L.ppb * 16 - 1) / ((int64_t)L.ppb * 16);
  gx = gx < 1 ? 1 : (gx > MAXG ? MAXG : gx);
  hipLaunchKernelGGL((bn_partial_kernel<T, MODE>), dim3((unsigned)gx, L.cblocks), dim3(256), 0, s, x, dy, res, P,
                     (int)C, ldx, lddy, ldr, L, mean, invstd, gamma, beta, relu, (double*)ws);
  hipLaunchKernelGGL(bn_partial_final_kernel, dim3((C + 31) / 32), dim3(256), 0, s, (const double*)ws, (int)gx,
                     (int)C, sums);
  return 0;
}

}  // namespace

extern "C" size_t ssseg_bn_workspace_bytes(int64_t C) { return sizeof(double) * 2 * MAXG * (size_t)C + 256; }

extern "C" int ssseg_bn_stats(const void* x, int64_t P, int64_t C, int64_t ldx, int dt, double* sums, void* ws,
                              size_t ws_bytes, ssseg_stream_t stream) {
  if (!x || !sums || P < 1 || C < 1 || C % CH || ldx % CH) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_bn_workspace_bytes(C)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (dt == SSSEG_BF16)
    run_partials<bf16_t, 0>((const bf16_t*)x, nullptr, nullptr, P, C, ldx, 0, 0, nullptr, nullptr, nullptr, nullptr, 0,
                            sums, ws, s);
  else if (dt == SSSEG_F32)
    run_partials<float, 0>((const float*)x, nullptr, nullptr, P, C, ldx, 0, 0, nullptr, nullptr, nullptr, nullptr, 0,
                           sums, ws, s);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_finalize(const double* sums, int64_t C, double count, float eps, float momentum, float* mean_out,
                                 float* invstd_out, float* running_mean, float* running_var,
                                 int64_t* num_batches_tracked, ssseg_stream_t stream) {
  if (!sums || !mean_out || !invstd_out || C < 1 || count <= 0) return SSSEG_EINVAL;
  if ((running_mean == nullptr) != (running_var == nullptr)) return SSSEG_EINVAL;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, (int)C, count,
                     eps, momentum, mean_out, invstd_out, running_mean, running_var, num_batches_tracked);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_eval_params(const float* running_mean, const float* running_var, float eps, int64_t C,
                                    float* mean_out, float* invstd_out, ssseg_stream_t stream) {
  if (!running_mean || !running_var || !mean_out || !invstd_out || C < 1) return SSSEG_EINVAL;
  hipLaunchKernelGGL(bn_eval_params_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, running_mean,
                     running_var, eps, (int)C, mean_out, invstd_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_apply(const void* x, const void* residual, void* y, int64_t P, int64_t C, int64_t ldx,
                              int64_t ldr, int64_t ldy, const float* mean, const float* invstd, const float* gamma,
                              const float* beta, int relu, int dt, ssseg_stream_t stream) {
  if (!x || !y || !mean || !invstd || P < 1 || C < 1 || C % CH || ldx % CH || ldy % CH || (residual && ldr % CH))
    return SSSEG_EINVAL;
  const int64_t total = P * (C / CH);
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(ssseg_grid(total, 256, 256 * 16)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<bf16_t>, g, b, 0, s, (const bf16_t*)x, (const bf16_t*)residual, (bf16_t*)y, P,
                       (int)C, ldx, ldr, ldy, mean, invstd, gamma, beta, relu);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(bn_apply_kernel<float>, g, b, 0, s, (const float*)x, (const float*)residual, (float*)y, P,
                       (int)C, ldx, ldr, ldy, mean, invstd, gamma, beta, relu);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_bwd_reduce(const void* dy, const void* x, const void* residual, int64_t P, int64_t C,
                                   int64_t ldx, int64_t ldr, int64_t lddy, const float* mean, const float* invstd,
                                   const float* gamma, const float* beta, int relu, int dt, double* sums, void* ws,
                                   size_t ws_bytes, ssseg_stream_t stream) {
  if (!dy || !x || !sums || !mean || !invstd || P < 1 || C < 1 || C % CH || ldx % CH || lddy % CH) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_bn_workspace_bytes(C)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (dt == SSSEG_BF16)
    run_partials<bf16_t, 1>((const bf16_t*)x, (const bf16_t*)dy, (const bf16_t*)residual, P, C, ldx, lddy, ldr, mean,
                            invstd, gamma, beta, relu, sums, ws, s);
  else if (dt == SSSEG_F32)
    run_partials<float, 1>((const float*)x, (const float*)dy, (const float*)residual, P, C, ldx, lddy, ldr, mean,
                           invstd, gamma, beta, relu, sums, ws, s);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_param_grad(const double* sums, int64_t C, float* dgamma, float* dbeta, ssseg_stream_t stream) {
  if (!sums || C < 1) return SSSEG_EINVAL;
  if (!dgamma && !dbeta) return 0;
  hipLaunchKernelGGL(bn_param_grad_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, (int)C,
                     dgamma, dbeta);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_bwd_apply(const void* dy, const void* x, const void* residual, void* dx, void* dres, int64_t P,
                                  int64_t C, int64_t ldx, int64_t ldr, int64_t lddy, int64_t lddx, const float* mean,
                                  const float* invstd, const float* gamma, const float* beta, int relu, int train,
                                  const double* sums, double count, int dt, ssseg_stream_t stream) {
  if (!dy || !x || !dx || !mean || !invstd || P < 1 || C < 1 || C % CH || (train && (!sums || count <= 0)))
    return SSSEG_EINVAL;
  const int64_t total = P * (C / CH);
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(ssseg_grid(total, 256, 256 * 16)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16_t>, g, b, 0, s, (const bf16_t*)dy, (const bf16_t*)x,
                       (const bf16_t*)residual, (bf16_t*)dx, (bf16_t*)dres, P, (int)C, ldx, ldr, lddy, lddx, mean,
                       invstd, gamma, beta, relu, train, sums, count);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, g, b, 0, s, (const float*)dy, (const float*)x,
                       (const float*)residual, (float*)dx, (float*)dres, P, (int)C, ldx, ldr, lddy, lddx, mean,
                       invstd, gamma, beta, relu, train, sums, count);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}
