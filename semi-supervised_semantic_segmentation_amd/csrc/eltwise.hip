// HBM-bound elementwise / reduction kernels of the training step:
//   layout + dtype conversion at the model boundary, BCE-with-logits (losses.py:41-48),
//   consistency loss (train.py:97-108), teacher EMA (mean_teacher.py:5-18),
//   clip_grad_norm_ + SGD momentum step (train.py:122-124, default_config.py:151-154).
// Reductions: grid-strided partials in fp64 -> one finalize block (deterministic, no atomics).
#include "common.h"

namespace {

constexpr int RED_BLOCKS = 1024;
constexpr int RED_THREADS = 256;

template <typename TI, typename TO>
__global__ void nchw_to_nhwc_kernel(const TI* x, TO* y, int64_t C, int64_t HW, int64_t Cp, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i % Cp, pix = (i / Cp) % HW, n = i / (Cp * HW);
    const float v = c < C ? io<TI>::ld(x, (n * C + c) * HW + pix) : 0.f;
    io<TO>::st(y, i, v);
  }
}

// one thread per pixel, 8 output channels per store (Cp % 8 == 0): the NCHW planes are read coalesced across
// threads (consecutive pixels), the NHWC row written in 16-byte (bf16 / fp16) or 2 x 16-byte (fp32) stores,
// one 64-bit index division per pixel instead of three per element
template <typename TO> struct St8;
template <> struct St8<bf16_t> {
  __device__ __forceinline__ static void st(bf16_t* p, const float (&v)[8]) {
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (unsigned)f32_to_bf16(v[2 * i]) | ((unsigned)f32_to_bf16(v[2 * i + 1]) << 16);
    *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct St8<f16_t> {
  __device__ __forceinline__ static void st(f16_t* p, const float (&v)[8]) { H16::st8(p, v); }
};
template <> struct St8<float> {
  __device__ __forceinline__ static void st(float* p, const float (&v)[8]) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

template <typename TI, typename TO>
__global__ void nchw_to_nhwc_pix_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t C, int64_t HW,
                                        int64_t Cp, int64_t P) {
  for (int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pix < P; pix += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = pix / HW, p = pix - n * HW;
    const TI* src = x + n * C * HW + p;
    for (int64_t c0 = 0; c0 < Cp; c0 += 8) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = c0 + e < C ? io<TI>::ld(src, (c0 + e) * HW) : 0.f;
      St8<TO>::st(y + pix * Cp + c0, v);
    }
  }
}

template <typename TI, typename TO>
__global__ void nhwc_to_nchw_kernel(const TI* x, TO* y, int64_t C, int64_t HW, int64_t ldc, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = i % HW, c = (i / HW) % C, n = i / (C * HW);
    io<TO>::st(y, i, io<TI>::ld(x, (n * HW + pix) * ldc + c));
  }
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* x, TO* y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    io<TO>::st(y, i, io<TI>::ld(x, i));
}

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.f / (1.f + expf(-x)); }

// ---- BCE with logits ----
__global__ void __launch_bounds__(RED_THREADS) bce_partial_kernel(const float* x, const float* t, int64_t n,
                                                                  double* part) {
  __shared__ double red[RED_THREADS / 64];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i], tt = t[i];
    const float l = fmaxf(v, 0.f) - v * tt + log1pf(expf(-fabsf(v)));
    acc += (double)l;
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(RED_THREADS) bce_final_kernel(const double* part, int nparts, int64_t n, float* out) {
  __shared__ double red[RED_THREADS / 64];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = (float)(acc / (double)n);
}

__global__ void bce_bwd_kernel(const float* x, const float* t, int64_t n, const float* gout, float* gx) {
  const float scale = gout[0] / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gx[i] = (sigmoidf_ref(x[i]) - t[i]) * scale;
}

// ---- consistency loss ----
__global__ void __launch_bounds__(RED_THREADS) cons_partial_kernel(const float* s, const float* t, int64_t C,
                                                                   int64_t HW, int64_t npix, float thr,
                                                                   double* part) {
  __shared__ double red[RED_THREADS / 64];
  double num = 0.0, cnt = 0.0;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < npix; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = q / HW, pix = q % HW;
    const float* sp = s + b * C * HW + pix;
    const float* tp = t + b * C * HW + pix;
    float mx = -INFINITY, d2 = 0.f;
    for (int64_t c = 0; c < C; ++c) {
      const float pt = sigmoidf_ref(tp[c * HW]);
      const float ps = sigmoidf_ref(sp[c * HW]);
      const float d = ps - pt;
      d2 += d * d;
      mx = fmaxf(mx, pt);
    }
    if (mx > thr) {
      num += (double)d2;
      cnt += 1.0;
    }
  }
  num = block_sum(num, red);
  cnt = block_sum(cnt, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = num;
    part[2 * blockIdx.x + 1] = cnt;
  }
}

__global__ void __launch_bounds__(RED_THREADS) cons_final_kernel(const double* part, int nparts, int64_t npix,
                                                                 float* out3) {
  __shared__ double red[RED_THREADS / 64];
  double num = 0.0, cnt = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    num += part[2 * i];
    cnt += part[2 * i + 1];
  }
  num = block_sum(num, red);
  cnt = block_sum(cnt, red);
  if (threadIdx.x == 0) {
    out3[0] = (float)num / (float)cnt;   // 0/0 = NaN when no pixel is confident (train.py:106)
    out3[1] = (float)(cnt / (double)npix);
    out3[2] = (float)cnt;
  }
}

__global__ void cons_bwd_kernel(const float* s, const float* t, int64_t C, int64_t HW, int64_t npix, float thr,
                                const float* out3, const float* gout, float* gs) {
  const float scale = gout[0] / out3[2];
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < npix; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = q / HW, pix = q % HW;
    const float* sp = s + b * C * HW + pix;
    const float* tp = t + b * C * HW + pix;
    float mx = -INFINITY;
    for (int64_t c = 0; c < C; ++c) mx = fmaxf(mx, sigmoidf_ref(tp[c * HW]));
    const float cm = mx > thr ? 1.f : 0.f;
    float* gp = gs + b * C * HW + pix;
    for (int64_t c = 0; c < C; ++c) {
      const float ps = sigmoidf_ref(sp[c * HW]);
      const float pt = sigmoidf_ref(tp[c * HW]);
      gp[c * HW] = 2.f * (ps - pt) * cm * scale * (ps * (1.f - ps));
    }
  }
}

// ---- EMA: t = round(ema*a); ema = fma(p, 1-a, t)  (bit-exact with torch CPU mul_().add_(alpha=)) ----
__global__ void ema_kernel(float* __restrict__ ema, const float* __restrict__ p, int64_t n, float a, float beta) {
  const int64_t n4 = n / 4;
  float4* e4 = reinterpret_cast<float4*>(ema);
  const float4* p4 = reinterpret_cast<const float4*>(p);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 e = e4[i];
    const float4 q = p4[i];
    e.x = fmaf(q.x, beta, __fmul_rn(e.x, a));
    e.y = fmaf(q.y, beta, __fmul_rn(e.y, a));
    e.z = fmaf(q.z, beta, __fmul_rn(e.z, a));
    e.w = fmaf(q.w, beta, __fmul_rn(e.w, a));
    e4[i] = e;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ema[i] = fmaf(p[i], beta, __fmul_rn(ema[i], a));
}

// ---- squared norm ----
__global__ void __launch_bounds__(RED_THREADS) sq_partial_kernel(const float* x, int64_t n, double* part) {
  __shared__ double red[RED_THREADS / 64];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[i];
    acc += v * v;
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(RED_THREADS) sq_final_kernel(const double* part, int nparts, float* out) {
  __shared__ double red[RED_THREADS / 64];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] += (float)acc;
}

// ---- clip + SGD ----
__global__ void sgd_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ buf, bf16_t* shadow,
                           int64_t n, float lr, float mom, float wd, float max_norm, const float* sqnorm, int first,
                           const float* amp) {
  float coef = 1.f;
  if (amp) {   // loss-scaled gradients (fp16 mode): unscale; a non-finite norm skips the whole step
    if (!isfinite(sqnorm[0])) return;
    coef = amp[3];
  }
  if (max_norm > 0.f) {
    const float total = sqrtf(sqnorm[0]) * coef;
    coef *= fminf(max_norm / (total + 1e-6f), 1.f);
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = __fmul_rn(g[i], coef);
    g[i] = gi;
    const float pi = p[i];
    const float d = wd != 0.f ? fmaf(pi, wd, gi) : gi;
    float b;
    if (mom != 0.f) {
      b = first ? d : __fadd_rn(__fmul_rn(buf[i], mom), d);
      buf[i] = b;
    } else {
      b = d;
    }
    const float np = fmaf(b, -lr, pi);
    p[i] = np;
    if (shadow) shadow[i] = f32_to_bf16(np);
  }
}

__global__ void sigmoid_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = sigmoidf_ref(x[i]);
}

__global__ void sigmoid_bwd_kernel(const float* __restrict__ y, const float* __restrict__ gy, float* __restrict__ gx,
                                   int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = y[i];
    gx[i] = gy[i] * (v * (1.f - v));
  }
}

// dynamic loss scale (the fp16 compute mode): state = [scale, growth tracker, found_inf, 1/scale]
__global__ void amp_update_kernel(float* state, const float* sqnorm, float growth, float backoff, int interval) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float sc = state[0];
  if (!isfinite(sqnorm[0])) {
    // floor at 1: a persistently non-finite loss (the reference's 0/0 consistency NaN survives its epoch gate)
    // would otherwise halve S to 0 in ~150 steps, and 1/S = inf then turns the next finite step's update into NaN
    sc = fmaxf(sc * backoff, 1.f);
    state[1] = 0.f;
    state[2] = 1.f;
  } else {
    state[2] = 0.f;
    state[1] += 1.f;
    if (state[1] >= (float)interval) {
      sc *= growth;
      state[1] = 0.f;
    }
  }
  state[0] = sc;
  state[3] = 1.f / sc;
}

__global__ void scale_by_kernel(const float* __restrict__ x, const float* __restrict__ s, float* __restrict__ y,
                                int64_t n) {
  const float a = s[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = x[i] * a;
}

// out = a*x + b*y (y optional): the loss-term arithmetic of the step (weights, 1/virtual batch, epoch gate) and
// its backward, so no framework elementwise kernel runs on the hot path
__global__ void axpby_kernel(const float* __restrict__ x, float a, const float* __restrict__ y, float b,
                             float* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = y ? fmaf(a, x[i], b * y[i]) : a * x[i];
}

__global__ void scale_kernel(float* __restrict__ x, int64_t n, float a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = __fmul_rn(x[i], a);
}

}  // namespace

extern "C" int ssseg_sigmoid_fwd(const float* x, float* y, int64_t n, ssseg_stream_t stream) {
  if (!x || !y || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(sigmoid_fwd_kernel, dim3(ssseg_grid(n, 256)), dim3(256), 0, (hipStream_t)stream, x, y, n);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_sigmoid_bwd(const float* y, const float* gy, float* gx, int64_t n, ssseg_stream_t stream) {
  if (!y || !gy || !gx || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(sigmoid_bwd_kernel, dim3(ssseg_grid(n, 256)), dim3(256), 0, (hipStream_t)stream, y, gy, gx, n);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_amp_update(float* state, const float* sqnorm, float growth, float backoff, int interval,
                                ssseg_stream_t stream) {
  if (!state || !sqnorm || interval < 1) return SSSEG_EINVAL;
  hipLaunchKernelGGL(amp_update_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, state, sqnorm, growth, backoff,
                     interval);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_scale_by(const float* x, const float* s, float* y, int64_t n, ssseg_stream_t stream) {
  if (!x || !s || !y || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(scale_by_kernel, dim3(ssseg_grid(n, 256)), dim3(256), 0, (hipStream_t)stream, x, s, y, n);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_axpby(const float* x, float a, const float* y, float b, float* out, int64_t n,
                           ssseg_stream_t stream) {
  if (!x || !out || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(axpby_kernel, dim3(ssseg_grid(n, 256)), dim3(256), 0, (hipStream_t)stream, x, a, y, b, out, n);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_scale_f32(float* x, int64_t n, float a, ssseg_stream_t stream) {
  if (!x || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(scale_kernel, dim3(ssseg_grid(n, 256, 256 * 8)), dim3(256), 0, (hipStream_t)stream, x, n, a);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t ssseg_reduce_workspace_bytes(int64_t) { return sizeof(double) * 2 * RED_BLOCKS; }

static int red_blocks(int64_t n) { return ssseg_grid(n, RED_THREADS, RED_BLOCKS); }

extern "C" int ssseg_nchw_to_nhwc(const void* x, void* y, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Cp,
                                  int dt_in, int dt_out, ssseg_stream_t stream) {
  if (!x || !y || Cp < C) return SSSEG_EINVAL;
  const int64_t total = N * H * W * Cp;
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (Cp % 8 == 0) {
    const int64_t P = N * H * W;
    const dim3 gp(ssseg_grid(P, 256)), bp(256);
    if (dt_in == SSSEG_F32 && dt_out == SSSEG_BF16)
      hipLaunchKernelGGL((nchw_to_nhwc_pix_kernel<float, bf16_t>), gp, bp, 0, s, (const float*)x, (bf16_t*)y, C, H * W,
                         Cp, P);
    else if (dt_in == SSSEG_F32 && dt_out == SSSEG_F32)
      hipLaunchKernelGGL((nchw_to_nhwc_pix_kernel<float, float>), gp, bp, 0, s, (const float*)x, (float*)y, C, H * W,
                         Cp, P);
    else if (dt_in == SSSEG_F32 && dt_out == SSSEG_F16)
      hipLaunchKernelGGL((nchw_to_nhwc_pix_kernel<float, f16_t>), gp, bp, 0, s, (const float*)x, (f16_t*)y, C, H * W,
                         Cp, P);
    else
      goto generic;
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
generic:
  const dim3 g(ssseg_grid(total, 256)), b(256);
  if (dt_in == SSSEG_F32 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<float, float>), g, b, 0, s, (const float*)x, (float*)y, C, H * W, Cp, total);
  else if (dt_in == SSSEG_F32 && dt_out == SSSEG_BF16)
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<float, bf16_t>), g, b, 0, s, (const float*)x, (bf16_t*)y, C, H * W, Cp, total);
  else if (dt_in == SSSEG_BF16 && dt_out == SSSEG_BF16)
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<bf16_t, bf16_t>), g, b, 0, s, (const bf16_t*)x, (bf16_t*)y, C, H * W, Cp, total);
  else if (dt_in == SSSEG_BF16 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<bf16_t, float>), g, b, 0, s, (const bf16_t*)x, (float*)y, C, H * W, Cp, total);
  else if (dt_in == SSSEG_F32 && dt_out == SSSEG_F16)
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<float, f16_t>), g, b, 0, s, (const float*)x, (f16_t*)y, C, H * W, Cp, total);
  else if (dt_in == SSSEG_F16 && dt_out == SSSEG_F16)
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<f16_t, f16_t>), g, b, 0, s, (const f16_t*)x, (f16_t*)y, C, H * W, Cp, total);
  else if (dt_in == SSSEG_F16 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<f16_t, float>), g, b, 0, s, (const f16_t*)x, (float*)y, C, H * W, Cp, total);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_nhwc_to_nchw(const void* x, void* y, int64_t N, int64_t C, int64_t H, int64_t W, int64_t ldc,
                                  int dt_in, int dt_out, ssseg_stream_t stream) {
  if (!x || !y || ldc < C) return SSSEG_EINVAL;
  const int64_t total = N * H * W * C;
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(ssseg_grid(total, 256)), b(256);
  if (dt_in == SSSEG_F32 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((nhwc_to_nchw_kernel<float, float>), g, b, 0, s, (const float*)x, (float*)y, C, H * W, ldc, total);
  else if (dt_in == SSSEG_BF16 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((nhwc_to_nchw_kernel<bf16_t, float>), g, b, 0, s, (const bf16_t*)x, (float*)y, C, H * W, ldc, total);
  else if (dt_in == SSSEG_F32 && dt_out == SSSEG_BF16)
    hipLaunchKernelGGL((nhwc_to_nchw_kernel<float, bf16_t>), g, b, 0, s, (const float*)x, (bf16_t*)y, C, H * W, ldc, total);
  else if (dt_in == SSSEG_BF16 && dt_out == SSSEG_BF16)
    hipLaunchKernelGGL((nhwc_to_nchw_kernel<bf16_t, bf16_t>), g, b, 0, s, (const bf16_t*)x, (bf16_t*)y, C, H * W, ldc, total);
  else if (dt_in == SSSEG_F16 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((nhwc_to_nchw_kernel<f16_t, float>), g, b, 0, s, (const f16_t*)x, (float*)y, C, H * W, ldc, total);
  else if (dt_in == SSSEG_F32 && dt_out == SSSEG_F16)
    hipLaunchKernelGGL((nhwc_to_nchw_kernel<float, f16_t>), g, b, 0, s, (const float*)x, (f16_t*)y, C, H * W, ldc, total);
  else if (dt_in == SSSEG_F16 && dt_out == SSSEG_F16)
    hipLaunchKernelGGL((nhwc_to_nchw_kernel<f16_t, f16_t>), g, b, 0, s, (const f16_t*)x, (f16_t*)y, C, H * W, ldc, total);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_cast(const void* x, void* y, int64_t n, int dt_in, int dt_out, ssseg_stream_t stream) {
  if (!x || !y || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(ssseg_grid(n, 256)), b(256);
  if (dt_in == SSSEG_F32 && dt_out == SSSEG_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16_t>), g, b, 0, s, (const float*)x, (bf16_t*)y, n);
  else if (dt_in == SSSEG_BF16 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((cast_kernel<bf16_t, float>), g, b, 0, s, (const bf16_t*)x, (float*)y, n);
  else if (dt_in == SSSEG_F32 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), g, b, 0, s, (const float*)x, (float*)y, n);
  else if (dt_in == SSSEG_BF16 && dt_out == SSSEG_BF16)
    hipLaunchKernelGGL((cast_kernel<bf16_t, bf16_t>), g, b, 0, s, (const bf16_t*)x, (bf16_t*)y, n);
  else if (dt_in == SSSEG_F32 && dt_out == SSSEG_F16)
    hipLaunchKernelGGL((cast_kernel<float, f16_t>), g, b, 0, s, (const float*)x, (f16_t*)y, n);
  else if (dt_in == SSSEG_F16 && dt_out == SSSEG_F32)
    hipLaunchKernelGGL((cast_kernel<f16_t, float>), g, b, 0, s, (const f16_t*)x, (float*)y, n);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bce_logits_fwd(const float* x, const float* t, int64_t n, float* loss_out, void* ws,
                                    size_t ws_bytes, ssseg_stream_t stream) {
  if (!x || !t || !loss_out || n <= 0) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_reduce_workspace_bytes(n)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int nb = red_blocks(n);
  hipLaunchKernelGGL(bce_partial_kernel, dim3(nb), dim3(RED_THREADS), 0, s, x, t, n, (double*)ws);
  hipLaunchKernelGGL(bce_final_kernel, dim3(1), dim3(RED_THREADS), 0, s, (const double*)ws, nb, n, loss_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bce_logits_bwd(const float* x, const float* t, int64_t n, const float* gout, float* gx,
                                    ssseg_stream_t stream) {
  if (!x || !t || !gout || !gx || n <= 0) return SSSEG_EINVAL;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3(ssseg_grid(n, 256)), dim3(256), 0, (hipStream_t)stream, x, t, n, gout, gx);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_consistency_fwd(const float* s, const float* t, int64_t B, int64_t C, int64_t HW, float thr,
                                     float* out3, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!s || !t || !out3 || B <= 0 || C <= 0 || HW <= 0) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_reduce_workspace_bytes(B * HW)) return SSSEG_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int64_t npix = B * HW;
  const int nb = red_blocks(npix);
  hipLaunchKernelGGL(cons_partial_kernel, dim3(nb), dim3(RED_THREADS), 0, st, s, t, C, HW, npix, thr, (double*)ws);
  hipLaunchKernelGGL(cons_final_kernel, dim3(1), dim3(RED_THREADS), 0, st, (const double*)ws, nb, npix, out3);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_consistency_bwd(const float* s, const float* t, int64_t B, int64_t C, int64_t HW, float thr,
                                     const float* out3, const float* gout, float* gs, ssseg_stream_t stream) {
  if (!s || !t || !out3 || !gout || !gs || B <= 0 || C <= 0 || HW <= 0) return SSSEG_EINVAL;
  const int64_t npix = B * HW;
  hipLaunchKernelGGL(cons_bwd_kernel, dim3(ssseg_grid(npix, 256)), dim3(256), 0, (hipStream_t)stream, s, t, C, HW,
                     npix, thr, out3, gout, gs);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_ema_update(float* ema, const float* param, int64_t n, double alpha, ssseg_stream_t stream) {
  if (!ema || !param || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  if ((((uintptr_t)ema) | ((uintptr_t)param)) & 15) return SSSEG_EINVAL;
  const float a = (float)alpha, beta = (float)(1.0 - alpha);
  hipLaunchKernelGGL(ema_kernel, dim3(ssseg_grid(n / 4 + 1, 256, 256 * 8)), dim3(256), 0, (hipStream_t)stream, ema,
                     param, n, a, beta);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_sqnorm_accum(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes,
                                  ssseg_stream_t stream) {
  if (!x || !out || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  if (!ws || ws_bytes < ssseg_reduce_workspace_bytes(n)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int nb = red_blocks(n);
  hipLaunchKernelGGL(sq_partial_kernel, dim3(nb), dim3(RED_THREADS), 0, s, x, n, (double*)ws);
  hipLaunchKernelGGL(sq_final_kernel, dim3(1), dim3(RED_THREADS), 0, s, (const double*)ws, nb, out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_sgd_step(float* param, float* grad, float* momentum_buf, uint16_t* bf16_shadow, int64_t n,
                              float lr, float momentum, float weight_decay, float max_norm, const float* sqnorm,
                              int first_step, const float* amp_state, ssseg_stream_t stream) {
  if (!param || !grad || n < 0 || (momentum != 0.f && !momentum_buf) || ((max_norm > 0.f || amp_state) && !sqnorm))
    return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(sgd_kernel, dim3(ssseg_grid(n, 256, 256 * 8)), dim3(256), 0, (hipStream_t)stream, param, grad,
                     momentum_buf, (bf16_t*)bf16_shadow, n, lr, momentum, weight_decay, max_norm, sqnorm,
                     first_step, amp_state);
  SSSEG_LAUNCH_CHECK();
  return 0;
}
