// Depthwise convolution (groups == channels, one R x S filter per channel) over NHWC activations:
// MobileNetV2's ConvBNReLU(hidden, hidden, stride, groups=hidden) (mobilenetv2.py:34-39,58).
// HBM-bound: one thread owns a 16-byte channel chunk (8 bf16 / 4 f32) of one pixel and walks the taps.
//
// Descriptor (ssseg_conv_desc) as for the conv engine with K == C (channels, padded), weights packed
// [R*S][ldw] in the compute dtype (ssseg_weight_pack layout 1 with Kd = 1), no output phases:
//   y[n][oy][ox][c] = act(scale[c] * sum_{r,s} x[n][oy*sy + r*dy + py][ox*sx + s*dx + px][c] * w[r*S+s][c]
//                         + shift[c] + res[...])
//   dgrad: dx[n][iy][ix][c] = sum over (r, s, oy, ox) with iy = oy*sy + r*dy + py ... of dy * w
//   wgrad: dw[c][0][r][s] (+)= sum_{n,oy,ox} dy[n][oy][ox][c] * x[n][iy][ix][c]
// Deterministic: wgrad partials per pixel block are reduced in fixed order.
#include "common.h"

namespace {

template <typename T> struct DV;
template <> struct DV<bf16_t> {
  static constexpr int V = 8;
  __device__ __forceinline__ static void ld(const bf16_t* p, float (&v)[8]) {
    const uint4 q = *(const uint4*)p;
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void st(bf16_t* p, const float (&v)[8]) {
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (unsigned)f32_to_bf16(v[2 * i]) | ((unsigned)f32_to_bf16(v[2 * i + 1]) << 16);
    *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct DV<f16_t> {
  static constexpr int V = 8;
  __device__ __forceinline__ static void ld(const f16_t* p, float (&v)[8]) { H16::ld8(p, v); }
  __device__ __forceinline__ static void st(f16_t* p, const float (&v)[8]) { H16::st8(p, v); }
};
template <> struct DV<float> {
  static constexpr int V = 4;
  __device__ __forceinline__ static void ld(const float* p, float (&v)[4]) {
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[4]) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
};

struct DG {
  int N, H, W, C, ldx, OH, OW, R, S, sy, sx, dy, dx, py, px, ldy, ldw;
};

template <typename T>
__global__ void __launch_bounds__(256) dw_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w, T* __restrict__ y,
                                                     DG g, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, const T* __restrict__ res, int ldr,
                                                     T* __restrict__ aux, int act, float slope) {
  constexpr int V = DV<T>::V;
  const int CV = g.C / V;
  const int total = g.N * g.OH * g.OW * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV, c0 = cv * V;
    int q = i / CV;
    const int ox = q % g.OW;
    q /= g.OW;
    const int oy = q % g.OH, n = q / g.OH;
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int iy = oy * g.sy + r * g.dy + g.py;
      if ((unsigned)iy >= (unsigned)g.H) continue;
      for (int s = 0; s < g.S; ++s) {
        const int ix = ox * g.sx + s * g.dx + g.px;
        if ((unsigned)ix >= (unsigned)g.W) continue;
        float xv[V], wv[V];
        DV<T>::ld(x + ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldx + c0, xv);
        DV<T>::ld(w + (int64_t)(r * g.S + s) * g.ldw + c0, wv);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = fmaf(xv[e], wv[e], acc[e]);
      }
    }
    const int64_t op = (int64_t)(n * g.OH + oy) * g.OW + ox;
    float r8[V];
#pragma unroll
    for (int e = 0; e < V; ++e) r8[e] = 0.f;
    if (res) DV<T>::ld(res + op * ldr + c0, r8);
    if (aux) DV<T>::st(aux + op * g.ldy + c0, acc);
    float o[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      float a = acc[e];
      if (scale) a *= scale[c0 + e];
      if (shift) a += shift[c0 + e];
      o[e] = act_fwd(a + r8[e], act, slope);
    }
    DV<T>::st(y + op * g.ldy + c0, o);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dw_dgrad_kernel(const T* __restrict__ gy, const T* __restrict__ w,
                                                       T* __restrict__ gx, DG g) {
  constexpr int V = DV<T>::V;
  const int CV = g.C / V;
  const int total = g.N * g.H * g.W * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV, c0 = cv * V;
    int q = i / CV;
    const int ix = q % g.W;
    q /= g.W;
    const int iy = q % g.H, n = q / g.H;
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int ty = iy - r * g.dy - g.py;   // = oy * sy
      if (ty < 0 || ty % g.sy) continue;
      const int oy = ty / g.sy;
      if (oy >= g.OH) continue;
      for (int s = 0; s < g.S; ++s) {
        const int tx = ix - s * g.dx - g.px;
        if (tx < 0 || tx % g.sx) continue;
        const int ox = tx / g.sx;
        if (ox >= g.OW) continue;
        float gv[V], wv[V];
        DV<T>::ld(gy + ((int64_t)(n * g.OH + oy) * g.OW + ox) * g.ldy + c0, gv);
        DV<T>::ld(w + (int64_t)(r * g.S + s) * g.ldw + c0, wv);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = fmaf(gv[e], wv[e], acc[e]);
      }
    }
    DV<T>::st(gx + ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldx + c0, acc);
  }
}

constexpr int MAXRS = 49;   // up to 7x7 filters
constexpr int WG_BLOCKS = 256;

// per-block partial weight gradients: part[blk][tap][C]; block = cpb chunk columns x ppb pixel rows
template <typename T>
__global__ void __launch_bounds__(256) dw_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ gy, DG g, int cpb,
                                                       float* __restrict__ part) {
  constexpr int V = DV<T>::V;
  __shared__ float red[256][V + 1];
  const int CV = g.C / V;
  const int t = threadIdx.x;
  const int cl = t % cpb, pl = t / cpb, ppb = 256 / cpb;
  const int cv = blockIdx.y * cpb + cl;
  const bool active = pl < ppb && cv < CV;
  const int c0 = cv * V;
  const int P = g.N * g.OH * g.OW;
  const int RS = g.R * g.S;
  for (int tap = 0; tap < RS; ++tap) {
    const int r = tap / g.S, s = tap - (tap / g.S) * g.S;
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    if (active) {
      for (int p = blockIdx.x * ppb + pl; p < P; p += gridDim.x * ppb) {
        const int ox = p % g.OW, q = p / g.OW, oy = q % g.OH, n = q / g.OH;
        const int iy = oy * g.sy + r * g.dy + g.py, ix = ox * g.sx + s * g.dx + g.px;
        if ((unsigned)iy >= (unsigned)g.H || (unsigned)ix >= (unsigned)g.W) continue;
        float xv[V], gv[V];
        DV<T>::ld(x + ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldx + c0, xv);
        DV<T>::ld(gy + (int64_t)p * g.ldy + c0, gv);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = fmaf(xv[e], gv[e], acc[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) red[t][e] = acc[e];
    __syncthreads();
    for (int idx = t; idx < cpb * V; idx += 256) {
      const int ch = idx / V, e = idx % V;
      const int c = (blockIdx.y * cpb + ch) * V + e;
      if (c >= g.C) continue;
      float sum = 0.f;
      for (int k = 0; k < ppb; ++k) sum += red[k * cpb + ch][e];
      part[((int64_t)blockIdx.x * RS + tap) * g.C + c] = sum;
    }
    __syncthreads();
  }
}

// dw[c][0][r][s] (+)= sum over pixel blocks (fixed order), c < c_real
__global__ void dw_wgrad_reduce_kernel(const float* __restrict__ part, int nblk, int RS, int C, int c_real,
                                       float* __restrict__ dw, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= RS * C) return;
  const int tap = i / C, c = i % C;
  if (c >= c_real) return;
  float s0 = 0.f, s1 = 0.f;
  int b = 0;
  for (; b + 1 < nblk; b += 2) {
    s0 += part[((int64_t)b * RS + tap) * C + c];
    s1 += part[((int64_t)(b + 1) * RS + tap) * C + c];
  }
  if (b < nblk) s0 += part[((int64_t)b * RS + tap) * C + c];
  const int64_t o = (int64_t)c * RS + tap;
  dw[o] = accumulate ? dw[o] + (s0 + s1) : (s0 + s1);
}

bool make_dg(const ssseg_conv_desc* d, DG& g, int dt) {
  if (!d) return false;
  const int64_t v[] = {d->N, d->H, d->W, d->C, d->ldx, d->OH, d->OW, d->K, d->R, d->S, d->ldy, d->ldw};
  for (int64_t e : v)
    if (e < 0 || e > 0x7fffffff) return false;
  if (d->K != d->C || d->outH != d->OH || d->outW != d->OW || d->osy != 1 || d->osx != 1 || d->ooy || d->oox)
    return false;
  const int vec = (dt == SSSEG_F32 ? 4 : 8);
  if (d->C % vec || d->ldx % vec || d->ldy % vec || d->ldw % vec || d->ldw < d->C) return false;
  if (d->R < 1 || d->S < 1 || d->R * d->S > MAXRS || d->sy < 1 || d->sx < 1) return false;
  if (d->N * d->H * d->W * d->ldx >= 0x7fffffffLL || d->N * d->OH * d->OW * d->ldy >= 0x7fffffffLL) return false;
  g = DG{(int)d->N, (int)d->H, (int)d->W, (int)d->C, (int)d->ldx, (int)d->OH, (int)d->OW, (int)d->R, (int)d->S,
         (int)d->sy, (int)d->sx, (int)d->dy, (int)d->dx, (int)d->py, (int)d->px, (int)d->ldy, (int)d->ldw};
  return true;
}

int wgrad_blocks(const DG& g) {
  const int P = g.N * g.OH * g.OW;
  int b = (P + 255) / 256;
  return b < 1 ? 1 : (b > WG_BLOCKS ? WG_BLOCKS : b);
}

}  // namespace

extern "C" int ssseg_dwconv_fwd(const void* x, const void* w, void* y, const ssseg_conv_desc* d, int dt,
                                const ssseg_conv_epilogue* epi, ssseg_stream_t stream) {
  DG g;
  if (!x || !w || !y || !make_dg(d, g, dt)) return SSSEG_EINVAL;
  const ssseg_conv_epilogue none = {nullptr, nullptr, nullptr, 0, nullptr, 0, 0.f};
  const ssseg_conv_epilogue& e = epi ? *epi : none;
  if (e.relu < 0 || e.relu > SSSEG_ACT_LEAKY || (e.residual && (e.ldr < g.C || e.ldr % 8))) return SSSEG_EINVAL;
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  const int64_t total = (int64_t)g.N * g.OH * g.OW * (g.C / V);
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(ssseg_grid(total, 256, 1 << 20)), blk(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(dw_fwd_kernel<bf16_t>, grid, blk, 0, s, (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, g, e.scale,
                       e.shift, (const bf16_t*)e.residual, (int)e.ldr, (bf16_t*)e.aux, e.relu, e.slope);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(dw_fwd_kernel<f16_t>, grid, blk, 0, s, (const f16_t*)x, (const f16_t*)w, (f16_t*)y, g, e.scale,
                       e.shift, (const f16_t*)e.residual, (int)e.ldr, (f16_t*)e.aux, e.relu, e.slope);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(dw_fwd_kernel<float>, grid, blk, 0, s, (const float*)x, (const float*)w, (float*)y, g, e.scale,
                       e.shift, (const float*)e.residual, (int)e.ldr, (float*)e.aux, e.relu, e.slope);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_dwconv_dgrad(const void* dy, const void* w, void* dx, const ssseg_conv_desc* d, int dt,
                                  ssseg_stream_t stream) {
  DG g;
  if (!dy || !w || !dx || !make_dg(d, g, dt)) return SSSEG_EINVAL;
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  const int64_t total = (int64_t)g.N * g.H * g.W * (g.C / V);
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(ssseg_grid(total, 256, 1 << 20)), blk(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(dw_dgrad_kernel<bf16_t>, grid, blk, 0, s, (const bf16_t*)dy, (const bf16_t*)w, (bf16_t*)dx, g);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(dw_dgrad_kernel<f16_t>, grid, blk, 0, s, (const f16_t*)dy, (const f16_t*)w, (f16_t*)dx, g);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(dw_dgrad_kernel<float>, grid, blk, 0, s, (const float*)dy, (const float*)w, (float*)dx, g);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t ssseg_dwconv_wgrad_workspace_bytes(const ssseg_conv_desc* d, int dt) {
  DG g;
  if (!make_dg(d, g, dt)) return 0;
  return (size_t)wgrad_blocks(g) * g.R * g.S * g.C * sizeof(float) + 256;
}

extern "C" int ssseg_dwconv_wgrad(const void* x, const void* dy, float* dw, const ssseg_conv_desc* d, int dt,
                                  int64_t c_real, int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  DG g;
  if (!x || !dy || !dw || !make_dg(d, g, dt) || c_real < 1 || c_real > g.C) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_dwconv_wgrad_workspace_bytes(d, dt)) return SSSEG_EWORKSPACE;
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  const int CV = g.C / V;
  const int cpb = CV < 256 ? CV : 256;
  const int nblk = wgrad_blocks(g);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(nblk, (CV + cpb - 1) / cpb);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(dw_wgrad_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)dy, g, cpb,
                       (float*)ws);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(dw_wgrad_kernel<f16_t>, grid, dim3(256), 0, s, (const f16_t*)x, (const f16_t*)dy, g, cpb,
                       (float*)ws);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(dw_wgrad_kernel<float>, grid, dim3(256), 0, s, (const float*)x, (const float*)dy, g, cpb,
                       (float*)ws);
  else
    return SSSEG_EUNSUPPORTED;
  const int RS = g.R * g.S;
  hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3((RS * g.C + 255) / 256), dim3(256), 0, s, (const float*)ws, nblk, RS,
                     g.C, (int)c_real, dw, accumulate);
  SSSEG_LAUNCH_CHECK();
  return 0;
}
