// Average pooling, global average pooling, n-ary add (+activation), dropout and the multi-scale attention
// blend — the remaining non-conv primitives of the C3-C5 model families, gfx950.
//   AvgPool2d(2, 2)                       hardnet.py:157
//   AdaptiveAvgPool2d(1) (ASPP pooling)   torchvision DeepLabV3 head behind deeplabv3.py:9,43
//   sum of fused branches (+ ReLU)        higher_hrnet.py:473-486 (TransitionFuse add / add_relu)
//   Dropout(0.5) (ASPP projection)        torchvision DeepLabV3 head
//   up(lo)*sigmoid(a) + hi*(1-sigmoid(a)) multiscale_attention.py:52-54
// NHWC activations are processed in 16-byte channel chunks (8 bf16 / 4 f32; the physical channel count is a
// multiple of the chunk), so every activation load and store is a full dwordx4.
#include "common.h"

namespace {

template <typename T> struct CV16;
template <> struct CV16<bf16_t> {
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
template <> struct CV16<f16_t> {
  static constexpr int V = 8;
  __device__ __forceinline__ static void ld(const f16_t* p, float (&v)[8]) { H16::ld8(p, v); }
  __device__ __forceinline__ static void st(f16_t* p, const float (&v)[8]) { H16::st8(p, v); }
};
template <> struct CV16<float> {
  static constexpr int V = 4;
  __device__ __forceinline__ static void ld(const float* p, float (&v)[4]) {
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[4]) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
};

// ---- AvgPool2d(k, s, p), ceil_mode False, count_include_pad True (PyTorch's defaults) --------------------
// divisor = window clipped to the padded map [-p, H+p) (PyTorch avg_pool2d); taps summed in (kh, kw) order
// in fp32, then one division — the order of the CPU kernel.
template <typename T>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int OH,
                                   int OW, int k, int s, int p) {
  constexpr int V = CV16<T>::V;
  const int CV = C / V;
  const int total = N * OH * OW * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int q = i / CV;
    const int ow = q % OW;
    q /= OW;
    const int oh = q % OH, n = q / OH;
    int hs = oh * s - p, ws = ow * s - p;
    int he = min(hs + k, H + p), we = min(ws + k, W + p);
    const float div = (float)((he - hs) * (we - ws));
    hs = max(hs, 0);
    ws = max(ws, 0);
    he = min(he, H);
    we = min(we, W);
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int ih = hs; ih < he; ++ih)
      for (int iw = ws; iw < we; ++iw) {
        float v[V];
        CV16<T>::ld(x + ((int64_t)(n * H + ih) * W + iw) * C + cv * V, v);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += v[e];
      }
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = acc[e] / div;
    CV16<T>::st(y + (int64_t)i * V, acc);
  }
}

// gx[ih][iw] = sum over the windows covering (ih, iw) of gy / divisor (deterministic gather)
template <typename T>
__global__ void avgpool_bwd_kernel(const T* __restrict__ gy, T* __restrict__ gx, int N, int H, int W, int C, int OH,
                                   int OW, int k, int s, int p) {
  constexpr int V = CV16<T>::V;
  const int CV = C / V;
  const int total = N * H * W * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int q = i / CV;
    const int iw = q % W;
    q /= W;
    const int ih = q % H, n = q / H;
    const int oh0 = max(0, (ih + p - k + s) / s), oh1 = min(OH - 1, (ih + p) / s);
    const int ow0 = max(0, (iw + p - k + s) / s), ow1 = min(OW - 1, (iw + p) / s);
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int hs = oh * s - p;
      if (ih < hs || ih >= hs + k) continue;
      const int hdiv = min(hs + k, H + p) - hs;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int ws = ow * s - p;
        if (iw < ws || iw >= ws + k) continue;
        const float div = (float)(hdiv * (min(ws + k, W + p) - ws));
        float g[V];
        CV16<T>::ld(gy + ((int64_t)(n * OH + oh) * OW + ow) * C + cv * V, g);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += g[e] / div;
      }
    }
    CV16<T>::st(gx + (int64_t)i * V, acc);
  }
}

// ---- AdaptiveAvgPool2d(1): y[n][c] = mean over the HW pixels ------------------------------------------------
// pass 1: grid (N, groups of 64 channel chunks, pixel splits); 256 threads = 64 chunks x 4 pixel rows, fp32
// partial sums per (n, split, channel); pass 2 sums the splits in fixed order (deterministic) and divides.
constexpr int GAP_SPLITS_MAX = 64;

template <typename T>
__global__ void __launch_bounds__(256) gap_partial_kernel(const T* __restrict__ x, float* __restrict__ part, int HW,
                                                          int C, int splits) {
  constexpr int V = CV16<T>::V;
  __shared__ float red[4][64][V];
  const int t = threadIdx.x, cl = t & 63, row = t >> 6;
  const int n = blockIdx.x, sp = blockIdx.z;
  const int c0 = (blockIdx.y * 64 + cl) * V;
  const int per = (HW + splits - 1) / splits;
  const int p0 = sp * per, p1 = min(HW, p0 + per);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  if (c0 < C) {
    const T* xb = x + (int64_t)n * HW * C + c0;
    int pix = p0 + row;
    for (; pix + 12 < p1; pix += 16) {   // 4 independent loads in flight
      float a[V], b[V], c[V], d[V];
      CV16<T>::ld(xb + (int64_t)pix * C, a);
      CV16<T>::ld(xb + (int64_t)(pix + 4) * C, b);
      CV16<T>::ld(xb + (int64_t)(pix + 8) * C, c);
      CV16<T>::ld(xb + (int64_t)(pix + 12) * C, d);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += (a[e] + b[e]) + (c[e] + d[e]);
    }
    for (; pix < p1; pix += 4) {
      float a[V];
      CV16<T>::ld(xb + (int64_t)pix * C, a);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += a[e];
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) red[row][cl][e] = acc[e];
  __syncthreads();
  if (row == 0 && c0 < C) {
    float* o = part + ((int64_t)n * splits + sp) * C + c0;
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = (red[0][cl][e] + red[1][cl][e]) + (red[2][cl][e] + red[3][cl][e]);
  }
}

template <typename T>
__global__ void gap_final_kernel(const float* __restrict__ part, T* __restrict__ y, int N, int C, int splits,
                                 float inv_hw, int64_t ldy) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i % C;
  float s = 0.f;
  for (int sp = 0; sp < splits; ++sp) s += part[((int64_t)n * splits + sp) * C + c];
  io<T>::st(y, (int64_t)n * ldy + c, s * inv_hw);
}

template <typename T>
__global__ void gap_bwd_kernel(const T* __restrict__ gy, T* __restrict__ gx, int N, int HW, int C, int64_t ldgy,
                               float inv_hw) {
  constexpr int V = CV16<T>::V;
  const int CV = C / V;
  const int64_t total = (int64_t)N * HW * CV;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    const int n = (int)(i / ((int64_t)HW * CV));
    float g[V];
    CV16<T>::ld(gy + (int64_t)n * ldgy + cv * V, g);
#pragma unroll
    for (int e = 0; e < V; ++e) g[e] *= inv_hw;
    CV16<T>::st(gx + i * V, g);
  }
}

// ---- y = act(x0 + x1 + ... + x_{n-1}), summed left to right in fp32 (the reference's add chain) --------------
struct Ptr8 {
  const void* p[8];
};

template <typename T>
__global__ void add_n_kernel(Ptr8 xs, int n, T* __restrict__ y, int64_t nchunks, int act, float slope) {
  constexpr int V = CV16<T>::V;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nchunks; i += (int64_t)gridDim.x * blockDim.x) {
    float acc[V];
    CV16<T>::ld((const T*)xs.p[0] + i * V, acc);
    for (int j = 1; j < n; ++j) {
      float v[V];
      CV16<T>::ld((const T*)xs.p[j] + i * V, v);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = act_fwd(acc[e], act, slope);
    CV16<T>::st(y + i * V, acc);
  }
}

// ---- Dropout: keep with probability 1-p, kept values scaled by 1/(1-p) -----------------------------------------
// Counter-based (Philox-4x32-10, counter = offset + i/4, key = seed): the backward regenerates the same mask
// from (seed, offset), so no mask is stored.
__device__ __forceinline__ void philox4(unsigned (&c)[4], uint64_t seed) {
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const unsigned hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
    const unsigned hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
    const unsigned n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n4, float p, float scale,
                               uint64_t seed, uint64_t offset, const unsigned long long* __restrict__ offset_dev) {
  if (offset_dev) offset = (uint64_t)*offset_dev;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t ctr = offset + (uint64_t)q;
    unsigned c[4] = {(unsigned)ctr, (unsigned)(ctr >> 32), 0x5eedu, 0u};
    philox4(c, seed);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float u = (float)(c[e] >> 8) * (1.0f / 16777216.0f);
      const float v = io<T>::ld(x, q * 4 + e);
      io<T>::st(y, q * 4 + e, u >= p ? v * scale : 0.f);
    }
  }
}

// ---- multi-scale attention blend (fp32, arbitrary 4-D strides) ------------------------------------------------
struct S4 {
  int64_t n, c, h, w;
};

__device__ __forceinline__ float sigmoidf_(float a) { return 1.f / (1.f + expf(-a)); }

__global__ void att_blend_fwd_kernel(const float* __restrict__ lo, S4 ls, const float* __restrict__ hi, S4 hs,
                                     const float* __restrict__ att, S4 as, float* __restrict__ out, int N, int C, int H,
                                     int W) {
  const int64_t total = (int64_t)N * C * H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    int64_t q = i / W;
    const int h = (int)(q % H);
    q /= H;
    const int c = (int)(q % C), n = (int)(q / C);
    const float s = sigmoidf_(att[n * as.n + h * as.h + w * as.w]);
    const float l = lo[n * ls.n + c * ls.c + h * ls.h + w * ls.w], r = hi[n * hs.n + c * hs.c + h * hs.h + w * hs.w];
    out[i] = __fadd_rn(__fmul_rn(l, s), __fmul_rn(r, __fsub_rn(1.f, s)));   // out*m + hi*(1-m), no contraction
  }
}

// one thread per pixel: glo = g*s, ghi = g*(1-s), gatt = sum_c (g*lo - g*hi) * (1-s)*s
__global__ void att_blend_bwd_kernel(const float* __restrict__ g, S4 gs, const float* __restrict__ lo, S4 ls,
                                     const float* __restrict__ hi, S4 hs, const float* __restrict__ att, S4 as,
                                     float* __restrict__ glo, float* __restrict__ ghi, float* __restrict__ gatt, int N,
                                     int C, int H, int W) {
  const int64_t total = (int64_t)N * H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    const int64_t q = i / W;
    const int h = (int)(q % H), n = (int)(q / H);
    const float s = sigmoidf_(att[n * as.n + h * as.h + w * as.w]);
    const float sm = __fsub_rn(1.f, s);
    float acc = 0.f;
    for (int c = 0; c < C; ++c) {
      const float gv = g[n * gs.n + c * gs.c + h * gs.h + w * gs.w];
      const float l = lo[n * ls.n + c * ls.c + h * ls.h + w * ls.w], r = hi[n * hs.n + c * hs.c + h * hs.h + w * hs.w];
      const int64_t o = (((int64_t)n * C + c) * H + h) * W + w;
      if (glo) glo[o] = gv * s;
      if (ghi) ghi[o] = gv * sm;
      acc += gv * l - gv * r;
    }
    if (gatt) gatt[i] = acc * sm * s;
  }
}

S4 s4(const int64_t* v) { return S4{v[0], v[1], v[2], v[3]}; }

}  // namespace

extern "C" int ssseg_avgpool_fwd(const void* x, void* y, int64_t N, int64_t H, int64_t W, int64_t C, int64_t OH,
                                 int64_t OW, int64_t k, int64_t s, int64_t p, int dt, ssseg_stream_t stream) {
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  if (!x || !y || k < 1 || s < 1 || p < 0 || 2 * p > k || C % V || N < 0 || OH < 1 || OW < 1) return SSSEG_EINVAL;
  const int64_t total = N * OH * OW * (C / V);
  if (total == 0) return 0;
  if (total >= 0x7fffffffLL || N * H * W * C >= (1LL << 40)) return SSSEG_EUNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(ssseg_grid(total, 256, 1 << 20)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)x, (bf16_t*)y, (int)N, (int)H, (int)W,
                       (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<f16_t>, g, b, 0, st, (const f16_t*)x, (f16_t*)y, (int)N, (int)H, (int)W,
                       (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(avgpool_fwd_kernel<float>, g, b, 0, st, (const float*)x, (float*)y, (int)N, (int)H, (int)W,
                       (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_avgpool_bwd(const void* gy, void* gx, int64_t N, int64_t H, int64_t W, int64_t C, int64_t OH,
                                 int64_t OW, int64_t k, int64_t s, int64_t p, int dt, ssseg_stream_t stream) {
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  if (!gy || !gx || k < 1 || s < 1 || p < 0 || 2 * p > k || C % V || N < 0 || H < 1 || W < 1) return SSSEG_EINVAL;
  const int64_t total = N * H * W * (C / V);
  if (total == 0) return 0;
  if (total >= 0x7fffffffLL) return SSSEG_EUNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(ssseg_grid(total, 256, 1 << 20)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(avgpool_bwd_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)gy, (bf16_t*)gx, (int)N, (int)H,
                       (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(avgpool_bwd_kernel<f16_t>, g, b, 0, st, (const f16_t*)gy, (f16_t*)gx, (int)N, (int)H,
                       (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(avgpool_bwd_kernel<float>, g, b, 0, st, (const float*)gy, (float*)gx, (int)N, (int)H, (int)W,
                       (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

static int gap_splits(int64_t HW) {
  int64_t sp = (HW + 255) / 256;
  return (int)(sp < 1 ? 1 : (sp > GAP_SPLITS_MAX ? GAP_SPLITS_MAX : sp));
}

extern "C" size_t ssseg_global_avgpool_workspace_bytes(int64_t N, int64_t HW, int64_t C) {
  return sizeof(float) * (size_t)(N * gap_splits(HW) * C) + 256;
}

extern "C" int ssseg_global_avgpool_fwd(const void* x, void* y, int64_t N, int64_t HW, int64_t C, int64_t ldy, int dt,
                                        void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  if (!x || !y || N < 1 || HW < 1 || C < 1 || C % V || ldy < C) return SSSEG_EINVAL;
  if (N > 65535 || N * HW * C >= (1LL << 40)) return SSSEG_EUNSUPPORTED;
  if (!ws || ws_bytes < ssseg_global_avgpool_workspace_bytes(N, HW, C)) return SSSEG_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int splits = gap_splits(HW);
  const dim3 g((unsigned)N, (unsigned)((C / V + 63) / 64), (unsigned)splits);
  const float inv = (float)(1.0 / (double)HW);
  if (dt == SSSEG_BF16) {
    hipLaunchKernelGGL(gap_partial_kernel<bf16_t>, g, dim3(256), 0, st, (const bf16_t*)x, (float*)ws, (int)HW, (int)C,
                       splits);
    hipLaunchKernelGGL(gap_final_kernel<bf16_t>, dim3((unsigned)((N * C + 255) / 256)), dim3(256), 0, st,
                       (const float*)ws, (bf16_t*)y, (int)N, (int)C, splits, inv, ldy);
  } else if (dt == SSSEG_F16) {
    hipLaunchKernelGGL(gap_partial_kernel<f16_t>, g, dim3(256), 0, st, (const f16_t*)x, (float*)ws, (int)HW, (int)C,
                       splits);
    hipLaunchKernelGGL(gap_final_kernel<f16_t>, dim3((unsigned)((N * C + 255) / 256)), dim3(256), 0, st,
                       (const float*)ws, (f16_t*)y, (int)N, (int)C, splits, inv, ldy);
  } else if (dt == SSSEG_F32) {
    hipLaunchKernelGGL(gap_partial_kernel<float>, g, dim3(256), 0, st, (const float*)x, (float*)ws, (int)HW, (int)C,
                       splits);
    hipLaunchKernelGGL(gap_final_kernel<float>, dim3((unsigned)((N * C + 255) / 256)), dim3(256), 0, st,
                       (const float*)ws, (float*)y, (int)N, (int)C, splits, inv, ldy);
  } else {
    return SSSEG_EUNSUPPORTED;
  }
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_global_avgpool_bwd(const void* gy, void* gx, int64_t N, int64_t HW, int64_t C, int64_t ldgy,
                                        int dt, ssseg_stream_t stream) {
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  if (!gy || !gx || N < 1 || HW < 1 || C < 1 || C % V || ldgy < C || ldgy % V) return SSSEG_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int64_t total = N * HW * (C / V);
  const float inv = (float)(1.0 / (double)HW);
  const dim3 g(ssseg_grid(total, 256, 1 << 20)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(gap_bwd_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)gy, (bf16_t*)gx, (int)N, (int)HW, (int)C,
                       ldgy, inv);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(gap_bwd_kernel<f16_t>, g, b, 0, st, (const f16_t*)gy, (f16_t*)gx, (int)N, (int)HW, (int)C,
                       ldgy, inv);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(gap_bwd_kernel<float>, g, b, 0, st, (const float*)gy, (float*)gx, (int)N, (int)HW, (int)C, ldgy,
                       inv);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_add_n(const void* const* xs_host, int n, void* y, int64_t numel, int act, float slope, int dt,
                           ssseg_stream_t stream) {
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  if (!xs_host || !y || n < 1 || n > 8 || numel < 0 || numel % V || act < 0 || act > SSSEG_ACT_LEAKY)
    return SSSEG_EINVAL;
  Ptr8 p{};
  for (int i = 0; i < n; ++i) {
    if (!xs_host[i] || ((uintptr_t)xs_host[i] & 15)) return SSSEG_EINVAL;
    p.p[i] = xs_host[i];
  }
  if ((uintptr_t)y & 15) return SSSEG_EINVAL;
  const int64_t nch = numel / V;
  if (nch == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(ssseg_grid(nch, 256, 1 << 20)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(add_n_kernel<bf16_t>, g, b, 0, st, p, n, (bf16_t*)y, nch, act, slope);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(add_n_kernel<f16_t>, g, b, 0, st, p, n, (f16_t*)y, nch, act, slope);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(add_n_kernel<float>, g, b, 0, st, p, n, (float*)y, nch, act, slope);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

namespace {
int dropout_launch(const void* x, void* y, int64_t n, float p, uint64_t seed, uint64_t offset,
                   const unsigned long long* offset_dev, int dt, ssseg_stream_t stream) {
  if (!x || !y || n < 0 || n % 4 || !(p >= 0.f && p < 1.f)) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const float scale = 1.f / (1.f - p);
  const dim3 g(ssseg_grid(n / 4, 256, 1 << 20)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(dropout_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)x, (bf16_t*)y, n / 4, p, scale, seed, offset,
                       offset_dev);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(dropout_kernel<f16_t>, g, b, 0, st, (const f16_t*)x, (f16_t*)y, n / 4, p, scale, seed, offset,
                       offset_dev);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(dropout_kernel<float>, g, b, 0, st, (const float*)x, (float*)y, n / 4, p, scale, seed, offset,
                       offset_dev);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

__global__ void rng_take_kernel(unsigned long long* counter, unsigned long long* snap, unsigned long long inc) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const unsigned long long v = *counter;
    snap[0] = v;
    counter[0] = v + inc;
  }
}
}  // namespace

extern "C" int ssseg_dropout(const void* x, void* y, int64_t n, float p, uint64_t seed, uint64_t offset, int dt,
                             ssseg_stream_t stream) {
  return dropout_launch(x, y, n, p, seed, offset, nullptr, dt, stream);
}

extern "C" int ssseg_dropout_dev(const void* x, void* y, int64_t n, float p, uint64_t seed,
                                 const unsigned long long* offset_dev, int dt, ssseg_stream_t stream) {
  if (!offset_dev) return SSSEG_EINVAL;
  return dropout_launch(x, y, n, p, seed, 0, offset_dev, dt, stream);
}

extern "C" int ssseg_rng_take(unsigned long long* counter, unsigned long long* snap, uint64_t inc,
                              ssseg_stream_t stream) {
  if (!counter || !snap) return SSSEG_EINVAL;
  hipLaunchKernelGGL(rng_take_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, counter, snap,
                     (unsigned long long)inc);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_att_blend_fwd(const float* lo, const int64_t* lo_strides4_host, const float* hi,
                                   const int64_t* hi_strides4_host, const float* att, const int64_t* att_strides4_host,
                                   float* out, int64_t N, int64_t C, int64_t H, int64_t W, ssseg_stream_t stream) {
  if (!lo || !hi || !att || !out || !lo_strides4_host || !hi_strides4_host || !att_strides4_host || N < 0 || C < 0 ||
      H < 0 || W < 0)
    return SSSEG_EINVAL;
  const int64_t total = N * C * H * W;
  if (total == 0) return 0;
  hipLaunchKernelGGL(att_blend_fwd_kernel, dim3(ssseg_grid(total, 256, 1 << 16)), dim3(256), 0, (hipStream_t)stream,
                     lo, s4(lo_strides4_host), hi, s4(hi_strides4_host), att, s4(att_strides4_host), out, (int)N, (int)C,
                     (int)H, (int)W);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_att_blend_bwd(const float* gout, const int64_t* g_strides4_host, const float* lo,
                                   const int64_t* lo_strides4_host, const float* hi, const int64_t* hi_strides4_host,
                                   const float* att, const int64_t* att_strides4_host, float* glo, float* ghi,
                                   float* gatt, int64_t N, int64_t C, int64_t H, int64_t W, ssseg_stream_t stream) {
  if (!gout || !lo || !hi || !att || !g_strides4_host || !lo_strides4_host || !hi_strides4_host ||
      !att_strides4_host || N < 0 || C < 0 || H < 0 || W < 0)
    return SSSEG_EINVAL;
  const int64_t total = N * H * W;
  if (total == 0) return 0;
  hipLaunchKernelGGL(att_blend_bwd_kernel, dim3(ssseg_grid(total, 256, 1 << 16)), dim3(256), 0, (hipStream_t)stream,
                     gout, s4(g_strides4_host), lo, s4(lo_strides4_host), hi, s4(hi_strides4_host), att,
                     s4(att_strides4_host), glo, ghi, gatt, (int)N, (int)C, (int)H, (int)W);
  SSSEG_LAUNCH_CHECK();
  return 0;
}
