// Max pooling (ResNet stem MaxPool2d(3,2,1); simple_unet.py:18 MaxPool2d(2,2,ceil_mode=True)) and the
// NHWC window copy used for torch.cat / _center_crop (unet.py:40-45, simple_unet.py:86-91), gfx950.
#include "common.h"

namespace {

template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int N, int H,
                                   int W, int C, int OH, int OW, int k, int s, int p) {
  const int64_t total = (int64_t)N * OH * OW * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    int64_t q = i / C;
    const int ow = (int)(q % OW);
    q /= OW;
    const int oh = (int)(q % OH);
    const int n = (int)(q / OH);
    // PyTorch CPU order: maxval = -inf, maxindex = first valid tap; update when v > maxval or v is NaN
    float m = -INFINITY;
    int best = -1;
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * s - p + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * s - p + kw;
        if (iw < 0 || iw >= W) continue;
        const float v = io<T>::ld(x, (((int64_t)n * H + ih) * W + iw) * C + c);
        if (best < 0) best = kh * k + kw;
        if (v > m || v != v) {
          m = v;
          best = kh * k + kw;
        }
      }
    }
    io<T>::st(y, i, m);
    idx[i] = (uint8_t)best;
  }
}

template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ gy, const uint8_t* __restrict__ idx, const T* __restrict__ res,
                                   T* __restrict__ gx, int N, int H, int W, int C, int OH, int OW, int k, int s, int p) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    int64_t q = i / C;
    const int iw = (int)(q % W);
    q /= W;
    const int ih = (int)(q % H);
    const int n = (int)(q / H);
    const int oh0 = max(0, (ih + p - k + s) / s), oh1 = min(OH - 1, (ih + p) / s);
    const int ow0 = max(0, (iw + p - k + s) / s), ow1 = min(OW - 1, (iw + p) / s);
    float acc = res ? io<T>::ld(res, i) : 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = ih - (oh * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = iw - (ow * s - p);
        if (kw < 0 || kw >= k) continue;
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c;
        if (idx[o] == kh * k + kw) acc += io<T>::ld(gy, o);
      }
    }
    io<T>::st(gx, i, acc);
  }
}

// 16-byte channel-chunk variants (C % (16/sizeof(T)) == 0, < 2^31 chunks): one thread per (pixel, chunk),
// 32-bit index math, the window's taps loaded as 16-byte vectors, argmax bytes stored 8/4 at a time.
template <typename T> struct VC;
template <> struct VC<bf16_t> {
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
template <> struct VC<f16_t> {
  static constexpr int V = 8;
  __device__ __forceinline__ static void ld(const f16_t* p, float (&v)[8]) { H16::ld8(p, v); }
  __device__ __forceinline__ static void st(f16_t* p, const float (&v)[8]) { H16::st8(p, v); }
};
template <> struct VC<float> {
  static constexpr int V = 4;
  __device__ __forceinline__ static void ld(const float* p, float (&v)[4]) {
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[4]) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
};

template <int V> struct IdxVec;
template <> struct IdxVec<8> {
  __device__ __forceinline__ static void st(uint8_t* p, const int (&b)[8]) {
    unsigned lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo |= (unsigned)(b[i] & 255) << (8 * i);
      hi |= (unsigned)(b[4 + i] & 255) << (8 * i);
    }
    *(uint2*)p = make_uint2(lo, hi);
  }
  __device__ __forceinline__ static void ld(const uint8_t* p, int (&b)[8]) {
    const uint2 q = *(const uint2*)p;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      b[i] = (q.x >> (8 * i)) & 255;
      b[4 + i] = (q.y >> (8 * i)) & 255;
    }
  }
};
template <> struct IdxVec<4> {
  __device__ __forceinline__ static void st(uint8_t* p, const int (&b)[4]) {
    unsigned w = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) w |= (unsigned)(b[i] & 255) << (8 * i);
    *(unsigned*)p = w;
  }
  __device__ __forceinline__ static void ld(const uint8_t* p, int (&b)[4]) {
    const unsigned w = *(const unsigned*)p;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = (w >> (8 * i)) & 255;
  }
};

template <typename T>
__global__ void maxpool_fwd_vec_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int N,
                                       int H, int W, int C, int OH, int OW, int k, int s, int p) {
  constexpr int V = VC<T>::V;
  const int CV = C / V;
  const int total = N * OH * OW * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int q = i / CV;
    const int ow = q % OW;
    q /= OW;
    const int oh = q % OH, n = q / OH;
    float m[V];
    int best[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      m[e] = -INFINITY;
      best[e] = -1;
    }
    if (k == 3) {   // the ResNet stem's 3x3 pool: all nine taps' loads in flight together (clamped addresses), then
                    // the same first-valid-tap / greater-or-NaN scan in tap order as the general loop below
      using CK = Chunk<T, V>;
      typename CK::raw qv[9];
      bool ok[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ih = oh * s - p + t / 3, iw = ow * s - p + t % 3;
        ok[t] = ih >= 0 && ih < H && iw >= 0 && iw < W;
        const int ch = min(max(ih, 0), H - 1), cw = min(max(iw, 0), W - 1);
        qv[t] = CK::ld(x + ((int64_t)(n * H + ch) * W + cw) * C + cv * V);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (!ok[t]) continue;
        float v[V];
        CK::cvt(qv[t], v);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          if (best[e] < 0) best[e] = t;
          if (v[e] > m[e] || v[e] != v[e]) {
            m[e] = v[e];
            best[e] = t;
          }
        }
      }
      const int64_t o = (int64_t)i * V;
      VC<T>::st(y + o, m);
      IdxVec<V>::st(idx + o, best);
      continue;
    }
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * s - p + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * s - p + kw;
        if (iw < 0 || iw >= W) continue;
        float v[V];
        VC<T>::ld(x + ((int64_t)(n * H + ih) * W + iw) * C + cv * V, v);
        const int tap = kh * k + kw;
#pragma unroll
        for (int e = 0; e < V; ++e) {   // PyTorch order: first valid tap, then v > max or NaN
          if (best[e] < 0) best[e] = tap;
          if (v[e] > m[e] || v[e] != v[e]) {
            m[e] = v[e];
            best[e] = tap;
          }
        }
      }
    }
    const int64_t o = (int64_t)i * V;
    VC<T>::st(y + o, m);
    IdxVec<V>::st(idx + o, best);
  }
}

template <typename T>
__global__ void maxpool_bwd_vec_kernel(const T* __restrict__ gy, const uint8_t* __restrict__ idx,
                                       const T* __restrict__ res, T* __restrict__ gx, int N, int H, int W, int C,
                                       int OH, int OW, int k, int s, int p) {
  constexpr int V = VC<T>::V;
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
    if (res)
      VC<T>::ld(res + (int64_t)i * V, acc);   // the parked gradient of x (GradJoin), added in the same pass
    else
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = 0.f;
    if (V == 8 && k == 3 && s == 2) {   // <= 2 x 2 windows reach a pixel: their index and gradient loads in flight together
                              // (clamped), then the general loop's additions in its (oh, ow) order
      using CK = Chunk<T, V>;
      typename CK::raw qg[4];
      uint2 qi[4];
      bool ok[4];
      int tap[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int oh = oh0 + (c >> 1), ow = ow0 + (c & 1);
        const int kh = ih - (oh * s - p), kw = iw - (ow * s - p);
        ok[c] = oh <= oh1 && ow <= ow1 && kh >= 0 && kh < k && kw >= 0 && kw < k;
        tap[c] = kh * k + kw;
        const int64_t o = ((int64_t)(n * OH + min(oh, OH - 1)) * OW + min(ow, OW - 1)) * C + cv * V;
        qi[c] = *(const uint2*)(idx + o);
        qg[c] = CK::ld(gy + o);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (!ok[c]) continue;
        float g[V];
        CK::cvt(qg[c], g);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const int b = (int)((e < 4 ? qi[c].x >> (8 * e) : qi[c].y >> (8 * (e - 4))) & 255u);
          acc[e] += b == tap[c] ? g[e] : 0.f;
        }
      }
      VC<T>::st(gx + (int64_t)i * V, acc);
      continue;
    }
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = ih - (oh * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = iw - (ow * s - p);
        if (kw < 0 || kw >= k) continue;
        const int64_t o = ((int64_t)(n * OH + oh) * OW + ow) * C + cv * V;
        int b[V];
        IdxVec<V>::ld(idx + o, b);
        float g[V];
        VC<T>::ld(gy + o, g);
        const int tap = kh * k + kw;
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += b[e] == tap ? g[e] : 0.f;
      }
    }
    VC<T>::st(gx + (int64_t)i * V, acc);
  }
}

template <typename T>
__global__ void nhwc_copy_kernel(const T* __restrict__ src, T* __restrict__ dst, int N, int H, int W, int C, int sH,
                                 int sW, int64_t sld, int soy, int sox, int dH, int dW, int64_t dld, int doy, int dox) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    int64_t q = i / C;
    const int w = (int)(q % W);
    q /= W;
    const int h = (int)(q % H);
    const int n = (int)(q / H);
    const T v = src[(((int64_t)n * sH + h + soy) * sW + w + sox) * sld + c];
    dst[(((int64_t)n * dH + h + doy) * dW + w + dox) * dld + c] = v;
  }
}

// 16-byte vector variant (C, sld, dld multiples of 16/sizeof(T) elements)
__global__ void nhwc_copy_v16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int N, int H, int W, int C4,
                                     int sH, int sW, int64_t sld4, int soy, int sox, int dH, int dW, int64_t dld4, int doy,
                                     int dox) {
  const int64_t total = (int64_t)N * H * W * C4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4);
    int64_t q = i / C4;
    const int w = (int)(q % W);
    q /= W;
    const int h = (int)(q % H);
    const int n = (int)(q / H);
    dst[(((int64_t)n * dH + h + doy) * dW + w + dox) * dld4 + c] = src[(((int64_t)n * sH + h + soy) * sW + w + sox) * sld4 + c];
  }
}

}  // namespace

extern "C" int ssseg_maxpool_fwd(const void* x, void* y, uint8_t* idx, int64_t N, int64_t H, int64_t W, int64_t C,
                                 int64_t OH, int64_t OW, int64_t k, int64_t s, int64_t p, int dt, ssseg_stream_t stream) {
  if (!x || !y || !idx || k < 1 || k > 15 || s < 1 || p < 0) return SSSEG_EINVAL;
  const int64_t total = N * OH * OW * C;
  if (total == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  if (C % V == 0 && total / V < 0x7fffffffLL && N * H * W * C < (1LL << 40)) {
    const dim3 gv(ssseg_grid(total / V, 256, 1 << 20)), bv(256);
    if (dt == SSSEG_BF16)
      hipLaunchKernelGGL(maxpool_fwd_vec_kernel<bf16_t>, gv, bv, 0, st, (const bf16_t*)x, (bf16_t*)y, idx, (int)N,
                         (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
    else if (dt == SSSEG_F16)
      hipLaunchKernelGGL(maxpool_fwd_vec_kernel<f16_t>, gv, bv, 0, st, (const f16_t*)x, (f16_t*)y, idx, (int)N,
                         (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
    else if (dt == SSSEG_F32)
      hipLaunchKernelGGL(maxpool_fwd_vec_kernel<float>, gv, bv, 0, st, (const float*)x, (float*)y, idx, (int)N, (int)H,
                         (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
    else
      return SSSEG_EUNSUPPORTED;
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  const dim3 g(ssseg_grid(total, 256)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)x, (bf16_t*)y, idx, (int)N, (int)H,
                       (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<f16_t>, g, b, 0, st, (const f16_t*)x, (f16_t*)y, idx, (int)N, (int)H,
                       (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, g, b, 0, st, (const float*)x, (float*)y, idx, (int)N, (int)H, (int)W,
                       (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_maxpool_bwd(const void* gy, const uint8_t* idx, void* gx, int64_t N, int64_t H, int64_t W,
                                 int64_t C, int64_t OH, int64_t OW, int64_t k, int64_t s, int64_t p, int dt,
                                 ssseg_stream_t stream) {
  return ssseg_maxpool_bwd_res(gy, idx, nullptr, gx, N, H, W, C, OH, OW, k, s, p, dt, stream);
}

extern "C" int ssseg_maxpool_bwd_res(const void* gy, const uint8_t* idx, const void* res, void* gx, int64_t N, int64_t H,
                                     int64_t W, int64_t C, int64_t OH, int64_t OW, int64_t k, int64_t s, int64_t p,
                                     int dt, ssseg_stream_t stream) {
  if (!gy || !gx || !idx || k < 1 || s < 1 || p < 0) return SSSEG_EINVAL;
  const int64_t total = N * H * W * C;
  if (total == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int V = (dt == SSSEG_F32 ? 4 : 8);
  if (C % V == 0 && total / V < 0x7fffffffLL && N * OH * OW * C < 0x7fffffffLL * V) {
    const dim3 gv(ssseg_grid(total / V, 256, 1 << 20)), bv(256);
    if (dt == SSSEG_BF16)
      hipLaunchKernelGGL(maxpool_bwd_vec_kernel<bf16_t>, gv, bv, 0, st, (const bf16_t*)gy, idx, (const bf16_t*)res, (bf16_t*)gx, (int)N,
                         (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
    else if (dt == SSSEG_F16)
      hipLaunchKernelGGL(maxpool_bwd_vec_kernel<f16_t>, gv, bv, 0, st, (const f16_t*)gy, idx, (const f16_t*)res, (f16_t*)gx, (int)N,
                         (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
    else if (dt == SSSEG_F32)
      hipLaunchKernelGGL(maxpool_bwd_vec_kernel<float>, gv, bv, 0, st, (const float*)gy, idx, (const float*)res, (float*)gx, (int)N,
                         (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
    else
      return SSSEG_EUNSUPPORTED;
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  const dim3 g(ssseg_grid(total, 256)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)gy, idx, (const bf16_t*)res, (bf16_t*)gx, (int)N, (int)H,
                       (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<f16_t>, g, b, 0, st, (const f16_t*)gy, idx, (const f16_t*)res, (f16_t*)gx, (int)N, (int)H,
                       (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, g, b, 0, st, (const float*)gy, idx, (const float*)res, (float*)gx, (int)N, (int)H,
                       (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_nhwc_copy(const void* src, void* dst, int64_t N, int64_t H, int64_t W, int64_t C, int64_t sH,
                               int64_t sW, int64_t sld, int64_t soy, int64_t sox, int64_t dH, int64_t dW, int64_t dld,
                               int64_t doy, int64_t dox, int dt, ssseg_stream_t stream) {
  if (!src || !dst || C < 0 || soy < 0 || sox < 0 || doy < 0 || dox < 0 || H + soy > sH || W + sox > sW ||
      H + doy > dH || W + dox > dW)
    return SSSEG_EINVAL;
  const int64_t total = N * H * W * C;
  if (total == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int esz = (dt == SSSEG_F32 ? 4 : 2);
  const int v = 16 / esz;
  if (C % v == 0 && sld % v == 0 && dld % v == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int64_t t4 = total / v;
    hipLaunchKernelGGL(nhwc_copy_v16_kernel, dim3(ssseg_grid(t4, 256)), dim3(256), 0, st, (const uint4*)src,
                       (uint4*)dst, (int)N, (int)H, (int)W, (int)(C / v), (int)sH, (int)sW, sld / v, (int)soy, (int)sox,
                       (int)dH, (int)dW, dld / v, (int)doy, (int)dox);
  } else if (dt == SSSEG_BF16) {
    hipLaunchKernelGGL(nhwc_copy_kernel<bf16_t>, dim3(ssseg_grid(total, 256)), dim3(256), 0, st,
                       (const bf16_t*)src, (bf16_t*)dst, (int)N, (int)H, (int)W, (int)C, (int)sH, (int)sW, sld, (int)soy,
                       (int)sox, (int)dH, (int)dW, dld, (int)doy, (int)dox);
  } else if (dt == SSSEG_F16) {
    hipLaunchKernelGGL(nhwc_copy_kernel<f16_t>, dim3(ssseg_grid(total, 256)), dim3(256), 0, st,
                       (const f16_t*)src, (f16_t*)dst, (int)N, (int)H, (int)W, (int)C, (int)sH, (int)sW, sld, (int)soy,
                       (int)sox, (int)dH, (int)dW, dld, (int)doy, (int)dox);
  } else if (dt == SSSEG_F32) {
    hipLaunchKernelGGL(nhwc_copy_kernel<float>, dim3(ssseg_grid(total, 256)), dim3(256), 0, st,
                       (const float*)src, (float*)dst, (int)N, (int)H, (int)W, (int)C, (int)sH, (int)sW, sld, (int)soy,
                       (int)sox, (int)dH, (int)dW, dld, (int)doy, (int)dox);
  } else {
    return SSSEG_EUNSUPPORTED;
  }
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_zero(void* p, size_t bytes, ssseg_stream_t stream) {
  if (!p) return SSSEG_EINVAL;
  if (bytes == 0) return 0;
  SSSEG_TRY(hipMemsetAsync(p, 0, bytes, (hipStream_t)stream));
  return 0;
}

namespace {
template <typename T>
__global__ void act_bwd_kernel(const T* __restrict__ gy, const T* __restrict__ y, T* __restrict__ gx, int64_t n, int act,
                               float slope) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    io<T>::st(gx, i, act_bwd(io<T>::ld(gy, i), io<T>::ld(y, i), act, slope));
}
}  // namespace

extern "C" int ssseg_act_bwd(const void* gy, const void* y, void* gx, int64_t n, int act, float slope, int dt,
                             ssseg_stream_t stream) {
  if (!gy || !y || !gx || n < 0 || act < 0 || act > SSSEG_ACT_LEAKY) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(ssseg_grid(n, 256)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(act_bwd_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)gy, (const bf16_t*)y, (bf16_t*)gx, n, act,
                       slope);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(act_bwd_kernel<f16_t>, g, b, 0, st, (const f16_t*)gy, (const f16_t*)y, (f16_t*)gx, n, act,
                       slope);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(act_bwd_kernel<float>, g, b, 0, st, (const float*)gy, (const float*)y, (float*)gx, n, act, slope);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_relu_bwd(const void* gy, const void* y, void* gx, int64_t n, int dt, ssseg_stream_t stream) {
  return ssseg_act_bwd(gy, y, gx, n, SSSEG_ACT_RELU, 0.f, dt, stream);
}
