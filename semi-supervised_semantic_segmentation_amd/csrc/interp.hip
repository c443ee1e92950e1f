// Bilinear interpolation forward/backward (F.interpolate mode='bilinear'), gfx950.
// Call sites: losses.py:18 and train.py:71,74,93 (align_corners=False, to the image size),
// unet.py:26 / simple_unet.py:71 (nn.Upsample(scale_factor=2, align_corners=True)).
// Source-index arithmetic follows PyTorch's area_pixel_compute_source_index in fp32; the 2-D blend
// is evaluated as (x00*w0 + x01*w1)*h0 + (x10*w0 + x11*w1)*h1 with explicit roundings, the order of
// the CPU kernel.  Backward is a deterministic gather over the outputs that read each input pixel.
#include "common.h"

// Built with -ffp-contract=off (Makefile): HIP's __fadd_rn / __fmul_rn are plain operators, contractible into FMAs
// differently per kernel; the vector and generic kernels must agree bitwise, and PyTorch's CPU kernel rounds every
// product.

namespace {

struct Strides {
  int64_t n, c, h, w;
};

struct Axis {
  int in, out;
  float scale;
  bool align;
};

// every operation rounded explicitly: no FMA contraction, whose choice may differ between kernels (the vector and
// the generic kernels must agree bitwise) and which PyTorch's CPU kernel does not do
__device__ __forceinline__ void src_index(const Axis& a, int d, int& i0, int& i1, float& l0, float& l1) {
  float src;
  if (a.align) {
    src = __fmul_rn(a.scale, (float)d);
  } else {
    src = __fsub_rn(__fmul_rn(a.scale, __fadd_rn((float)d, 0.5f)), 0.5f);
    src = src < 0.f ? 0.f : src;
  }
  i0 = min((int)src, a.in - 1);
  l1 = fminf(fmaxf(__fsub_rn(src, (float)i0), 0.f), 1.f);
  i1 = i0 + (i0 < a.in - 1 ? 1 : 0);
  l0 = __fsub_rn(1.f, l1);
}

static Axis make_axis(int64_t in, int64_t out, bool align) {
  Axis a;
  a.in = (int)in;
  a.out = (int)out;
  a.align = align;
  if (align)
    a.scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  else
    a.scale = (float)in / (float)out;
  return a;
}

// I: index type of the element decode (int when N*C*Ho*Wo < 2^31: 64-bit divisions cost ~10x the 32-bit ones)
template <typename T, typename I>
__global__ void bilinear_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t N_, int64_t C_, Axis ah, Axis aw,
                                    Strides xs, Strides ys, int c_fastest) {
  const I N = (I)N_, C = (I)C_, Ho = ah.out, Wo = aw.out, total = N * C * Ho * Wo;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    I n, c, oh, ow;
    if (c_fastest) {
      c = i % C; ow = (i / C) % Wo; oh = (i / (C * Wo)) % Ho; n = i / (C * Wo * Ho);
    } else {
      ow = i % Wo; oh = (i / Wo) % Ho; c = (i / (Wo * Ho)) % C; n = i / (Wo * Ho * C);
    }
    int h0, h1, w0, w1;
    float lh0, lh1, lw0, lw1;
    src_index(ah, (int)oh, h0, h1, lh0, lh1);
    src_index(aw, (int)ow, w0, w1, lw0, lw1);
    const T* xb = x + (int64_t)n * xs.n + (int64_t)c * xs.c;
    const float x00 = io<T>::ld(xb, h0 * xs.h + w0 * xs.w), x01 = io<T>::ld(xb, h0 * xs.h + w1 * xs.w);
    const float x10 = io<T>::ld(xb, h1 * xs.h + w0 * xs.w), x11 = io<T>::ld(xb, h1 * xs.h + w1 * xs.w);
    const float t0 = __fadd_rn(__fmul_rn(x00, lw0), __fmul_rn(x01, lw1));
    const float t1 = __fadd_rn(__fmul_rn(x10, lw0), __fmul_rn(x11, lw1));
    const float v = __fadd_rn(__fmul_rn(t0, lh0), __fmul_rn(t1, lh1));
    io<T>::st(y, (int64_t)n * ys.n + (int64_t)c * ys.c + (int64_t)oh * ys.h + (int64_t)ow * ys.w, v);
  }
}

// fp32 logits resizes (train.py:71,74,93, losses.py:18: the head's 2-channel logits, NHWC with a padded pixel
// stride, to the image size): one thread per output pixel and ALL channels (C <= 4), so the source indices and
// weights are computed once per pixel and each input pixel's channels come from one sector.  Per channel the
// arithmetic is the generic kernel's (same roundings, same order): bit-identical results.
template <typename T, int C>
__global__ void bilinear_fwd_pix_kernel(const T* __restrict__ x, T* __restrict__ y, Axis ah, Axis aw, Strides xs,
                                        Strides ys) {
  const int ow = blockIdx.x * blockDim.x + threadIdx.x, oh = blockIdx.y, n = blockIdx.z;
  if (ow >= aw.out) return;
  int h0, h1, w0, w1;
  float lh0, lh1, lw0, lw1;
  src_index(ah, oh, h0, h1, lh0, lh1);
  src_index(aw, ow, w0, w1, lw0, lw1);
  const T* xb = x + (int64_t)n * xs.n;
  const int64_t o00 = h0 * xs.h + w0 * xs.w, o01 = h0 * xs.h + w1 * xs.w;
  const int64_t o10 = h1 * xs.h + w0 * xs.w, o11 = h1 * xs.h + w1 * xs.w;
  float v[C][4];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    v[c][0] = io<T>::ld(xb, o00 + c * xs.c);
    v[c][1] = io<T>::ld(xb, o01 + c * xs.c);
    v[c][2] = io<T>::ld(xb, o10 + c * xs.c);
    v[c][3] = io<T>::ld(xb, o11 + c * xs.c);
  }
  T* yb = y + (int64_t)n * ys.n + (int64_t)oh * ys.h + (int64_t)ow * ys.w;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float t0 = __fadd_rn(__fmul_rn(v[c][0], lw0), __fmul_rn(v[c][1], lw1));
    const float t1 = __fadd_rn(__fmul_rn(v[c][2], lw0), __fmul_rn(v[c][3], lw1));
    io<T>::st(yb, (int64_t)c * ys.c, __fadd_rn(__fmul_rn(t0, lh0), __fmul_rn(t1, lh1)));
  }
}

// outputs o whose source pair (i0, i1) contains input i lie within [lo, hi]
__device__ __forceinline__ void out_window(const Axis& a, int i, int& lo, int& hi) {
  if (a.scale <= 0.f) {
    lo = 0;
    hi = a.out - 1;
    return;
  }
  const float inv = 1.f / a.scale;
  float c0, c1;
  if (a.align) {
    c0 = (float)(i - 1) * inv;
    c1 = (float)(i + 1) * inv;
  } else {
    c0 = ((float)(i - 1) + 0.5f) * inv - 0.5f;
    c1 = ((float)(i + 1) + 0.5f) * inv - 0.5f;
  }
  lo = max((int)floorf(c0) - 1, 0);
  hi = min((int)ceilf(c1) + 1, a.out - 1);
}

template <typename T, typename I>
__global__ void bilinear_bwd_kernel(const T* __restrict__ gy, T* __restrict__ gx, int64_t N_, int64_t C_, Axis ah,
                                    Axis aw, Strides gys, Strides gxs, int c_fastest) {
  const I N = (I)N_, C = (I)C_, H = ah.in, W = aw.in, total = N * C * H * W;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    I n, c, h, w;
    if (c_fastest) {
      c = i % C; w = (i / C) % W; h = (i / (C * W)) % H; n = i / (C * W * H);
    } else {
      w = i % W; h = (i / W) % H; c = (i / (W * H)) % C; n = i / (W * H * C);
    }
    int ohlo, ohhi, owlo, owhi;
    out_window(ah, (int)h, ohlo, ohhi);
    out_window(aw, (int)w, owlo, owhi);
    const T* gb = gy + (int64_t)n * gys.n + (int64_t)c * gys.c;
    float acc = 0.f;
    for (int oh = ohlo; oh <= ohhi; ++oh) {
      int h0, h1;
      float l0, l1;
      src_index(ah, oh, h0, h1, l0, l1);
      const float wh = (h0 == h ? l0 : 0.f) + (h1 == h ? l1 : 0.f);
      if (wh == 0.f) continue;
      float row = 0.f;
      for (int ow = owlo; ow <= owhi; ++ow) {
        int w0, w1;
        float m0, m1;
        src_index(aw, ow, w0, w1, m0, m1);
        const float ww = (w0 == w ? m0 : 0.f) + (w1 == w ? m1 : 0.f);
        if (ww != 0.f) row = fmaf(io<T>::ld(gb, (int64_t)oh * gys.h + (int64_t)ow * gys.w), ww, row);
      }
      acc = fmaf(row, wh, acc);
    }
    io<T>::st(gx, (int64_t)n * gxs.n + (int64_t)c * gxs.c + (int64_t)h * gxs.h + (int64_t)w * gxs.w, acc);
  }
}

// backward of bilinear_fwd_pix_kernel: one thread per input pixel and all C <= 4 channels (the output window and
// its weights computed once per pixel); per channel the generic kernel's gather in the same order: bit-identical
template <typename T, int C>
__global__ void bilinear_bwd_pix_kernel(const T* __restrict__ gy, T* __restrict__ gx, Axis ah, Axis aw, Strides gys,
                                        Strides gxs) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x, h = blockIdx.y, n = blockIdx.z;
  if (w >= aw.in) return;
  int ohlo, ohhi, owlo, owhi;
  out_window(ah, h, ohlo, ohhi);
  out_window(aw, w, owlo, owhi);
  const T* gb = gy + (int64_t)n * gys.n;
  float acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
  for (int oh = ohlo; oh <= ohhi; ++oh) {
    int h0, h1;
    float l0, l1;
    src_index(ah, oh, h0, h1, l0, l1);
    const float wh = (h0 == h ? l0 : 0.f) + (h1 == h ? l1 : 0.f);
    if (wh == 0.f) continue;
    float row[C];
#pragma unroll
    for (int c = 0; c < C; ++c) row[c] = 0.f;
    for (int ow = owlo; ow <= owhi; ++ow) {
      int w0, w1;
      float m0, m1;
      src_index(aw, ow, w0, w1, m0, m1);
      const float ww = (w0 == w ? m0 : 0.f) + (w1 == w ? m1 : 0.f);
      if (ww != 0.f) {
        const int64_t o = (int64_t)oh * gys.h + (int64_t)ow * gys.w;
#pragma unroll
        for (int c = 0; c < C; ++c) row[c] = fmaf(io<T>::ld(gb, o + c * gys.c), ww, row[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = fmaf(row[c], wh, acc[c]);
  }
  T* xb = gx + (int64_t)n * gxs.n + (int64_t)h * gxs.h + (int64_t)w * gxs.w;
#pragma unroll
  for (int c = 0; c < C; ++c) io<T>::st(xb, (int64_t)c * gxs.c, acc[c]);
}

// 16-bit NHWC activations (the HRNet / UNet feature maps: channels fastest, C % 8 == 0, 16-byte aligned rows): one
// thread per (pixel, 8-channel chunk), blockIdx.y = output row, blockIdx.z = image -- no per-element index decode,
// 16-byte loads and stores.  Per channel the arithmetic is the generic kernels' (same roundings, same order), so
// the results are bit-identical to them.
template <typename T>
__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
  T o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) io<T>::st(o, e, v[e]);
  return *(const uint4*)o;
}

template <typename T>
__global__ void __launch_bounds__(256) bilinear_fwd_nhwc_kernel(const T* __restrict__ x, T* __restrict__ y, int C8,
                                                                Axis ah, Axis aw, Strides xs, Strides ys) {
  const int oh = blockIdx.y, n = blockIdx.z;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= aw.out * C8) return;
  const int ow = idx / C8, c = (idx - ow * C8) * 8;
  int h0, h1, w0, w1;
  float lh0, lh1, lw0, lw1;
  src_index(ah, oh, h0, h1, lh0, lh1);
  src_index(aw, ow, w0, w1, lw0, lw1);
  const T* xb = x + (int64_t)n * xs.n + c;
  const typename Chunk<T, 8>::raw q00 = Chunk<T, 8>::ld(xb + (int64_t)h0 * xs.h + (int64_t)w0 * xs.w),
                                  q01 = Chunk<T, 8>::ld(xb + (int64_t)h0 * xs.h + (int64_t)w1 * xs.w),
                                  q10 = Chunk<T, 8>::ld(xb + (int64_t)h1 * xs.h + (int64_t)w0 * xs.w),
                                  q11 = Chunk<T, 8>::ld(xb + (int64_t)h1 * xs.h + (int64_t)w1 * xs.w);
  float a00[8], a01[8], a10[8], a11[8], v[8];
  Chunk<T, 8>::cvt(q00, a00);
  Chunk<T, 8>::cvt(q01, a01);
  Chunk<T, 8>::cvt(q10, a10);
  Chunk<T, 8>::cvt(q11, a11);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t0 = __fadd_rn(__fmul_rn(a00[e], lw0), __fmul_rn(a01[e], lw1));
    const float t1 = __fadd_rn(__fmul_rn(a10[e], lw0), __fmul_rn(a11[e], lw1));
    v[e] = __fadd_rn(__fmul_rn(t0, lh0), __fmul_rn(t1, lh1));
  }
  *(uint4*)(y + (int64_t)n * ys.n + (int64_t)oh * ys.h + (int64_t)ow * ys.w + c) = pack8<T>(v);
}

template <typename T>
__global__ void __launch_bounds__(256) bilinear_bwd_nhwc_kernel(const T* __restrict__ gy, T* __restrict__ gx, int C8,
                                                                Axis ah, Axis aw, Strides gys, Strides gxs) {
  const int h = blockIdx.y, n = blockIdx.z;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= aw.in * C8) return;
  const int w = idx / C8, c = (idx - w * C8) * 8;
  int ohlo, ohhi, owlo, owhi;
  out_window(ah, h, ohlo, ohhi);
  out_window(aw, w, owlo, owhi);
  const T* gb = gy + (int64_t)n * gys.n + c;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int oh = ohlo; oh <= ohhi; ++oh) {
    int h0, h1;
    float l0, l1;
    src_index(ah, oh, h0, h1, l0, l1);
    const float wh = (h0 == h ? l0 : 0.f) + (h1 == h ? l1 : 0.f);
    if (wh == 0.f) continue;
    float row[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) row[e] = 0.f;
    for (int ow = owlo; ow <= owhi; ++ow) {
      int w0, w1;
      float m0, m1;
      src_index(aw, ow, w0, w1, m0, m1);
      const float ww = (w0 == w ? m0 : 0.f) + (w1 == w ? m1 : 0.f);
      if (ww != 0.f) {
        float g[8];
        Chunk<T, 8>::cvt(Chunk<T, 8>::ld(gb + (int64_t)oh * gys.h + (int64_t)ow * gys.w), g);
#pragma unroll
        for (int e = 0; e < 8; ++e) row[e] = fmaf(g[e], ww, row[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = fmaf(row[e], wh, acc[e]);
  }
  *(uint4*)(gx + (int64_t)n * gxs.n + (int64_t)h * gxs.h + (int64_t)w * gxs.w + c) = pack8<T>(acc);
}

// The same input gradient in two separable passes (bitwise the one-pass kernel: that kernel already sums each output
// row over its columns first, row[] = sum_ow g * ww in ow order, then acc = sum_oh row * wh in oh order, skipping rows
// with wh == 0; here pass 1 stores those row sums in fp32 for every (oh, w), pass 2 combines them).  The one-pass kernel
// has one thread per INPUT chunk walking a (2^k + 1)^2 output window with dependent loads -- 81 of them per thread for
// HRNet's 8x fuse upsampling, over a grid of only N x h x w x C/8 threads (43 us average in C4's step); each pass here
// walks one axis (<= 2^k + 1 loads) over a grid of N x Ho x w (resp. N x h x w) chunks.
template <typename T>
__global__ void __launch_bounds__(256) bilinear_bwd_rows_nhwc_kernel(const T* __restrict__ gy, float* __restrict__ rs,
                                                                     int C8, int Ho, Axis aw, Strides gys) {
  const int oh = blockIdx.y, n = blockIdx.z;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= aw.in * C8) return;
  const int w = idx / C8, c = (idx - w * C8) * 8;
  int owlo, owhi;
  out_window(aw, w, owlo, owhi);
  const T* gb = gy + (int64_t)n * gys.n + (int64_t)oh * gys.h + c;
  float row[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) row[e] = 0.f;
  for (int ow = owlo; ow <= owhi; ++ow) {
    int w0, w1;
    float m0, m1;
    src_index(aw, ow, w0, w1, m0, m1);
    const float ww = (w0 == w ? m0 : 0.f) + (w1 == w ? m1 : 0.f);
    if (ww != 0.f) {
      float g[8];
      Chunk<T, 8>::cvt(Chunk<T, 8>::ld(gb + (int64_t)ow * gys.w), g);
#pragma unroll
      for (int e = 0; e < 8; ++e) row[e] = fmaf(g[e], ww, row[e]);
    }
  }
  float* r = rs + (((int64_t)n * Ho + oh) * aw.in + w) * (C8 * 8) + c;
  *(float4*)r = make_float4(row[0], row[1], row[2], row[3]);
  *(float4*)(r + 4) = make_float4(row[4], row[5], row[6], row[7]);
}

template <typename T>
__global__ void __launch_bounds__(256) bilinear_bwd_cols_nhwc_kernel(const float* __restrict__ rs, T* __restrict__ gx,
                                                                     int C8, int Ho, Axis ah, int Wi, Strides gxs) {
  const int h = blockIdx.y, n = blockIdx.z;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= Wi * C8) return;
  const int w = idx / C8, c = (idx - w * C8) * 8;
  int ohlo, ohhi;
  out_window(ah, h, ohlo, ohhi);
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int oh = ohlo; oh <= ohhi; ++oh) {
    int h0, h1;
    float l0, l1;
    src_index(ah, oh, h0, h1, l0, l1);
    const float wh = (h0 == h ? l0 : 0.f) + (h1 == h ? l1 : 0.f);
    if (wh == 0.f) continue;
    const float* r = rs + (((int64_t)n * Ho + oh) * Wi + w) * (C8 * 8) + c;
    const float4 a = *(const float4*)r, b = *(const float4*)(r + 4);
    const float row[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = fmaf(row[e], wh, acc[e]);
  }
  *(uint4*)(gx + (int64_t)n * gxs.n + (int64_t)h * gxs.h + (int64_t)w * gxs.w + c) = pack8<T>(acc);
}

// the NHWC kernels apply: 16-bit, channels fastest in both tensors, 16-byte aligned chunks, grid dims in range
static bool nhwc_ok(const void* a, const void* b, int64_t N, int64_t C, int64_t rows, int64_t cols, const Strides& as,
                    const Strides& bs, int dt) {
  if (dt != SSSEG_BF16 && dt != SSSEG_F16) return false;
  if (as.c != 1 || bs.c != 1 || C % 8 || C < 8) return false;
  if (((uintptr_t)a | (uintptr_t)b) % 16) return false;
  if ((as.n | as.h | as.w | bs.n | bs.h | bs.w) % 8) return false;
  return N <= 65535 && rows <= 65535 && cols * (C / 8) < 0x7fffffffLL;
}

static Strides to_strides(const int64_t* s) { return Strides{s[0], s[1], s[2], s[3]}; }

// the per-pixel fp32 kernels apply: C <= 4 channels, grid dims in range (SSSEG_BIL_PIX=0 turns them off for A/B)
static bool pix_ok(int64_t N, int64_t C, int64_t rows, int64_t cols, int dt) {
  static const bool on = [] {
    const char* e = getenv("SSSEG_BIL_PIX");
    return !(e && e[0] == '0');
  }();
  return on && dt == SSSEG_F32 && C >= 1 && C <= 4 && N <= 65535 && rows <= 65535 && cols < (1 << 24);
}

}  // namespace

extern "C" int ssseg_bilinear_fwd(const void* x, void* y, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Ho,
                                  int64_t Wo, const int64_t* xs4, const int64_t* ys4, int align_corners, int dt,
                                  ssseg_stream_t stream) {
  if (!x || !y || !xs4 || !ys4 || N < 0 || C < 0 || H < 1 || W < 1 || Ho < 1 || Wo < 1) return SSSEG_EINVAL;
  const int64_t total = N * C * Ho * Wo;
  if (total == 0) return 0;
  const Axis ah = make_axis(H, Ho, align_corners), aw = make_axis(W, Wo, align_corners);
  const Strides xs = to_strides(xs4), ys = to_strides(ys4);
  const int cf = ys.c == 1 && C > 1;
  hipStream_t s = (hipStream_t)stream;
  if (nhwc_ok(x, y, N, C, Ho, Wo, xs, ys, dt)) {
    const int C8 = (int)(C / 8);
    const dim3 g((unsigned)((Wo * C8 + 255) / 256), (unsigned)Ho, (unsigned)N), b(256);
    if (dt == SSSEG_BF16)
      hipLaunchKernelGGL(bilinear_fwd_nhwc_kernel<bf16_t>, g, b, 0, s, (const bf16_t*)x, (bf16_t*)y, C8, ah, aw, xs, ys);
    else
      hipLaunchKernelGGL(bilinear_fwd_nhwc_kernel<f16_t>, g, b, 0, s, (const f16_t*)x, (f16_t*)y, C8, ah, aw, xs, ys);
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  if (pix_ok(N, C, Ho, Wo, dt)) {   // few channels (the logits): one thread per output pixel, all channels
    const dim3 g((unsigned)((Wo + 255) / 256), (unsigned)Ho, (unsigned)N), b(256);
    auto k = C == 1 ? bilinear_fwd_pix_kernel<float, 1> : C == 2 ? bilinear_fwd_pix_kernel<float, 2>
           : C == 3 ? bilinear_fwd_pix_kernel<float, 3> : bilinear_fwd_pix_kernel<float, 4>;
    hipLaunchKernelGGL(k, g, b, 0, s, (const float*)x, (float*)y, ah, aw, xs, ys);
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  const dim3 g(ssseg_grid(total, 256, 256 * 32)), b(256);
  const bool i32 = total < 0x7fffffffLL - (1LL << 24);   // i + grid stride stays in int range
#define BIL_FWD(T)                                                                                                   \
  if (i32)                                                                                                           \
    hipLaunchKernelGGL((bilinear_fwd_kernel<T, int>), g, b, 0, s, (const T*)x, (T*)y, N, C, ah, aw, xs, ys, cf);     \
  else                                                                                                               \
    hipLaunchKernelGGL((bilinear_fwd_kernel<T, int64_t>), g, b, 0, s, (const T*)x, (T*)y, N, C, ah, aw, xs, ys, cf);
  if (dt == SSSEG_F32) {
    BIL_FWD(float)
  } else if (dt == SSSEG_BF16) {
    BIL_FWD(bf16_t)
  } else if (dt == SSSEG_F16) {
    BIL_FWD(f16_t)
  } else {
    return SSSEG_EUNSUPPORTED;
  }
#undef BIL_FWD
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t ssseg_bilinear_bwd_workspace_bytes(int64_t N, int64_t C, int64_t W, int64_t Ho) {
  if (N < 1 || C < 1 || W < 1 || Ho < 1) return 0;
  return (size_t)N * Ho * W * ((C + 7) / 8 * 8) * sizeof(float) + 256;
}

extern "C" int ssseg_bilinear_bwd_ws(const void* gy, void* gx, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Ho,
                                     int64_t Wo, const int64_t* gys4, const int64_t* gxs4, int align_corners, int dt,
                                     void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!gy || !gx || !gys4 || !gxs4 || N < 0 || C < 0 || H < 1 || W < 1 || Ho < 1 || Wo < 1) return SSSEG_EINVAL;
  if (N * C * H * W == 0) return 0;
  const Strides gys = to_strides(gys4), gxs = to_strides(gxs4);
  if (!ws || !nhwc_ok(gy, gx, N, C, H, W, gys, gxs, dt) || !nhwc_ok(gy, gx, N, C, Ho, W, gys, gxs, dt))
    return ssseg_bilinear_bwd(gy, gx, N, C, H, W, Ho, Wo, gys4, gxs4, align_corners, dt, stream);
  if (ws_bytes < ssseg_bilinear_bwd_workspace_bytes(N, C, W, Ho) || ((uintptr_t)ws & 15)) return SSSEG_EWORKSPACE;
  const Axis ah = make_axis(H, Ho, align_corners), aw = make_axis(W, Wo, align_corners);
  const int C8 = (int)(C / 8);
  hipStream_t s = (hipStream_t)stream;
  const dim3 g1((unsigned)((W * C8 + 255) / 256), (unsigned)Ho, (unsigned)N), b(256);
  const dim3 g2((unsigned)((W * C8 + 255) / 256), (unsigned)H, (unsigned)N);
  if (dt == SSSEG_BF16) {
    hipLaunchKernelGGL(bilinear_bwd_rows_nhwc_kernel<bf16_t>, g1, b, 0, s, (const bf16_t*)gy, (float*)ws, C8, (int)Ho,
                       aw, gys);
    hipLaunchKernelGGL(bilinear_bwd_cols_nhwc_kernel<bf16_t>, g2, b, 0, s, (const float*)ws, (bf16_t*)gx, C8, (int)Ho,
                       ah, (int)W, gxs);
  } else {
    hipLaunchKernelGGL(bilinear_bwd_rows_nhwc_kernel<f16_t>, g1, b, 0, s, (const f16_t*)gy, (float*)ws, C8, (int)Ho,
                       aw, gys);
    hipLaunchKernelGGL(bilinear_bwd_cols_nhwc_kernel<f16_t>, g2, b, 0, s, (const float*)ws, (f16_t*)gx, C8, (int)Ho,
                       ah, (int)W, gxs);
  }
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bilinear_bwd(const void* gy, void* gx, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Ho,
                                  int64_t Wo, const int64_t* gys4, const int64_t* gxs4, int align_corners, int dt,
                                  ssseg_stream_t stream) {
  if (!gy || !gx || !gys4 || !gxs4 || N < 0 || C < 0 || H < 1 || W < 1 || Ho < 1 || Wo < 1) return SSSEG_EINVAL;
  const int64_t total = N * C * H * W;
  if (total == 0) return 0;
  const Axis ah = make_axis(H, Ho, align_corners), aw = make_axis(W, Wo, align_corners);
  const Strides gys = to_strides(gys4), gxs = to_strides(gxs4);
  const int cf = gxs.c == 1 && C > 1;
  hipStream_t s = (hipStream_t)stream;
  if (nhwc_ok(gy, gx, N, C, H, W, gys, gxs, dt)) {
    const int C8 = (int)(C / 8);
    const dim3 g((unsigned)((W * C8 + 255) / 256), (unsigned)H, (unsigned)N), b(256);
    if (dt == SSSEG_BF16)
      hipLaunchKernelGGL(bilinear_bwd_nhwc_kernel<bf16_t>, g, b, 0, s, (const bf16_t*)gy, (bf16_t*)gx, C8, ah, aw, gys,
                         gxs);
    else
      hipLaunchKernelGGL(bilinear_bwd_nhwc_kernel<f16_t>, g, b, 0, s, (const f16_t*)gy, (f16_t*)gx, C8, ah, aw, gys,
                         gxs);
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  if (pix_ok(N, C, H, W, dt)) {
    const dim3 g((unsigned)((W + 255) / 256), (unsigned)H, (unsigned)N), b(256);
    auto k = C == 1 ? bilinear_bwd_pix_kernel<float, 1> : C == 2 ? bilinear_bwd_pix_kernel<float, 2>
           : C == 3 ? bilinear_bwd_pix_kernel<float, 3> : bilinear_bwd_pix_kernel<float, 4>;
    hipLaunchKernelGGL(k, g, b, 0, s, (const float*)gy, (float*)gx, ah, aw, gys, gxs);
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  const dim3 g(ssseg_grid(total, 256, 256 * 32)), b(256);
  const bool i32 = total < 0x7fffffffLL - (1LL << 24);   // i + grid stride stays in int range
#define BIL_BWD(T)                                                                                                     \
  if (i32)                                                                                                             \
    hipLaunchKernelGGL((bilinear_bwd_kernel<T, int>), g, b, 0, s, (const T*)gy, (T*)gx, N, C, ah, aw, gys, gxs, cf);   \
  else                                                                                                                 \
    hipLaunchKernelGGL((bilinear_bwd_kernel<T, int64_t>), g, b, 0, s, (const T*)gy, (T*)gx, N, C, ah, aw, gys, gxs, cf);
  if (dt == SSSEG_F32) {
    BIL_BWD(float)
  } else if (dt == SSSEG_BF16) {
    BIL_BWD(bf16_t)
  } else if (dt == SSSEG_F16) {
    BIL_BWD(f16_t)
  } else {
    return SSSEG_EUNSUPPORTED;
  }
#undef BIL_BWD
  SSSEG_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------------------------------------
// Rotation about the image centre (reversible_augmentations.Rotate, reference reversible_augmentations.py:5-23,
// kornia.rotate): y(p) = bilinear sample of x at M^-1 p, zeros outside, pixel centres on integer coordinates.
// M is OpenCV's / kornia's get_rotation_matrix2d(centre, angle, 1) (positive angle = counter-clockwise);
// the inverse map of a rotation is the rotation by -angle about the same centre.  NCHW fp32.
// Backward scatters each output gradient to its four taps (float atomics: this path is off the hot loop).
// ------------------------------------------------------------------------------------------------
namespace {

struct RotMap {
  float a, b, cx, cy;   // source = (a*(x-cx) + b*(y-cy) + cx, -b*(x-cx) + a*(y-cy) + cy)
};

__device__ __forceinline__ void rot_src(const RotMap& m, int x, int y, float& sx, float& sy) {
  const float dx = (float)x - m.cx, dy = (float)y - m.cy;
  sx = fmaf(m.a, dx, m.b * dy) + m.cx;
  sy = fmaf(-m.b, dx, m.a * dy) + m.cy;
}

__global__ void rotate_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t NC, int H, int W,
                                  RotMap m) {
  const int64_t total = NC * H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int px = (int)(i % W), py = (int)((i / W) % H);
    const int64_t plane = i / ((int64_t)H * W);
    float sx, sy;
    rot_src(m, px, py, sx, sy);
    const float fx = floorf(sx), fy = floorf(sy);
    const int x0 = (int)fx, y0 = (int)fy;
    const float wx = sx - fx, wy = sy - fy;
    const float* p = x + plane * H * W;
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
      const float w = ((t & 1) ? wx : 1.f - wx) * ((t >> 1) ? wy : 1.f - wy);
      if ((unsigned)xx < (unsigned)W && (unsigned)yy < (unsigned)H) v = fmaf(w, p[(int64_t)yy * W + xx], v);
    }
    y[i] = v;
  }
}

__global__ void rotate_bwd_kernel(const float* __restrict__ gy, float* __restrict__ gx, int64_t NC, int H, int W,
                                  RotMap m) {
  const int64_t total = NC * H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int px = (int)(i % W), py = (int)((i / W) % H);
    const int64_t plane = i / ((int64_t)H * W);
    float sx, sy;
    rot_src(m, px, py, sx, sy);
    const float fx = floorf(sx), fy = floorf(sy);
    const int x0 = (int)fx, y0 = (int)fy;
    const float wx = sx - fx, wy = sy - fy;
    const float g = gy[i];
    float* p = gx + plane * H * W;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
      const float w = ((t & 1) ? wx : 1.f - wx) * ((t >> 1) ? wy : 1.f - wy);
      if ((unsigned)xx < (unsigned)W && (unsigned)yy < (unsigned)H) atomicAdd(p + (int64_t)yy * W + xx, w * g);
    }
  }
}

RotMap rot_map(double angle_deg, int64_t H, int64_t W) {
  const double th = angle_deg * 3.14159265358979323846 / 180.0;
  RotMap m;
  // inverse map of the counter-clockwise rotation by `angle` (y axis pointing down): rotate back by -angle
  m.a = (float)cos(th);
  m.b = (float)(-sin(th));
  m.cx = (float)(W - 1) * 0.5f;
  m.cy = (float)(H - 1) * 0.5f;
  return m;
}

}  // namespace

extern "C" int ssseg_rotate_fwd(const float* x, float* y, int64_t N, int64_t C, int64_t H, int64_t W, double angle_deg,
                                ssseg_stream_t stream) {
  if (!x || !y || N < 0 || C < 0 || H < 1 || W < 1 || H > 0x7fffffff || W > 0x7fffffff) return SSSEG_EINVAL;
  const int64_t total = N * C * H * W;
  if (total == 0) return 0;
  hipLaunchKernelGGL(rotate_fwd_kernel, dim3(ssseg_grid(total, 256)), dim3(256), 0, (hipStream_t)stream, x, y, N * C,
                     (int)H, (int)W, rot_map(angle_deg, H, W));
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_rotate_bwd(const float* gy, float* gx, int64_t N, int64_t C, int64_t H, int64_t W, double angle_deg,
                                ssseg_stream_t stream) {
  if (!gy || !gx || N < 0 || C < 0 || H < 1 || W < 1 || H > 0x7fffffff || W > 0x7fffffff) return SSSEG_EINVAL;
  const int64_t total = N * C * H * W;
  if (total == 0) return 0;
  SSSEG_TRY(hipMemsetAsync(gx, 0, sizeof(float) * total, (hipStream_t)stream));
  hipLaunchKernelGGL(rotate_bwd_kernel, dim3(ssseg_grid(total, 256)), dim3(256), 0, (hipStream_t)stream, gy, gx, N * C,
                     (int)H, (int)W, rot_map(angle_deg, H, W));
  SSSEG_LAUNCH_CHECK();
  return 0;
}
