// Device train-time augmentations: a batched restatement of the albumentations pipelines of the reference config
// (configs/default_config.py:179-205 train['augmentations'], :206-212 train['unsupervised_augmentations']) after
// the host's LongestMaxSize + PadIfNeeded (data/transforms.py).  The host (data/device_augment.py) draws every
// random parameter in the pipeline's order with Python's `random` (as albumentations does) and uploads one record
// per sample; these kernels apply them to the whole batch in HBM:
//   ssseg_aug_warp       Rotate(15) o RandomResizedCrop o HorizontalFlip composed into one affine map, then one of
//                        ElasticTransform / GridDistortion / OpticalDistortion as a per-pixel coordinate map; image
//                        bilinear (OpenCV pixel-centre convention), mask nearest, reflect-101 border -- ONE
//                        resampling where albumentations resamples per transform (it also applies the distortion
//                        after the colour ops; the colour ops are per pixel, so only the blur's order differs)
//   ssseg_aug_color      RandomBrightnessContrast, ToGray, RGBShift / HueSaturationValue on the uint8 value grid
//   ssseg_aug_blur       separable Gaussian (GaussianBlur; the ElasticTransform displacement fields)
//   ssseg_aug_iso_finish ISONoise (HLS hue / luminance noise, per-image luminance std) and ToFloat -> NCHW [0, 1]
// albumentations and cv2 are absent from this image: parity with them is unpinned; the kernels are checked against
// the numpy restatement in oracle/augment_ref.py (tests/test_augment.py).
#include "common.h"

namespace {

__device__ __forceinline__ void philox(unsigned (&c)[4], uint64_t seed) {
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
// uniform in (0, 1]
__device__ __forceinline__ float u01(unsigned v) { return ((float)(v >> 8) + 1.0f) * (1.0f / 16777216.0f); }

// reflect-101 (OpenCV BORDER_REFLECT_101: ... c b | a b c ... | d c ...) and scipy 'reflect' (... b a | a b ...)
__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while ((unsigned)i >= (unsigned)n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}
__device__ __forceinline__ int reflect_sym(int i, int n) {
  while ((unsigned)i >= (unsigned)n) i = i < 0 ? -i - 1 : 2 * n - 1 - i;
  return i;
}

__device__ __forceinline__ float clamp255(float v) { return fminf(fmaxf(v, 0.f), 255.f); }
__device__ __forceinline__ float round_u8(float v) { return rintf(clamp255(v)); }

// crop-grid output pixel -> input-image coordinates (before the affine)
__device__ __forceinline__ void distort(const ssseg_aug_warp_params& p, int x, int y, int Wo, int Ho,
                                        const float* gmaps, const float* fields, int n, float& qx, float& qy) {
  qx = (float)x;
  qy = (float)y;
  if (p.distort == 1) {   // ElasticTransform: remap by (x + dx, y + dy) of the randomly affine-warped crop
    const float* f = fields + ((int64_t)p.field * Ho * Wo + (int64_t)y * Wo + x) * 2;
    const float ex = qx + f[0], ey = qy + f[1];
    qx = p.m[0] * ex + p.m[1] * ey + p.m[2];
    qy = p.m[3] * ex + p.m[4] * ey + p.m[5];
  } else if (p.distort == 2) {   // GridDistortion: separable piecewise-linear stretch of each axis
    const float* g = gmaps + (int64_t)n * (Wo + Ho);
    qx = g[x];
    qy = g[Wo + y];
  } else if (p.distort == 3) {   // OpticalDistortion: cv2.initUndistortRectifyMap with distortion (k, k, 0, 0, 0)
    const float u = (qx - p.cx) / p.fx, v = (qy - p.cy) / p.fy;
    const float r2 = u * u + v * v, kr = 1.f + p.k * r2 + p.k * r2 * r2;
    qx = p.fx * u * kr + p.cx;
    qy = p.fy * v * kr + p.cy;
  }
}

__global__ void aug_warp_kernel(const uint8_t* __restrict__ img, const uint8_t* __restrict__ mask, int Cm, int N, int H,
                                int W, float* __restrict__ out_img, float* __restrict__ out_mask, int Ho, int Wo,
                                const ssseg_aug_warp_params* __restrict__ params, const float* __restrict__ gmaps,
                                const float* __restrict__ fields, int nchw01) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, n = blockIdx.z;
  if (x >= Wo) return;
  const ssseg_aug_warp_params p = params[n];
  float qx, qy;
  distort(p, x, y, Wo, Ho, gmaps, fields, n, qx, qy);
  const float sx = p.a[0] * qx + p.a[1] * qy + p.a[2], sy = p.a[3] * qx + p.a[4] * qy + p.a[5];
  const int64_t opix = ((int64_t)n * Ho + y) * Wo + x, plane = (int64_t)Ho * Wo;
  // image: bilinear (cv2.INTER_LINEAR), border reflect-101 or constant 0
  const float fx0 = floorf(sx), fy0 = floorf(sy);
  const float lx = sx - fx0, ly = sy - fy0;
  const int ix = (int)fx0, iy = (int)fy0;
  const uint8_t* ib = img + (int64_t)n * H * W * 3;
  float v[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    int xx = ix + (t & 1), yy = iy + (t >> 1);
    const float wgt = ((t & 1) ? lx : 1.f - lx) * ((t >> 1) ? ly : 1.f - ly);
    if (p.border == 1) {
      xx = reflect101(xx, W);
      yy = reflect101(yy, H);
    } else if ((unsigned)xx >= (unsigned)W || (unsigned)yy >= (unsigned)H) {
      continue;
    }
    const uint8_t* px = ib + ((int64_t)yy * W + xx) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] += wgt * (float)px[c];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float r = round_u8(v[c]);   // the uint8 result of the resampling
    if (nchw01) out_img[(int64_t)n * 3 * plane + c * plane + (int64_t)y * Wo + x] = r * (1.f / 255.f);
    else out_img[opix * 3 + c] = r;
  }
  if (mask) {   // nearest (cvRound of the source coordinate), same border; ToFloat -> NCHW [0, 1]
    int mx = __float2int_rn(sx), my = __float2int_rn(sy);
    bool ok = true;
    if (p.border == 1) {
      mx = reflect101(mx, W);
      my = reflect101(my, H);
    } else {
      ok = (unsigned)mx < (unsigned)W && (unsigned)my < (unsigned)H;
    }
    const uint8_t* mb = mask + (((int64_t)n * H + my) * W + mx) * Cm;
    for (int c = 0; c < Cm; ++c)
      out_mask[((int64_t)n * Cm + c) * plane + (int64_t)y * Wo + x] = ok ? (float)mb[c] * (1.f / 255.f) : 0.f;
  }
}

// RGB (0..255) <-> OpenCV 8-bit HSV (H in [0, 180), S, V in [0, 255])
__device__ __forceinline__ void rgb2hsv8(float r, float g, float b, float& h, float& s, float& v) {
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b)), d = mx - mn;
  v = mx;
  s = mx > 0.f ? 255.f * d / mx : 0.f;
  float hd = 0.f;
  if (d > 0.f) {
    if (mx == r) hd = 60.f * (g - b) / d;
    else if (mx == g) hd = 120.f + 60.f * (b - r) / d;
    else hd = 240.f + 60.f * (r - g) / d;
    if (hd < 0.f) hd += 360.f;
  }
  h = rintf(hd * 0.5f);
  if (h >= 180.f) h -= 180.f;
  s = rintf(s);
  v = rintf(v);
}
__device__ __forceinline__ void hsv82rgb(float h, float s, float v, float& r, float& g, float& b) {
  const float hd = h * 2.f, sf = s / 255.f;
  const float c = v * sf, hp = hd / 60.f;
  const float x = c * (1.f - fabsf(fmodf(hp, 2.f) - 1.f)), m = v - c;
  float r1 = 0.f, g1 = 0.f, b1 = 0.f;
  const int sector = (int)floorf(hp) % 6;
  switch (sector) {
    case 0: r1 = c; g1 = x; break;
    case 1: r1 = x; g1 = c; break;
    case 2: g1 = c; b1 = x; break;
    case 3: g1 = x; b1 = c; break;
    case 4: r1 = x; b1 = c; break;
    default: r1 = c; b1 = x; break;
  }
  r = round_u8(r1 + m);
  g = round_u8(g1 + m);
  b = round_u8(b1 + m);
}

__global__ void aug_color_kernel(float* __restrict__ img, int64_t HW, const ssseg_aug_color_params* __restrict__ params) {
  const int n = blockIdx.y;
  const ssseg_aug_color_params p = params[n];
  if (!p.bc && !p.gray && !p.rgb && !p.hsv) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += (int64_t)gridDim.x * blockDim.x) {
    float* px = img + ((int64_t)n * HW + i) * 3;
    float r = px[0], g = px[1], b = px[2];
    if (p.bc) {   // brightness_contrast_adjust (uint8 LUT): clip(v * alpha + beta * 255), then astype(uint8)
      r = floorf(clamp255(r * p.alpha + p.beta * 255.f));
      g = floorf(clamp255(g * p.alpha + p.beta * 255.f));
      b = floorf(clamp255(b * p.alpha + p.beta * 255.f));
    }
    if (p.gray) {   // ToGray: cv2 COLOR_RGB2GRAY on uint8 -- Q14 fixed point (0.299, 0.587, 0.114) = (4899, 9617,
                    // 1868) / 2^14, rounded (+2^13) -- replicated to 3 channels (GRAY2RGB); r, g, b are integers here
      const int y = ((int)r * 4899 + (int)g * 9617 + (int)b * 1868 + 8192) >> 14;
      r = g = b = (float)y;
    }
    if (p.rgb) {   // RGBShift (uint8 LUT): clip(v + shift).astype(uint8)
      r = floorf(clamp255(r + p.shift[0]));
      g = floorf(clamp255(g + p.shift[1]));
      b = floorf(clamp255(b + p.shift[2]));
    }
    if (p.hsv) {   // HueSaturationValue on 8-bit HSV (uint8 LUTs): hue mod 180, sat / val clip, then astype(uint8)
      float h, s, v;
      rgb2hsv8(r, g, b, h, s, v);
      h = fmodf(h + p.hsv_shift[0], 180.f);
      if (h < 0.f) h += 180.f;
      h = floorf(h);
      s = floorf(clamp255(s + p.hsv_shift[1]));
      v = floorf(clamp255(v + p.hsv_shift[2]));
      hsv82rgb(h, s, v, r, g, b);
    }
    px[0] = r;
    px[1] = g;
    px[2] = b;
  }
}

// separable Gaussian, one axis: out[n][y][x][c] = sum_k w[n][k] * in[n][refl(y or x + k - r)][..][c]
template <bool VERT>
__global__ void aug_blur_kernel(const float* __restrict__ in, float* __restrict__ out, int H, int W, int C,
                                const int* __restrict__ radius, const float* __restrict__ weights, int wmax, int sym,
                                int round8) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, n = blockIdx.z;
  if (x >= W) return;
  const int r = radius[n];
  const float* w = weights + (int64_t)n * wmax;
  const float* ib = in + (int64_t)n * H * W * C;
  float* ob = out + (((int64_t)n * H + y) * W + x) * C;
  for (int c = 0; c < C; ++c) {
    float acc;
    if (r == 0) {
      acc = ib[((int64_t)y * W + x) * C + c];
    } else {
      acc = 0.f;
      for (int k = -r; k <= r; ++k) {
        const int yy = VERT ? (sym ? reflect_sym(y + k, H) : reflect101(y + k, H)) : y;
        const int xx = VERT ? x : (sym ? reflect_sym(x + k, W) : reflect101(x + k, W));
        acc = fmaf(w[k + r], ib[((int64_t)yy * W + xx) * C + c], acc);
      }
      if (round8 && VERT) acc = round_u8(acc);
    }
    ob[c] = acc;
  }
}

// RGB [0, 1] -> HLS (H in degrees, L, S in [0, 1]) and back (cv2.COLOR_RGB2HLS / HLS2RGB on float32)
__device__ __forceinline__ void rgb2hls(float r, float g, float b, float& h, float& l, float& s) {
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b)), d = mx - mn;
  l = 0.5f * (mx + mn);
  h = 0.f;
  s = 0.f;
  if (d > 1e-12f) {
    s = l < 0.5f ? d / (mx + mn) : d / (2.f - mx - mn);
    if (mx == r) h = 60.f * (g - b) / d;
    else if (mx == g) h = 120.f + 60.f * (b - r) / d;
    else h = 240.f + 60.f * (r - g) / d;
    if (h < 0.f) h += 360.f;
  }
}
__device__ __forceinline__ float hls_c(float p, float q, float t) {
  if (t < 0.f) t += 360.f;
  if (t >= 360.f) t -= 360.f;
  if (t < 60.f) return p + (q - p) * t / 60.f;
  if (t < 180.f) return q;
  if (t < 240.f) return p + (q - p) * (240.f - t) / 60.f;
  return p;
}
__device__ __forceinline__ void hls2rgb(float h, float l, float s, float& r, float& g, float& b) {
  if (s <= 0.f) {
    r = g = b = l;
    return;
  }
  const float q = l < 0.5f ? l * (1.f + s) : l + s - l * s, p = 2.f * l - q;
  r = hls_c(p, q, h + 120.f);
  g = hls_c(p, q, h);
  b = hls_c(p, q, h - 120.f);
}

// per-image sums of the HLS luminance (fp64): st[n] = (sum L, sum L^2)
__global__ void aug_lum_stats_kernel(const float* __restrict__ img, int64_t HW, const ssseg_aug_color_params* params,
                                     double* __restrict__ st) {
  const int n = blockIdx.y;
  if (!params[n].iso) return;
  __shared__ double red[2][256];
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += (int64_t)gridDim.x * blockDim.x) {
    const float* px = img + ((int64_t)n * HW + i) * 3;
    const float r = px[0] / 255.f, g = px[1] / 255.f, b = px[2] / 255.f;
    const double l = 0.5 * ((double)fmaxf(r, fmaxf(g, b)) + (double)fminf(r, fminf(g, b)));
    s1 += l;
    s2 += l * l;
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    atomicAdd(st + 2 * n, red[0][0]);
    atomicAdd(st + 2 * n + 1, red[1][0]);
  }
}

// Poisson(lambda) by inversion (lambda <= 80: e^-lambda stays a normal float)
__device__ __forceinline__ float poisson(float lambda, float u) {
  float p = expf(-lambda), F = p;
  int k = 0;
  while (u > F && k < 1024) {
    ++k;
    p *= lambda / (float)k;
    F += p;
    if (p < 1e-30f && (float)k > lambda) break;
  }
  return (float)k;
}

// ISONoise (per ISO sample) + ToFloat: NHWC [0, 255] -> NCHW [0, 1]
__global__ void aug_iso_finish_kernel(const float* __restrict__ img, float* __restrict__ out, int64_t HW,
                                      const ssseg_aug_color_params* __restrict__ params, const double* __restrict__ st,
                                      uint64_t seed) {
  const int n = blockIdx.y;
  const ssseg_aug_color_params p = params[n];
  float lam = 0.f;
  if (p.iso) {
    const double m = st[2 * n] / (double)HW, var = fmax(st[2 * n + 1] / (double)HW - m * m, 0.0);
    lam = fminf((float)sqrt(var) * p.iso_intensity * 255.f, 80.f);
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += (int64_t)gridDim.x * blockDim.x) {
    const float* px = img + ((int64_t)n * HW + i) * 3;
    float r = px[0], g = px[1], b = px[2];
    if (p.iso) {
      unsigned c[4] = {(unsigned)i, (unsigned)(i >> 32), (unsigned)n, 0x150u};
      philox(c, seed);
      const float u1 = u01(c[0]), u2 = u01(c[1]), u3 = u01(c[2]);
      const float nrm = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
      float h, l, s;
      rgb2hls(r / 255.f, g / 255.f, b / 255.f, h, l, s);
      h += nrm * p.iso_color_std;
      if (h < 0.f) h += 360.f;
      if (h > 360.f) h -= 360.f;
      l += (poisson(lam, u3) / 255.f) * (1.f - l);
      hls2rgb(h, l, s, r, g, b);
      r = floorf(clamp255(r * 255.f));   // image.astype(np.uint8)
      g = floorf(clamp255(g * 255.f));
      b = floorf(clamp255(b * 255.f));
    }
    const int64_t base = (int64_t)n * 3 * HW + i;
    out[base] = r * (1.f / 255.f);
    out[base + HW] = g * (1.f / 255.f);
    out[base + 2 * HW] = b * (1.f / 255.f);
  }
}

// uniform(-1, 1) displacement noise for the ElasticTransform fields: f[n][y][x][2]
__global__ void aug_uniform_field_kernel(float* __restrict__ f, int64_t total, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned c[4] = {(unsigned)i, (unsigned)(i >> 32), 0xe1a5u, 0u};
    philox(c, seed);
    f[i] = u01(c[0]) * 2.f - 1.f;
  }
}

}  // namespace

extern "C" int ssseg_aug_warp(const uint8_t* img, const uint8_t* mask, int64_t mask_c, int64_t N, int64_t H, int64_t W,
                              float* out_img, float* out_mask, int64_t Ho, int64_t Wo,
                              const ssseg_aug_warp_params* params, const float* gmaps, const float* fields,
                              int out_nchw01, ssseg_stream_t stream) {
  if (!img || !out_img || !params || N < 1 || H < 1 || W < 1 || Ho < 1 || Wo < 1 || N > 65535 || Ho > 65535 ||
      (mask && (!out_mask || mask_c < 1)) || H * W * 3 > 0x7fffffffLL)
    return SSSEG_EINVAL;
  const dim3 g((unsigned)((Wo + 127) / 128), (unsigned)Ho, (unsigned)N), b(128);
  hipLaunchKernelGGL(aug_warp_kernel, g, b, 0, (hipStream_t)stream, img, mask, (int)mask_c, (int)N, (int)H, (int)W,
                     out_img, out_mask, (int)Ho, (int)Wo, params, gmaps, fields, out_nchw01);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_aug_color(float* img, int64_t N, int64_t H, int64_t W, const ssseg_aug_color_params* params,
                               ssseg_stream_t stream) {
  if (!img || !params || N < 1 || H < 1 || W < 1 || N > 65535) return SSSEG_EINVAL;
  const int64_t HW = H * W;
  const dim3 g((unsigned)std::min<int64_t>((HW + 255) / 256, 1024), (unsigned)N), b(256);
  hipLaunchKernelGGL(aug_color_kernel, g, b, 0, (hipStream_t)stream, img, HW, params);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_aug_blur(float* x, float* tmp, int64_t N, int64_t H, int64_t W, int64_t C, const int32_t* radius,
                              const float* weights, int64_t wmax, int sym_border, int round_u8_out,
                              ssseg_stream_t stream) {
  if (!x || !tmp || !radius || !weights || N < 1 || H < 1 || W < 1 || C < 1 || N > 65535 || H > 65535 || wmax < 1)
    return SSSEG_EINVAL;
  const dim3 g((unsigned)((W + 127) / 128), (unsigned)H, (unsigned)N), b(128);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(aug_blur_kernel<false>, g, b, 0, s, (const float*)x, tmp, (int)H, (int)W, (int)C, radius, weights,
                     (int)wmax, sym_border, round_u8_out);
  hipLaunchKernelGGL(aug_blur_kernel<true>, g, b, 0, s, (const float*)tmp, x, (int)H, (int)W, (int)C, radius, weights,
                     (int)wmax, sym_border, round_u8_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_aug_iso_finish(const float* img, float* out, int64_t N, int64_t H, int64_t W,
                                    const ssseg_aug_color_params* params, double* stats_ws, uint64_t seed,
                                    ssseg_stream_t stream) {
  if (!img || !out || !params || !stats_ws || N < 1 || H < 1 || W < 1 || N > 65535) return SSSEG_EINVAL;
  const int64_t HW = H * W;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(stats_ws, 0, sizeof(double) * 2 * N, s) != hipSuccess) return SSSEG_EINVAL;
  const dim3 g((unsigned)std::min<int64_t>((HW + 255) / 256, 512), (unsigned)N), b(256);
  hipLaunchKernelGGL(aug_lum_stats_kernel, g, b, 0, s, img, HW, params, stats_ws);
  hipLaunchKernelGGL(aug_iso_finish_kernel, g, b, 0, s, img, out, HW, params, (const double*)stats_ws, seed);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_aug_uniform_field(float* f, int64_t n, uint64_t seed, ssseg_stream_t stream) {
  if (!f || n < 1) return SSSEG_EINVAL;
  hipLaunchKernelGGL(aug_uniform_field_kernel, dim3(ssseg_grid(n, 256)), dim3(256), 0, (hipStream_t)stream, f, n, seed);
  SSSEG_LAUNCH_CHECK();
  return 0;
}
