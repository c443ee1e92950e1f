// CowMix mask generation (reference cowmix.py:6-69) and pixel mixing (cowmix.py:72-73) for gfx950.
//
// Pipeline per call (all on `stream`, no host sync, graph-capturable):
//   memset(stats) -> taps (K from max sigma on device) -> vertical pass (noise -> tmp)
//   -> horizontal pass (tmp -> field, + per-sample sum / sum of squares in fp64)
//   -> finalize (thr = erfinv(2p-1)*sqrt(2)*std + mean) -> threshold (mask = field > thr)
// Both passes stage a row/column window of the input in LDS and run the taps in the reference's
// order (k = 0..K-1), fp32 fused multiply-add.  HBM traffic: read noise, write+read tmp, write+read
// field, write mask = 6 * 4 B per pixel (the field round trip is needed for the global statistics).
#include "common.h"

namespace {

constexpr int KCAP = 1023;       // max window (sigma_max <= 170); larger K writes NaN masks
constexpr int KC = 128;          // taps staged per chunk

struct CowmixWs {
  double* stats;   // [B][2]
  int* K;          // [1] (+ padding)
  float* taps;     // [B][KCAP]
  float* tmp;      // [B][H][W]
  float* thr;      // [B]
};

static size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

static size_t carve(CowmixWs* w, void* base, int64_t B, int64_t H, int64_t W) {
  char* p = (char*)base;
  size_t off = 0;
  if (w) w->stats = (double*)(p + off);
  off = align16(off + sizeof(double) * 2 * B);
  if (w) w->K = (int*)(p + off);
  off = align16(off + 16);
  if (w) w->taps = (float*)(p + off);
  off = align16(off + sizeof(float) * KCAP * B);
  if (w) w->tmp = (float*)(p + off);
  off = align16(off + sizeof(float) * B * H * W);
  if (w) w->thr = (float*)(p + off);
  off = align16(off + sizeof(float) * B);
  return off;
}

// K = int(round(max sigma * 3) * 2) + 1 (cowmix.py:30; Python round = half-to-even = rint),
// taps_b[k] = exp(-x_k^2 / (2 sigma_b^2)) / sum, x_k = k + floor(-K/2) (+0.5 if K even) (cowmix.py:6-11).
// One block per sample b (every block derives K from all B sigmas itself; block 0 publishes it).
__global__ void __launch_bounds__(256) cowmix_taps_kernel(const float* sigma, int B, float* taps, int* Kout) {
  __shared__ float smax;
  __shared__ float red[4];
  if (threadIdx.x == 0) {
    float m = sigma[0];
    for (int i = 1; i < B; ++i) m = fmaxf(m, sigma[i]);
    smax = m;
  }
  __syncthreads();
  const double r = rint((double)smax * 3.0);
  long long Kl = (long long)r * 2 + 1;
  const int K = (Kl > KCAP || Kl < 1) ? -1 : (int)Kl;
  if (blockIdx.x == 0 && threadIdx.x == 0) *Kout = K;
  if (K < 0) return;
  const int x_first = (-K) >> 1;        // floor(-K/2)
  const float half = (K % 2 == 0) ? 0.5f : 0.f;
  const int b = blockIdx.x;
  const float s = sigma[b];
  const float denom = 2.f * (s * s);
  float part = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float x = (float)(x_first + k) + half;
    const float g = expf(-(x * x) / denom);
    taps[(size_t)b * KCAP + k] = g;
    part += g;
  }
  const float tot = block_sum(part, red);
  for (int k = threadIdx.x; k < K; k += blockDim.x) taps[(size_t)b * KCAP + k] /= tot;
}

// Vertical pass: out[b][y][x] = sum_k g[k] * in[b][y - K/2 + k][x] (zero outside).
// Block: 64 columns x 64 rows; thread (ty, tx) owns column tx and rows ty*16 .. ty*16+15.  Register window: per 8 taps
// a thread reads the 23 staged rows its 16 outputs x 8 taps touch once (not 128 LDS reads), then 128 FMAs in the
// same order per output (k ascending): bit-identical to the one-read-per-FMA loop it replaces (64 -> LDS-light).
constexpr int VTH = 64;
__global__ void __launch_bounds__(256) cowmix_vblur_kernel(const float* __restrict__ in, const float* __restrict__ taps,
                                                           const int* Kp, float* __restrict__ out, int H, int W) {
  __shared__ float tile[(VTH + KC - 1) * 64];
  __shared__ float tp[KC];
  const int K = *Kp;
  if (K < 0) return;
  const int b = blockIdx.z, x0 = blockIdx.x * 64, y0 = blockIdx.y * VTH;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int pad = K >> 1, x = x0 + tx;
  const float* src = in + (size_t)b * H * W;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (int k0 = 0; k0 < K; k0 += KC) {
    const int kc = min(KC, K - k0);
    if (threadIdx.x < kc) tp[threadIdx.x] = taps[(size_t)b * KCAP + k0 + threadIdx.x];
    const int rows = VTH + kc - 1;
    for (int r = ty; r < rows; r += 4) {
      const int iy = y0 - pad + k0 + r;
      tile[r * 64 + tx] = (iy >= 0 && iy < H && x < W) ? src[(size_t)iy * W + x] : 0.f;
    }
    __syncthreads();
    const float* col = tile + (ty * 16) * 64 + tx;
    int k = 0;
    for (; k + 8 <= kc; k += 8) {
      float win[23];
#pragma unroll
      for (int i = 0; i < 23; ++i) win[i] = col[(k + i) * 64];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float g = tp[k + u];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = fmaf(g, win[u + j], acc[j]);
      }
    }
    for (; k < kc; ++k) {
      const float g = tp[k];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = fmaf(g, col[(j + k) * 64], acc[j]);
    }
    __syncthreads();
  }
  if (x < W) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int y = y0 + ty * 16 + j;
      if (y < H) out[((size_t)b * H + y) * W + x] = acc[j];
    }
  }
}

// Horizontal pass + per-sample statistics.  Block: 8 rows x 256 columns; thread (ty, tx) owns row ty and the two runs
// of 4 consecutive columns 4 tx .. 4 tx + 3 and 128 + 4 tx .. 128 + 4 tx + 3 (lanes 16 bytes apart: conflict-free
// 16-byte LDS reads; the row stride is 4 banks off the next row's).  Register window: per 8 taps a thread reads the 12
// staged values each run's 4 outputs x 8 taps touch (three 16-byte reads), then 32 FMAs per run in the same order per
// output (k ascending): bit-identical to the one-read-per-FMA loop.
constexpr int HTW = 256, HROWS = 8, HLD = HTW + KC + 4;
__global__ void __launch_bounds__(256) cowmix_hblur_kernel(const float* __restrict__ in, const float* __restrict__ taps,
                                                           const int* Kp, float* __restrict__ out, double* stats,
                                                           int H, int W) {
  __shared__ __attribute__((aligned(16))) float tile[HROWS * HLD];
  __shared__ float tp[KC];
  __shared__ double red[4];
  const int K = *Kp;
  if (K < 0) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int b = blockIdx.z, x0 = blockIdx.x * HTW, y = blockIdx.y * HROWS + ty;
  const int pad = K >> 1;
  const float* src = in + ((size_t)b * H + min(y, H - 1)) * W;
  float acc[2][4];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[g][j] = 0.f;
  for (int k0 = 0; k0 < K; k0 += KC) {
    const int kc = min(KC, K - k0);
    if (threadIdx.x < kc) tp[threadIdx.x] = taps[(size_t)b * KCAP + k0 + threadIdx.x];
    const int cols = HTW + kc - 1;
    for (int c = tx; c < cols; c += 32) {
      const int ix = x0 - pad + k0 + c;
      tile[ty * HLD + c] = (ix >= 0 && ix < W && y < H) ? src[ix] : 0.f;
    }
    __syncthreads();
    const float* row = tile + ty * HLD + 4 * tx;
    int k = 0;
    for (; k + 8 <= kc; k += 8) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        float win[12];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float4 v = *(const float4*)(row + 128 * g + k + 4 * i);
          win[4 * i] = v.x;
          win[4 * i + 1] = v.y;
          win[4 * i + 2] = v.z;
          win[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float gk = tp[k + u];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[g][j] = fmaf(gk, win[u + j], acc[g][j]);
        }
      }
    }
    for (; k < kc; ++k) {
      const float gk = tp[k];
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[g][j] = fmaf(gk, row[128 * g + k + j], acc[g][j]);
    }
    __syncthreads();
  }
  double s1 = 0.0, s2 = 0.0;
  if (y < H) {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int x = x0 + 128 * g + 4 * tx + j;
        if (x < W) {
          out[((size_t)b * H + y) * W + x] = acc[g][j];
          s1 += (double)acc[g][j];
          s2 += (double)acc[g][j] * (double)acc[g][j];
        }
      }
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red);
  if (threadIdx.x == 0) {
    atomicAdd(&stats[2 * b], s1);
    atomicAdd(&stats[2 * b + 1], s2);
  }
}

// thr = erfinv(2p-1) * sqrt(2) * std + mean, float32 like cowmix.py:64-66; std unbiased (N-1).
__global__ void cowmix_finalize_kernel(const double* stats, const float* p, const int* Kp, int B, int64_t N,
                                       float* thr, float* thr_out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double n = (double)N;
  const double s1 = stats[2 * b], s2 = stats[2 * b + 1];
  const double mean = s1 / n;
  double var = (s2 - s1 * mean) / (n - 1.0);
  var = var < 0.0 ? 0.0 : var;
  const float meanf = (float)mean, stdf = (float)sqrt(var);
  const float factor = erfinvf(2.f * p[b] - 1.f) * 1.41421354f;  // (float)math.sqrt(2.0)
  float t = factor * stdf + meanf;
  if (*Kp < 0) t = __int_as_float(0x7fc00000);
  thr[b] = t;
  if (thr_out) thr_out[b] = t;
}

__global__ void cowmix_threshold_kernel(const float* field, const float* thr, float* mask, int64_t HW, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const float t = thr[i / HW];
    const float f = field[i];
    mask[i] = (f > t) ? 1.f : (t != t ? t : 0.f);
  }
}

// ------------------------------------------------------------------------------------------------
// Philox-4x32-10 normal(0,1) (Box-Muller) for throughput-mode noise.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox_round(unsigned (&c)[4], unsigned k0, unsigned k1) {
  const unsigned M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  unsigned hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
  unsigned hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
  unsigned n0 = hi1 ^ c[1] ^ k0, n1 = lo1, n2 = hi0 ^ c[3] ^ k1, n3 = lo0;
  c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
}

// the Philox counter offset from device memory (graph-replayable draws: every replay reads the advanced counter) or
// from the argument
__device__ __forceinline__ uint64_t rng_offset(const unsigned long long* dev, uint64_t host, uint64_t add) {
  return (dev ? (uint64_t)*dev : host) + add;
}

__global__ void normal_kernel(float* out, int64_t n, uint64_t seed, uint64_t offset,
                              const unsigned long long* offset_dev = nullptr, uint64_t add = 0) {
  offset = rng_offset(offset_dev, offset, add);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q * 4 < n; q += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t ctr = offset + (uint64_t)q;
    unsigned c[4] = {(unsigned)ctr, (unsigned)(ctr >> 32), 0u, 0u};
    unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      philox_round(c, k0, k1);
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    float z[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float u1 = ((float)(c[2 * h] >> 8) + 0.5f) * (1.0f / 16777216.0f);
      const float u2 = (float)(c[2 * h + 1] >> 8) * (1.0f / 16777216.0f);
      const float rad = sqrtf(-2.f * logf(u1));
      float s, co;
      sincosf(6.283185307179586f * u2, &s, &co);
      z[2 * h] = rad * co;
      z[2 * h + 1] = rad * s;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (q * 4 + j < n) out[q * 4 + j] = z[j];
  }
}

// p_b = lo + u*(hi-lo), sigma_b = exp(llo + u'*(lhi-llo)) from Philox uniforms (stream 1 of the key)
__global__ void cowmix_draw_kernel(float* p, float* sigma, int B, float lo, float hi, float llo, float lhi, uint64_t seed,
                                   uint64_t offset, const unsigned long long* offset_dev = nullptr) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  offset = rng_offset(offset_dev, offset, 0);
  unsigned c[4] = {(unsigned)(offset + b), (unsigned)((offset + b) >> 32), 1u, 0u};
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const float u1 = (float)(c[0] >> 8) * (1.0f / 16777216.0f), u2 = (float)(c[1] >> 8) * (1.0f / 16777216.0f);
  p[b] = lo + u1 * (hi - lo);
  sigma[b] = expf(llo + u2 * (lhi - llo));
}

__global__ void rng_advance_kernel(unsigned long long* offset_dev, unsigned long long inc) { *offset_dev += inc; }

template <typename T>
__global__ void mix_kernel(const T* a, const T* b, const float* m, T* out, int64_t C, int64_t HW, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = i % HW, n = i / (C * HW);
    const float mm = m[n * HW + pix];
    const float v = io<T>::ld(a, i) * mm + io<T>::ld(b, i) * (1.f - mm);
    io<T>::st(out, i, v);
  }
}

}  // namespace

extern "C" size_t ssseg_cowmix_workspace_bytes(int64_t B, int64_t H, int64_t W) {
  return carve(nullptr, nullptr, B, H, W);
}

extern "C" int ssseg_cowmix_mask(const float* noise, const float* sigma, const float* p, int64_t B, int64_t H,
                                 int64_t W, float* mask_out, float* field_out, float* thr_out, void* workspace,
                                 size_t workspace_bytes, ssseg_stream_t stream) {
  if (B < 1 || H < 1 || W < 1 || !noise || !sigma || !p || !mask_out) return SSSEG_EINVAL;
  if (!workspace || workspace_bytes < ssseg_cowmix_workspace_bytes(B, H, W)) return SSSEG_EWORKSPACE;
  if (B > 65535 || H > (1 << 24)) return SSSEG_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  CowmixWs w;
  carve(&w, workspace, B, H, W);
  float* field = field_out ? field_out : mask_out;   // threshold pass is in-place safe
  SSSEG_TRY(hipMemsetAsync(w.stats, 0, sizeof(double) * 2 * B, s));
  hipLaunchKernelGGL(cowmix_taps_kernel, dim3((unsigned)B), dim3(256), 0, s, sigma, (int)B, w.taps, w.K);
  hipLaunchKernelGGL(cowmix_vblur_kernel, dim3((W + 63) / 64, (H + VTH - 1) / VTH, B), dim3(256), 0, s, noise,
                     w.taps, w.K, w.tmp, (int)H, (int)W);
  hipLaunchKernelGGL(cowmix_hblur_kernel, dim3((W + HTW - 1) / HTW, (H + HROWS - 1) / HROWS, B), dim3(256), 0, s, w.tmp,
                     w.taps,
                     w.K, field, w.stats, (int)H, (int)W);
  hipLaunchKernelGGL(cowmix_finalize_kernel, dim3((B + 63) / 64), dim3(64), 0, s, w.stats, p, w.K, (int)B, H * W,
                     w.thr, thr_out);
  const int64_t total = B * H * W;
  hipLaunchKernelGGL(cowmix_threshold_kernel, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, field, w.thr, mask_out,
                     H * W, total);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_normal_f32(float* out, int64_t n, uint64_t seed, uint64_t offset, ssseg_stream_t stream) {
  if (!out || n < 0) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(normal_kernel, dim3(ssseg_grid((n + 3) / 4, 256)), dim3(256), 0, (hipStream_t)stream, out, n,
                     seed, offset);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_cowmix_draw(float* p, float* sigma, float* noise, int64_t B, int64_t HW, double prop_lo,
                                 double prop_hi, double sigma_lo, double sigma_hi, uint64_t seed, uint64_t offset,
                                 ssseg_stream_t stream) {
  if (!p || !sigma || !noise || B < 1 || HW < 1 || sigma_lo <= 0 || sigma_hi <= 0) return SSSEG_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cowmix_draw_kernel, dim3((B + 63) / 64), dim3(64), 0, s, p, sigma, (int)B, (float)prop_lo,
                     (float)prop_hi, (float)log(sigma_lo), (float)log(sigma_hi), seed, offset);
  const int64_t n = B * HW;
  hipLaunchKernelGGL(normal_kernel, dim3(ssseg_grid((n + 3) / 4, 256)), dim3(256), 0, s, noise, n, seed,
                     offset + (uint64_t)B);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_cowmix_draw_dev(float* p, float* sigma, float* noise, int64_t B, int64_t HW, double prop_lo,
                                     double prop_hi, double sigma_lo, double sigma_hi, uint64_t seed,
                                     unsigned long long* offset_dev, ssseg_stream_t stream) {
  if (!p || !sigma || !noise || !offset_dev || B < 1 || HW < 1 || sigma_lo <= 0 || sigma_hi <= 0) return SSSEG_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cowmix_draw_kernel, dim3((B + 63) / 64), dim3(64), 0, s, p, sigma, (int)B, (float)prop_lo,
                     (float)prop_hi, (float)log(sigma_lo), (float)log(sigma_hi), seed, (uint64_t)0,
                     (const unsigned long long*)offset_dev);
  const int64_t n = B * HW;
  hipLaunchKernelGGL(normal_kernel, dim3(ssseg_grid((n + 3) / 4, 256)), dim3(256), 0, s, noise, n, seed, (uint64_t)0,
                     (const unsigned long long*)offset_dev, (uint64_t)B);
  // the same advance as the host-counter form: B + ceil(B*HW / 4) + 1
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, s, offset_dev,
                     (unsigned long long)(B + (n + 3) / 4 + 1));
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_mix(const void* a, const void* b, const float* mask, void* out, int64_t B, int64_t C,
                         int64_t HW, int dt, ssseg_stream_t stream) {
  if (!a || !b || !mask || !out || B < 0 || C < 0 || HW < 0) return SSSEG_EINVAL;
  const int64_t total = B * C * HW;
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dt == SSSEG_F32)
    hipLaunchKernelGGL(mix_kernel<float>, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, (const float*)a,
                       (const float*)b, mask, (float*)out, C, HW, total);
  else if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(mix_kernel<bf16_t>, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, (const bf16_t*)a,
                       (const bf16_t*)b, mask, (bf16_t*)out, C, HW, total);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(mix_kernel<f16_t>, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, (const f16_t*)a,
                       (const f16_t*)b, mask, (f16_t*)out, C, HW, total);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}
