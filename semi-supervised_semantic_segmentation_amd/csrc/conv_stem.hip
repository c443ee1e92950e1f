// conv_stem.hip: the first convolution of an encoder (3-channel image in, e.g. the ResNet-50 stem 7x7/s2/p3,
// resnet.py Stem; the reference's encoders start the same way), gfx950.
//
// The generic engine pads the 3 input channels to the 8-channel NHWC vector and contracts k = (r, s, c) over
// 7 x 7 x 8 = 392 (13 MFMA k-steps of 32, 62 % of them multiplying zeros), through a register-staged tile
// (C % 64 != 0 keeps it off the LDS-DMA path).  Here k runs (s, c) inside one filter row r: the 4 channels
// 0..3 of the S <= 8 taps of row r are one 32-deep k-step (s*4 + c; channel 3 and taps >= S are zero), so
// the whole filter is R k-steps (7 for the stem: 1.9x less MFMA work); each lane's MFMA operand (taps 2q, 2q+1
// of its pixel, 4 channels each) comes from the block's image patch, staged once in LDS with coalesced loads.
// The packed weights [K][R][S*4] (ssseg_weight_pack with Cp = 4) sit in LDS as [BN][R][32] for the block.
// Epilogue: the engine's LDS-staged store_tile_lds (affine / residual / activation / raw copy / fused BN
// statistics, coalesced 16-byte row stores).
// Different k grouping from the engine's variants, so results match them to fp32 rounding, not bitwise.
#include "conv_kernels.h"

namespace {

constexpr int STEM_FM = 2, STEM_FN = 4, STEM_BM = 4 * STEM_FM * 16, STEM_BN = 64;
constexpr int STEM_PW = (STEM_BM - 1) * 2 + 8;   // staged image columns per filter row (stride <= 2, S <= 8)

// One block = 128 consecutive output pixels of ONE output row (host: OW % 128 == 0) x 64 channels.  The R image
// rows x STEM_PW columns the block's windows cover are staged once in LDS (channels 0..3 = 8 bytes per pixel,
// coalesced loads); each lane's MFMA operand (taps 2q, 2q+1 of its pixel in filter row r) is two ds_read_b64.
template <typename T16, int R, bool STATS>
__global__ void __launch_bounds__(256) stem_conv_kernel(const T16* __restrict__ x, const T16* __restrict__ w4,
                                                        T16* __restrict__ y, ConvGeom g, Epi<T16> ep) {
  constexpr int FM = STEM_FM, FN = STEM_FN, BM = STEM_BM, BN = STEM_BN;
  constexpr int BSZ = BN * R * 32 * 2;                       // weights [BN][R][32], bytes
  constexpr int PSZ = R * STEM_PW * 8;                       // image patch [R][PW] x 8 bytes
  constexpr int ESZ = BM * (BN * 4 + 16);                    // staged epilogue (store_tile_lds)
  constexpr int SMEM = (BSZ + PSZ) > ESZ ? (BSZ + PSZ) : ESZ;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n0 = blockIdx.y * BN;
  const long long m0 = (long long)blockIdx.x * BM;
  const int gq = lane >> 4, li = lane & 15;
  const int ox0 = (int)(m0 % g.OW);
  const int qrow = (int)(m0 / g.OW);
  const int oy = qrow % g.OH, img = qrow / g.OH;
  const int iy0 = oy * g.sy + g.py, ix0 = ox0 * g.sx + g.px;   // py, px: minus the padding
  const int pw = (BM - 1) * g.sx + g.S;                      // columns actually used

  // stage the image patch (zero outside the image) and the weights: every global load of the block is issued
  // before the first LDS write (a load-then-store loop would wait for each load in turn)
  constexpr int KP = (R * STEM_PW + 255) / 256;            // patch pixels per thread
  constexpr int KW = (BN * R * 8 + 255) / 256;             // weight 8-byte slots per thread ([BN][R][8] slots)
  uint2* P = (uint2*)(smem + BSZ);
  uint2 pv[KP], wv[KW];
  bool pok[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int i = t + 256 * k;
    const int r = i / pw, c = i - r * pw;
    const int iy = iy0 + r, ix = ix0 + c;
    pok[k] = i < R * pw && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
    const long long off = pok[k] ? (((long long)img * g.H + iy) * g.W + ix) * g.ldx : 0;
    pv[k] = *(const uint2*)(x + off);
  }
  const int SK = g.S * 4;
  const unsigned short* wsrc = (const unsigned short*)w4;
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    const int i = t + 256 * k;
    const int q = i & 7, r = (i >> 3) % R, nn = (i >> 3) / R;
    const int n = n0 + nn;
    const bool v = i < BN * R * 8 && n < g.K && q < g.S;
    wv[k] = v ? *(const uint2*)(wsrc + ((long long)n * R + r) * SK + 4 * q) : make_uint2(0u, 0u);
  }
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int i = t + 256 * k;
    if (i < R * pw) {
      const int r = i / pw, c = i - r * pw;
      P[r * STEM_PW + c] = pok[k] ? pv[k] : make_uint2(0u, 0u);
    }
  }
  unsigned short* Bs = (unsigned short*)smem;
  uint2* B8 = (uint2*)smem;                                  // [BN][R][8] 8-byte slots = [BN][R][32] shorts
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    const int i = t + 256 * k;
    if (i < BN * R * 8) B8[i] = wv[k];
  }
  __syncthreads();

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool h0 = 2 * gq < g.S, h1 = 2 * gq + 1 < g.S;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    bf16x8 af[FN], bfr[FM];
#pragma unroll
    for (int i = 0; i < FN; ++i) af[i] = *(const bf16x8*)(Bs + ((i * 16 + li) * R + r) * 32 + 8 * gq);
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int c = (wave * (FM * 16) + j * 16 + li) * g.sx + 2 * gq;   // patch column of tap 2gq
      const uint2 lo = h0 ? P[r * STEM_PW + c] : make_uint2(0u, 0u);
      const uint2 hi = h1 ? P[r * STEM_PW + c + 1] : make_uint2(0u, 0u);
      bfr[j] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc[i][j] = M16<T16>::mma(af[i], bfr[j], acc[i][j]);
  }
  // LDS-staged coalesced epilogue (waits for every wave's LDS reads first)
  store_tile_lds<T16, BM, BN, FM, FN, 256, STATS>(acc, smem, m0, n0, wave * (FM * 16), 0, lane, g, y, ep);
}

template <typename T16, int R>
void launch_stem(const void* x, const void* w4, void* y, const ConvGeom& g, const Epi<T16>& ep, hipStream_t s) {
  const dim3 grid((unsigned)(g.M / STEM_BM), (unsigned)((g.K + STEM_BN - 1) / STEM_BN));
  if (ep.stats)
    hipLaunchKernelGGL((stem_conv_kernel<T16, R, true>), grid, dim3(256), 0, s, (const T16*)x, (const T16*)w4, (T16*)y,
                       g, ep);
  else
    hipLaunchKernelGGL((stem_conv_kernel<T16, R, false>), grid, dim3(256), 0, s, (const T16*)x, (const T16*)w4,
                       (T16*)y, g, ep);
}

template <typename T16>
int dispatch_stem(const void* x, const void* w4, void* y, const ConvGeom& g, const Epi<T16>& ep, hipStream_t s) {
  switch (g.R) {
    case 7: launch_stem<T16, 7>(x, w4, y, g, ep, s); return 0;
    case 3: launch_stem<T16, 3>(x, w4, y, g, ep, s); return 0;
    default: return SSSEG_EUNSUPPORTED;
  }
}

}  // namespace

extern "C" int ssseg_conv_stem_epi(const void* x, const void* w4, void* y, const ssseg_conv_desc* d, int dt,
                                   const ssseg_conv_epilogue* epi, ssseg_stream_t stream) {
  ConvGeom g;
  if (!make_geom(d, g) || !x || !w4 || !y) return SSSEG_EINVAL;
  if (dt != SSSEG_BF16 && dt != SSSEG_F16) return SSSEG_EUNSUPPORTED;
  // taps: S <= 8 per filter row, dilation 1; input: >= 4 physical channels, 8-byte aligned pixel rows
  if (g.S < 1 || g.S > 8 || g.dy != 1 || g.dx != 1 || g.C < 4 || g.ldx % 4 || g.ldx < g.C) return SSSEG_EINVAL;
  // a block is 128 pixels of one output row, stride <= 2 (the staged patch width)
  if (g.OW % STEM_BM || g.sx < 1 || g.sx > 2 || g.sy < 1) return SSSEG_EINVAL;
  if (g.K < 1 || g.K % 16 || g.ldy % 4 || g.N < 1 || g.OH < 1 || g.OW < 1 || g.M >= 0x7fffffffLL) return SSSEG_EINVAL;
  const ssseg_conv_epilogue none = {nullptr, nullptr, nullptr, 0, nullptr, 0, 0.f, nullptr, 0, nullptr};
  const ssseg_conv_epilogue& e = epi ? *epi : none;
  if (e.residual && (e.ldr < g.K || e.ldr % 4)) return SSSEG_EINVAL;
  if (e.stats && (!e.stats_rows_host || e.stats_ld < 1 || e.stats_ld > g.K)) return SSSEG_EINVAL;
  if (e.stats && (e.scale || e.residual || e.relu || e.aux)) return SSSEG_EINVAL;
  if (e.relu < 0 || e.relu > SSSEG_ACT_LEAKY) return SSSEG_EINVAL;
  if (e.stats_rows_host) *e.stats_rows_host = 0;
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if (dt == SSSEG_BF16) {
    const Epi<bf16_t> eb{e.scale, e.shift, (const bf16_t*)e.residual, (int)e.ldr, e.relu, (bf16_t*)e.aux, e.slope,
                         e.stats, (int)e.stats_ld};
    rc = dispatch_stem<bf16_t>(x, w4, y, g, eb, s);
  } else {
    const Epi<f16_t> eh{e.scale, e.shift, (const f16_t*)e.residual, (int)e.ldr, e.relu, (f16_t*)e.aux, e.slope,
                        e.stats, (int)e.stats_ld};
    rc = dispatch_stem<f16_t>(x, w4, y, g, eh, s);
  }
  if (rc) return rc;
  if (e.stats_rows_host && e.stats) *e.stats_rows_host = (g.M + STEM_BM - 1) / STEM_BM;
  SSSEG_LAUNCH_CHECK();
  return 0;
}
