// Pointwise (1x1 / stride-1 / unpadded) contraction over 64 or 128 input channels: variants 26 (64-pixel wave
// tiles) and 27 (32-pixel wave tiles) of the engine's autotuner (conv.hip).  ResNet-50's bottleneck expansions and
// their input gradients (64 -> 256 @16x128^2, 128 -> 512 @16x64^2, 256 -> 64 dgrad, ...): one k-tile per output tile,
// so the LDS-DMA kernels spend a launch on load -> 8 MFMAs -> LDS-staged epilogue chains with two or three blocks per
// CU and ~10 tile rounds in sequence, 2 TB/s on a layer whose bytes are 4x its flops' worth.
//
// Here nothing is staged and no wave waits for another: each wave keeps one 64-channel slice of the weights in
// registers (loaded once: its slice is fixed for the launch), loads its pixels' channel chunks straight into MFMA
// B fragments, and walks its pixel tiles with the next tile's loads issued before the current tile's epilogue.  The
// epilogue works on the accumulator registers directly (lane = 4 consecutive output channels of one pixel: one 8-byte
// store per fragment; the four fragments of a pixel fill its 128-byte output segment back to back in L2).
//
// k-sequence: channels 0..C-1 in 32-deep MFMA steps, lane group g supplying channels 8g..8g+7 of each step, weights
// as operand A -- the gather kernels' sequence for a 1x1 layer; the epilogue is store_tile_lds's arithmetic
// (acc * scale + shift + residual, then the activation, one rounding): outputs are the other variants' bit for bit
// (tests/test_hip_layers.py::test_conv_variants_bitwise).
//
// Work split: item = (pixel tile, 64-channel slice), slice fastest; wave gw of the 4G launched (XCD-aware block
// order: the waves sharing a pixel tile sit on one XCD and share its L2) runs items gw, gw + 4G, ...  With 4G a
// multiple of the slice count nK, a wave's slice never changes and the nK consecutive waves of "group" gw / nK cover
// all channels of the same pixel tiles.  Fused BatchNorm statistics: each wave sums its tiles (fp32 per tile, a
// 16-lane DPP reduce-scatter, then fp64 across tiles) and writes its 64 channels of statistics row `group` once at the end
// -- 4G / nK rows per launch (conv.hip reports that count), no per-tile partial-row writes, no cross-wave reduction.
#include "conv_kernels.h"

namespace {

__device__ __forceinline__ void act4(float (&v)[4], int act, float slope) {
  if (act == SSSEG_ACT_RELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  } else if (act == SSSEG_ACT_RELU6) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fminf(fmaxf(v[e], 0.f), 6.f);
  } else if (act == SSSEG_ACT_LEAKY) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * slope;
  }
}

template <typename TO> struct Pack4;
template <> struct Pack4<bf16_t> {
  __device__ __forceinline__ static uint2 pk(const float (&v)[4]) {
    return make_uint2((unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16),
                      (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16));
  }
};
template <> struct Pack4<f16_t> {
  __device__ __forceinline__ static uint2 pk(const float (&v)[4]) {
    const f16x2_t a = {(f16_t)v[0], (f16_t)v[1]}, b = {(f16_t)v[2], (f16_t)v[3]};
    return make_uint2(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b));
  }
};

// odd 16-lane rows of a <-> even rows of b
__device__ __forceinline__ void swap16(uint2& a, uint2& b) {
  const auto x = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto y = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  a = make_uint2(x[0], y[0]);
  b = make_uint2(x[1], y[1]);
}

// partner lane's value within a 16-lane row (DPP): row_mirror (l <-> 15 - l), row_half_mirror (l <-> 7 - l within 8),
// quad_perm xor 2, quad_perm xor 1
template <int CTL> __device__ __forceinline__ float dpp_partner(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTL, 0xF, 0xF, false));
}

// reduce-scatter of 16 per-lane values over a 16-lane row by recursive halving: lane li ends with the row's sum of
// value li (index i * 4 + e of s[4][4]).  Each step a lane keeps the half of its values whose index bit matches its
// own lane bit and adds the partner's copy of that half: 8 + 4 + 2 + 1 partner reads instead of 16 full row sums.
__device__ __forceinline__ float row16_scatter(const float (&s)[4][4], int li) {
  float v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = s[k >> 2][k & 3];
  const bool b3 = li & 8, b2 = li & 4, b1 = li & 2, b0 = li & 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float keep = b3 ? v[k + 8] : v[k], send = b3 ? v[k] : v[k + 8];
    v[k] = keep + dpp_partner<0x140>(send);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float keep = b2 ? v[k + 4] : v[k], send = b2 ? v[k] : v[k + 4];
    v[k] = keep + dpp_partner<0x141>(send);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float keep = b1 ? v[k + 2] : v[k], send = b1 ? v[k] : v[k + 2];
    v[k] = keep + dpp_partner<0x4E>(send);
  }
  const float keep = b0 ? v[1] : v[0], send = b0 ? v[0] : v[1];
  return keep + dpp_partner<0xB1>(send);
}

// KC: 32-deep k-steps (C / 32); FJ: 16-pixel fragments per wave tile
template <typename TO, int KC, int FJ, bool STATS, bool RES>
__global__ void __launch_bounds__(256, 2) pw_kernel(const TO* __restrict__ x, const TO* __restrict__ w,
                                                    TO* __restrict__ y, ConvGeom g, Epi<TO> ep, int nK, int ngroups,
                                                    int nptiles) {
  constexpr int TP = FJ * 16;
  using CK = Chunk<TO, 4>;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int gw = xcd_tile(blockIdx.x, gridDim.x) * 4 + wave;
  const int slice = gw % nK, grp = gw / nK;
  const int n0 = slice * 64;

  bf16x8 wf[4][KC];   // output channel n0 + 16 i + li, channels 32 kc + 8 lg .. + 7
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      wf[i][kc] = *(const bf16x8*)(w + (long long)(n0 + 16 * i + li) * g.ldw + kc * 32 + lg * 8);
  float sc[4][4], sh[4][4];   // lane's channels n0 + 16 i + 4 lg + e
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + 16 * i + 4 * lg + e;
      sc[i][e] = ep.scale ? ep.scale[n] : 1.f;
      sh[i][e] = ep.shift ? ep.shift[n] : 0.f;
    }

  // pixel rows past M load row M - 1 (every load unconditional) and store nothing
  auto load_tile = [&](int pt, bf16x8 (&b)[FJ][KC], typename CK::raw (&r)[FJ][4]) {
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      long long m = (long long)pt * TP + 16 * j + li;
      m = m < g.M ? m : g.M - 1;
      const TO* p = x + m * g.ldx + lg * 8;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) b[j][kc] = *(const bf16x8*)(p + kc * 32);
      if constexpr (RES)
#pragma unroll
        for (int i = 0; i < 4; ++i) r[j][i] = CK::ld(ep.res + m * ep.ldr + n0 + 16 * i + 4 * lg);
    }
  };

  double d1 = 0.0, d2 = 0.0;   // STATS: fp64 sums of channel n0 + 16 (li >> 2) + 4 lg + (li & 3)
  bf16x8 b[FJ][KC];
  typename CK::raw r[FJ][4];
  int pt = grp;
  if (pt < nptiles) load_tile(pt, b, r);
  for (; pt < nptiles; pt += ngroups) {
    f32x4 acc[4][FJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = M16<TO>::mma(wf[i][kc], b[j][kc], acc[i][j]);
    typename CK::raw rt[FJ][4];
    if constexpr (RES)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) rt[j][i] = r[j][i];
    // the next tile's operands are in flight during this tile's epilogue
    if (pt + ngroups < nptiles) load_tile(pt + ngroups, b, r);

    float s1[4][4], s2[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) s1[i][e] = s2[i][e] = 0.f;
    // fragments j, j + 1 in pairs: after the affine / activation each lane packs its 4 channels of both, and one
    // permlane16 swap per dword gives the even rows (lane groups 0, 2) 8 consecutive channels of fragment j's pixel
    // and the odd rows the same 8 channels of fragment j + 1's: one 16-byte store per pair instead of two 8-byte ones
#pragma unroll
    for (int j = 0; j < FJ; j += 2) {
      const long long mj = (long long)pt * TP + 16 * j + li;
      const long long ms = mj + ((lg & 1) ? 16 : 0);   // this lane's pixel after the swap
      const bool live0 = mj < g.M, live1 = mj + 16 < g.M, lives = ms < g.M;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float rr[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (RES) CK::cvt(rt[j + h][i], rr);
#pragma unroll
          for (int e = 0; e < 4; ++e)   // store_tile_lds's expression
            v[h][e] = acc[i][j + h][e] * sc[i][e] + sh[i][e] + rr[e];
          act4(v[h], ep.relu, ep.slope);
          if constexpr (STATS) {
            const bool live = h ? live1 : live0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float q = live ? stored<TO>(v[h][e]) : 0.f;
              s1[i][e] += q;
              s2[i][e] += q * q;
            }
          }
        }
        const long long o = ms * g.ldy + n0 + 16 * i + 8 * (lg >> 1);
        uint2 a = Pack4<TO>::pk(v[0]), b = Pack4<TO>::pk(v[1]);
        swap16(a, b);
        if (lives) *(uint4*)(y + o) = make_uint4(a.x, a.y, b.x, b.y);
        if (ep.aux) {
          const float r0[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          const float r1[4] = {acc[i][j + 1][0], acc[i][j + 1][1], acc[i][j + 1][2], acc[i][j + 1][3]};
          uint2 c = Pack4<TO>::pk(r0), d = Pack4<TO>::pk(r1);
          swap16(c, d);
          if (lives) *(uint4*)(ep.aux + o) = make_uint4(c.x, c.y, d.x, d.y);
        }
      }
    }
    if constexpr (STATS) {
      d1 += (double)row16_scatter(s1, li);
      d2 += (double)row16_scatter(s2, li);
    }
  }
  if constexpr (STATS) {
    const int n = n0 + 16 * (li >> 2) + 4 * lg + (li & 3);
    if (n < ep.sld) {
      ep.stats[(long long)(2 * grp) * ep.sld + n] = d1;
      ep.stats[(long long)(2 * grp + 1) * ep.sld + n] = d2;
    }
  }
}

template <typename TO, int KC, int FJ>
void launch_kc(const TO* x, const TO* w, TO* y, const ConvGeom& g, const Epi<TO>& ep, unsigned grid, int nK,
               int ngroups, int nptiles, hipStream_t s) {
  const bool st = ep.stats != nullptr, res = ep.res != nullptr;
  if (st)
    hipLaunchKernelGGL((pw_kernel<TO, KC, FJ, true, false>), dim3(grid), dim3(256), 0, s, x, w, y, g, ep, nK,
                       ngroups, nptiles);
  else if (res)
    hipLaunchKernelGGL((pw_kernel<TO, KC, FJ, false, true>), dim3(grid), dim3(256), 0, s, x, w, y, g, ep, nK,
                       ngroups, nptiles);
  else
    hipLaunchKernelGGL((pw_kernel<TO, KC, FJ, false, false>), dim3(grid), dim3(256), 0, s, x, w, y, g, ep, nK,
                       ngroups, nptiles);
}

// the 64-pixel form: C = 64, no residual
template <typename TO>
void launch_kc4(const TO* x, const TO* w, TO* y, const ConvGeom& g, const Epi<TO>& ep, unsigned grid, int nK,
                int ngroups, int nptiles, hipStream_t s) {
  if (ep.stats)
    hipLaunchKernelGGL((pw_kernel<TO, 2, 4, true, false>), dim3(grid), dim3(256), 0, s, x, w, y, g, ep, nK, ngroups,
                       nptiles);
  else
    hipLaunchKernelGGL((pw_kernel<TO, 2, 4, false, false>), dim3(grid), dim3(256), 0, s, x, w, y, g, ep, nK,
                       ngroups, nptiles);
}

}  // namespace

thread_local long long t_pw_rows = -1;

template <typename TO>
int launch_pw(int fj, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, hipStream_t s,
              float* ws, const PhaseTab* ph, const void* x2) {
  if (g_knobs[13] < 0 || ws || ph || x2 || !g.aident || !g.oident || ep.y2 || ep.rmask) return -1;
  if ((g.C != 64 && g.C != 128) || g.ldx < g.C || g.ldx % 8 || g.ldw != g.C || g.K % 64 || g.ldy % 8) return -1;
  if (ep.res && (ep.ldr % 4 || ep.ldr < g.K)) return -1;
  if (ep.stats && (ep.scale || ep.res || ep.aux)) return -1;   // host contract (conv.hip)
  // 64-pixel tiles: 64 channels without a residual only (the 128-channel and residual forms spill at 2 waves / SIMD)
  if (fj == 4 && (g.C != 64 || ep.res)) return -1;
  const int nK = g.K / 64;
  if (nK != 1 && nK != 2 && nK != 4 && nK != 8 && nK != 16) return -1;
  const int tp = fj * 16;
  const long long nptiles = (g.M + tp - 1) / tp, items = nptiles * nK;
  if (nptiles > 0x7fffffffLL || g.M * g.ldx > 0x7fffffffLL * 8) return -1;
  // two resident 4-wave blocks per CU: 512 blocks fill the chip once (three per CU for the 32-pixel 64-channel form,
  // which fits 3 waves / SIMD, measured no faster); 4G must be a multiple of nK (fixed slice per wave) and the
  // statistics rows 4G / nK must fit the caller's table (ceil(M / 64) rows)
  const long long q = nK > 4 ? nK / 4 : 1;
  long long G = std::min<long long>(512, items / 4);
  G -= G % q;
  if (ep.stats) G = std::min<long long>(G, (g.M + 63) / 64 * nK / 4 / q * q);
  if (G < 1) return -1;
  const int ngroups = (int)(4 * G / nK);
  const TO *xt = (const TO*)x, *wt = (const TO*)w;
  TO* yt = (TO*)y;
  if (fj == 4) {
    launch_kc4<TO>(xt, wt, yt, g, ep, (unsigned)G, nK, ngroups, (int)nptiles, s);
  } else {
    if (g.C == 64) launch_kc<TO, 2, 2>(xt, wt, yt, g, ep, (unsigned)G, nK, ngroups, (int)nptiles, s);
    else launch_kc<TO, 4, 2>(xt, wt, yt, g, ep, (unsigned)G, nK, ngroups, (int)nptiles, s);
  }
  t_pw_rows = ngroups;
  return 64;
}

template int launch_pw<bf16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&, hipStream_t,
                               float*, const PhaseTab*, const void*);
template int launch_pw<f16_t>(int, const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&, hipStream_t,
                              float*, const PhaseTab*, const void*);
