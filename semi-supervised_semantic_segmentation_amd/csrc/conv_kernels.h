// conv_kernels.h: device code of the implicit-GEMM convolution engine (shared by conv*.hip).
// Implicit-GEMM convolution engine for gfx950 (MFMA 16x16x32 bf16 / 16x16x4 f32), NHWC activations.
//
// One gather-GEMM kernel covers every contraction of the conv layers on the hot path
// (unet.py:8,21-22,27,85; simple_unet.py:64-72,118; encoder convs):
//   y[m][n] = sum_k A[m][k] * B[n][k]
//   m = output position (img, oy, ox) of a GEMM grid OHxOW, written to pixel (oy*osy+ooy, ox*osx+oox)
//   k = (r, s, c):  A = x[img][oy*sy + r*dy + py][ox*sx + s*dx + px][c]  (0 outside),  B = packed weights
// Forward conv, stride-1 dgrad (flipped taps), strided dgrad and ConvTranspose2d(4,2,1) forward
// (stride-phase decomposition: one launch per output phase, dilation -1) are all this kernel with
// different descriptors and weight packings (ssseg_weight_pack).
// Weight gradients use a second kernel (split-K over pixels, fp32 slabs, deterministic reduce).
//
// Tiling: 256 threads = 4 waves; block tile BM pixels x BN channels x 64 bytes of k; LDS double
// buffer with register-staged global loads (issue next tile's loads before the MFMAs, write them to
// the other buffer after), one barrier per k-tile.  The MFMA A operand is the weight tile and the B
// operand the pixel tile, so each lane's accumulator holds 4 consecutive output channels of one
// pixel: the NHWC epilogue stores them with one 8/16-byte write.
#pragma once
#include <algorithm>
#include <type_traits>

#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16x16x32 MFMA on 16-bit operands held as 8 x 16-bit lanes (the LDS fragments are read as raw bits):
// bf16 (v_mfma_f32_16x16x32_bf16) or IEEE half (v_mfma_f32_16x16x32_f16, same rate: the fp16 mode)
template <typename T16> struct M16;
template <> struct M16<bf16_t> {
  __device__ __forceinline__ static f32x4 mma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct M16<f16_t> {
  __device__ __forceinline__ static f32x4 mma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  }
};
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct ConvGeom {
  int N, H, W, C, ldx;
  int OH, OW, K;
  int R, S, sy, sx, dy, dx, py, px;
  int outH, outW, osy, osx, ooy, oox, ldy;
  int ldw;
  long long M;   // N*OH*OW
  int KK;        // R*S*C
  // division by OW / OH as multiply-high + shift (set by make_geom; exact for 0 <= n < 2^31): the output-pixel
  // decode m -> (img, oy, ox) of every tile row otherwise costs two integer divisions (~40 VALU each)
  unsigned mow, moh;
  int sow, soh;
  unsigned mn64, mn128, mn256, mS;   // magic divisors: n-tile counts ceil(K/64), ceil(K/128), ceil(K/256), filter width S
  int sn64, sn128, sn256, sS;
  int oident;   // output pixel == GEMM row (stride-1 output grid, no offsets): no decode in the epilogue
  int aident;   // 1x1 stride-1 unpadded gather over the same grid: A row m is input pixel m
  // virtual channel concat of the input (unet.py:44 torch.cat feeding conv3_0): channels [0, 64*c1b) come from x
  // (pixel stride ldx), channels [64*c1b, C) from a second tensor x2 (pixel stride ldx2), same N x H x W.  No
  // second source: c1b >= C / 64.
  int c1b, ldx2;
  unsigned mC;   // magic divisor: channel count C (the general-k LDS-DMA loader's k -> (tap, channel) split)
  int sC;
};

// magic multiplier for unsigned division by d >= 1: n / d = (umulhi(n, m) + n) >> s for n < 2^31
static inline void fdiv_init(int d, unsigned& m, int& s) {
  int l = 0;
  while ((1ll << l) < (long long)d) ++l;
  m = (unsigned)((((unsigned long long)1 << (32 + l)) / (unsigned long long)d) - ((unsigned long long)1 << 32) + 1);
  s = l;
}
__device__ __forceinline__ int fdiv(int n, unsigned m, int s) {
  return (int)((__umulhi((unsigned)n, m) + (unsigned)n) >> s);
}
// output-pixel decode of GEMM row m (0 <= m < M < 2^31)
__device__ __forceinline__ void decode_m(const ConvGeom& g, int m, int& img, int& oy, int& ox) {
  const int q = fdiv(m, g.mow, g.sow);
  ox = m - q * g.OW;
  img = fdiv(q, g.moh, g.soh);
  oy = q - img * g.OH;
}
// output pixel (row of y) of GEMM row m: m itself on the identity grid (every forward conv, stride-1 dgrad)
__device__ __forceinline__ long long out_pixel(const ConvGeom& g, int m) {
  if (g.oident) return m;
  int img, oy, ox;
  decode_m(g, m, img, oy, ox);
  return ((long long)img * g.outH + oy * g.osy + g.ooy) * g.outW + ox * g.osx + g.oox;
}

static inline bool make_geom(const ssseg_conv_desc* d, ConvGeom& g) {
  if (!d) return false;
  const int64_t vals[] = {d->N, d->H, d->W, d->C, d->ldx, d->OH, d->OW, d->K, d->R, d->S, d->outH, d->outW, d->ldy,
                          d->ldw};
  for (int64_t v : vals)
    if (v < 0 || v > (int64_t)0x7fffffff) return false;
  g.N = (int)d->N; g.H = (int)d->H; g.W = (int)d->W; g.C = (int)d->C; g.ldx = (int)d->ldx;
  g.OH = (int)d->OH; g.OW = (int)d->OW; g.K = (int)d->K;
  g.R = (int)d->R; g.S = (int)d->S; g.sy = (int)d->sy; g.sx = (int)d->sx; g.dy = (int)d->dy; g.dx = (int)d->dx;
  g.py = (int)d->py; g.px = (int)d->px;
  g.outH = (int)d->outH; g.outW = (int)d->outW; g.osy = (int)d->osy; g.osx = (int)d->osx; g.ooy = (int)d->ooy;
  g.oox = (int)d->oox; g.ldy = (int)d->ldy; g.ldw = (int)d->ldw;
  g.M = (long long)d->N * d->OH * d->OW;
  g.KK = (int)(d->R * d->S * d->C);
  fdiv_init(g.OW > 0 ? g.OW : 1, g.mow, g.sow);
  fdiv_init(g.OH > 0 ? g.OH : 1, g.moh, g.soh);
  fdiv_init(g.K > 0 ? (g.K + 63) / 64 : 1, g.mn64, g.sn64);
  fdiv_init(g.K > 0 ? (g.K + 127) / 128 : 1, g.mn128, g.sn128);
  fdiv_init(g.K > 0 ? (g.K + 255) / 256 : 1, g.mn256, g.sn256);
  fdiv_init(g.S > 0 ? g.S : 1, g.mS, g.sS);
  fdiv_init(g.C > 0 ? g.C : 1, g.mC, g.sC);
  g.oident = g.osy == 1 && g.osx == 1 && g.ooy == 0 && g.oox == 0 && g.outH == g.OH && g.outW == g.OW;
  g.aident = g.R == 1 && g.S == 1 && g.sy == 1 && g.sx == 1 && g.py == 0 && g.px == 0 && g.H == g.OH &&
             g.W == g.OW;
  g.c1b = 0x40000000;
  g.ldx2 = 0;
  return true;
}

template <typename T> struct MF;
template <> struct MF<bf16_t> {
  static constexpr int VEC = 8;
  typedef bf16x8 frag;
  __device__ __forceinline__ static void mma(const frag& a, const frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MF<f16_t> {
  static constexpr int VEC = 8;
  typedef f16x8 frag;
  __device__ __forceinline__ static void mma(const frag& a, const frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct MF<float> {
  static constexpr int VEC = 4;
  typedef f32x4 frag;
  // k inside a 16-element chunk is permuted consistently for A and B: MFMA e consumes element e
  __device__ __forceinline__ static void mma(const frag& a, const frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  }
};

template <typename TO> struct Store4;
template <> struct Store4<float> {
  __device__ __forceinline__ static void st(float* p, const float (&v)[4]) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
};
template <> struct Store4<f16_t> {
  __device__ __forceinline__ static void st(f16_t* p, const float (&v)[4]) { H16::st4(p, v); }
};
template <> struct Store4<bf16_t> {
  __device__ __forceinline__ static void st(bf16_t* p, const float (&v)[4]) {
    uint2 u;
    u.x = (unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16);
    u.y = (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16);
    *(uint2*)p = u;
  }
};

// epilogue: y = act(acc * scale[n] + shift[n] + res[pixel][n]); scale null = 1, shift null = 0
// (conv bias -> shift; a folded eval BatchNorm -> scale/shift; Bottleneck identity -> res)
template <typename TO>
struct Epi {
  const float* scale;
  const float* shift;
  const TO* res;
  int ldr;
  int relu;    // activation code SSSEG_ACT_*
  TO* aux;     // optional copy of the raw accumulator (pre-affine conv output), pixel stride ldy
  float slope;
  double* stats;   // optional BatchNorm statistics partials of the stored output: row (2*mtile) = sum y,
  int sld;         // row (2*mtile+1) = sum y^2, channels [0, sld) (sld = the BN's channel count)
  // split output (the input gradient of a virtual concat, ssseg_conv_igemm_epi_vsplit): channels [oc1, K) go to y2
  // (pixel stride ldy2) at channel n - oc1; oc1 % 8 == 0, so no 4- or 8-channel group straddles the seam
  TO* y2 = nullptr;
  int oc1 = 0x40000000;
  int ldy2 = 0;
  // rmask (SSSEG_ACT_RELU / SSSEG_ACT_LEAKY): res is not added but is the forward output of the input's producer (of the
  // first part's, for a split output), whose activation backward is applied in place: channels [0, oc1) are stored as
  // (res > 0 ? v : 0) or (res > 0 ? v : v * rslope), channels >= oc1 read no res
  int rmask = 0;
  float rslope = 0.f;   // rmask == SSSEG_ACT_LEAKY: (res > 0 ? v : v * rslope) (the producer's LeakyReLU backward)
  // gstat (with rmask and stats): the statistics rows hold (sum m, sum m * res) of the masked gradient m BEFORE the
  // scale, rounded to TO -- the two sums a BatchNorm backward reduces (res = its output y, from which x_hat follows
  // wherever m != 0); the stored value is scale * m
  int gstat = 0;
  int sdbg = 0;  // experiment switch for the fused statistics (knob 12): 1 no sums, 2 no tile_stats, 4 no row write,
                  // 8 no cross-lane shuffles
};

// where output channel n of pixel op is stored (y, or the second part of a split output)
template <typename TO>
__device__ __forceinline__ TO* out_at(const Epi<TO>& ep, TO* y, int ldy, long long op, int n) {
  return n >= ep.oc1 ? ep.y2 + op * ep.ldy2 + (n - ep.oc1) : y + op * ldy + n;
}

// the value a later pass reads back from the stored output (the BN statistics are those of that value)
template <typename TO> __device__ __forceinline__ float stored(float v);
template <> __device__ __forceinline__ float stored<float>(float v) { return v; }
template <> __device__ __forceinline__ float stored<bf16_t>(float v) { return bf16_to_f32(f32_to_bf16(v)); }
template <> __device__ __forceinline__ float stored<f16_t>(float v) { return (float)(f16_t)v; }

// sum over a 16-lane DPP row (quad_perm xor 1, xor 2, row_half_mirror, row_mirror): every lane of the row ends with
// the same value, in a fixed order, without LDS traffic
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

// Per-tile BatchNorm statistics partials from the epilogue (fused training BN statistics, replaces a separate
// read of the conv output).  Each thread holds fp64 (sum, sumsq) of V consecutive channels starting at
// channel offset cofs within the tile, over some of the tile's rows; lanes holding the same channels are those
// whose lane index agrees in the bits below `lstride` (a power of two): xor-shuffle over the higher bits,
// then the NW waves' partials meet in LDS (fixed order: deterministic) and row mtile of the partial table is
// written for channels [n0, n0 + BN).  Every thread of the block must call this (two barriers).
template <int V, int BN, int NW, typename SA>
__device__ __forceinline__ void tile_stats(SA (&s1)[V], SA (&s2)[V], int lstride, bool holder, int cofs,
                                           char* smem, long long mtile, int n0, double* __restrict__ stats, int sld,
                                           int dbg = 0) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    if (o < lstride || (dbg & 8)) break;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      s1[e] += __shfl_xor(s1[e], o, 64);
      s2[e] += __shfl_xor(s2[e], o, 64);
    }
  }
  lds_barrier();   // LDS free (the caller's last LDS reads are done); the y stores keep draining
  double* red = (double*)smem;   // [NW][BN][2]
  const int w = threadIdx.x >> 6;
  if (holder)
#pragma unroll
    for (int e = 0; e < V; ++e) {
      red[(w * BN + cofs + e) * 2] = (double)s1[e];
      red[(w * BN + cofs + e) * 2 + 1] = (double)s2[e];
    }
  lds_barrier();
  for (int c = threadIdx.x; c < BN; c += NW * 64) {
    const int n = n0 + c;
    if (n >= sld || (dbg & 4)) continue;
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      a += red[(k * BN + c) * 2];
      b += red[(k * BN + c) * 2 + 1];
    }
    stats[(mtile * 2) * sld + n] = a;
    stats[(mtile * 2 + 1) * sld + n] = b;
  }
}

// Output phases of one transposed conv (ConvTranspose2d(4,2,1): four 2x2-tap phases) in ONE launch: blockIdx.y =
// phase, each with its own input offset, output sub-grid and packed weights (same K, taps and weight stride).
// A 16x16-input layer has only 32-128 tiles per phase: one launch fills the chip where four could not.
struct PhaseTab {
  int n;                          // phases (1: a plain launch)
  int py[4], px[4], ooy[4], oox[4];
  const void* w[4];
};

template <typename TO> struct Load4;
template <> struct Load4<float> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[4]) {
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
};
template <> struct Load4<f16_t> {
  __device__ __forceinline__ static void ld(const f16_t* p, float (&v)[4]) { H16::ld4(p, v); }
};
template <> struct Load4<bf16_t> {
  __device__ __forceinline__ static void ld(const bf16_t* p, float (&v)[4]) {
    const uint2 q = *(const uint2*)p;
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  }
};

// Writes one wave's FN x FM fragments: y[pixel(m)][n..n+3] = act(acc*scale + shift + res), NHWC.
// The per-channel affine of a fragment column is loaded once, and every residual of the column is loaded
// before the first store (the stores may alias the residual as far as the compiler knows, so it could not
// batch those loads itself): one HBM round trip per column instead of one per pixel.
template <typename TO, int FM, int FN, bool ST = false>
__device__ __forceinline__ void store_tile(const f32x4 (&acc)[FN][FM], long long mb, int nb, int lane,
                                           const ConvGeom& g, TO* __restrict__ y, const Epi<TO>& ep,
                                           double (*st1)[4] = nullptr, double (*st2)[4] = nullptr) {
  long long op[FM];   // output pixel of fragment row j (-1: past M)
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const long long m = mb + j * 16 + (lane & 15);
    op[j] = -1;
    if (m < g.M) {
      op[j] = out_pixel(g, (int)m);   // M < 2^31 (geom_ok)
    }
  }
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = nb + i * 16 + (lane >> 4) * 4;
    if (n >= g.K) continue;
    const bool full = n + 3 < g.K;
    float sc[4], sh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool in = n + e < g.K;
      sc[e] = (ep.scale && in) ? ep.scale[n + e] : 1.f;
      sh[e] = (ep.shift && in) ? ep.shift[n + e] : 0.f;
    }
    float r[FM][4];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      r[j][0] = r[j][1] = r[j][2] = r[j][3] = 0.f;
      if (ep.res && op[j] >= 0 && n < ep.oc1) {
        const TO* rp = ep.res + op[j] * ep.ldr + n;
        if (full && (ep.ldr & 3) == 0)
          Load4<TO>::ld(rp, r[j]);
        else
#pragma unroll
          for (int e = 0; e < 4; ++e)   // fixed trip count: r stays in registers (a runtime bound spills it)
            if (n + e < g.K) r[j][e] = io<TO>::ld(rp, e);
      }
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      if (op[j] < 0) continue;
      if (ep.aux) {
        const float a4[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (full && (g.ldy & 3) == 0)
          Store4<TO>::st(ep.aux + op[j] * g.ldy + n, a4);
        else
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < g.K) io<TO>::st(ep.aux, op[j] * g.ldy + n + e, a4[e]);
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = acc[i][j][e];
        if (ep.scale) a *= sc[e];
        if (ep.shift) a += sh[e];
        if (!ep.rmask) a += r[j][e];
        a = act_fwd(a, ep.relu, ep.slope);
        if (ep.rmask && n < ep.oc1 && !(r[j][e] > 0.f)) a = ep.rmask == SSSEG_ACT_LEAKY ? a * ep.rslope : 0.f;
        v[e] = a;
        if constexpr (ST) {   // compile-time: the statistics arrays stay in registers
          if (n + e < g.K) {
            if (ep.gstat) {   // (sum m, sum m * res) of the unscaled masked gradient m
              float m = acc[i][j][e];
              if (n < ep.oc1 && !(r[j][e] > 0.f)) m = ep.rmask == SSSEG_ACT_LEAKY ? m * ep.rslope : 0.f;
              const double q = (double)stored<TO>(m);
              st1[i][e] += q;
              st2[i][e] += q * (double)r[j][e];
            } else {
              const double q = (double)stored<TO>(a);
              st1[i][e] += q;
              st2[i][e] += q * q;
            }
          }
        }
      }
      TO* yp = out_at(ep, y, g.ldy, op[j], n);
      if (full && (g.ldy & 3) == 0) {
        Store4<TO>::st(yp, v);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < g.K) io<TO>::st(yp, e, v[e]);
      }
    }
  }
}

// LDS-staged epilogue for the LDS-DMA kernel: the raw fp32 accumulators go to LDS (rows padded by 16 B:
// conflict-free float4 writes), then each thread finishes 8 consecutive channels of one pixel with 16-byte
// residual loads and 16-byte (bf16) / 2x16-byte (f32) stores, so a pixel row is written in full lines.
// Same arithmetic as store_tile (fp32 acc*scale + shift + res, then act, then one rounding).
// act_fwd over 8 values with the (uniform) activation code tested once, not per value
__device__ __forceinline__ void act8(float (&v)[8], int act, float slope) {
  if (act == SSSEG_ACT_RELU) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  } else if (act == SSSEG_ACT_RELU6) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fminf(fmaxf(v[e], 0.f), 6.f);
  } else if (act == SSSEG_ACT_LEAKY) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * slope;
  }
}

template <typename TO> struct Out8;
template <> struct Out8<bf16_t> {
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
template <> struct Out8<f16_t> {
  __device__ __forceinline__ static void ld(const f16_t* p, float (&v)[8]) { H16::ld8(p, v); }
  __device__ __forceinline__ static void st(f16_t* p, const float (&v)[8]) { H16::st8(p, v); }
};
template <> struct Out8<float> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[8]) {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[8]) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <int NP> struct PreRes {   // residual chunks an epilogue thread loaded ahead of the main loop
  u32x4 v[NP];
  bool on;
};

// T2D (the halo-tiled 3x3 kernel, conv_hconv3.hip): the tile is t2.rows image rows x 2^t2.lw columns of image t2.n starting
// at (t2.y0, t2.x0) instead of BM consecutive GEMM rows; its statistics row is t2.tile (output grid == GEMM grid)
struct Tile2D {
  int n, y0, x0, rows;
  long long tile;
  int lw = 6;   // log2 of the tile width (64 columns; 32 / 16 on the 32^2 / 16^2 maps)
};

template <typename TO, int BM, int BN, int FM, int FN, int NT, bool STATS, int NPRE = 1, bool T2D = false>
__device__ __forceinline__ void store_tile_lds(const f32x4 (&acc)[FN][FM], char* smem, long long m0, int n0, int wmo,
                                               int wno, int lane, const ConvGeom& g, TO* __restrict__ y,
                                               const Epi<TO>& ep, PreRes<NPRE> pre = PreRes<NPRE>{{}, false},
                                               Tile2D t2 = Tile2D{0, 0, 0, 0, 0}) {
  // pre: this thread's residual chunks, already loaded by the caller (one per pass; used where `full`)
  constexpr int LDR = BN * 4 + 16;   // bytes per staged pixel row
  // REGST: the fused BatchNorm statistics come from the accumulators, before the staging: per lane fp32 sums of the
  // stored value over its FM fragment rows (acc + shift: a conv feeding a training BN has no scale / residual /
  // activation -- host contract), a 16-lane DPP row sum, and each wave's (sum, sumsq) of its WTN channels goes into
  // the 16 pad bytes of the staged rows: slot (wm * BN + channel) * 2, 4 floats per row.  No extra barrier, no LDS
  // shuffles and nothing live across the store pass (the store-pass summation it replaces kept 16 sums live there
  // and reduced them with 48 LDS permutes + 2 barriers per tile).  ep.sdbg & 16 = that older path (A/B).
  constexpr int WTM = FM * 16, WM_ = BM / WTM;
  constexpr bool REGST = STATS && BN <= 32 * FM;
  const bool regst = REGST && !(ep.sdbg & 16) && !ep.gstat;   // (gradient statistics: the store pass, below)
  float rs1[REGST ? FN : 1][4], rs2[REGST ? FN : 1][4];
  if constexpr (REGST) {
    if (regst) {
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int nb = n0 + wno + i * 16 + (lane >> 4) * 4;
        float sh[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sh[e] = (ep.shift && nb + e < g.K) ? ep.shift[nb + e] : 0.f;
          rs1[i][e] = rs2[i][e] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int row = wmo + j * 16 + (lane & 15);
          const bool rv = T2D ? (row >> t2.lw) < t2.rows : m0 + row < g.M;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float q = (rv && nb + e < g.K) ? stored<TO>(acc[i][j][e] + sh[e]) : 0.f;
            rs1[i][e] += q;
            rs2[i][e] += q * q;
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          rs1[i][e] = row16_sum(rs1[i][e]);
          rs2[i][e] = row16_sum(rs2[i][e]);
        }
      }
    }
  }
  __syncthreads();                   // every wave is done with the LDS ring
#pragma unroll
  for (int j = 0; j < FM; ++j)
#pragma unroll
    for (int i = 0; i < FN; ++i)
      *(f32x4*)(smem + (wmo + j * 16 + (lane & 15)) * LDR + (wno + i * 16 + (lane >> 4) * 4) * 4) = acc[i][j];
  if constexpr (REGST) {
    if (regst && (lane & 15) == 0) {
      const int wmi = wmo / WTM;
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int slot = (wmi * BN + wno + i * 16 + (lane >> 4) * 4 + e) * 2;
          *(float2*)(smem + (slot >> 2) * LDR + BN * 4 + (slot & 3) * 4) = make_float2(rs1[i][e], rs2[i][e]);
        }
    }
  }
  __syncthreads();
  if constexpr (REGST) {
    if (regst) {
      for (int c = threadIdx.x; c < BN; c += NT) {
        const int n = n0 + c;
        if (n >= ep.sld || (ep.sdbg & 4)) continue;
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int w = 0; w < WM_; ++w) {
          const int slot = (w * BN + c) * 2;
          const float2 v = *(const float2*)(smem + (slot >> 2) * LDR + BN * 4 + (slot & 3) * 4);
          a += (double)v.x;
          b += (double)v.y;
        }
        const long long mt = T2D ? t2.tile : m0 / BM;
        ep.stats[(mt * 2) * ep.sld + n] = a;
        ep.stats[(mt * 2 + 1) * ep.sld + n] = b;
      }
    }
  }
  constexpr int CPR = BN / 8;                 // 8-channel chunks per row
  static_assert(NT % CPR == 0 && 64 % CPR == 0, "epilogue: one fixed channel chunk per thread");
  constexpr int RPP = NT / CPR, NP = (BM + RPP - 1) / RPP;   // rows per pass, passes
  const int ch = threadIdx.x % CPR, r0 = threadIdx.x / CPR;
  const int n = n0 + ch * 8;
  // STATS: the fused BatchNorm statistics are summed in the store pass itself, from the values it stores (the conv
  // feeding a training BatchNorm has no scale / residual / activation in its epilogue -- host contract -- so that
  // is acc + shift).  Per-thread sums over <= BM / RPP rows in the accumulator type SA (fp32 for bf16 outputs:
  // exact products of 8-bit mantissas, <= 32 terms), fp64 across threads and tiles.  (A second pass over the staged
  // tile after the stores cost ~1.9 us per tile: 50 -> 80 us on the 64->256 1x1 @16x128^2 forward.)
  using SA = typename std::conditional<sizeof(TO) == 2, float, double>::type;
  SA s1[STATS ? 8 : 1], s2[STATS ? 8 : 1];
#pragma unroll
  for (int e = 0; e < (STATS ? 8 : 1); ++e) s1[e] = s2[e] = (SA)0;
  if (n < g.K) {
    const bool vec = (g.ldy & 7) == 0 && (!ep.res || (ep.ldr & 7) == 0);
    const bool full = vec && n + 7 < g.K;
    // this thread's 8 channels are the same in every pass: the affine is loaded once, and all residual
    // rows are in flight before the first store
    float sc[8], sh[8];
    if (full && ep.scale && ((reinterpret_cast<uintptr_t>(ep.scale) & 15) == 0)) {   // two 16-byte loads
      const float4 a = *(const float4*)(ep.scale + n), b = *(const float4*)(ep.scale + n + 4);
      sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w; sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) sc[e] = (ep.scale && n + e < g.K) ? ep.scale[n + e] : 1.f;
    }
    if (full && ep.shift && ((reinterpret_cast<uintptr_t>(ep.shift) & 15) == 0)) {
      const float4 a = *(const float4*)(ep.shift + n), b = *(const float4*)(ep.shift + n + 4);
      sh[0] = a.x; sh[1] = a.y; sh[2] = a.z; sh[3] = a.w; sh[4] = b.x; sh[5] = b.y; sh[6] = b.z; sh[7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) sh[e] = (ep.shift && n + e < g.K) ? ep.shift[n + e] : 0.f;
    }
    long long op[NP];
    float r[NP][8];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int row = r0 + p * RPP;
      op[p] = -1;
      if constexpr (T2D) {
        if (row < BM && (row >> t2.lw) < t2.rows)
          op[p] = ((long long)t2.n * g.outH + t2.y0 + (row >> t2.lw)) * g.outW + t2.x0 + (row & ((1 << t2.lw) - 1));
      } else {
        const long long m = m0 + row;
        if (row < BM && m < g.M) {
          op[p] = out_pixel(g, (int)m);   // M < 2^31 (geom_ok)
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) r[p][e] = 0.f;
      if (ep.res && op[p] >= 0 && n < ep.oc1) {
        if (full) {
          if constexpr (sizeof(TO) == 2) {
            if (pre.on) {
              const u32x4 q = pre.v[p < NPRE ? p : 0];
              Chunk<TO, 8>::cvt(make_uint4(q.x, q.y, q.z, q.w), r[p]);
            } else {
              Out8<TO>::ld(ep.res + op[p] * ep.ldr + n, r[p]);
            }
          } else {
            Out8<TO>::ld(ep.res + op[p] * ep.ldr + n, r[p]);
          }
        } else
#pragma unroll
          for (int e = 0; e < 8; ++e)   // fixed trip count: r stays in registers (a runtime bound spills it)
            if (n + e < g.K) r[p][e] = io<TO>::ld(ep.res, op[p] * ep.ldr + n + e);
      }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if (op[p] < 0) continue;
      const float* a = (const float*)(smem + (r0 + p * RPP) * LDR + ch * 32);
      float v[8];
      const float4 a0 = *(const float4*)a, a1 = *(const float4*)(a + 4);
      const float raw[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      // affine + residual, then ONE uniform activation switch per chunk (not one per value)
      if (ep.rmask) {   // split output with the first part's ReLU backward (no residual add)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = raw[e] * sc[e] + sh[e];
        act8(v, ep.relu, ep.slope);
        if (n < ep.oc1) {
          const float ms = ep.rmask == SSSEG_ACT_LEAKY ? ep.rslope : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = r[p][e] > 0.f ? v[e] : v[e] * ms;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = raw[e] * sc[e] + sh[e] + r[p][e];   // scale 1 / shift 0 when absent
        act8(v, ep.relu, ep.slope);
      }
      if constexpr (STATS) {
        if (ep.gstat) {   // (sum m, sum m * res) of the unscaled masked gradient (bf16 x bf16: exact fp32 products)
          const float ms = ep.rmask == SSSEG_ACT_LEAKY ? ep.rslope : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float m = (n < ep.oc1 && !(r[p][e] > 0.f)) ? (ep.rmask == SSSEG_ACT_LEAKY ? raw[e] * ms : 0.f)
                                                              : raw[e];
            const SA q = n + e < g.K ? (SA)stored<TO>(m) : (SA)0;
            s1[e] += q;
            s2[e] += q * (SA)r[p][e];
          }
        } else if (!regst && !(ep.sdbg & 1)) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const SA q = n + e < g.K ? (SA)stored<TO>(v[e]) : (SA)0;
            s1[e] += q;
            s2[e] += q * q;
          }
        }
      }
      const long long o = op[p] * g.ldy + n;
      TO* yp = out_at(ep, y, g.ldy, op[p], n);   // (a split output has no aux: host contract)
      if (full) {
        Out8<TO>::st(yp, v);
        if (ep.aux) Out8<TO>::st(ep.aux + o, raw);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (n + e >= g.K) continue;
          io<TO>::st(yp, e, v[e]);
          if (ep.aux) io<TO>::st(ep.aux, o + e, raw[e]);
        }
      }
    }
  }
  if constexpr (STATS)
    if (!regst && !(ep.sdbg & 2))
      tile_stats<8, BN, NT / 64, SA>(s1, s2, CPR, (threadIdx.x & 63) < CPR, ch * 8, smem, T2D ? t2.tile : m0 / BM, n0,
                                     ep.stats, ep.sld, ep.sdbg);
}

// fused statistics after store_tile (register epilogue): lane holds fp64 sums of fragment column i's 4
// channels over its FM rows; lanes 16 apart hold other channel groups, lanes differing in bits 0-3 other rows
template <int FN, int BN, int NW>
__device__ __forceinline__ void frag_stats(double (&st1)[FN][4], double (&st2)[FN][4], int wno, char* smem,
                                           long long mtile, int n0, double* stats, int sld) {
  const int lane = threadIdx.x & 63;
  // reduce over the 16 row lanes of each channel group first (xor 8, 4, 2, 1)
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        st1[i][e] += __shfl_xor(st1[i][e], o, 64);
        st2[i][e] += __shfl_xor(st2[i][e], o, 64);
      }
  lds_barrier();
  double* red = (double*)smem;   // [NW][BN][2], zero where a wave holds no channel
  for (int k = threadIdx.x; k < NW * BN * 2; k += NW * 64) red[k] = 0.0;
  lds_barrier();
  const int w = threadIdx.x >> 6;
  if ((lane & 15) == 0)
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = wno + i * 16 + (lane >> 4) * 4 + e;
        red[(w * BN + c) * 2] = st1[i][e];
        red[(w * BN + c) * 2 + 1] = st2[i][e];
      }
  lds_barrier();
  for (int c = threadIdx.x; c < BN; c += NW * 64) {
    const int n = n0 + c;
    if (n >= sld) continue;
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      a += red[(k * BN + c) * 2];
      b += red[(k * BN + c) * 2 + 1];
    }
    stats[(mtile * 2) * sld + n] = a;
    stats[(mtile * 2 + 1) * sld + n] = b;
  }
}

// XCD-aware remap of a 1-D grid (bijective for any grid size): consecutive tile ids land on one XCD
__device__ __forceinline__ int xcd_tile(int bid, int ntiles) {
  const int xcd = bid & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

constexpr int ROWB = 80;   // 64 data bytes + 16 pad per LDS row

// ------------------------------------------------------------------------------------------------
// forward / dgrad / transposed-conv gather GEMM
// ------------------------------------------------------------------------------------------------
extern int g_knobs[17];   // runtime variant switches (ssseg_set_knob), defined in conv.hip
// 0: reg-staged pipeline depth; 1: split-K cap (-1 off = default, 0 auto: the autotuner also times each variant with
// its split plan, fp32-atomic partials + finalize, and keeps it where faster); 2: 64x64 small-M tiles (reg-staged path);
// 3: bf16 LDS-DMA path (0 on, -1 off); 4: variant (0 auto, 1..10 / 12..23 LDS-DMA config, 11 register-staged, 24 the
// halo-tiled 3x3 kernel where it applies, 25 its 32-channel form, 26 / 27 the pointwise kernels);
// 5: autotune unseen geometries (1 on, 0 = static heuristic); knob 6 = 1 clears the variant cache;
// 7: LDS-staged coalesced epilogue in the LDS-DMA kernel (0 on, -1 off);
// 8: bf16 weight gradient on the LDS-DMA kernel (0 on, -1 = register-staged wgrad_kernel);
// 9: LDS-DMA weight-gradient tile variant (0 = the static plan, 1.. = a forced WGRAD_CFGS entry, conv_wgrad.hip);
// 10: weight-gradient split count scale in percent (100 = the plan's); 11: halo-tiled 3x3 kernels (conv_wgrad_halo.hip,
// conv_hconv3.hip; 0 on, -1 = the split-K weight gradient and no variant 24); 12: fused-statistics experiment switch
// (Epi::sdbg, LDS-DMA configs; 0 = normal); 13: pointwise kernels (conv_pw.hip, variants 26 / 27; 0 on, -1 off)

// STATS: the epilogue also writes the fused BatchNorm statistics partials (a separate instantiation: the fp64
// sums raise the register count, which must not cost the launches that do not need them)
template <typename T, typename TO, int BM, int BN, int WM, int WN, bool DEEP, bool STATS = false>
__global__ void __launch_bounds__(256, DEEP ? 2 : 1) igemm_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                                  TO* __restrict__ y, ConvGeom g, Epi<TO> ep,
                                                                  int splits, float* __restrict__ ws) {
  constexpr int VEC = MF<T>::VEC;
  constexpr int BK = 64 / (int)sizeof(T);
  constexpr int A_PER = BM / 64;                 // pixel rows per thread (4 chunks per row)
  constexpr int B_IT = (BN * 4 + 255) / 256;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1, "tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * ROWB];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware remap of the 1-D grid: consecutive tile ids (the N tiles of one M tile, then the next
  // M tile) go to the same XCD so the gathered input rows are re-read from that XCD's L2.
  const int nnt = (g.K + BN - 1) / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const long long m0 = (long long)(tile / nnt) * BM;
  const int n0 = (tile % nnt) * BN;
  const int chunk = t & 3;
  const int RS = g.R * g.S;
  // split-K: this block reduces k-tiles [kt0, kt1) of the contraction (blockIdx.y = split index)
  const int nk_all = (g.KK + BK - 1) / BK;
  const int kper = (nk_all + splits - 1) / splits;
  const int kt0 = blockIdx.y * kper;
  const int kt1 = min(nk_all, kt0 + kper);

  int a_n[A_PER], a_oy[A_PER], a_ox[A_PER];
  bool a_ok[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const long long m = m0 + (t >> 2) + 64 * i;
    a_ok[i] = m < g.M;
    const long long mm = a_ok[i] ? m : 0;
    decode_m(g, (int)mm, a_n[i], a_oy[i], a_ox[i]);
  }
  // k-state of this thread's chunk: k = tap*C + kc, tap = r*S + s (advanced by every load, in order).
  // 16-bit operands with C % 64 == 0 run the LDS-DMA kernel's order (64-channel block major, tap minor, two
  // 32-deep halves per block and tap), so every variant accumulates the same MFMA k-sequence (bitwise equal).
  const bool cm = sizeof(T) == 2 && (g.C & 63) == 0;
  int tap, kc, r, s, half = 0;
  if (cm) {
    const int cb = kt0 / (2 * RS), rem = kt0 - cb * 2 * RS;
    tap = rem >> 1;
    half = rem & 1;
    kc = cb * 64 + half * BK + chunk * VEC;
  } else {
    const int k_first = kt0 * BK + chunk * VEC;
    tap = min(k_first / g.C, RS);
    kc = k_first - tap * g.C;
  }
  r = tap / max(g.S, 1);
  s = tap - r * g.S;
  const int nk = max(kt1 - kt0, 0);

  auto load = [&](uint4 (&ra)[A_PER], uint4 (&rb)[B_IT], int kt) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int iy = a_oy[i] * g.sy + r * g.dy + g.py;
      const int ix = a_ox[i] * g.sx + s * g.dx + g.px;
      const bool ok = a_ok[i] && tap < RS && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      ra[i] = ok ? *(const uint4*)(x + ((long long)(a_n[i] * g.H + iy) * g.W + ix) * g.ldx + kc) : make_uint4(0, 0, 0, 0);
    }
    // B rows: the same k as this thread's A chunk (id & 3 == t & 3)
    const int kb = tap < RS ? tap * g.C + kc : g.KK;
#pragma unroll
    for (int j = 0; j < B_IT; ++j) {
      const int id = t + 256 * j;
      rb[j] = make_uint4(0, 0, 0, 0);
      if (id < BN * 4) {
        const int n = n0 + (id >> 2);
        if (n < g.K && kb < g.KK) rb[j] = *(const uint4*)(w + (long long)n * g.ldw + kb);
      }
    }
    (void)kt;
    if (cm) {
      if (!half) {
        half = 1;
        kc += BK;
      } else {
        half = 0;
        kc -= BK;
        ++tap;
        if (++s == g.S) { s = 0; ++r; }
        if (tap == RS) { tap = 0; r = 0; s = 0; kc += 2 * BK; }
      }
    } else {
      kc += BK;
      while (kc >= g.C && tap < RS) {
        kc -= g.C; ++tap;
        if (++s == g.S) { s = 0; ++r; }
      }
    }
  };
  auto store = [&](const uint4 (&ra)[A_PER], const uint4 (&rb)[B_IT], int buf) {
    char* As = smem + buf * (BM + BN) * ROWB;
    char* Bs = As + BM * ROWB;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) *(uint4*)(As + ((t >> 2) + 64 * i) * ROWB + chunk * 16) = ra[i];
#pragma unroll
    for (int j = 0; j < B_IT; ++j) {
      const int id = t + 256 * j;
      if (id < BN * 4) *(uint4*)(Bs + (id >> 2) * ROWB + (id & 3) * 16) = rb[j];
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* As = smem + buf * (BM + BN) * ROWB;
    const char* Bs = As + BM * ROWB;
    typename MF<T>::frag af[FN], bfr[FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
      af[i] = *(const typename MF<T>::frag*)(Bs + (wn * WTN + i * 16 + (lane & 15)) * ROWB + (lane >> 4) * 16);
#pragma unroll
    for (int j = 0; j < FM; ++j)
      bfr[j] = *(const typename MF<T>::frag*)(As + (wm * WTM + j * 16 + (lane & 15)) * ROWB + (lane >> 4) * 16);
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) MF<T>::mma(af[i], bfr[j], acc[i][j]);
  };

  if constexpr (DEEP) {
    // two register sets: tile kt+2 is in flight while tile kt is multiplied and tile kt+1 is staged
    uint4 ra0[A_PER], rb0[B_IT], ra1[A_PER], rb1[B_IT];
    if (nk > 0) load(ra0, rb0, 0);
    if (nk > 1) load(ra1, rb1, 1);
    if (nk > 0) store(ra0, rb0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      if (kt + 2 < nk) load(ra0, rb0, kt + 2);
      compute(0);
      if (kt + 1 < nk) store(ra1, rb1, 1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      if (kt + 3 < nk) load(ra1, rb1, kt + 3);
      compute(1);
      if (kt + 2 < nk) store(ra0, rb0, 0);
      __syncthreads();
    }
  } else {
    // one register set: tile kt+1 is in flight while tile kt is multiplied
    uint4 ra0[A_PER], rb0[B_IT];
    if (nk > 0) {
      load(ra0, rb0, 0);
      store(ra0, rb0, 0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load(ra0, rb0, kt + 1);
      compute(kt & 1);
      if (kt + 1 < nk) store(ra0, rb0, (kt + 1) & 1);
      __syncthreads();
    }
  }

  // epilogue: lane holds channels n..n+3 (n = 4*(lane>>4) within a 16-wide fragment) of pixel lane&15
  if (splits > 1) {   // fp32 partials into ws[m][K]; finalize applies the epilogue and writes y
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const long long m = m0 + wm * WTM + j * 16 + (lane & 15);
      if (m >= g.M) continue;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * WTN + i * 16 + (lane >> 4) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < g.K) atomicAdd(ws + m * g.K + n + e, acc[i][j][e]);
      }
    }
    return;
  }
  if constexpr (STATS) {
    double st1[FN][4], st2[FN][4];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) st1[i][e] = st2[i][e] = 0.0;
    store_tile<TO, FM, FN, true>(acc, m0 + wm * WTM, n0 + wn * WTN, lane, g, y, ep, st1, st2);
    frag_stats<FN, BN, 4>(st1, st2, wn * WTN, smem, m0 / BM, n0, ep.stats, ep.sld);
    return;
  }
  store_tile<TO, FM, FN>(acc, m0 + wm * WTM, n0 + wn * WTN, lane, g, y, ep);
}

// ------------------------------------------------------------------------------------------------
// bf16 gather GEMM, LDS-DMA pipeline (gfx950), for C % 64 == 0.  Same contraction and epilogue as
// igemm_kernel.  k runs channel-block major, tap minor, and a k-tile (BK = 64) never straddles a tap, so the
// tap (r, s) and channel block c0 are wave-uniform scalars.  Tiles are staged by buffer_load ... lds
// (16 B per lane straight into LDS, no VGPR round trip) into an NS-deep LDS ring: NS-1 tiles are in
// flight while one is multiplied, one raw barrier per k-tile, counted vmcnt.  Per-lane byte offsets are
// rebuilt only when the tap changes (padding pixels get an out-of-range offset: the buffer unit
// returns zeros); inside a tap only the scalar soffset moves.  The LDS image is lane-linear (one
// wave-instruction = 8 rows x 128 B); the bank swizzle (16-byte chunk c of row r stored at
// c ^ ((r >> 1) & 7)) is applied on the per-lane source offset, and fragment reads apply the same XOR.
// ------------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void bldslds16(__amdgpu_buffer_rsrc_t rs, char* lds_wave_base, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)lds_wave_base, 16, voff, soff, 0, 0);
}

// The same LDS-DMA issued from inline asm, i.e. invisible to hipcc's s_waitcnt bookkeeping.  Kernels whose LDS reads
// are ds_read_b64_tr_b16 need it: the transposed-read builtin carries no LDS alias scope, so for every such read hipcc
// inserts an s_waitcnt vmcnt(0) on ALL outstanding LDS-DMA -- including the ring's prefetch issued just before the
// compute, which serialises the pipeline (seen in the .s of wgrad_glds_kernel and wgrad_halo3_kernel; the ds_read_b128
// fragments of igemm_glds_kernel carry the scope and get no such wait).  Completion is then counted only by the kernel's
// own vmcnt_wait<> ring waits.  M0 (the LDS destination) is compiler-reserved: set and restored inside the statement.
__device__ __forceinline__ void bldslds16_nt(__amdgpu_buffer_rsrc_t rs, char* lds_wave_base, unsigned voff,
                                             unsigned soff) {
  const unsigned la = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds_wave_base);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(la), "s"(soff)
      : "memory");
}

template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until the ring's oldest tile landed when `ahead` (<= D - 1) later tiles of NL vmcnt units each may stay in flight
template <int NL, int D>
__device__ __forceinline__ void ring_wait(int ahead) {
  if (D >= 3 && ahead >= 2) vmcnt_wait<2 * NL>();
  else if (D >= 2 && ahead >= 1) vmcnt_wait<NL>();
  else vmcnt_wait<0>();
}

constexpr unsigned OOB = 0x80000000u;   // > any num_records we build: the load returns zeros

// ---- deterministic split-K (S k-slices per output tile, combined inside the launch) ---------------------------------
// Tickets: one u32 per (phase, tile) in the library's ticket pool (ticket_slots: zero at load, a range per launch,
// every ticket reset to zero by the block that draws last -- no memset launch before a split launch).
// Workspace: [unused ticket-sized region, padded to 256 B]
// [slabs: per (phase, tile) S slices x NW waves x FN*FM fragments x 64 lanes x 16 B of fp32 partials].
// Every slice block writes its partial accumulators with write-through (sc1) 16-byte stores, every wave drains its
// stores, then one lane adds to the tile's ticket (agent scope); the block that draws S-1 is the last one and sums the
// S partials with sc1 loads (they bypass this CU's L1, which may hold stale lines of an earlier launch's slabs) in
// slice order 0, 1, ..., S-1 -- a fixed order, whichever block arrives last: the result is bitwise reproducible and the
// same for every tile config (cdna_hip_programming.md §5 'In-launch split-K reduction', §6 Guideline 16, R1 form).
constexpr int DSPLIT_MAX_FRAGS = 8;   // per wave: the combine keeps 2-3 accumulator sets live

__host__ __device__ inline long long dsplit_ticket_bytes(long long ntiles) { return (ntiles * 4 + 255) / 256 * 256; }

template <int FN, int FM, int NW>
__device__ __forceinline__ bool dsplit_combine(f32x4 (&acc)[FN][FM], float* ws, unsigned* tick, int tg, int slice,
                                               int splits, int ntiles, char* smem) {
  constexpr int F = FN * FM;
  constexpr unsigned TILE_BYTES = NW * F * 1024;   // one slice's partial tile
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  char* base = (char*)ws + dsplit_ticket_bytes(ntiles) + (long long)tg * splits * TILE_BYTES;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(splits * TILE_BYTES), 0x00020000);
  const unsigned vo = (unsigned)((wave * F * 64 + lane) * 16);
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, vo + (i * FM + j) * 1024,
                                             slice * TILE_BYTES, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its partial left the CU
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(tick + tg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool is_last = old == (unsigned)(splits - 1);
    // every slice has drawn: the last one leaves the ticket at zero for the next launch that uses this pool slot
    if (is_last) __hip_atomic_store(tick + tg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *(volatile int*)smem = is_last;
  }
  __syncthreads();
  const bool last = *(volatile int*)smem != 0;
  if (!last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the loads below the ticket
  for (int s = 0; s < splits; ++s) {
    u32x4 v[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
        v[i][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + (i * FM + j) * 1024, s * TILE_BYTES, 16);
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const f32x4 p = __builtin_bit_cast(f32x4, v[i][j]);
        acc[i][j] = s ? acc[i][j] + p : p;
      }
  }
  return true;
}

// KM (k mode): 0 = 64-channel k-tiles (C % 64 == 0, channel block major, tap minor: the tile's tap and channel block
// are scalars); 1 = the same over a virtual concat input (ConvGeom.c1b / ldx2): k-tiles of channel block >= c1b
// gather from x2 (a scalar choice per k-tile: the block never straddles the seam because both parts are whole
// 64-channel blocks); 2 = general k (any C % 8 == 0: HRNet-W32's 32-channel branches, HarDNet's growth layers):
// k runs linearly, k = tap * C + c, exactly like the register-staged kernel, so a 64-deep k-tile may hold several
// taps -- every lane splits its own 16-byte chunk's k into (tap, channel) and gathers from that tap's pixel
// minimum waves per SIMD the register allocator must leave room for, where registers (not LDS) bound the occupancy:
// the single-slot 128x64 tile (the 1x1 expansions' choice, a load -> 8 MFMA -> store chain per tile) fits four blocks
// per CU in LDS (34.8 KB each) but its 140 registers allowed three -- capped at 128 it runs four (64->256 1x1
// @16x128^2: 56 -> 48 us, with fused statistics 78 -> 69 us); the 8-wave 256x64 two-slot tile fits two blocks in LDS
// (80 KB each) but its statistics instantiation's 132 registers allowed one; the 8-wave 128x64 two-slot tile fits
// three blocks (48 KB) but its 88-92 registers allowed two
#ifndef SSSEG_GLDS_OCC_MODE
#define SSSEG_GLDS_OCC_MODE 1   // 0: no caps, 2: also the 8-wave 128x64 tile at 6 waves (spills; A/B builds)
#endif
#define GLDS_OCC(BM, BN, NW, NS)                                                                                   \
  (SSSEG_GLDS_OCC_MODE == 0 ? 1                                                                                  \
   : (((BM) == 128 && (BN) == 64 && (NW) == 4 && (NS) == 1) ||                                                   \
      ((BM) == 256 && (BN) == 64 && (NW) == 8 && (NS) == 2))                                                     \
       ? 4                                                                                                       \
       : ((SSSEG_GLDS_OCC_MODE >= 2 && (BM) == 128 && (BN) == 64 && (NW) == 8 && (NS) == 2) ? 6 : 1))
template <typename TO, int BM, int BN, int WM, int WN, int NW, int NS, bool STATS, int KM = 0>
__global__ void __launch_bounds__(NW * 64, GLDS_OCC(BM, BN, NW, NS)) igemm_glds_kernel(const TO* __restrict__ x,
                                                                const TO* __restrict__ w, TO* __restrict__ y,
                                                                ConvGeom g, Epi<TO> ep, unsigned xbytes,
                                                                unsigned wbytes, int g_epi_lds, int splits,
                                                                float* __restrict__ ws, unsigned* tix, PhaseTab ph,
                                                                const TO* __restrict__ x2, unsigned x2bytes) {
  constexpr int ROW = 128;                       // bytes per LDS row = 64 bf16 of k
  constexpr bool VC = KM == 1, GK = KM == 2;
  constexpr int STAGE = (BM + BN) * ROW;
  constexpr int AI = BM / 8 / NW;                // A (pixel) wave-instructions per wave per stage
  constexpr int BI = BN / 8 / NW;                // B (weight) wave-instructions per wave per stage
  constexpr int NL = AI + BI;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  static_assert(WM * WN == NW && FM >= 1 && FN >= 1 && AI >= 1 && BI >= 1 && NS >= 1 && NS <= 4, "tile");
  // NS == 1 (single-slot ring, for nk == 1..2: 1x1 convs over 64-128 channels): the slot is sized to also
  // hold the staged epilogue, and occupancy (4-9 workgroups per CU) hides the load -> MFMA -> store chain
  constexpr int EPI = BM * (BN * 4 + 16);
  constexpr int SMEM = (NS == 1 && EPI > STAGE) ? EPI : NS * STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  // wave index as a scalar: the LDS-DMA destinations (per-wave LDS bases) then need no readfirstlane per load
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int nnt = (g.K + BN - 1) / BN;
  // deterministic split-K (splits = S > 1, a power of two): block id -> (output tile, k-slice); the S slices of a tile
  // are consecutive in the XCD-remapped order (one XCD, next to the n-tiles of the same pixel tile)
  const int lsp = 31 - __builtin_clz((unsigned)splits);
  const int bid = xcd_tile(blockIdx.x, gridDim.x);
  const int tile = bid >> lsp, slice = bid & (splits - 1);
  static_assert(BN == 64 || BN == 128 || BN == 256, "n-tile divisor magic");
  const int mt_ = fdiv(tile, BN == 64 ? g.mn64 : (BN == 128 ? g.mn128 : g.mn256),
                       BN == 64 ? g.sn64 : (BN == 128 ? g.sn128 : g.sn256));   // tile / nnt
  const long long m0 = (long long)mt_ * BM;
  const int n0 = (tile - mt_ * nnt) * BN;
  if (ph.n > 1) {   // this block's output phase: offsets, sub-grid, weights, statistics rows
    const int p = blockIdx.y;
    g.py = ph.py[p];
    g.px = ph.px[p];
    g.ooy = ph.ooy[p];
    g.oox = ph.oox[p];
    w = (const TO*)ph.w[p];
    if (ep.stats) ep.stats += (long long)p * ((g.M + BM - 1) / BM) * 2 * ep.sld;
  }
  const int RS = g.R * g.S;
  const int cpt = g.C >> 6;                      // k-tiles per tap
  // split-K (low-tile layers): this block reduces k-tiles [kt0, kt0 + nk) in order; the partition depends on the
  // contraction and S only (never on the tile config), so every config sums the same slices
  const int nk_all = GK ? (g.KK + 63) >> 6 : RS * cpt;
  int kt0 = 0, nk = nk_all;   // the common unsplit launch: no divisions
  if (splits > 1) {
    const int kper = (nk_all + splits - 1) / splits;
    kt0 = min(nk_all, slice * kper);
    nk = min(nk_all, kt0 + kper) - kt0;
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, (int)wbytes, 0x00020000);
  __amdgpu_buffer_rsrc_t xr2 = xr;
  if constexpr (VC) xr2 = __builtin_amdgcn_make_buffer_rsrc((void*)x2, (short)0, (int)x2bytes, 0x00020000);

  // lane rows: A row 8*(wave*AI + ii) + (lane>>3), B row 8*(wave*BI + jj) + (lane>>3); the lane loads
  // logical chunk (lane & 7) ^ swz(row) = (lane & 7) ^ (lane >> 4) ^ 4*(instruction parity)
  const int c_even = (lane & 7) ^ (lane >> 4);
  int a_off[AI], a_iy[AI], a_ix[AI];
  int a_pix[VC ? AI : 1];   // VC: input pixel index of the row (the byte offset differs per source)
  int a_k[GK ? AI : 1];     // GK: k of this lane's chunk in the next k-tile to issue
#pragma unroll
  for (int ii = 0; ii < AI; ++ii) {
    const int inst = wave * AI + ii;
    const int ch = c_even ^ ((inst & 1) * 4);
    const long long m = m0 + 8 * inst + (lane >> 3);
    int pix = 0;
    if (m < g.M && g.aident) {   // 1x1 / stride 1 / no padding: input pixel m, always in bounds
      a_iy[ii] = 0;
      a_ix[ii] = 0;
      pix = (int)m;
    } else if (m < g.M) {
      int img, oy, ox;   // M < 2^31 (geom_ok): 32-bit decode
      decode_m(g, (int)m, img, oy, ox);
      a_iy[ii] = oy * g.sy + g.py;
      a_ix[ii] = ox * g.sx + g.px;
      pix = (img * g.H + a_iy[ii]) * g.W + a_ix[ii];
    } else {
      a_iy[ii] = -0x40000000;   // never in bounds
      a_ix[ii] = 0;
    }
    a_off[ii] = pix * g.ldx * 2 + (GK ? 0 : ch * 16);
    if constexpr (VC) a_pix[ii] = pix * g.ldx2 * 2 + ch * 16;
    if constexpr (GK) a_k[ii] = kt0 * 64 + ch * 8;
  }
  unsigned b_off[BI];
#pragma unroll
  for (int jj = 0; jj < BI; ++jj) {
    const int inst = wave * BI + jj;
    const int ch = c_even ^ ((inst & 1) * 4);
    const int n = n0 + 8 * inst + (lane >> 3);
    b_off[jj] = n < g.K ? (unsigned)(n * g.ldw * 2 + ch * 16) : OOB;
  }

  unsigned a_cur[AI];   // byte offsets of this lane's A rows for the current tap (OOB = padding)
  unsigned a_cur2[VC ? AI : 1];   // VC: the same rows in x2
  auto set_tap = [&](int tap) {
    const int r = fdiv(tap, g.mS, g.sS), s_ = tap - r * g.S;
    const int dyy = r * g.dy, dxx = s_ * g.dx;
    const int toff = (dyy * g.W + dxx) * g.ldx * 2;
#pragma unroll
    for (int ii = 0; ii < AI; ++ii) {
      const int iy = a_iy[ii] + dyy, ix = a_ix[ii] + dxx;
      const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      a_cur[ii] = ok ? (unsigned)(a_off[ii] + toff) : OOB;
      if constexpr (VC) a_cur2[ii] = ok ? (unsigned)(a_pix[ii] + (dyy * g.W + dxx) * g.ldx2 * 2) : OOB;
    }
  };

  // k-tile order: channel block major, tap minor (kt = cb * RS + tap).  The taps of one 64-channel block re-read
  // the same input lines RS times in a row, so those re-reads hit L2 (PMC: a tap-major sweep over all C kept
  // BM x C x 2 B per block live -- 50 MB over the chip at 384 channels -- and its re-reads went to the Infinity
  // Cache at 2.6x the L2 latency, which is what bounds the LDS-DMA stream: ~90 outstanding lines per CU)
  // GK: the (tap, channel) of each lane's chunk k; k >= KK (the last tile's tail) is a padding tap (zeros), so
  // the weight bytes loaded there (the next row's head) only ever meet zeros
  auto set_k = [&]() {
#pragma unroll
    for (int ii = 0; ii < AI; ++ii) {
      const int k = a_k[ii];
      const int tap = fdiv(k, g.mC, g.sC), c = k - tap * g.C;
      const int r = fdiv(tap, g.mS, g.sS), s_ = tap - r * g.S;
      const int dyy = r * g.dy, dxx = s_ * g.dx;
      const int iy = a_iy[ii] + dyy, ix = a_ix[ii] + dxx;
      const bool ok = tap < RS && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      a_cur[ii] = ok ? (unsigned)(a_off[ii] + ((dyy * g.W + dxx) * g.ldx + c) * 2) : OOB;
    }
  };
  int ld_tap = kt0 ? kt0 % RS : 0, ld_c = kt0 ? kt0 / RS : 0;   // next: tap, channel block
  int ld_kt = kt0;                                              // GK: next k-tile
  if constexpr (GK) set_k();
  else set_tap(ld_tap);
  auto issue = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + BM * ROW;
    if constexpr (GK) {
      const unsigned sb = (unsigned)__builtin_amdgcn_readfirstlane(ld_kt * 128);
#pragma unroll
      for (int ii = 0; ii < AI; ++ii) bldslds16(xr, As + (wave * AI + ii) * 1024, a_cur[ii], 0u);
#pragma unroll
      for (int jj = 0; jj < BI; ++jj) bldslds16(wr, Bs + (wave * BI + jj) * 1024, b_off[jj], sb);
      ++ld_kt;
#pragma unroll
      for (int ii = 0; ii < AI; ++ii) a_k[ii] += 64;
      set_k();
      return;
    }
    // wave-uniform soffsets, stated as such (otherwise the compiler may keep the k-state in VGPRs and wrap every
    // LDS-DMA issue in a readfirstlane waterfall loop)
    const unsigned sa = (unsigned)__builtin_amdgcn_readfirstlane(ld_c * 128),
                   sb = (unsigned)__builtin_amdgcn_readfirstlane((ld_tap * cpt + ld_c) * 128);
    if (VC && ld_c >= g.c1b) {   // channel block of the second source (scalar branch)
      const unsigned sa2 = (unsigned)(ld_c - g.c1b) * 128u;
#pragma unroll
      for (int ii = 0; ii < AI; ++ii) bldslds16(xr2, As + (wave * AI + ii) * 1024, a_cur2[ii], sa2);
    } else {
#pragma unroll
      for (int ii = 0; ii < AI; ++ii) bldslds16(xr, As + (wave * AI + ii) * 1024, a_cur[ii], sa);
    }
#pragma unroll
    for (int jj = 0; jj < BI; ++jj) bldslds16(wr, Bs + (wave * BI + jj) * 1024, b_off[jj], sb);
    if (++ld_tap == RS) {
      ld_tap = 0;
      ++ld_c;
    }
    if (RS > 1) set_tap(ld_tap);
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // single-slot configs (one or two k-tiles: the 1x1 layers) with a residual: the LDS-staged epilogue's
  // residual chunks are loaded here, in flight with the operand DMA, instead of after the MFMAs -- one dependent
  // HBM round trip less per tile in a kernel whose tiles are a load -> multiply -> store chain
  constexpr int EP_CPR = BN / 8, EP_RPP = NW * 64 / EP_CPR, EP_NP = (BM + EP_RPP - 1) / EP_RPP;
  constexpr bool PRE = NS == 1 && EPI <= SMEM && (NW * 64) % EP_CPR == 0 && 64 % EP_CPR == 0;
  PreRes<PRE ? EP_NP : 1> pre;
  pre.on = false;
  if constexpr (PRE) {
    if (ep.res && splits == 1) {
      const int ch = t % EP_CPR, r0 = t / EP_CPR;
      const int n = n0 + ch * 8;
      pre.on = (g.ldy & 7) == 0 && (ep.ldr & 7) == 0 && n + 7 < g.K && n < ep.oc1;
#pragma unroll
      for (int p = 0; p < EP_NP; ++p) {
        const int row = r0 + p * EP_RPP;
        const long long m = m0 + row;
        pre.v[p] = u32x4{0u, 0u, 0u, 0u};
        if (pre.on && row < BM && m < g.M) {
          const long long op = out_pixel(g, (int)m);   // M < 2^31 (geom_ok)
          pre.v[p] = *(const u32x4*)(ep.res + op * ep.ldr + n);
        }
      }
    }
  }
  const int rsw = ((lane & 15) >> 1) & 7;   // read-side swizzle of this lane's fragment row
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * ROW;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int pc = ((ks * 4 + (lane >> 4)) ^ rsw) * 16;
      bf16x8 af[FN], bfr[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i) af[i] = *(const bf16x8*)(Bs + (wn * WTN + i * 16 + (lane & 15)) * ROW + pc);
#pragma unroll
      for (int j = 0; j < FM; ++j) bfr[j] = *(const bf16x8*)(As + (wm * WTM + j * 16 + (lane & 15)) * ROW + pc);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = M16<TO>::mma(af[i], bfr[j], acc[i][j]);
    }
  };

  if constexpr (NS == 1) {
    for (int kt = 0; kt < nk; ++kt) {
      if (kt) __builtin_amdgcn_s_barrier();   // every wave is done reading the slot
      issue(0);
      vmcnt_wait<0>();
      __builtin_amdgcn_s_barrier();           // every wave's part of tile kt landed
      compute(0);
    }
  } else {
    constexpr int D = NS - 1;   // tiles in flight ahead of the one being multiplied
#pragma unroll
    for (int p = 0; p < D; ++p)
      if (p < nk) issue(p);
    for (int kt = 0; kt < nk; ++kt) {
      // wait for tile kt: the tiles issued after it (at most D-1) may stay in flight
      const int ahead = min(nk - 1, kt + D - 1) - kt;
      if (D >= 3 && ahead >= 2) vmcnt_wait<2 * NL>();
      else if (D >= 2 && ahead >= 1) vmcnt_wait<NL>();
      else vmcnt_wait<0>();
      __builtin_amdgcn_s_barrier();   // every wave's tile kt landed; ring slot (kt+D)%NS is free
      if (kt + D < nk) issue((kt + D) % NS);
      compute(kt % NS);
    }
  }
  if constexpr (FN * FM <= DSPLIT_MAX_FRAGS) {
    if (splits > 1) {   // the last-arriving slice of the tile sums all S partials in slice order, then the epilogue
      const int tpp = (int)(gridDim.x >> lsp);   // tiles per phase
      if (!dsplit_combine<FN, FM, NW>(acc, ws, tix, (ph.n > 1 ? (int)blockIdx.y : 0) * tpp + tile, slice, splits,
                                      tpp * (int)gridDim.y, smem))
        return;
    }
  }
  if constexpr (EPI <= SMEM) {
    // the LDS-staged epilogue whenever the staged tile fits the ring (the register epilogue is not even compiled
    // then: as dead code it cost the statistics instantiations a scratch frame)
    (void)g_epi_lds;
    store_tile_lds<TO, BM, BN, FM, FN, NW * 64, STATS, PRE ? EP_NP : 1>(acc, smem, m0, n0, wm * WTM, wn * WTN, lane,
                                                                        g, y, ep, pre);
  } else if constexpr (STATS) {
    double st1[FN][4], st2[FN][4];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) st1[i][e] = st2[i][e] = 0.0;
    store_tile<TO, FM, FN, true>(acc, m0 + wm * WTM, n0 + wn * WTN, lane, g, y, ep, st1, st2);
    frag_stats<FN, BN, NW>(st1, st2, wn * WTN, smem, m0 / BM, n0, ep.stats, ep.sld);
  } else {
    store_tile<TO, FM, FN>(acc, m0 + wm * WTM, n0 + wn * WTN, lane, g, y, ep);
  }
}

// split-K finalize: y[pixel(m)][n] = act(ws[m][n] * scale[n] + shift[n] + res[pixel(m)][n])
template <typename TO>
__global__ void splitk_finalize_kernel(const float* __restrict__ ws, TO* __restrict__ y, ConvGeom g, Epi<TO> ep) {
  const long long total = g.M * g.K;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(i % g.K);
    const long long m = i / g.K;
    const long long op = out_pixel(g, (int)m);   // M < 2^31 (geom_ok)
    float v = ws[i];
    if (ep.aux) io<TO>::st(ep.aux, op * g.ldy + n, v);
    if (ep.scale) v *= ep.scale[n];
    if (ep.shift) v += ep.shift[n];
    const float r = (ep.res && n < ep.oc1) ? io<TO>::ld(ep.res, op * ep.ldr + n) : 0.f;
    if (!ep.rmask) v += r;
    v = act_fwd(v, ep.relu, ep.slope);
    if (ep.rmask && n < ep.oc1 && !(r > 0.f)) v = ep.rmask == SSSEG_ACT_LEAKY ? v * ep.rslope : 0.f;
    io<TO>::st(out_at(ep, y, g.ldy, op, n), 0, v);
  }
}

// output pixels of a phase whose tap set is empty (e.g. odd rows of a 1x1/s2 dgrad): epilogue of 0
// 8 channels per thread (K % 8 == 0, 16-byte aligned rows): one 16-byte store per chunk
template <typename TO>
__global__ void phase_zero_vec_kernel(TO* y, ConvGeom g, Epi<TO> ep) {
  const int kc = g.K >> 3;
  const long long total = g.M * kc;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(i % kc) * 8;
    const long long m = i / kc;
    const long long op = out_pixel(g, (int)m);   // M < 2^31 (geom_ok)
    float r[8], v[8];
    if (ep.res && !ep.rmask) Out8<TO>::ld(ep.res + op * ep.ldr + n, r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = ep.shift ? ep.shift[n + e] : 0.f;
      if (ep.res && !ep.rmask) t += r[e];
      v[e] = act_fwd(t, ep.relu, ep.slope);
    }
    if (ep.aux) {
      const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      Out8<TO>::st(ep.aux + op * g.ldy + n, z);
    }
    Out8<TO>::st(out_at(ep, y, g.ldy, op, n), v);
  }
}

template <typename TO>
__global__ void phase_zero_kernel(TO* y, ConvGeom g, Epi<TO> ep) {
  const long long total = g.M * g.K;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(i % g.K);
    const long long m = i / g.K;
    const long long op = out_pixel(g, (int)m);   // M < 2^31 (geom_ok)
    float v = ep.shift ? ep.shift[n] : 0.f;
    if (ep.aux) io<TO>::st(ep.aux, op * g.ldy + n, 0.f);
    if (ep.res && !ep.rmask) v += io<TO>::ld(ep.res, op * ep.ldr + n);
    v = act_fwd(v, ep.relu, ep.slope);
    io<TO>::st(out_at(ep, y, g.ldy, op, n), 0, v);
  }
}

template <typename T, int BM, int BN>
inline int plan_splits(const ConvGeom& g);

template <typename TO>
__global__ void splitk_finalize_kernel(const float* __restrict__ ws, TO* __restrict__ y, ConvGeom g, Epi<TO> ep);

// S of the deterministic split-K for the launch being dispatched (conv.hip dispatch_igemm sets it: 1 = unsplit); a
// config whose per-wave fragment count exceeds DSPLIT_MAX_FRAGS cannot run a split launch (-1)
extern thread_local int t_dsplit;

// n consecutive self-resetting tickets of the library's pool (conv.hip): ranges rotate over the pool, so launches in
// flight together (a few streams) never share one
unsigned* ticket_slots(long long n);

template <typename TO, int BM, int BN, int WM, int WN, int NW, int NS, int VC>
int launch_glds_vc(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                   unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2, unsigned x2b) {
  static_assert(sizeof(TO) == 2, "LDS-DMA configs: 16-bit activations in and out (fp32-output heads have K <= 16)");
  constexpr int FRAGS = (BM / WM / 16) * (BN / WN / 16);
  const long long tiles = ((g.M + BM - 1) / BM) * ((g.K + BN - 1) / BN);
  const int epi = (int)(g_knobs[7] == 0);
  const TO* xa = (const TO*)x2;
  const PhaseTab one{1, {0}, {0}, {0}, {0}, {nullptr}};
  const bool phased = ph && ph->n > 1;   // all output phases in one launch (blockIdx.y = phase)
  const PhaseTab& pt = phased ? *ph : one;
  const unsigned nph = phased ? (unsigned)ph->n : 1u;
  const int sp = ws ? t_dsplit : 1;
  if (sp > 1 && (FRAGS > DSPLIT_MAX_FRAGS || tiles * sp > 0x7fffffffLL)) return -1;
  unsigned* tix = sp > 1 ? ticket_slots(tiles * nph) : nullptr;
  if (sp > 1 && !tix) return -1;
  const dim3 grid((unsigned)(tiles * sp), nph);
  if (ep.stats)
    hipLaunchKernelGGL((igemm_glds_kernel<TO, BM, BN, WM, WN, NW, NS, true, VC>), grid, dim3(NW * 64), 0, s,
                       (const TO*)x, (const TO*)w, (TO*)y, g, ep, xb, wb, epi, sp, ws, tix, pt, xa, x2b);
  else
    hipLaunchKernelGGL((igemm_glds_kernel<TO, BM, BN, WM, WN, NW, NS, false, VC>), grid, dim3(NW * 64), 0, s,
                       (const TO*)x, (const TO*)w, (TO*)y, g, ep, xb, wb, epi, sp, ws, tix, pt, xa, x2b);
  return BM;
}

// bytes of the deterministic split-K workspace of S slices over any LDS-DMA config (tiles of BM <= 256, BN <= 128 with
// at most DSPLIT_MAX_FRAGS fragments per wave: a slice tile holds at most BM x BN fp32 partials, and the tile grid
// covers at most (M + 255) x (K + 127) outputs per phase); tickets for the smallest tile (64 x 64)
static inline size_t dsplit_ws_bytes(const ConvGeom& g, int nph, int S) {
  if (S <= 1) return 0;
  const long long t64 = (long long)nph * ((g.M + 63) / 64) * ((g.K + 63) / 64);
  return (size_t)(dsplit_ticket_bytes(t64) + (long long)S * nph * (g.M + 255) * (g.K + 127) * 4);
}

// x2 != nullptr: the virtual-concat instantiation (second input source, ConvGeom.c1b / ldx2)
template <typename TO, int BM, int BN, int WM, int WN, int NW, int NS>
int launch_glds(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb, unsigned wb,
                hipStream_t s, float* ws, const PhaseTab* ph, const void* x2 = nullptr, unsigned x2b = 0) {
  if (x2) return launch_glds_vc<TO, BM, BN, WM, WN, NW, NS, 1>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
  if (g.C & 63) {   // general k: instantiated for the 64-wide n-tiles only (the C % 64 != 0 layers have K <= 98)
    if constexpr (BN == 64) return launch_glds_vc<TO, BM, BN, WM, WN, NW, NS, 2>(x, w, y, g, ep, xb, wb, s, ws, ph, nullptr, 0);
    return -1;
  }
  return launch_glds_vc<TO, BM, BN, WM, WN, NW, NS, 0>(x, w, y, g, ep, xb, wb, s, ws, ph, nullptr, 0);
}


// LDS-DMA configs, one translation unit per group (conv_glds_*.hip) so the engine compiles in parallel.
// Each returns the tile height BM of the launched config (the fused BN statistics write ceil(M/BM) rows).
template <typename TO>
int launch_glds_grp_a(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2 = nullptr,
                      unsigned x2b = 0);
template <typename TO>
int launch_glds_grp_b(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2 = nullptr,
                      unsigned x2b = 0);
template <typename TO>
int launch_glds_grp_d(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2 = nullptr,
                      unsigned x2b = 0);
template <typename TO>
int launch_glds_grp_e(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2 = nullptr,
                      unsigned x2b = 0);
template <typename TO>
int launch_glds_grp_c(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                      unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2 = nullptr,
                      unsigned x2b = 0);


template <typename T, int BM, int BN>
inline int plan_splits(const ConvGeom& g) {
  const long long tiles = ((g.M + BM - 1) / BM) * ((g.K + BN - 1) / BN);
  const int nk = (g.KK + 64 / (int)sizeof(T) - 1) / (64 / (int)sizeof(T));
  if (g_knobs[1] < 0 || tiles >= 512 || nk < 32) return 1;
  long long sp = (1024 + tiles - 1) / tiles;
  sp = std::min<long long>(sp, nk / 16);
  if (g_knobs[1] > 0) sp = std::min<long long>(sp, g_knobs[1]);
  return (int)std::max<long long>(1, std::min<long long>(sp, 64));
}


// halo-tiled 3x3 / stride-1 / pad-1 forward (and stride-1 input-gradient) contraction, LDS-DMA variant 24 of the
// autotuner (conv_hconv3.hip); returns the tile height 256, or -1 where it cannot run the launch
template <typename TO>
int launch_hconv3(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                  unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2, unsigned x2b,
                  int mode = 0);

// the same for 32 input and 32 output channels (conv_hconv3s.hip), variant 25; 256 or -1
template <typename TO>
int launch_hconv3s(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                   hipStream_t s, float* ws, const PhaseTab* ph, const void* x2);

// pointwise 1x1 / stride-1 contraction over 64 or 128 channels (conv_pw.hip), variants 26 (fj = 4: 64-pixel wave
// tiles) and 27 (fj = 2: 32-pixel tiles); returns 64 or -1.  With fused statistics it writes t_pw_rows partial rows
// (set by every launch of it; run_variant resets it to -1 before each launch)
template <typename TO>
int launch_pw(int fj, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, hipStream_t s,
              float* ws, const PhaseTab* ph, const void* x2);
extern thread_local long long t_pw_rows;

// halo-tiled 3x3 / stride-1 weight gradient (conv_wgrad_halo.hip)
struct HaloSeg {
  const void* x;    // input (pixel stride ldx), channels [0, c1) of a virtual concat (all C without one)
  const void* x2;   // a virtual concat's second part (channels >= c1, pixel stride ldx2), else null
  const void* dy;   // output gradient (pixel stride ldy)
  unsigned xbytes, x2bytes, dbytes;
};
struct HaloArgs {
  HaloSeg seg[2];
  int H, W, C, K, ldx, ldx2, ldy, c1;
  int ncb, nkb, nstrips;
  long long steps[2], sps[2];   // row steps per segment, row steps per split
  int splits, s1;               // total splits, splits of segment 0
  float* slab;                  // [splits][K][9 * C] fp32 partials (splits > 1)
  float* dw;                    // splits == 1: dW written directly in `layout` (0 = [K][3][3][C], 1 = OIHW)
  int c_real, k_real, layout, accumulate;
};
struct HaloPlan {
  int ncb, nkb, nstrips, splits, s1;
  long long steps[2], sps[2];
};
bool halo3_eligible(const ConvGeom& g, int dt);
HaloPlan halo3_plan(const ConvGeom& g, long long n1, long long n2);
size_t halo3_ws_bytes(const ConvGeom& g, long long n1, long long n2);
void launch_wgrad_halo3(int dt, const HaloArgs& a, hipStream_t s);

// register-staged kernel launches (conv_reg_*.hip): returns the tile height BM
template <typename T, typename TO>
int dispatch_regstaged(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, float* ws,
                       hipStream_t s);
