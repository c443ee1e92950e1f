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
#include <algorithm>
#include <mutex>
#include <unordered_map>

#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct ConvGeom {
  int N, H, W, C, ldx;
  int OH, OW, K;
  int R, S, sy, sx, dy, dx, py, px;
  int outH, outW, osy, osx, ooy, oox, ldy;
  int ldw;
  long long M;   // N*OH*OW
  int KK;        // R*S*C
};

static bool make_geom(const ssseg_conv_desc* d, ConvGeom& g) {
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
};

template <typename TO> struct Load4;
template <> struct Load4<float> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[4]) {
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
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
template <typename TO, int FM, int FN>
__device__ __forceinline__ void store_tile(const f32x4 (&acc)[FN][FM], long long mb, int nb, int lane,
                                           const ConvGeom& g, TO* __restrict__ y, const Epi<TO>& ep) {
  long long op[FM];   // output pixel of fragment row j (-1: past M)
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const long long m = mb + j * 16 + (lane & 15);
    op[j] = -1;
    if (m < g.M) {
      const int ox = (int)m % g.OW;    // 32-bit decode: geom_ok guarantees M < 2^31
      const int q = (int)m / g.OW;
      const int oy = q % g.OH, img = q / g.OH;
      op[j] = ((long long)img * g.outH + oy * g.osy + g.ooy) * g.outW + ox * g.osx + g.oox;
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
      if (ep.res && op[j] >= 0) {
        const TO* rp = ep.res + op[j] * ep.ldr + n;
        if (full && (ep.ldr & 3) == 0)
          Load4<TO>::ld(rp, r[j]);
        else
          for (int e = 0; e < 4 && n + e < g.K; ++e) r[j][e] = io<TO>::ld(rp, e);
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
          for (int e = 0; e < 4 && n + e < g.K; ++e) io<TO>::st(ep.aux, op[j] * g.ldy + n + e, a4[e]);
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = acc[i][j][e];
        if (ep.scale) a *= sc[e];
        if (ep.shift) a += sh[e];
        a += r[j][e];
        a = act_fwd(a, ep.relu, ep.slope);
        v[e] = a;
      }
      TO* yp = y + op[j] * g.ldy;
      if (full && (g.ldy & 3) == 0) {
        Store4<TO>::st(yp + n, v);
      } else {
        for (int e = 0; e < 4 && n + e < g.K; ++e) io<TO>::st(yp, n + e, v[e]);
      }
    }
  }
}

// LDS-staged epilogue for the LDS-DMA kernel: the raw fp32 accumulators go to LDS (rows padded by 16 B:
// conflict-free float4 writes), then each thread finishes 8 consecutive channels of one pixel with 16-byte
// residual loads and 16-byte (bf16) / 2x16-byte (f32) stores, so a pixel row is written in full lines.
// Same arithmetic as store_tile (fp32 acc*scale + shift + res, then act, then one rounding).
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

template <typename TO, int BM, int BN, int FM, int FN, int NT>
__device__ __forceinline__ void store_tile_lds(const f32x4 (&acc)[FN][FM], char* smem, long long m0, int n0, int wmo,
                                               int wno, int lane, const ConvGeom& g, TO* __restrict__ y,
                                               const Epi<TO>& ep) {
  constexpr int LDR = BN * 4 + 16;   // bytes per staged pixel row
  __syncthreads();                   // every wave is done with the LDS ring
#pragma unroll
  for (int j = 0; j < FM; ++j)
#pragma unroll
    for (int i = 0; i < FN; ++i)
      *(f32x4*)(smem + (wmo + j * 16 + (lane & 15)) * LDR + (wno + i * 16 + (lane >> 4) * 4) * 4) = acc[i][j];
  __syncthreads();
  constexpr int CPR = BN / 8;                 // 8-channel chunks per row
  static_assert(NT % CPR == 0, "epilogue: one fixed channel chunk per thread");
  constexpr int RPP = NT / CPR, NP = (BM + RPP - 1) / RPP;   // rows per pass, passes
  const int ch = threadIdx.x % CPR, r0 = threadIdx.x / CPR;
  const int n = n0 + ch * 8;
  if (n >= g.K) return;
  const bool vec = (g.ldy & 7) == 0 && (!ep.res || (ep.ldr & 7) == 0);
  const bool full = vec && n + 7 < g.K;
  // this thread's 8 channels are the same in every pass: the affine is loaded once, and all residual
  // rows are in flight before the first store
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bool in = n + e < g.K;
    sc[e] = (ep.scale && in) ? ep.scale[n + e] : 1.f;
    sh[e] = (ep.shift && in) ? ep.shift[n + e] : 0.f;
  }
  long long op[NP];
  float r[NP][8];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int row = r0 + p * RPP;
    const long long m = m0 + row;
    op[p] = -1;
    if (row < BM && m < g.M) {
      const int ox = (int)m % g.OW;    // 32-bit decode: geom_ok guarantees M < 2^31
      const int q = (int)m / g.OW;
      const int oy = q % g.OH, img = q / g.OH;
      op[p] = ((long long)img * g.outH + oy * g.osy + g.ooy) * g.outW + ox * g.osx + g.oox;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) r[p][e] = 0.f;
    if (ep.res && op[p] >= 0) {
      if (full)
        Out8<TO>::ld(ep.res + op[p] * ep.ldr + n, r[p]);
      else
        for (int e = 0; e < 8 && n + e < g.K; ++e) r[p][e] = io<TO>::ld(ep.res, op[p] * ep.ldr + n + e);
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if (op[p] < 0) continue;
    const float* a = (const float*)(smem + (r0 + p * RPP) * LDR + ch * 32);
    float v[8];
    const float4 a0 = *(const float4*)a, a1 = *(const float4*)(a + 4);
    const float raw[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = raw[e];
      if (ep.scale) t *= sc[e];
      if (ep.shift) t += sh[e];
      t += r[p][e];
      t = act_fwd(t, ep.relu, ep.slope);
      v[e] = t;
    }
    const long long o = op[p] * g.ldy + n;
    if (full) {
      Out8<TO>::st(y + o, v);
      if (ep.aux) Out8<TO>::st(ep.aux + o, raw);
    } else {
      for (int e = 0; e < 8 && n + e < g.K; ++e) {
        io<TO>::st(y, o + e, v[e]);
        if (ep.aux) io<TO>::st(ep.aux, o + e, raw[e]);
      }
    }
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
int g_knobs[9] = {0, -1, 0, 0, 0, 1, 0, 0, 0};   // runtime variant switches (ssseg_set_knob)
// 0: reg-staged pipeline depth; 1: split-K cap (-1 off); 2: 64x64 small-M tiles (reg-staged path);
// 3: bf16 LDS-DMA path (0 on, -1 off); 4: variant (0 auto, 1..10 / 12..17 LDS-DMA config, 11 register-staged);
// 5: autotune unseen geometries (1 on, 0 = static heuristic); knob 6 = 1 clears the variant cache;
// 7: LDS-staged coalesced epilogue in the LDS-DMA kernel (0 on, -1 off);
// 8: bf16 weight gradient on the LDS-DMA kernel (0 on, -1 = register-staged wgrad_kernel)

template <typename T, typename TO, int BM, int BN, int WM, int WN, bool DEEP>
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
    a_ox[i] = (int)mm % g.OW;
    const int q = (int)mm / g.OW;
    a_oy[i] = q % g.OH;
    a_n[i] = q / g.OH;
  }
  // k-state of this thread's chunk: k = tap*C + kc, tap = r*S + s (advanced by every load, in order)
  const int k_first = kt0 * BK + chunk * VEC;
  int tap = min(k_first / g.C, RS), kc = k_first - tap * g.C, r = tap / max(g.S, 1), s = tap - r * g.S;
  const int nk = max(kt1 - kt0, 0);

  auto load = [&](uint4 (&ra)[A_PER], uint4 (&rb)[B_IT], int kt) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int iy = a_oy[i] * g.sy + r * g.dy + g.py;
      const int ix = a_ox[i] * g.sx + s * g.dx + g.px;
      const bool ok = a_ok[i] && tap < RS && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      ra[i] = ok ? *(const uint4*)(x + ((long long)(a_n[i] * g.H + iy) * g.W + ix) * g.ldx + kc) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < B_IT; ++j) {
      const int id = t + 256 * j;
      rb[j] = make_uint4(0, 0, 0, 0);
      if (id < BN * 4) {
        const int n = n0 + (id >> 2);
        const int k = (kt0 + kt) * BK + (id & 3) * VEC;
        if (n < g.K && k < g.KK) rb[j] = *(const uint4*)(w + (long long)n * g.ldw + k);
      }
    }
    kc += BK;
    while (kc >= g.C && tap < RS) {
      kc -= g.C; ++tap;
      if (++s == g.S) { s = 0; ++r; }
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
  store_tile<TO, FM, FN>(acc, m0 + wm * WTM, n0 + wn * WTN, lane, g, y, ep);
}

// ------------------------------------------------------------------------------------------------
// bf16 gather GEMM, LDS-DMA pipeline (gfx950), for C % 64 == 0.  Same contraction and epilogue as
// igemm_kernel.  k runs tap-major (k = tap*C + c) and a k-tile (BK = 64) never straddles a tap, so the
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

template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr unsigned OOB = 0x80000000u;   // > any num_records we build: the load returns zeros

template <typename TO, int BM, int BN, int WM, int WN, int NW, int NS>
__global__ void __launch_bounds__(NW * 64, 1) igemm_glds_kernel(const bf16_t* __restrict__ x,
                                                                const bf16_t* __restrict__ w, TO* __restrict__ y,
                                                                ConvGeom g, Epi<TO> ep, unsigned xbytes,
                                                                unsigned wbytes, int g_epi_lds) {
  constexpr int ROW = 128;                       // bytes per LDS row = 64 bf16 of k
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

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nnt = (g.K + BN - 1) / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const long long m0 = (long long)(tile / nnt) * BM;
  const int n0 = (tile % nnt) * BN;
  const int RS = g.R * g.S;
  const int cpt = g.C >> 6;                      // k-tiles per tap
  const int nk = RS * cpt;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, (int)wbytes, 0x00020000);

  // lane rows: A row 8*(wave*AI + ii) + (lane>>3), B row 8*(wave*BI + jj) + (lane>>3); the lane loads
  // logical chunk (lane & 7) ^ swz(row) = (lane & 7) ^ (lane >> 4) ^ 4*(instruction parity)
  const int c_even = (lane & 7) ^ (lane >> 4);
  int a_off[AI], a_iy[AI], a_ix[AI];
#pragma unroll
  for (int ii = 0; ii < AI; ++ii) {
    const int inst = wave * AI + ii;
    const int ch = c_even ^ ((inst & 1) * 4);
    const long long m = m0 + 8 * inst + (lane >> 3);
    if (m < g.M) {
      const int ox = (int)m % g.OW;
      const int q = (int)m / g.OW;
      const int oy = q % g.OH, img = q / g.OH;
      a_iy[ii] = oy * g.sy + g.py;
      a_ix[ii] = ox * g.sx + g.px;
      a_off[ii] = ((img * g.H + a_iy[ii]) * g.W + a_ix[ii]) * g.ldx * 2 + ch * 16;
    } else {
      a_iy[ii] = -0x40000000;   // never in bounds
      a_ix[ii] = 0;
      a_off[ii] = 0;
    }
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
  auto set_tap = [&](int tap) {
    const int r = tap / g.S, s_ = tap - (tap / g.S) * g.S;
    const int dyy = r * g.dy, dxx = s_ * g.dx;
    const int toff = (dyy * g.W + dxx) * g.ldx * 2;
#pragma unroll
    for (int ii = 0; ii < AI; ++ii) {
      const int iy = a_iy[ii] + dyy, ix = a_ix[ii] + dxx;
      const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      a_cur[ii] = ok ? (unsigned)(a_off[ii] + toff) : OOB;
    }
  };

  int ld_tap = 0, ld_c = 0, ld_kt = 0;   // k-tile being staged next: tap, channel block, index
  set_tap(0);
  auto issue = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + BM * ROW;
    const unsigned sa = (unsigned)ld_c * 128u, sb = (unsigned)ld_kt * 128u;
#pragma unroll
    for (int ii = 0; ii < AI; ++ii) bldslds16(xr, As + (wave * AI + ii) * 1024, a_cur[ii], sa);
#pragma unroll
    for (int jj = 0; jj < BI; ++jj) bldslds16(wr, Bs + (wave * BI + jj) * 1024, b_off[jj], sb);
    ++ld_kt;
    if (++ld_c == cpt) {
      ld_c = 0;
      if (++ld_tap < RS) set_tap(ld_tap);
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

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
        for (int j = 0; j < FM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
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
  if constexpr (EPI <= SMEM) {
    if (g_epi_lds)
      store_tile_lds<TO, BM, BN, FM, FN, NW * 64>(acc, smem, m0, n0, wm * WTM, wn * WTN, lane, g, y, ep);
    else
      store_tile<TO, FM, FN>(acc, m0 + wm * WTM, n0 + wn * WTN, lane, g, y, ep);
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
    const int ox = (int)m % g.OW;    // 32-bit decode: geom_ok guarantees M < 2^31
    const int q = (int)m / g.OW;
    const int oy = q % g.OH, img = q / g.OH;
    const long long op = ((long long)img * g.outH + oy * g.osy + g.ooy) * g.outW + ox * g.osx + g.oox;
    float v = ws[i];
    if (ep.aux) io<TO>::st(ep.aux, op * g.ldy + n, v);
    if (ep.scale) v *= ep.scale[n];
    if (ep.shift) v += ep.shift[n];
    if (ep.res) v += io<TO>::ld(ep.res, op * ep.ldr + n);
    v = act_fwd(v, ep.relu, ep.slope);
    io<TO>::st(y, op * g.ldy + n, v);
  }
}

// output pixels of a phase whose tap set is empty (e.g. odd rows of a 1x1/s2 dgrad): epilogue of 0
template <typename TO>
__global__ void phase_zero_kernel(TO* y, ConvGeom g, Epi<TO> ep) {
  const long long total = g.M * g.K;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(i % g.K);
    const long long m = i / g.K;
    const int ox = (int)m % g.OW;    // 32-bit decode: geom_ok guarantees M < 2^31
    const int q = (int)m / g.OW;
    const int oy = q % g.OH, img = q / g.OH;
    const long long op = ((long long)img * g.outH + oy * g.osy + g.ooy) * g.outW + ox * g.osx + g.oox;
    float v = ep.shift ? ep.shift[n] : 0.f;
    if (ep.aux) io<TO>::st(ep.aux, op * g.ldy + n, 0.f);
    if (ep.res) v += io<TO>::ld(ep.res, op * ep.ldr + n);
    v = act_fwd(v, ep.relu, ep.slope);
    io<TO>::st(y, op * g.ldy + n, v);
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient: dW[co][kk] = sum_p dY[p][co] * x_col[p][kk], kk = (r, s, c)
// MFMA A = x_col^T (rows kk), B = dY (cols co).  LDS tiles are stored pixel-major as loaded and the
// k-contiguous fragments come from ds_read_b64_tr_b16 (bf16) / strided ds_read_b32 (f32).
// Split-K over pixels; every split writes an fp32 slab tile, a reduce kernel sums the slabs.
// ------------------------------------------------------------------------------------------------
template <typename T> struct WG;
template <> struct WG<bf16_t> {
  static constexpr int BKP = 64;                   // pixels per k-tile (two 32-deep MFMA steps)
  static constexpr int PADB = 32;                  // row pad bytes (row stride == 8 dwords mod 64)
};
template <> struct WG<float> {
  static constexpr int BKP = 16;
  static constexpr int PADB = 64;                  // row stride == 16 dwords mod 32
};

// MFMA k index (8g + j) -> LDS row, conflict-free for the transpose reads
__device__ __forceinline__ int kperm(int g, int j) { return 16 * (g >> 1) + 8 * (j >> 2) + 4 * (g & 1) + (j & 3); }

struct WDirect {   // splits == 1: write dW in its final layout (no slab, no reduce launch)
  float* dw;
  int c_real, k_real, layout, accumulate;
};

template <typename T, int BMW, int BNW>
__global__ void __launch_bounds__(256) wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                    float* __restrict__ slab, ConvGeom g, long long pix_per_split,
                                                    WDirect dd) {
  constexpr int VEC = MF<T>::VEC;
  constexpr int BKP = WG<T>::BKP;
  constexpr int ROWX = BMW * (int)sizeof(T) + WG<T>::PADB;
  constexpr int ROWD = BNW * (int)sizeof(T) + WG<T>::PADB;
  constexpr int XCH = BMW / VEC, DCH = BNW / VEC;          // 16-byte chunks per row
  constexpr int X_IT = BKP * XCH / 256, D_IT = BKP * DCH / 256;
  static_assert(X_IT >= 1 && D_IT >= 1 && (256 % XCH) == 0 && (256 % DCH) == 0, "wgrad tile");
  constexpr int WTM = BMW / 2, WTN = BNW / 2, FM = WTM / 16, FN = WTN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * BKP * (ROWX + ROWD)];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int kk0 = blockIdx.x * BMW, co0 = blockIdx.y * BNW;
  const long long p_begin = (long long)blockIdx.z * pix_per_split;
  const long long p_end = min(p_begin + pix_per_split, g.M);

  // x_col chunk of this thread: fixed (r, s, c)
  const int xc = t % XCH;
  const int kkx = kk0 + xc * VEC;
  const bool kk_ok = kkx < g.KK;
  const int tapx = kk_ok ? kkx / g.C : 0, cx = kk_ok ? kkx % g.C : 0;
  const int rx = tapx / g.S, sx_ = tapx % g.S;
  const int dc = t % DCH;
  const int cod = co0 + dc * VEC;
  const bool co_ok = cod < g.K;

  // pixel state per loaded x row, advanced incrementally (no per-tile division): row pixel
  // p = p_begin + t/XCH + i*(256/XCH) + kt*BKP, decoded once into (img, oy, ox)
  long long xp[X_IT];
  int ximg[X_IT], xoy[X_IT], xox[X_IT];
  long long dp[D_IT];
#pragma unroll
  for (int i = 0; i < X_IT; ++i) {
    xp[i] = p_begin + t / XCH + i * (256 / XCH);
    const long long pp = xp[i] < g.M ? xp[i] : 0;
    xox[i] = (int)(pp % g.OW);
    const long long q = pp / g.OW;
    xoy[i] = (int)(q % g.OH);
    ximg[i] = (int)(q / g.OH);
  }
#pragma unroll
  for (int i = 0; i < D_IT; ++i) dp[i] = p_begin + t / DCH + i * (256 / DCH);

  uint4 rx_[X_IT], rd_[D_IT];
  auto load = [&]() {
#pragma unroll
    for (int i = 0; i < X_IT; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (xp[i] < p_end && kk_ok) {
        const int iy = xoy[i] * g.sy + rx * g.dy + g.py, ix = xox[i] * g.sx + sx_ * g.dx + g.px;
        if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
          v = *(const uint4*)(x + ((long long)(ximg[i] * g.H + iy) * g.W + ix) * g.ldx + cx);
      }
      rx_[i] = v;
      xp[i] += BKP;
      xox[i] += BKP;
      while (xox[i] >= g.OW) {
        xox[i] -= g.OW;
        if (++xoy[i] == g.OH) {
          xoy[i] = 0;
          ++ximg[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < D_IT; ++i) {
      const long long p = dp[i];
      rd_[i] = (p < p_end && co_ok) ? *(const uint4*)(dy + p * g.ldy + cod) : make_uint4(0, 0, 0, 0);
      dp[i] += BKP;
    }
  };
  auto store = [&](int buf) {
    char* Xs = smem + buf * BKP * (ROWX + ROWD);
    char* Ds = Xs + BKP * ROWX;
#pragma unroll
    for (int i = 0; i < X_IT; ++i) *(uint4*)(Xs + (t / XCH + i * (256 / XCH)) * ROWX + xc * 16) = rx_[i];
#pragma unroll
    for (int i = 0; i < D_IT; ++i) *(uint4*)(Ds + (t / DCH + i * (256 / DCH)) * ROWD + dc * 16) = rd_[i];
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const long long npix = p_end > p_begin ? p_end - p_begin : 0;
  const int nk = (int)((npix + BKP - 1) / BKP);
  if (nk > 0) {
    load();
    store(0);
    __syncthreads();
  }
  const int gq = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load();
    const char* Xs = smem + buf * BKP * (ROWX + ROWD);
    const char* Ds = Xs + BKP * ROWX;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int ks = 0; ks < BKP / 32; ++ks) {
      bf16x8 af[FM], bfr[FN];
      const int r0 = ks * 32 + kperm(gq, q4), r1 = ks * 32 + kperm(gq, 4 + q4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int col = wm * WTM + i * 16 + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + r0 * ROWX + col * 2));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + r1 * ROWX + col * 2));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * WTN + j * 16 + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + r0 * ROWD + col * 2));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + r1 * ROWD + col * 2));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BKP / 4; ++ks) {
        const int row = ks * 4 + gq;
        float af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = *(const float*)(Xs + row * ROWX + (wm * WTM + i * 16 + li) * 4);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = *(const float*)(Ds + row * ROWD + (wn * WTN + j * 16 + li) * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  // slab[split][co][kk]: lane holds kk .. kk+3 (rows) of channel co (column)
  if (dd.dw) {   // single split: final layout directly (0 = [K][R][S][C], 1 = [k_real][c_real][R][S]), += if accumulate
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int kkb = kk0 + wm * WTM + i * 16 + 4 * gq;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int co = co0 + wn * WTN + j * 16 + li;
        if (co >= dd.k_real) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kk = kkb + e;
          if (kk >= g.KK) continue;
          const int c = kk % g.C, tap = kk / g.C;
          if (c >= dd.c_real) continue;
          long long o;
          if (dd.layout == 0) o = ((long long)co * g.R * g.S + tap) * g.C + c;
          else o = (((long long)co * dd.c_real + c) * g.R + tap / g.S) * g.S + tap % g.S;
          dd.dw[o] = dd.accumulate ? dd.dw[o] + acc[i][j][e] : acc[i][j][e];
        }
      }
    }
    return;
  }
  float* sl = slab + (long long)blockIdx.z * g.K * g.KK;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int kk = kk0 + wm * WTM + i * 16 + 4 * gq;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int co = co0 + wn * WTN + j * 16 + li;
      if (co >= g.K || kk >= g.KK) continue;
      float* p = sl + (long long)co * g.KK + kk;
      if (kk + 3 < g.KK) {
        *(float4*)p = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      } else {
        for (int e = 0; e < 4 && kk + e < g.KK; ++e) p[e] = acc[i][j][e];
      }
    }
  }
}

// wgrad output of one wave: lane holds dW for kk .. kk+3 (rows) of channel co (column) per fragment.
// Single split (dd.dw set): final layout directly (0 = [K][R][S][C], 1 = [k_real][c_real][R][S]),
// += if accumulate; otherwise the fp32 slab tile slab[split][co][kk] that wgrad_reduce_kernel sums.
template <int FM, int FN>
__device__ __forceinline__ void wgrad_store(const f32x4 (&acc)[FM][FN], int kkb0, int cob0, int lane,
                                            const ConvGeom& g, float* __restrict__ slab, const WDirect& dd,
                                            int split) {
  const int gq = lane >> 4, li = lane & 15;
  if (dd.dw) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int kkb = kkb0 + i * 16 + 4 * gq;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int co = cob0 + j * 16 + li;
        if (co >= dd.k_real) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kk = kkb + e;
          if (kk >= g.KK) continue;
          const int c = kk % g.C, tap = kk / g.C;
          if (c >= dd.c_real) continue;
          long long o;
          if (dd.layout == 0) o = ((long long)co * g.R * g.S + tap) * g.C + c;
          else o = (((long long)co * dd.c_real + c) * g.R + tap / g.S) * g.S + tap % g.S;
          dd.dw[o] = dd.accumulate ? dd.dw[o] + acc[i][j][e] : acc[i][j][e];
        }
      }
    }
    return;
  }
  float* sl = slab + (long long)split * g.K * g.KK;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int kk = kkb0 + i * 16 + 4 * gq;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int co = cob0 + j * 16 + li;
      if (co >= g.K || kk >= g.KK) continue;
      float* p = sl + (long long)co * g.KK + kk;
      if (kk + 3 < g.KK) {
        *(float4*)p = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      } else {
        for (int e = 0; e < 4 && kk + e < g.KK; ++e) p[e] = acc[i][j][e];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient on an LDS-DMA pipeline (bf16, gfx950), for C % BMW == 0: a kk-tile never straddles a
// tap, so the tap (r, s) and the channel block c0 are block-uniform and each x row of a k-tile is one
// run of BMW channels of one pixel.  The 64-pixel k-tiles of x (gathered rows) and dY are staged by
// buffer_load ... lds (16 B per lane; padding pixels and rows past the split get an out-of-range offset
// and read as zeros) into an NS-deep ring, one raw barrier per k-tile with a counted vmcnt, as in
// igemm_glds_kernel.  LDS rows are unpadded (128 / 256 B); 16-byte chunk ch of row r is stored at
// ch ^ wswz(r) — applied on the source offset, since the DMA writes lane-linearly — and the
// ds_read_b64_tr_b16 fragment reads apply the same XOR.  With the k-slot -> pixel-row map wkp (a
// half-wave's two 4-row blocks 8 rows apart) every transposed read is bank-conflict-free.  Same
// contraction, split plan and output path as wgrad_kernel.
// ------------------------------------------------------------------------------------------------
template <int ROWB>
__device__ __forceinline__ int wswz(int r) {
  if constexpr (ROWB == 256) return ((r & 3) << 2) | ((r >> 2) & 3);
  else return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 1);
}
__device__ __forceinline__ int wkp(int g, int j) { return 16 * (g >> 1) + 8 * (g & 1) + 4 * (j >> 2) + (j & 3); }

template <int BMW, int BNW, int NS>
__global__ void __launch_bounds__(256) wgrad_glds_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                         float* __restrict__ slab, ConvGeom g, long long pix_per_split,
                                                         WDirect dd, unsigned xbytes, unsigned dbytes) {
  constexpr int BKP = 64;                                    // pixels per k-tile
  constexpr int ROWX = BMW * 2, ROWD = BNW * 2;              // LDS row bytes
  constexpr int XCPR = ROWX / 16, DCPR = ROWD / 16;          // 16-byte chunks per row
  constexpr int XI = BKP * XCPR / 256, DI = BKP * DCPR / 256;   // wave-instructions per wave per stage
  constexpr int NL = XI + DI;
  constexpr int STAGE = BKP * (ROWX + ROWD);
  constexpr int WTM = BMW / 2, WTN = BNW / 2, FM = WTM / 16, FN = WTN / 16;
  static_assert(XI >= 1 && DI >= 1 && NS >= 2 && NS <= 3, "wgrad glds tile");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // 1-D grid, XCD-aware: consecutive logical ids (the mt x nt tiles of one pixel split, which gather the
  // same x and dY rows) run on one XCD and share its L2
  const int mt = (g.KK + BMW - 1) / BMW, nt = (g.K + BNW - 1) / BNW;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int split = tile / (mt * nt), rem = tile - split * (mt * nt);
  const int kk0 = (rem % mt) * BMW, co0 = (rem / mt) * BNW;
  const long long p_begin = (long long)split * pix_per_split;
  const long long p_end = min(p_begin + pix_per_split, g.M);
  const int tap = kk0 / g.C, c0 = kk0 - tap * g.C;
  const int tr = tap / g.S, ts = tap - tr * g.S;
  const int offy = tr * g.dy + g.py, offx = ts * g.dx + g.px;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, (int)dbytes, 0x00020000);

  // x slot ii of this lane: LDS row (wave*XI + ii)*(64/XCPR) + lane/XCPR, logical chunk (lane%XCPR)^swz;
  // its pixel advances by BKP per k-tile (incremental decode, no per-tile division)
  long long xp[XI];
  int xoy[XI], xox[XI], ximg[XI], xcb[XI];
#pragma unroll
  for (int ii = 0; ii < XI; ++ii) {
    const int row = (wave * XI + ii) * (64 / XCPR) + lane / XCPR;
    xcb[ii] = (c0 + ((lane % XCPR) ^ wswz<ROWX>(row)) * 8) * 2;
    xp[ii] = p_begin + row;
    const long long pp = xp[ii] < g.M ? xp[ii] : 0;
    xox[ii] = (int)(pp % g.OW);
    const long long q = pp / g.OW;
    xoy[ii] = (int)(q % g.OH);
    ximg[ii] = (int)(q / g.OH);
  }
  long long dp[DI];
  int dcb[DI];
#pragma unroll
  for (int jj = 0; jj < DI; ++jj) {
    const int row = (wave * DI + jj) * (64 / DCPR) + lane / DCPR;
    const int co = co0 + ((lane % DCPR) ^ wswz<ROWD>(row)) * 8;
    dcb[jj] = co < g.K ? co * 2 : -1;
    dp[jj] = p_begin + row;
  }
  auto issue = [&](int buf) {
    char* Xs = smem + buf * STAGE;
    char* Ds = Xs + BKP * ROWX;
#pragma unroll
    for (int ii = 0; ii < XI; ++ii) {
      unsigned off = OOB;
      if (xp[ii] < p_end) {
        const int iy = xoy[ii] * g.sy + offy, ix = xox[ii] * g.sx + offx;
        if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
          off = (unsigned)(((ximg[ii] * g.H + iy) * g.W + ix) * g.ldx) * 2u + (unsigned)xcb[ii];
      }
      bldslds16(xr, Xs + (wave * XI + ii) * 1024, off, 0);
      xp[ii] += BKP;
      xox[ii] += BKP;
      while (xox[ii] >= g.OW) {
        xox[ii] -= g.OW;
        if (++xoy[ii] == g.OH) {
          xoy[ii] = 0;
          ++ximg[ii];
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < DI; ++jj) {
      const unsigned off = (dp[jj] < p_end && dcb[jj] >= 0) ? (unsigned)(dp[jj] * g.ldy * 2 + dcb[jj]) : OOB;
      bldslds16(dr, Ds + (wave * DI + jj) * 1024, off, 0);
      dp[jj] += BKP;
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int gq = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  auto compute = [&](int buf) {
    const char* Xs = smem + buf * STAGE;
    const char* Ds = Xs + BKP * ROWX;
#pragma unroll
    for (int ks = 0; ks < BKP / 32; ++ks) {
      const int r0 = ks * 32 + wkp(gq, q4), r1 = ks * 32 + wkp(gq, 4 + q4);
      const int sx0 = 16 * wswz<ROWX>(r0), sx1 = 16 * wswz<ROWX>(r1);
      const int sd0 = 16 * wswz<ROWD>(r0), sd1 = 16 * wswz<ROWD>(r1);
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int col = wm * WTM + i * 16 + 4 * p4;
        const int cb = 16 * (col >> 3), e8 = 2 * (col & 7);
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + r0 * ROWX + (cb ^ sx0) + e8));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + r1 * ROWX + (cb ^ sx1) + e8));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * WTN + j * 16 + 4 * p4;
        const int cb = 16 * (col >> 3), e8 = 2 * (col & 7);
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + r0 * ROWD + (cb ^ sd0) + e8));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + r1 * ROWD + (cb ^ sd1) + e8));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const long long npix = p_end > p_begin ? p_end - p_begin : 0;
  const int nk = (int)((npix + BKP - 1) / BKP);
  constexpr int D = NS - 1;   // k-tiles in flight ahead of the one being multiplied
#pragma unroll
  for (int p = 0; p < D; ++p)
    if (p < nk) issue(p);
  for (int kt = 0; kt < nk; ++kt) {
    if (D >= 2 && kt + 1 < nk) vmcnt_wait<NL>();   // tile kt landed, tile kt+1 may stay in flight
    else vmcnt_wait<0>();
    __builtin_amdgcn_s_barrier();                  // every wave's tile kt landed; slot (kt+D)%NS is free
    if (kt + D < nk) issue((kt + D) % NS);
    compute(kt % NS);
  }
  wgrad_store<FM, FN>(acc, kk0 + wm * WTM, co0 + wn * WTN, lane, g, slab, dd, split);
}

// sum the split slabs and write dW in the requested layout: 0 = [K][R][S][C] (packed, C = physical),
// 1 = [K][C_real][R][S] (PyTorch OIHW).  accumulate: dst += sum.
// A block owns 64 consecutive outputs (256-byte slab rows, coalesced) and spreads the splits over its 16
// waves: wave w sums splits w, w+16, ... in two chains (16 loads in flight per lane with the unroll), then
// the 16 partials are added in wave order through LDS — a fixed order, so the result is deterministic.
__global__ void __launch_bounds__(1024) wgrad_reduce_wide_kernel(const float* __restrict__ slab, int splits, int K, int R,
                                                            int S, int C, int c_real, int k_real,
                                                            float* __restrict__ dst, int layout, int accumulate) {
  __shared__ float red[16][64];
  const long long KK = (long long)R * S * C;
  const long long total = (long long)K * KK;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long i = (long long)blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f;
  if (i < total) {
    int z = w;
#pragma unroll 8
    for (; z + 16 < splits; z += 32) {
      a0 += slab[(long long)z * total + i];
      a1 += slab[(long long)(z + 16) * total + i];
    }
    if (z < splits) a0 += slab[(long long)z * total + i];
  }
  red[w][lane] = a0 + a1;
  __syncthreads();
  if (w != 0 || i >= total) return;
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) sum += red[k][lane];
  const int kk = (int)(i % KK), k = (int)(i / KK);
  const int c = kk % C, tap = kk / C, r = tap / S, s = tap % S;
  if (c >= c_real || k >= k_real) return;
  long long o;
  if (layout == 0) o = ((long long)k * R * S + tap) * C + c;
  else o = (((long long)k * c_real + c) * R + r) * S + s;
  dst[o] = accumulate ? dst[o] + sum : sum;
}

// few splits: one thread per output, 4 independent chains
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int K, int R, int S, int C, int c_real,
                                    int k_real, float* __restrict__ dst, int layout, int accumulate) {
  const long long KK = (long long)R * S * C;
  const long long total = (long long)K * KK;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int kk = (int)(i % KK), k = (int)(i / KK);
    const int c = kk % C, tap = kk / C, r = tap / S, s = tap % S;
    if (c >= c_real || k >= k_real) continue;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int z = 0;
    for (; z + 4 <= splits; z += 4) {
      s0 += slab[(long long)z * total + i];
      s1 += slab[(long long)(z + 1) * total + i];
      s2 += slab[(long long)(z + 2) * total + i];
      s3 += slab[(long long)(z + 3) * total + i];
    }
    for (; z < splits; ++z) s0 += slab[(long long)z * total + i];
    const float sum = (s0 + s1) + (s2 + s3);
    long long o;
    if (layout == 0) o = ((long long)k * R * S + tap) * C + c;
    else o = (((long long)k * c_real + c) * R + r) * S + s;
    dst[o] = accumulate ? dst[o] + sum : sum;
  }
}

// ------------------------------------------------------------------------------------------------
// weight packing: dst[k][rr][ss][c] (c < Cp; zero for c >= Cd) from an fp32 source
//   layout 0: src[k][c][r][s]  (Conv2d OIHW; ConvTranspose2d used as a conv over its output grad)
//   layout 1: src[c][k][r][s]  (transposed roles: conv dgrad, ConvTranspose2d forward)
//   r = r0 + rr*rstep, s = s0 + ss*sstep
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void weight_pack_kernel(const float* __restrict__ src, T* __restrict__ dst, int Kd, int Kr, int Cd, int Rs,
                                   int Ss, int Cp, int layout, int r0, int rstep, int Rn, int s0, int sstep, int Sn) {
  const long long total = (long long)Kd * Rn * Sn * Cp;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    long long q = i / Cp;
    const int ss = (int)(q % Sn);
    q /= Sn;
    const int rr = (int)(q % Rn);
    const int k = (int)(q / Rn);
    float v = 0.f;
    if (c < Cd && k < Kr) {
      const int r = r0 + rr * rstep, s = s0 + ss * sstep;
      const long long idx = layout == 0 ? (((long long)k * Cd + c) * Rs + r) * Ss + s
                                        : (((long long)c * Kr + k) * Rs + r) * Ss + s;
      v = src[idx];
    }
    io<T>::st(dst, i, v);
  }
}

// one launch repacks many convs: blockIdx.y = descriptor, blocks along x grid-stride over its elements
template <typename T>
__global__ void __launch_bounds__(256) weight_pack_batch_kernel(const ssseg_pack_desc* __restrict__ descs) {
  // 32-bit index math (the host checks every pack < 2^31 elements)
  const ssseg_pack_desc& d = descs[blockIdx.y];
  const int Cp = (int)d.Cp, Sn = (int)d.Sn, Rn = (int)d.Rn, Cd = (int)d.Cd, Kr = (int)d.Kr, Rs = (int)d.Rs,
            Ss = (int)d.Ss, r0 = (int)d.r0, rstep = (int)d.rstep, s0 = (int)d.s0, sstep = (int)d.sstep;
  const int total = (int)d.Kd * Rn * Sn * Cp;
  const bool l0 = d.layout == 0;
  const float* src = d.src;
  T* dst = (T*)d.dst;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % Cp;
    int q = i / Cp;
    const int ss = q % Sn;
    q /= Sn;
    const int rr = q % Rn, k = q / Rn;
    float v = 0.f;
    if (c < Cd && k < Kr) {
      const int r = r0 + rr * rstep, s = s0 + ss * sstep;
      v = src[l0 ? ((k * Cd + c) * Rs + r) * Ss + s : ((c * Kr + k) * Rs + r) * Ss + s];
    }
    io<T>::st(dst, i, v);
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
namespace {

template <typename T, int BM, int BN>
int plan_splits(const ConvGeom& g) {
  const long long tiles = ((g.M + BM - 1) / BM) * ((g.K + BN - 1) / BN);
  const int nk = (g.KK + 64 / (int)sizeof(T) - 1) / (64 / (int)sizeof(T));
  if (g_knobs[1] < 0 || tiles >= 512 || nk < 32) return 1;
  long long sp = (1024 + tiles - 1) / tiles;
  sp = std::min<long long>(sp, nk / 16);
  if (g_knobs[1] > 0) sp = std::min<long long>(sp, g_knobs[1]);
  return (int)std::max<long long>(1, std::min<long long>(sp, 64));
}

template <typename T, typename TO, int BM, int BN, int WM, int WN>
void launch_igemm(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, float* ws, int splits,
                  hipStream_t s) {
  const long long tiles = ((g.M + BM - 1) / BM) * ((g.K + BN - 1) / BN);
  const dim3 grid((unsigned)tiles, (unsigned)splits);
  if (splits > 1) (void)hipMemsetAsync(ws, 0, sizeof(float) * g.M * g.K, s);
  if (g_knobs[0] == 0)
    hipLaunchKernelGGL((igemm_kernel<T, TO, BM, BN, WM, WN, false>), grid, dim3(256), 0, s, (const T*)x, (const T*)w,
                       (TO*)y, g, ep, splits, ws);
  else
    hipLaunchKernelGGL((igemm_kernel<T, TO, BM, BN, WM, WN, true>), grid, dim3(256), 0, s, (const T*)x, (const T*)w,
                       (TO*)y, g, ep, splits, ws);
  if (splits > 1)
    hipLaunchKernelGGL(splitk_finalize_kernel<TO>, dim3(ssseg_grid(g.M * g.K, 256)), dim3(256), 0, s, ws, (TO*)y, g,
                       ep);
}

template <typename TO, int BM, int BN, int WM, int WN, int NW, int NS>
void launch_glds(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb, unsigned wb,
                 hipStream_t s) {
  const long long tiles = ((g.M + BM - 1) / BM) * ((g.K + BN - 1) / BN);
  hipLaunchKernelGGL((igemm_glds_kernel<TO, BM, BN, WM, WN, NW, NS>), dim3((unsigned)tiles), dim3(NW * 64), 0, s,
                     (const bf16_t*)x, (const bf16_t*)w, (TO*)y, g, ep, xb, wb, (int)(g_knobs[7] == 0));
}

template <typename TO>
void launch_glds_cfg(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep,
                     unsigned xb, unsigned wb, hipStream_t s) {
  switch (cfg) {
    case 1: launch_glds<TO, 256, 128, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s); break;
    case 2: launch_glds<TO, 256, 64, 4, 1, 4, 3>(x, w, y, g, ep, xb, wb, s); break;
    case 3: launch_glds<TO, 128, 128, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s); break;
    case 4: launch_glds<TO, 128, 64, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s); break;
    case 5: launch_glds<TO, 64, 64, 2, 2, 4, 3>(x, w, y, g, ep, xb, wb, s); break;
    case 6: launch_glds<TO, 256, 128, 4, 2, 8, 3>(x, w, y, g, ep, xb, wb, s); break;
    case 7: launch_glds<TO, 256, 64, 4, 2, 8, 3>(x, w, y, g, ep, xb, wb, s); break;
    case 8: launch_glds<TO, 128, 128, 2, 2, 4, 4>(x, w, y, g, ep, xb, wb, s); break;
    case 9: launch_glds<TO, 128, 64, 2, 2, 4, 4>(x, w, y, g, ep, xb, wb, s); break;
    // two-slot rings: 64 / 80 / 48 KB of LDS, so 2-3 workgroups share a CU and hide each other's
    // pipeline fill and epilogue (the short-k layers: 3x3 over 64-128 channels, nk = 9..18)
    case 12: launch_glds<TO, 128, 128, 2, 2, 4, 2>(x, w, y, g, ep, xb, wb, s); break;
    case 13: launch_glds<TO, 256, 64, 4, 1, 4, 2>(x, w, y, g, ep, xb, wb, s); break;
    case 14: launch_glds<TO, 128, 64, 2, 2, 4, 2>(x, w, y, g, ep, xb, wb, s); break;
    // one-slot / small two-slot rings for nk = 1..2 (1x1 expansions 64->256, 128->512): 35 / 17 / 32 KB
    // of LDS, 4-9 workgroups per CU; output-write bound, so occupancy is what hides the HBM latency
    case 15: launch_glds<TO, 128, 64, 2, 2, 4, 1>(x, w, y, g, ep, xb, wb, s); break;
    case 16: launch_glds<TO, 64, 64, 2, 2, 4, 1>(x, w, y, g, ep, xb, wb, s); break;
    case 17: launch_glds<TO, 64, 64, 2, 2, 4, 2>(x, w, y, g, ep, xb, wb, s); break;
    default: launch_glds<TO, 64, 64, 2, 2, 4, 4>(x, w, y, g, ep, xb, wb, s); break;
  }
}

template <typename T, typename TO>
void dispatch_regstaged(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, float* ws,
                        hipStream_t s) {
  const long long t128 = ((g.M + 127) / 128) * ((g.K + 127) / 128);
  const bool small = g_knobs[2] == 0 ? (t128 < 512) : (g_knobs[2] > 0);
  if (g.K <= 16)
    launch_igemm<T, TO, 256, 16, 4, 1>(x, w, y, g, ep, ws, ws ? plan_splits<T, 256, 16>(g) : 1, s);
  else if (g.K <= 64 && !small)
    launch_igemm<T, TO, 256, 64, 4, 1>(x, w, y, g, ep, ws, ws ? plan_splits<T, 256, 64>(g) : 1, s);
  else if (small)
    launch_igemm<T, TO, 64, 64, 2, 2>(x, w, y, g, ep, ws, ws ? plan_splits<T, 64, 64>(g) : 1, s);
  else
    launch_igemm<T, TO, 128, 128, 2, 2>(x, w, y, g, ep, ws, ws ? plan_splits<T, 128, 128>(g) : 1, s);
}

// ---- bf16 variant choice: per-geometry autotune cache ----------------------------------------
// Every variant accumulates the same 32-deep MFMA k-sequence in the same order, so the choice changes
// speed, never results (tests/test_hip_layers.py::test_conv_variants_bitwise).  Variant 0 is the
// register-staged kernel, 1..10 and 12..17 the LDS-DMA configs.  With knob 5 on (default) an unseen geometry is
// timed once over the candidates on the caller's stream (HIP events) and the fastest is cached.
constexpr int kCandidates[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 13, 14, 15, 16, 17};
std::unordered_map<unsigned long long, int> g_variant;
std::mutex g_variant_mu;

static unsigned long long geom_key(const ConvGeom& g, int tag) {
  const long long v[] = {g.N, g.H, g.W, g.C, g.ldx, g.OH, g.OW, g.K, g.R, g.S, g.sy, g.sx, g.dy, g.dx, g.py, g.px,
                         g.outH, g.outW, g.osy, g.osx, g.ldy, g.ldw, tag};
  unsigned long long h = 1469598103934665603ull;
  for (long long e : v) h = (h ^ (unsigned long long)e) * 1099511628211ull;
  return h;
}

static int heuristic_variant(const ConvGeom& g) {
  auto tiles = [&](int bm, int bn) { return ((g.M + bm - 1) / bm) * ((g.K + bn - 1) / bn); };
  if (g.KK <= 128) return 0;
  if (g.K > 64) return tiles(256, 128) >= 128 ? 6 : (tiles(128, 128) >= 256 ? 8 : 5);
  return tiles(64, 64) < 512 ? 10 : 0;
}

template <typename T, typename TO>
void run_variant(int v, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                 unsigned wb, hipStream_t s) {
  if (v == 0)
    dispatch_regstaged<T, TO>(x, w, y, g, ep, nullptr, s);
  else
    launch_glds_cfg<TO>(v, x, w, y, g, ep, xb, wb, s);
}

template <typename T, typename TO>
int tune_variant(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                 unsigned wb, hipStream_t s) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return heuristic_variant(g);
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return heuristic_variant(g);
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return heuristic_variant(g);
  }
  int best = heuristic_variant(g);
  float best_ms = 1e30f;
  static const bool log = getenv("SSSEG_TUNE_LOG") != nullptr;   // one line per tuned geometry (stderr)
  char line[512];
  int len = log ? snprintf(line, sizeof line, "tune N%d %dx%d C%d -> %dx%d K%d %dx%d s%d d%d out%dx%d/%d ep%d%d:",
                           g.N, g.H, g.W, g.C, g.OH, g.OW, g.K, g.R, g.S, g.sy, g.dy, g.outH, g.outW, g.osy,
                           ep.scale ? 1 : 0, ep.aux ? 1 : 0) : 0;
  for (int v : kCandidates) {
    run_variant<T, TO>(v, x, w, y, g, ep, xb, wb, s);   // warm (code load, caches)
    float ms = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0, s);
      run_variant<T, TO>(v, x, w, y, g, ep, xb, wb, s);
      (void)hipEventRecord(e1, s);
      float t = 1e30f;
      if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&t, e0, e1) == hipSuccess) ms = std::min(ms, t);
    }
    if (log && len > 0 && len < (int)sizeof line - 16) len += snprintf(line + len, sizeof line - len, " %d:%.0f", v, ms * 1e3f);
    if (ms < best_ms) {
      best_ms = ms;
      best = v;
    }
  }
  if (log) fprintf(stderr, "%s -> %d\n", line, best);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

template <typename T, typename TO>
void dispatch_igemm(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, float* ws,
                    hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    const long long xb = (long long)g.N * g.H * g.W * g.ldx * 2, wb = (long long)g.K * g.ldw * 2;
    if (g_knobs[3] == 0 && !ws && g.C % 64 == 0 && g.ldx % 8 == 0 && g.ldw % 8 == 0 && g.ldw == g.KK &&
        g.K > 16 && xb < 0x7fffffffLL && wb < 0x7fffffffLL) {
      int v = g_knobs[4];
      if (v < 0) v = 0;
      if (v == 0) {
        const unsigned long long key = geom_key(g, (int)sizeof(TO) * 4 + (ep.res ? 2 : 0) + (ep.scale ? 1 : 0));
        std::lock_guard<std::mutex> lk(g_variant_mu);
        auto it = g_variant.find(key);
        if (it != g_variant.end()) {
          v = it->second;
        } else {
          v = g_knobs[5] ? tune_variant<T, TO>(x, w, y, g, ep, (unsigned)xb, (unsigned)wb, s) : heuristic_variant(g);
          g_variant[key] = v;
        }
      } else if (g_knobs[4] == 11) {
        v = 0;   // forced register-staged
      }
      run_variant<T, TO>(v, x, w, y, g, ep, (unsigned)xb, (unsigned)wb, s);
      return;
    }
  }
  dispatch_regstaged<T, TO>(x, w, y, g, ep, ws, s);
}

struct WgradPlan {
  int bmw, bnw, mt, nt, splits;
  long long pps;
  bool glds;
};

template <typename T>
WgradPlan plan_wgrad(const ConvGeom& g, int bmw = 0) {
  WgradPlan p;
  p.glds = false;
  p.bnw = g.K <= 64 ? 64 : 128;
  p.bmw = bmw ? bmw : (g.KK <= 64 ? 64 : 128);   // (a 256x64 tile for Cout <= 64 measured slower: 263 -> 208 TF)
  p.mt = (g.KK + p.bmw - 1) / p.bmw;
  p.nt = (g.K + p.bnw - 1) / p.bnw;
  const long long tiles = (long long)p.mt * p.nt;
  const int bkp = WG<T>::BKP;
  const long long max_splits_by_work = std::max<long long>(1, g.M / (bkp * 8));   // >= 8 k-tiles per split
  long long want = std::max<long long>(1, (1024 + tiles - 1) / tiles);
  const long long slab_cap = std::max<long long>(1, (64ll << 20) / (4ll * g.K * g.KK + 1));  // <= 64 MiB of slabs
  // (capping splits by slab traffic measured slower: layer3/4 wgrads need the parallelism, 58 -> 150 us)
  long long sp = std::min(std::min(want, max_splits_by_work), slab_cap);
  sp = std::max<long long>(1, std::min<long long>(sp, 65535));
  p.pps = (g.M + sp - 1) / sp;
  p.pps = (p.pps + bkp - 1) / bkp * bkp;
  p.splits = (int)((g.M + p.pps - 1) / p.pps);
  if (p.splits < 1) p.splits = 1;
  return p;
}

template <typename T>
void launch_wgrad(const void* x, const void* dy, float* slab, const ConvGeom& g, const WgradPlan& p, WDirect dd,
                  hipStream_t s) {
  const dim3 grid(p.mt, p.nt, p.splits);
  if (p.bmw == 64 && p.bnw == 64)
    hipLaunchKernelGGL((wgrad_kernel<T, 64, 64>), grid, dim3(256), 0, s, (const T*)x, (const T*)dy, slab, g, p.pps, dd);
  else if (p.bmw == 64)
    hipLaunchKernelGGL((wgrad_kernel<T, 64, 128>), grid, dim3(256), 0, s, (const T*)x, (const T*)dy, slab, g, p.pps, dd);
  else if (p.bnw == 64)
    hipLaunchKernelGGL((wgrad_kernel<T, 128, 64>), grid, dim3(256), 0, s, (const T*)x, (const T*)dy, slab, g, p.pps, dd);
  else
    hipLaunchKernelGGL((wgrad_kernel<T, 128, 128>), grid, dim3(256), 0, s, (const T*)x, (const T*)dy, slab, g, p.pps, dd);
}

// LDS-DMA weight gradient: bf16, C % 64 == 0 (a 64- or 128-channel kk-tile inside one tap), operands < 2 GB
static bool wgrad_glds_ok(const ConvGeom& g, int dt) {
  if (dt != SSSEG_BF16 || g_knobs[8] != 0) return false;
  if (g.C % 64 || g.ldx % 8 || g.ldy % 8 || g.K % 8) return false;
  const long long xb = (long long)g.N * g.H * g.W * g.ldx * 2, db = g.M * g.ldy * 2;
  return xb < 0x7fffffffLL && db < 0x7fffffffLL;
}

static WgradPlan choose_wgrad(const ConvGeom& g, int dt) {
  WgradPlan p;
  if (wgrad_glds_ok(g, dt)) {
    p = plan_wgrad<bf16_t>(g, (g.C % 128 == 0 && g.KK > 64) ? 128 : 64);
    p.glds = true;
  } else {
    p = dt == SSSEG_BF16 ? plan_wgrad<bf16_t>(g) : plan_wgrad<float>(g);
  }
  return p;
}

template <int BMW, int BNW>
void launch_wgrad_glds_t(const void* x, const void* dy, float* slab, const ConvGeom& g, const WgradPlan& p, WDirect dd,
                         hipStream_t s) {
  constexpr int NS = 64 * (BMW + BNW) * 2 <= 24576 ? 3 : 2;   // 48 / 72 / 64 KB of LDS: 2-3 blocks per CU
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.ldx * 2), db = (unsigned)(g.M * g.ldy * 2);
  hipLaunchKernelGGL((wgrad_glds_kernel<BMW, BNW, NS>), dim3(p.mt * p.nt * p.splits), dim3(256), 0, s, (const bf16_t*)x,
                     (const bf16_t*)dy, slab, g, p.pps, dd, xb, db);
}

void launch_wgrad_glds(const void* x, const void* dy, float* slab, const ConvGeom& g, const WgradPlan& p, WDirect dd,
                       hipStream_t s) {
  if (p.bmw == 128 && p.bnw == 128) launch_wgrad_glds_t<128, 128>(x, dy, slab, g, p, dd, s);
  else if (p.bmw == 128) launch_wgrad_glds_t<128, 64>(x, dy, slab, g, p, dd, s);
  else if (p.bnw == 128) launch_wgrad_glds_t<64, 128>(x, dy, slab, g, p, dd, s);
  else launch_wgrad_glds_t<64, 64>(x, dy, slab, g, p, dd, s);
}

bool geom_ok(const ConvGeom& g, int dt) {
  const int vec = dt == SSSEG_BF16 ? 8 : 4;
  if (g.C % vec || g.ldx % vec || g.ldw % vec) return false;
  if (g.N < 1 || g.OH < 1 || g.OW < 1 || g.K < 1 || g.C < 1) return false;
  if (g.M >= 0x7fffffffLL) return false;   // kernels decode output positions with 32-bit math
  if (g.R < 0 || g.S < 0) return false;
  return true;
}

}  // namespace

extern "C" int ssseg_set_knob(int id, int value) {
  if (id < 0 || id >= 9) return SSSEG_EINVAL;
  if (id == 6 && value) {
    std::lock_guard<std::mutex> lk(g_variant_mu);
    g_variant.clear();
    return 0;
  }
  g_knobs[id] = value;
  return 0;
}

extern "C" size_t ssseg_conv_igemm_workspace_bytes(const ssseg_conv_desc* d, int dt) {
  ConvGeom g;
  if (!make_geom(d, g)) return 0;
  int sp;
  const long long t128 = ((g.M + 127) / 128) * ((g.K + 127) / 128);
  const bool small = g_knobs[2] == 0 ? (t128 < 512) : (g_knobs[2] > 0);
  if (g.K <= 16) sp = dt == SSSEG_BF16 ? plan_splits<bf16_t, 256, 16>(g) : plan_splits<float, 256, 16>(g);
  else if (g.K <= 64 && !small) sp = dt == SSSEG_BF16 ? plan_splits<bf16_t, 256, 64>(g) : plan_splits<float, 256, 64>(g);
  else if (small) sp = dt == SSSEG_BF16 ? plan_splits<bf16_t, 64, 64>(g) : plan_splits<float, 64, 64>(g);
  else sp = dt == SSSEG_BF16 ? plan_splits<bf16_t, 128, 128>(g) : plan_splits<float, 128, 128>(g);
  return sp > 1 ? (size_t)g.M * g.K * sizeof(float) : 0;
}

extern "C" int ssseg_conv_igemm_epi(const void* x, const void* w, void* y, const ssseg_conv_desc* d, int dt, int dt_out,
                                    const ssseg_conv_epilogue* epi, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  ConvGeom g;
  if (!make_geom(d, g) || !y) return SSSEG_EINVAL;
  if (!geom_ok(g, dt)) return SSSEG_EINVAL;
  const ssseg_conv_epilogue none = {nullptr, nullptr, nullptr, 0, nullptr, 0, 0.f};
  const ssseg_conv_epilogue& e = epi ? *epi : none;
  if (e.residual && (e.ldr < g.K || e.ldr > 0x7fffffff)) return SSSEG_EINVAL;
  if (g.M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (e.relu < 0 || e.relu > SSSEG_ACT_LEAKY) return SSSEG_EINVAL;
  const Epi<float> ef{e.scale, e.shift, (const float*)e.residual, (int)e.ldr, e.relu, (float*)e.aux, e.slope};
  const Epi<bf16_t> eb{e.scale, e.shift, (const bf16_t*)e.residual, (int)e.ldr, e.relu, (bf16_t*)e.aux, e.slope};
  if (g.KK == 0) {   // no taps reach this output phase: the contraction is zero
    if (dt_out == SSSEG_F32)
      hipLaunchKernelGGL(phase_zero_kernel<float>, dim3(ssseg_grid(g.M * g.K, 256)), dim3(256), 0, s, (float*)y, g, ef);
    else
      hipLaunchKernelGGL(phase_zero_kernel<bf16_t>, dim3(ssseg_grid(g.M * g.K, 256)), dim3(256), 0, s, (bf16_t*)y, g,
                         eb);
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  if (!x || !w) return SSSEG_EINVAL;
  const size_t need = ssseg_conv_igemm_workspace_bytes(d, dt);
  float* wsf = (need > 0 && ws && ws_bytes >= need) ? (float*)ws : nullptr;   // no workspace: no split-K
  if (dt == SSSEG_BF16 && dt_out == SSSEG_BF16)
    dispatch_igemm<bf16_t, bf16_t>(x, w, y, g, eb, wsf, s);
  else if (dt == SSSEG_BF16 && dt_out == SSSEG_F32)
    dispatch_igemm<bf16_t, float>(x, w, y, g, ef, wsf, s);
  else if (dt == SSSEG_F32 && dt_out == SSSEG_F32)
    dispatch_igemm<float, float>(x, w, y, g, ef, wsf, s);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_conv_igemm(const void* x, const void* w, void* y, const ssseg_conv_desc* d, int dt, int dt_out,
                                const float* bias, int relu, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  const ssseg_conv_epilogue e = {nullptr, bias, nullptr, 0, nullptr, relu ? SSSEG_ACT_RELU : 0, 0.f};
  return ssseg_conv_igemm_epi(x, w, y, d, dt, dt_out, &e, ws, ws_bytes, stream);
}

extern "C" size_t ssseg_conv_wgrad_workspace_bytes(const ssseg_conv_desc* d, int dt) {
  ConvGeom g;
  if (!make_geom(d, g)) return 0;
  const WgradPlan p = choose_wgrad(g, dt);
  return (size_t)p.splits * g.K * g.KK * sizeof(float) + 256;
}

extern "C" int ssseg_conv_wgrad(const void* x, const void* dy, float* dw, const ssseg_conv_desc* d, int dt,
                                int64_t c_real, int64_t k_real, int layout, int accumulate, void* ws, size_t ws_bytes,
                                ssseg_stream_t stream) {
  ConvGeom g;
  if (!make_geom(d, g) || !x || !dy || !dw) return SSSEG_EINVAL;
  if (!geom_ok(g, dt) || g.ldy % (dt == SSSEG_BF16 ? 8 : 4) || g.K % (dt == SSSEG_BF16 ? 8 : 4)) return SSSEG_EINVAL;
  if (c_real < 1 || c_real > g.C || k_real < 1 || k_real > g.K || (layout != 0 && layout != 1)) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_conv_wgrad_workspace_bytes(d, dt)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* slab = (float*)ws;
  WgradPlan p;
  if (dt != SSSEG_BF16 && dt != SSSEG_F32) return SSSEG_EUNSUPPORTED;
  p = choose_wgrad(g, dt);
  const WDirect dd{p.splits == 1 ? dw : nullptr, (int)c_real, (int)k_real, layout, accumulate};
  if (p.glds)
    launch_wgrad_glds(x, dy, slab, g, p, dd, s);
  else if (dt == SSSEG_BF16)
    launch_wgrad<bf16_t>(x, dy, slab, g, p, dd, s);
  else
    launch_wgrad<float>(x, dy, slab, g, p, dd, s);
  if (p.splits == 1) {
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  const long long total = (long long)g.K * g.KK;
  if (p.splits >= 64)   // many splits: spread them over the 16 waves of a block
    hipLaunchKernelGGL(wgrad_reduce_wide_kernel, dim3((unsigned)((total + 63) / 64)), dim3(1024), 0, s, slab, p.splits,
                       g.K, g.R, g.S, g.C, (int)c_real, (int)k_real, dw, layout, accumulate);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, slab, p.splits, g.K, g.R, g.S,
                       g.C, (int)c_real, (int)k_real, dw, layout, accumulate);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_weight_pack_batch(const ssseg_pack_desc* descs, int64_t n, int dt, ssseg_stream_t stream) {
  if (n < 0 || n > 65535 || (n > 0 && !descs)) return SSSEG_EINVAL;
  if (n == 0) return 0;
  const dim3 grid(256, (unsigned)n);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(weight_pack_batch_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, descs);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(weight_pack_batch_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, descs);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_weight_pack(const float* src, void* dst, int64_t Kd, int64_t Kr, int64_t Cd, int64_t Rs, int64_t Ss,
                                 int64_t Cp, int layout, int64_t r0, int64_t rstep, int64_t Rn, int64_t s0, int64_t sstep,
                                 int64_t Sn, int dt, ssseg_stream_t stream) {
  if (!src || !dst || Cp < Cd || Kd < 1 || Kr < 1 || Kr > Kd || Rn < 0 || Sn < 0 || (layout != 0 && layout != 1))
    return SSSEG_EINVAL;
  if (Rn > 0 && (r0 < 0 || r0 >= Rs || r0 + (Rn - 1) * rstep < 0 || r0 + (Rn - 1) * rstep >= Rs)) return SSSEG_EINVAL;
  if (Sn > 0 && (s0 < 0 || s0 >= Ss || s0 + (Sn - 1) * sstep < 0 || s0 + (Sn - 1) * sstep >= Ss)) return SSSEG_EINVAL;
  const long long total = Kd * Rn * Sn * Cp;
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(weight_pack_kernel<bf16_t>, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, src, (bf16_t*)dst,
                       (int)Kd, (int)Kr, (int)Cd, (int)Rs, (int)Ss, (int)Cp, layout, (int)r0, (int)rstep, (int)Rn,
                       (int)s0, (int)sstep, (int)Sn);
  else if (dt == SSSEG_F32)
    hipLaunchKernelGGL(weight_pack_kernel<float>, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, src, (float*)dst,
                       (int)Kd, (int)Kr, (int)Cd, (int)Rs, (int)Ss, (int)Cp, layout, (int)r0, (int)rstep, (int)Rn,
                       (int)s0, (int)sstep, (int)Sn);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}
