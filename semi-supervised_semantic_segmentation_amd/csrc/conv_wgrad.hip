// Weight gradients of the implicit-GEMM conv engine (split-K over pixels into fp32 slabs + deterministic
// reduce, or direct when one split suffices).  Split from conv.hip for parallel compilation.
#include <algorithm>
#include <vector>

#include "conv_kernels.h"

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
template <> struct WG<f16_t> : WG<bf16_t> {};
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
    decode_m(g, (int)pp, ximg[i], xoy[i], xox[i]);   // M < 2^31 (wg_geom_ok)
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
        for (int j = 0; j < FN; ++j) acc[i][j] = M16<T>::mma(af[i], bfr[j], acc[i][j]);
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

// Second pixel segment of a merged launch (ssseg_conv_wgrad2): the supervised and the consistency backward of
// one conv have the same geometry and differ only in their pixel sets, so their weight gradients are ONE
// contraction over the union of the pixels.  Splits [0, s1) read (x, dy, g.M), splits [s1, s1 + s2) read
// (x, dy, M) of this segment; every split writes its own slab and the reduce sums all of them in order.
struct WSeg2 {
  const void* x;
  const void* dy;
  long long M;
  unsigned xbytes, dbytes;
  int s1;   // first split of this segment (0: no second segment)
  // virtual concat input (ssseg_vcat): channels >= c1 of segment 1 / 2 come from xa / xb (pixel stride ldx2);
  // c1 = 0: none.  A kk-tile never straddles c1 (c1 % BMW == 0), so the source is a block-uniform choice.
  int c1, ldx2;
  const void* xa;
  const void* xb;
  unsigned xabytes, xbbytes;
};

// ST (straddle): the kk-tile may cross the seam of a virtual concat input (sg.c1 % BMW != 0, e.g. the UNet's
// 256^2 conv3_0 over [up 64 | skip 64] with a 128-wide kk-tile): every x piece is issued twice, by the lanes whose
// chunk lies before the seam from the first part and by the others from the second (EXEC-masked LDS-DMA: each
// lane lands its 16 bytes in the same slot as in the unsplit issue), so the tile and its MFMA sequence are those of
// the materialised concat.
// GK (general k, C % 64 != 0: HRNet-W32's 32-channel branches, HarDNet's growth layers): a kk-tile holds several
// taps, so every lane finds its own chunk's (tap, channel) once at the start (the kk-tile is fixed per block) and
// gathers from that tap's offset; kk >= KK (the last tile's tail) loads zeros
template <typename T16, int BMW, int BNW, int NS, int WM = 2, int WN = 2, int BKP = 64, bool ST = false, bool GK = false>
__global__ void __launch_bounds__(WM * WN * 64) wgrad_glds_kernel(const T16* __restrict__ x, const T16* __restrict__ dy,
                                                                   float* __restrict__ slab, ConvGeom g,
                                                                   long long pix_per_split, WDirect dd, unsigned xbytes,
                                                                   unsigned dbytes, WSeg2 sg) {
  // BKP pixels per k-tile; WM x WN waves, each owning a (BMW / WM) x (BNW / WN) block of dW
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int ROWX = BMW * 2, ROWD = BNW * 2;              // LDS row bytes
  constexpr int XCPR = ROWX / 16, DCPR = ROWD / 16;          // 16-byte chunks per row
  constexpr int XI = BKP * XCPR / NT, DI = BKP * DCPR / NT;  // wave-instructions per wave per stage
  constexpr int NL = (ST ? 2 : 1) * XI + DI;                 // vmcnt units per stage
  constexpr int STAGE = BKP * (ROWX + ROWD);
  constexpr int WTM = BMW / WM, WTN = BNW / WN, FM = WTM / 16, FN = WTN / 16;
  static_assert(XI >= 1 && DI >= 1 && NS >= 2 && NS <= 4 && FM >= 1 && FN >= 1 && BKP % 32 == 0, "wgrad glds tile");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  // wave index as a scalar: the LDS-DMA destinations (per-wave LDS bases) then need no readfirstlane per load
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // 1-D grid, XCD-aware: consecutive logical ids (the mt x nt tiles of one pixel split, which gather the
  // same x and dY rows) run on one XCD and share its L2
  const int mt = (g.KK + BMW - 1) / BMW, nt = (g.K + BNW - 1) / BNW;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int split = tile / (mt * nt), rem = tile - split * (mt * nt);
  const int kk0 = (rem % mt) * BMW, co0 = (rem / mt) * BNW;
  const bool seg2 = sg.s1 > 0 && split >= sg.s1;   // block-uniform
  const long long p_begin = (long long)(seg2 ? split - sg.s1 : split) * pix_per_split;
  const long long p_end = min(p_begin + pix_per_split, seg2 ? sg.M : g.M);
  const int tap = kk0 / g.C, c0 = kk0 - tap * g.C;
  const int tr = tap / g.S, ts = tap - tr * g.S;
  const int offy = tr * g.dy + g.py, offx = ts * g.dx + g.px;
  const bool src2 = sg.c1 > 0 && c0 >= sg.c1;      // block-uniform: this kk-tile reads the concat's second part
  const void* xbase = src2 ? (seg2 ? sg.xb : sg.xa) : (seg2 ? sg.x : (const void*)x);
  const unsigned xbyt = src2 ? (seg2 ? sg.xbbytes : sg.xabytes) : (seg2 ? sg.xbytes : xbytes);
  const int ldx = src2 ? sg.ldx2 : g.ldx, cb0 = src2 ? c0 - sg.c1 : c0;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)xbase, (short)0, (int)xbyt, 0x00020000);
  // ST: this tile straddles the seam (block-uniform); the second part's resource
  const bool strad = ST && sg.c1 > c0 && sg.c1 < c0 + BMW;
  __amdgpu_buffer_rsrc_t xr2 = xr;
  if constexpr (ST)
    xr2 = __builtin_amdgcn_make_buffer_rsrc(seg2 ? (void*)sg.xb : (void*)sg.xa, (short)0,
                                            (int)(seg2 ? sg.xbbytes : sg.xabytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(seg2 ? (void*)sg.dy : (void*)dy, (short)0,
                                                                      (int)(seg2 ? sg.dbytes : dbytes), 0x00020000);

  // x slot ii of this lane: LDS row (wave*XI + ii)*(64/XCPR) + lane/XCPR, logical chunk (lane%XCPR)^swz;
  // its pixel advances by BKP per k-tile (incremental decode, no per-tile division)
  long long xp[XI];
  int xoy[XI], xox[XI], ximg[XI], xcb[XI];
  int gofy[GK ? XI : 1], gofx[GK ? XI : 1];   // GK: this lane's tap offsets per piece
  bool xin2[ST ? XI : 1];   // ST: this lane's chunk of piece ii lies past the seam (second part)
#pragma unroll
  for (int ii = 0; ii < XI; ++ii) {
    const int row = (wave * XI + ii) * (64 / XCPR) + lane / XCPR;
    xcb[ii] = (cb0 + ((lane % XCPR) ^ wswz<ROWX>(row)) * 8) * 2;
    if constexpr (GK) {
      const int kk = kk0 + ((lane % XCPR) ^ wswz<ROWX>(row)) * 8;
      const int tp = fdiv(kk, g.mC, g.sC), c = kk - tp * g.C;
      const int r = fdiv(tp, g.mS, g.sS), s_ = tp - r * g.S;
      xcb[ii] = c * 2;
      gofy[ii] = tp < g.R * g.S ? r * g.dy + g.py : -0x40000000;   // padding tap: never in bounds
      gofx[ii] = s_ * g.dx + g.px;
    }
    if constexpr (ST) {
      xin2[ii] = strad && c0 + ((lane % XCPR) ^ wswz<ROWX>(row)) * 8 >= sg.c1;
      if (xin2[ii]) xcb[ii] -= sg.c1 * 2;   // channel offset inside the second part
    }
    xp[ii] = p_begin + row;
    const long long pp = xp[ii] < p_end ? xp[ii] : 0;
    decode_m(g, (int)pp, ximg[ii], xoy[ii], xox[ii]);   // M < 2^31 (wg_geom_ok)
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
      if constexpr (ST) {
        if (strad) {   // two EXEC-masked issues of the same piece (one vmcnt unit each, taken by every lane)
          unsigned o1 = OOB, o2 = OOB;
          if (xp[ii] < p_end) {
            const int iy = xoy[ii] * g.sy + offy, ix = xox[ii] * g.sx + offx;
            if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W) {
              const unsigned pix = (unsigned)((ximg[ii] * g.H + iy) * g.W + ix);
              o1 = pix * (unsigned)g.ldx * 2u + (unsigned)xcb[ii];
              o2 = pix * (unsigned)sg.ldx2 * 2u + (unsigned)xcb[ii];
            }
          }
          if (!xin2[ii]) bldslds16_nt(xr, Xs + (wave * XI + ii) * 1024, o1, 0);
          if (xin2[ii]) bldslds16_nt(xr2, Xs + (wave * XI + ii) * 1024, o2, 0);
        }
      }
      if (xp[ii] < p_end) {
        const int iy = xoy[ii] * g.sy + (GK ? gofy[ii] : offy), ix = xox[ii] * g.sx + (GK ? gofx[ii] : offx);
        if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
          off = (unsigned)(((ximg[ii] * g.H + iy) * g.W + ix) * ldx) * 2u + (unsigned)xcb[ii];
      }
      if (!strad) bldslds16_nt(xr, Xs + (wave * XI + ii) * 1024, off, 0);
      xp[ii] += BKP;
      if (BKP < g.OW) {   // at most one row wrap (wave-uniform test)
        xox[ii] += BKP;
        if (xox[ii] >= g.OW) {
          xox[ii] -= g.OW;
          if (++xoy[ii] == g.OH) {
            xoy[ii] = 0;
            ++ximg[ii];
          }
        }
      } else if (xp[ii] < p_end) {   // small maps: several rows per k-tile -- decode again (magic divisors)
        decode_m(g, (int)xp[ii], ximg[ii], xoy[ii], xox[ii]);
      }
    }
#pragma unroll
    for (int jj = 0; jj < DI; ++jj) {
      const unsigned off = (dp[jj] < p_end && dcb[jj] >= 0) ? (unsigned)(dp[jj] * g.ldy * 2 + dcb[jj]) : OOB;
      bldslds16_nt(dr, Ds + (wave * DI + jj) * 1024, off, 0);
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
        for (int j = 0; j < FN; ++j) acc[i][j] = M16<T16>::mma(af[i], bfr[j], acc[i][j]);
    }
  };

  const long long npix = p_end > p_begin ? p_end - p_begin : 0;
  const int nk = (int)((npix + BKP - 1) / BKP);
  constexpr int D = NS - 1;   // k-tiles in flight ahead of the one being multiplied
#pragma unroll
  for (int p = 0; p < D; ++p)
    if (p < nk) issue(p);
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed; the tiles issued after it (at most D - 1) may stay in flight.  An ST block whose kk-tile lies
    // wholly in one part of the concat (C > 128, e.g. [64 | 192]) issues each x piece once: XI + DI units per stage
    const int ahead = min(nk - 1, kt + D - 1) - kt;
    if (ST && !strad) ring_wait<XI + DI, D>(ahead);
    else ring_wait<NL, D>(ahead);
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

namespace {

struct WgradPlan {
  int bmw, bnw, mt, nt, splits;
  long long pps;
  bool glds;
  int cfg;          // LDS-DMA config (WGRAD_CFGS index), 0 = register-staged
  bool st = false;  // kk-tiles may straddle a virtual concat's seam (the ST kernel variant)
};

// LDS-DMA weight-gradient configs: tile (kk x co), ring depth, waves (WM x WN), pixels per k-tile.
// The static plan uses 1-4 (bmw by C % 128, bnw by K); 5.. are A/B candidates (knob 9).
struct WgradCfg {
  int bmw, bnw, ns, wm, wn, bkp;
  int pct = 100;   // split count in percent of plan_wgrad's (fewer, longer splits: less slab traffic)
};
constexpr WgradCfg WGRAD_CFGS[] = {
    {0, 0, 0, 0, 0, 0},
    {64, 64, 3, 2, 2, 64},     // 1: 48 KB LDS
    {128, 64, 3, 2, 2, 64},    // 2: 72 KB
    {64, 128, 3, 2, 2, 64},    // 3: 72 KB
    {128, 128, 2, 2, 2, 64},   // 4: 64 KB
    {128, 64, 3, 4, 2, 64},    // 5: 8 waves, 32x32 per wave
    {128, 128, 2, 2, 4, 64},   // 6: 8 waves, 64x32 per wave
    {128, 64, 2, 2, 2, 128},   // 7: 128-pixel k-tiles, 96 KB
    {64, 64, 3, 2, 2, 128},    // 8: 128-pixel k-tiles, 96 KB
    {256, 64, 2, 4, 2, 64},    // 9: 8 waves, 80 KB
    {128, 128, 3, 2, 4, 64},   // 10: 8 waves, 96 KB
    {64, 64, 4, 2, 2, 64},     // 11: 4-deep ring, 64 KB
    {128, 64, 4, 2, 2, 64},    // 12: 4-deep ring, 96 KB
    {64, 128, 4, 2, 2, 64},    // 13: 4-deep ring, 96 KB
    {64, 64, 3, 2, 4, 64},     // 14: 8 waves, 32x16 per wave
    {64, 128, 3, 2, 4, 64},    // 15: 8 waves, 32x32 per wave
    {64, 128, 3, 4, 2, 64},    // 16: 8 waves, 16x64 per wave
    {128, 128, 2, 4, 2, 64},   // 17: 8 waves, 32x64 per wave
    {128, 64, 2, 4, 2, 64},    // 18: 8 waves, 2-deep ring, 48 KB
    // the static plan's picks (tools/wgrad_variants.py on the C2 geometries, profiles/r3_wgrad_variants.txt): the
    // 8-wave tiles at half the splits beat the round-2 4-wave plan by 15-35 % on every layer with C % 128 == 0
    {128, 128, 2, 2, 4, 64, 50},   // 19: cfg 6 at 50 % of the splits
    {64, 128, 3, 4, 2, 64, 50},    // 20: cfg 16 at 50 % of the splits
};
constexpr int N_WGRAD_CFGS = (int)(sizeof(WGRAD_CFGS) / sizeof(WGRAD_CFGS[0]));

template <typename T>
WgradPlan plan_wgrad(const ConvGeom& g, int bmw = 0, long long slots = 0, int bnw = 0, int bkp_ = 0, int pct = 100) {
  WgradPlan p;
  p.glds = false;
  p.cfg = 0;
  p.bnw = bnw ? bnw : (g.K <= 64 ? 64 : 128);
  p.bmw = bmw ? bmw : (g.KK <= 64 ? 64 : 128);   // (a 256x64 tile for Cout <= 64 measured slower: 263 -> 208 TF)
  p.mt = (g.KK + p.bmw - 1) / p.bmw;
  p.nt = (g.K + p.bnw - 1) / p.bnw;
  const long long tiles = (long long)p.mt * p.nt;
  const int bkp = bkp_ ? bkp_ : WG<T>::BKP;
  const long long max_splits_by_work = std::max<long long>(1, g.M / (bkp * 8));   // >= 8 k-tiles per split
  long long want = std::max<long long>(1, (1024 + tiles - 1) / tiles);
  if (slots > 0 && tiles < 1024) {
    // every split does the same work, so blocks run in whole rounds of `slots` (resident blocks on the chip):
    // round the block count DOWN to R full rounds (R ~ 1024 / slots) -- 1026 blocks over 512 slots ran a
    // third, 2 %-full round (measured 0.70 of the rounds busy on the 128->64 3x3 @256^2 weight gradient)
    const long long rounds = std::max<long long>(1, (1024 + slots / 2) / slots);
    want = std::max<long long>(1, rounds * slots / tiles);
  }
  if (pct != 100) want = std::max<long long>(1, want * pct / 100);
  if (g_knobs[10] != 100 && g_knobs[10] > 0) want = std::max<long long>(1, want * g_knobs[10] / 100);
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

// LDS-DMA weight gradient: bf16, C % 64 == 0 (a 64- or 128-channel kk-tile inside one tap) or any C % 8 == 0 (the
// general-k tiles, 64 wide), operands < 2 GB
static bool wgrad_glds_ok(const ConvGeom& g, int dt) {
  if ((dt != SSSEG_BF16 && dt != SSSEG_F16) || g_knobs[8] != 0) return false;
  if (g.C % 8 || g.ldx % 8 || g.ldy % 8 || g.K % 8) return false;
  const long long xb = (long long)g.N * g.H * g.W * g.ldx * 2, db = g.M * g.ldy * 2;
  return xb < 0x7fffffffLL && db < 0x7fffffffLL;
}

long long wgrad_slots(int cfg);

// the static LDS-DMA config choice: kk-tile 128 where a tap holds whole 128-channel blocks, co-tile by K; 8-wave
// tiles (measured: profiles/r3_wgrad_variants.txt)
static int static_wgrad_cfg(const ConvGeom& g) {
  const int bmw = (g.C % 128 == 0 && g.KK > 64) ? 128 : 64;
  const int bnw = g.K <= 64 ? 64 : 128;
  return bmw == 64 ? (bnw == 64 ? 1 : 20) : (bnw == 64 ? 18 : 19);
}

// c1 > 0 (virtual concat input) with c1 % bmw != 0: a 128-wide kk-tile straddles the seam and runs the ST variant
// (st = true); other widths fall back to a 64-wide tile
static int wgrad_cfg_for(const ConvGeom& g, int c1 = 0, bool* st = nullptr) {
  int c = g_knobs[9];
  if (!(c > 0 && c < N_WGRAD_CFGS && (g.C % 64 ? WGRAD_CFGS[c].bmw == 64 : g.C % WGRAD_CFGS[c].bmw == 0)))
    c = static_wgrad_cfg(g);
  if (st) *st = false;
  if (c1 > 0 && c1 % WGRAD_CFGS[c].bmw) {
    if (WGRAD_CFGS[c].bmw == 128 && c1 % 64 == 0 && st) *st = true;
    else c = WGRAD_CFGS[c].bnw == 64 ? 1 : 20;
  }
  return c;
}

static WgradPlan plan_for_cfg(const ConvGeom& g, int c) {
  const WgradCfg& wc = WGRAD_CFGS[c];
  WgradPlan p = plan_wgrad<bf16_t>(g, wc.bmw, wgrad_slots(c), wc.bnw, wc.bkp, wc.pct);
  p.glds = true;
  p.cfg = c;
  return p;
}

static WgradPlan choose_wgrad(const ConvGeom& g, int dt) {
  if (wgrad_glds_ok(g, dt)) return plan_for_cfg(g, wgrad_cfg_for(g));
  return dt != SSSEG_F32 ? plan_wgrad<bf16_t>(g) : plan_wgrad<float>(g);
}

template <typename T16, int C, bool ST = false, bool GK = false>
constexpr auto wgrad_kernel_of() {
  return &wgrad_glds_kernel<T16, WGRAD_CFGS[C].bmw, WGRAD_CFGS[C].bnw, WGRAD_CFGS[C].ns, WGRAD_CFGS[C].wm,
                            WGRAD_CFGS[C].wn, WGRAD_CFGS[C].bkp, ST, GK>;
}

// resident blocks of an LDS-DMA wgrad config on the whole device (cached per config)
template <int C>
long long wgrad_slots_t() {
  static long long slots = -1;
  if (slots < 0) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wgrad_kernel_of<bf16_t, C>(),
                                                     WGRAD_CFGS[C].wm * WGRAD_CFGS[C].wn * 64, 0) != hipSuccess)
      return 0;   // unknown: the unquantized plan
    slots = (long long)per_cu * cus;
  }
  return slots;
}

template <int C = 1>
long long wgrad_slots_dispatch(int c) {
  if constexpr (C < N_WGRAD_CFGS) {
    if (c == C) return wgrad_slots_t<C>();
    return wgrad_slots_dispatch<C + 1>(c);
  } else {
    return 0;
  }
}

long long wgrad_slots(int cfg) { return wgrad_slots_dispatch<1>(cfg); }

template <typename T16, int C>
void launch_wgrad_glds_t(const void* x, const void* dy, float* slab, const ConvGeom& g, const WgradPlan& p, WDirect dd,
                         hipStream_t s, const WSeg2& sg) {
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.ldx * 2), db = (unsigned)(g.M * g.ldy * 2);
  if constexpr (WGRAD_CFGS[C].bmw == 64) {
    if (g.C % 64) {   // general k (wgrad_cfg_for picks 64-wide kk-tiles for these)
      hipLaunchKernelGGL((wgrad_kernel_of<T16, C, false, true>()), dim3(p.mt * p.nt * p.splits),
                         dim3(WGRAD_CFGS[C].wm * WGRAD_CFGS[C].wn * 64), 0, s, (const T16*)x, (const T16*)dy, slab, g,
                         p.pps, dd, xb, db, sg);
      return;
    }
  }
  if constexpr (WGRAD_CFGS[C].bmw == 128) {
    if (p.st) {   // kk-tiles straddling a virtual concat's seam
      hipLaunchKernelGGL((wgrad_kernel_of<T16, C, true>()), dim3(p.mt * p.nt * p.splits),
                         dim3(WGRAD_CFGS[C].wm * WGRAD_CFGS[C].wn * 64), 0, s, (const T16*)x, (const T16*)dy, slab, g,
                         p.pps, dd, xb, db, sg);
      return;
    }
  }
  hipLaunchKernelGGL((wgrad_kernel_of<T16, C>()), dim3(p.mt * p.nt * p.splits),
                     dim3(WGRAD_CFGS[C].wm * WGRAD_CFGS[C].wn * 64), 0, s, (const T16*)x, (const T16*)dy, slab, g,
                     p.pps, dd, xb, db, sg);
}

template <typename T16, int C = 1>
void launch_wgrad_glds_dispatch(const void* x, const void* dy, float* slab, const ConvGeom& g, const WgradPlan& p,
                                WDirect dd, hipStream_t s, const WSeg2& sg) {
  if constexpr (C < N_WGRAD_CFGS) {
    if (p.cfg == C) return launch_wgrad_glds_t<T16, C>(x, dy, slab, g, p, dd, s, sg);
    return launch_wgrad_glds_dispatch<T16, C + 1>(x, dy, slab, g, p, dd, s, sg);
  }
}

template <typename T16>
void launch_wgrad_glds(const void* x, const void* dy, float* slab, const ConvGeom& g, const WgradPlan& p, WDirect dd,
                       hipStream_t s, const WSeg2& sg = WSeg2{nullptr, nullptr, 0, 0, 0, 0, 0, 0, nullptr, nullptr, 0,
                                                               0}) {
  launch_wgrad_glds_dispatch<T16, 1>(x, dy, slab, g, p, dd, s, sg);
}


bool wg_geom_ok(const ConvGeom& g, int dt) {
  const int vec = dt == SSSEG_F32 ? 4 : 8;
  if (g.C % vec || g.ldx % vec || g.ldw % vec) return false;
  if (g.N < 1 || g.OH < 1 || g.OW < 1 || g.K < 1 || g.C < 1) return false;
  if (g.M >= 0x7fffffffLL) return false;
  if (g.R < 0 || g.S < 0) return false;
  return true;
}

}  // namespace

// largest slab workspace over the configs a launch of this geometry may use (the 64-wide kk-tile one is taken for a
// virtual concat input whose seam is not 128-aligned)
static size_t wgrad_ws_bytes(const ConvGeom& g, int dt) {
  const WgradPlan p = choose_wgrad(g, dt);
  size_t b = (size_t)p.splits * g.K * g.KK * sizeof(float);
  if (halo3_eligible(g, dt)) b = std::max(b, halo3_ws_bytes(g, g.N, 0));
  if (p.glds) {
    const WgradPlan q = plan_for_cfg(g, wgrad_cfg_for(g, 64));
    b = std::max(b, (size_t)q.splits * g.K * g.KK * sizeof(float));
  }
  return b + 256;
}

extern "C" size_t ssseg_conv_wgrad_workspace_bytes(const ssseg_conv_desc* d, int dt) {
  ConvGeom g;
  if (!make_geom(d, g)) return 0;
  return wgrad_ws_bytes(g, dt);
}

// ---- deferred split reductions (ssseg_wgrad_defer_reduce / ssseg_wgrad_reduce_flush) --------------------------------
// The weight gradients of a training step run back to back after the backward passes join (train.train_step's held
// calls); each one's split slabs were reduced by a launch of its own (66 per C2 step, 12-15 us each).  With deferral
// on, the reductions are recorded instead and one flush launches them together, up to RB_MAX per launch, the
// descriptors passed by value in the kernel arguments (no table upload: capturable).  Per output element the sum is
// the one wgrad_reduce_kernel / wgrad_reduce_wide_kernel computes (same chains, same order): bitwise the same dW.
struct ReduceDesc {
  const float* slab;
  float* dst;
  int splits, K, R, S, C, c_real, k_real;
  short layout, accumulate;
};
constexpr int RB_MAX = 40;
struct ReduceBatch {
  ReduceDesc d[RB_MAX];
  int n;
};
thread_local bool t_defer_reduce = false;
thread_local std::vector<ReduceDesc> t_pending_reduce;

__device__ __forceinline__ void reduce_store(const ReduceDesc& d, long long i, long long KK, float sum) {
  const int kk = (int)(i % KK), k = (int)(i / KK);
  const int c = kk % d.C, tap = kk / d.C, r = tap / d.S, s = tap % d.S;
  if (c >= d.c_real || k >= d.k_real) return;
  long long o;
  if (d.layout == 0) o = ((long long)k * d.R * d.S + tap) * d.C + c;
  else o = (((long long)k * d.c_real + c) * d.R + r) * d.S + s;
  d.dst[o] = d.accumulate ? d.dst[o] + sum : sum;
}

// blockIdx.y = descriptor; 1024 threads.  splits >= 64: the wide kernel's form (64 outputs per block, wave w sums
// splits w, w + 16, ... in two chains, then the 16 wave partials in order); else the plain kernel's (one output per
// thread, four chains over the splits), grid-stride over the descriptor's outputs
__global__ void __launch_bounds__(1024) wgrad_reduce_batch_kernel(ReduceBatch b) {
  const ReduceDesc& d = b.d[blockIdx.y];
  const long long KK = (long long)d.R * d.S * d.C, total = (long long)d.K * KK;
  if (d.splits >= 64) {
    __shared__ float red[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long i = (long long)blockIdx.x * 64 + lane;
    if ((long long)blockIdx.x * 64 >= total) return;   // (uniform)
    float a0 = 0.f, a1 = 0.f;
    if (i < total) {
      int z = w;
#pragma unroll 8
      for (; z + 16 < d.splits; z += 32) {
        a0 += d.slab[(long long)z * total + i];
        a1 += d.slab[(long long)(z + 16) * total + i];
      }
      if (z < d.splits) a0 += d.slab[(long long)z * total + i];
    }
    red[w][lane] = a0 + a1;
    __syncthreads();
    if (w != 0 || i >= total) return;
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) sum += red[k][lane];
    reduce_store(d, i, KK, sum);
    return;
  }
  for (long long i = (long long)blockIdx.x * 1024 + threadIdx.x; i < total; i += (long long)gridDim.x * 1024) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int z = 0;
    for (; z + 4 <= d.splits; z += 4) {
      s0 += d.slab[(long long)z * total + i];
      s1 += d.slab[(long long)(z + 1) * total + i];
      s2 += d.slab[(long long)(z + 2) * total + i];
      s3 += d.slab[(long long)(z + 3) * total + i];
    }
    for (; z < d.splits; ++z) s0 += d.slab[(long long)z * total + i];
    reduce_store(d, i, KK, (s0 + s1) + (s2 + s3));
  }
}

namespace {

void launch_reduce(const float* slab, const ConvGeom& g, int splits, int64_t c_real, int64_t k_real, float* dw,
                   int layout, int accumulate, hipStream_t s) {
  if (t_defer_reduce) {
    t_pending_reduce.push_back(ReduceDesc{slab, dw, splits, g.K, g.R, g.S, g.C, (int)c_real, (int)k_real,
                                          (short)layout, (short)accumulate});
    return;
  }
  const long long total = (long long)g.K * g.KK;
  if (splits >= 64)   // many splits: spread them over the 16 waves of a block
    hipLaunchKernelGGL(wgrad_reduce_wide_kernel, dim3((unsigned)((total + 63) / 64)), dim3(1024), 0, s, slab, splits,
                       g.K, g.R, g.S, g.C, (int)c_real, (int)k_real, dw, layout, accumulate);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, slab, splits, g.K, g.R, g.S,
                       g.C, (int)c_real, (int)k_real, dw, layout, accumulate);
}

// validates a virtual concat descriptor against the geometry and fills the WSeg2 second-source fields of one segment
bool vcat_ok(const ssseg_vcat* vc, const ConvGeom& g, int dt) {
  if (!vc) return true;
  return vc->x2 && vc->c1 > 0 && vc->c1 < g.C && vc->c1 % 64 == 0 && (g.C - vc->c1) % 64 == 0 && g.ldx >= vc->c1 &&
         vc->ldx2 >= g.C - vc->c1 && vc->ldx2 % 8 == 0 && vc->ldx2 <= 0x7fffffff && (dt == SSSEG_BF16 || dt == SSSEG_F16) &&
         (long long)g.N * g.H * g.W * vc->ldx2 * 2 < 0x7fffffffLL;
}

// the halo-tiled 3x3 weight gradient over one or two pixel segments (x2 / dy2 / n2: the merged launch's second)
void run_halo3(const ConvGeom& g, int dt, const void* x, const ssseg_vcat* vc, const void* dy, const void* x2,
               const ssseg_vcat* vc2, const void* dy2, long long n2, float* dw, int64_t c_real, int64_t k_real,
               int layout, int accumulate, float* slab, hipStream_t s) {
  const HaloPlan p = halo3_plan(g, g.N, n2);
  HaloArgs a{};
  const long long pix1 = (long long)g.N * g.H * g.W, pix2 = n2 * g.H * g.W;
  a.seg[0] = HaloSeg{x, vc ? vc->x2 : nullptr, dy, (unsigned)(pix1 * g.ldx * 2),
                     vc ? (unsigned)(pix1 * vc->ldx2 * 2) : 0u, (unsigned)(pix1 * g.ldy * 2)};
  if (n2 > 0)
    a.seg[1] = HaloSeg{x2, vc2 ? vc2->x2 : nullptr, dy2, (unsigned)(pix2 * g.ldx * 2),
                       vc2 ? (unsigned)(pix2 * vc2->ldx2 * 2) : 0u, (unsigned)(pix2 * g.ldy * 2)};
  a.H = g.H;
  a.W = g.W;
  a.C = g.C;
  a.K = g.K;
  a.ldx = g.ldx;
  a.ldx2 = vc ? (int)vc->ldx2 : 0;
  a.ldy = g.ldy;
  a.c1 = vc ? (int)vc->c1 : 0;
  a.ncb = p.ncb;
  a.nkb = p.nkb;
  a.nstrips = p.nstrips;
  a.steps[0] = p.steps[0];
  a.steps[1] = p.steps[1];
  a.sps[0] = p.sps[0];
  a.sps[1] = p.sps[1];
  a.splits = p.splits;
  a.s1 = p.s1;
  a.slab = slab;
  a.dw = p.splits == 1 ? dw : nullptr;
  a.c_real = (int)c_real;
  a.k_real = (int)k_real;
  a.layout = layout;
  a.accumulate = accumulate;
  launch_wgrad_halo3(dt, a, s);
  if (p.splits > 1) launch_reduce(slab, g, p.splits, c_real, k_real, dw, layout, accumulate, s);
}

// operands addressable with 32-bit byte offsets (the LDS-DMA buffer resources)
bool halo3_fits(const ConvGeom& g, long long n, const ssseg_vcat* vc) {
  if (!vc && g.ldx < g.C) return false;
  const long long pix = n * g.H * g.W;
  return pix * g.ldx * 2 < 0x7fffffffLL && pix * g.ldy * 2 < 0x7fffffffLL && (!vc || pix * vc->ldx2 * 2 < 0x7fffffffLL);
}

int wgrad_one(const void* x, const ssseg_vcat* vc, const void* dy, float* dw, const ssseg_conv_desc* d, int dt,
              int64_t c_real, int64_t k_real, int layout, int accumulate, void* ws, size_t ws_bytes,
              ssseg_stream_t stream) {
  ConvGeom g;
  if (!make_geom(d, g) || !x || !dy || !dw) return SSSEG_EINVAL;
  const int vec = dt == SSSEG_F32 ? 4 : 8;
  if (!wg_geom_ok(g, dt) || g.ldy % vec || g.K % vec) return SSSEG_EINVAL;
  if (c_real < 1 || c_real > g.C || k_real < 1 || k_real > g.K || (layout != 0 && layout != 1)) return SSSEG_EINVAL;
  if (!vcat_ok(vc, g, dt)) return SSSEG_EINVAL;
  if (!ws || ws_bytes < wgrad_ws_bytes(g, dt)) return SSSEG_EWORKSPACE;
  if (dt != SSSEG_BF16 && dt != SSSEG_F16 && dt != SSSEG_F32) return SSSEG_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  float* slab = (float*)ws;
  if (halo3_eligible(g, dt) && halo3_fits(g, g.N, vc)) {
    run_halo3(g, dt, x, vc, dy, nullptr, nullptr, nullptr, 0, dw, c_real, k_real, layout, accumulate, slab, s);
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  WgradPlan p = choose_wgrad(g, dt);
  // the register-staged kernel has no second source, and its plain loads cannot read a virtually padded
  // contraction (C > ldx: the host's vpad; the LDS-DMA reads are bounded by the buffer size)
  if (!p.glds && g.C > g.ldx) return SSSEG_EUNSUPPORTED;
  if (vc) {
    if (!p.glds) return SSSEG_EUNSUPPORTED;
    bool st = false;
    p = plan_for_cfg(g, wgrad_cfg_for(g, (int)vc->c1, &st));
    p.st = st;
  }
  const WDirect dd{p.splits == 1 ? dw : nullptr, (int)c_real, (int)k_real, layout, accumulate};
  WSeg2 sg{nullptr, nullptr, 0, 0, 0, 0, 0, 0, nullptr, nullptr, 0, 0};
  if (vc) {
    sg.c1 = (int)vc->c1;
    sg.ldx2 = (int)vc->ldx2;
    sg.xa = vc->x2;
    sg.xabytes = (unsigned)((long long)g.N * g.H * g.W * vc->ldx2 * 2);
  }
  if (p.glds && dt == SSSEG_F16)
    launch_wgrad_glds<f16_t>(x, dy, slab, g, p, dd, s, sg);
  else if (p.glds)
    launch_wgrad_glds<bf16_t>(x, dy, slab, g, p, dd, s, sg);
  else if (dt == SSSEG_BF16)
    launch_wgrad<bf16_t>(x, dy, slab, g, p, dd, s);
  else if (dt == SSSEG_F16)
    launch_wgrad<f16_t>(x, dy, slab, g, p, dd, s);
  else
    launch_wgrad<float>(x, dy, slab, g, p, dd, s);
  if (p.splits > 1) launch_reduce(slab, g, p.splits, c_real, k_real, dw, layout, accumulate, s);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

// merged launch plan of ssseg_conv_wgrad2: one split plan over the union of both pixel sets (as if the batch were
// n1 + n2), each segment cut into whole splits of that size.  False when either segment is not LDS-DMA eligible.
bool merged_plan(const ConvGeom& g1, int64_t n2, int dt, WgradPlan& p, int& s1, ConvGeom& g2, int c1 = 0,
                 bool allow_st = true) {
  if (n2 < 1 || n2 > 0x7fffffff || !wgrad_glds_ok(g1, dt)) return false;
  g2 = g1;
  g2.N = (int)n2;
  g2.M = n2 * (long long)g1.OH * g1.OW;
  if (g2.M >= 0x7fffffffLL || !wgrad_glds_ok(g2, dt)) return false;
  ConvGeom gm = g1;
  gm.M = g1.M + g2.M;
  bool st = false;
  p = plan_for_cfg(gm, wgrad_cfg_for(g1, c1, allow_st ? &st : nullptr));
  p.st = st;
  const int bkp = WGRAD_CFGS[p.cfg].bkp;
  // the plan's split count shared out in proportion to the segments' pixels, never more splits in total
  // (a split past the plan's rounds would start a nearly empty extra round)
  const long long sp = std::max(2, p.splits);
  long long a = std::min(sp - 1, std::max(1LL, (long long)((double)sp * g1.M / gm.M + 0.5)));
  long long pps = std::max((g1.M + a - 1) / a, (g2.M + (sp - a) - 1) / (sp - a));
  pps = (pps + bkp - 1) / bkp * bkp;
  p.pps = pps;
  s1 = (int)((g1.M + pps - 1) / pps);
  p.splits = s1 + (int)((g2.M + pps - 1) / pps);
  return true;
}

size_t wgrad2_ws_bytes(const ConvGeom& g, int64_t n2, int dt) {
  ConvGeom g2;
  WgradPlan p;
  int s1;
  size_t b = 0;
  for (int c1 : {0, 64})   // the static config and the 64-wide one a virtual concat may need
    if (merged_plan(g, n2, dt, p, s1, g2, c1)) b = std::max(b, (size_t)p.splits * g.K * g.KK * sizeof(float) + 256);
  if (halo3_eligible(g, dt)) b = std::max(b, halo3_ws_bytes(g, g.N, n2));
  if (b) return b;
  ConvGeom gb = g;
  gb.N = (int)n2;
  gb.M = n2 * (long long)g.OH * g.OW;
  return std::max(wgrad_ws_bytes(g, dt), wgrad_ws_bytes(gb, dt));
}

int wgrad_two(const void* x, const ssseg_vcat* vc, const void* dy, const void* x2, const ssseg_vcat* vc2,
              const void* dy2, int64_t n2, float* dw, const ssseg_conv_desc* d, int dt, int64_t c_real, int64_t k_real,
              int layout, int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  ConvGeom g, g2;
  if (!make_geom(d, g) || !x || !dy || !x2 || !dy2 || !dw || n2 < 1 || n2 > 0x7fffffff) return SSSEG_EINVAL;
  const int vec = dt == SSSEG_F32 ? 4 : 8;
  if (!wg_geom_ok(g, dt) || g.ldy % vec || g.K % vec) return SSSEG_EINVAL;
  if (c_real < 1 || c_real > g.C || k_real < 1 || k_real > g.K || (layout != 0 && layout != 1)) return SSSEG_EINVAL;
  if ((vc == nullptr) != (vc2 == nullptr) || (vc && (vc->c1 != vc2->c1 || vc->ldx2 != vc2->ldx2))) return SSSEG_EINVAL;
  ConvGeom gb = g;
  gb.N = (int)n2;
  gb.M = n2 * (long long)g.OH * g.OW;
  if (!vcat_ok(vc, g, dt) || !vcat_ok(vc2, gb, dt)) return SSSEG_EINVAL;
  if (!ws || ws_bytes < wgrad2_ws_bytes(g, n2, dt)) return SSSEG_EWORKSPACE;
  if (halo3_eligible(g, dt) && halo3_fits(g, g.N, vc) && halo3_fits(g, n2, vc2)) {
    run_halo3(g, dt, x, vc, dy, x2, vc2, dy2, n2, dw, c_real, k_real, layout, accumulate, (float*)ws,
              (hipStream_t)stream);
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  WgradPlan p;
  int s1;
  if (!merged_plan(g, n2, dt, p, s1, g2, vc ? (int)vc->c1 : 0)) {   // the two contributions one after the other
    if (vc) return SSSEG_EUNSUPPORTED;
    ssseg_conv_desc d2 = *d;
    d2.N = n2;
    const int rc = wgrad_one(x, nullptr, dy, dw, d, dt, c_real, k_real, layout, accumulate, ws, ws_bytes, stream);
    if (rc) return rc;
    return wgrad_one(x2, nullptr, dy2, dw, &d2, dt, c_real, k_real, layout, 1, ws, ws_bytes, stream);
  }
  hipStream_t s = (hipStream_t)stream;
  float* slab = (float*)ws;
  WSeg2 sg{x2, dy2, g2.M, (unsigned)((long long)g2.N * g2.H * g2.W * g2.ldx * 2), (unsigned)(g2.M * g2.ldy * 2), s1,
           0, 0, nullptr, nullptr, 0, 0};
  if (vc) {
    sg.c1 = (int)vc->c1;
    sg.ldx2 = (int)vc->ldx2;
    sg.xa = vc->x2;
    sg.xb = vc2->x2;
    sg.xabytes = (unsigned)((long long)g.N * g.H * g.W * vc->ldx2 * 2);
    sg.xbbytes = (unsigned)((long long)g2.N * g2.H * g2.W * vc->ldx2 * 2);
  }
  const WDirect dd{nullptr, (int)c_real, (int)k_real, layout, accumulate};
  if (dt == SSSEG_F16)
    launch_wgrad_glds<f16_t>(x, dy, slab, g, p, dd, s, sg);
  else
    launch_wgrad_glds<bf16_t>(x, dy, slab, g, p, dd, s, sg);
  launch_reduce(slab, g, p.splits, c_real, k_real, dw, layout, accumulate, s);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

}  // namespace

extern "C" int ssseg_conv_wgrad(const void* x, const void* dy, float* dw, const ssseg_conv_desc* d, int dt,
                                int64_t c_real, int64_t k_real, int layout, int accumulate, void* ws, size_t ws_bytes,
                                ssseg_stream_t stream) {
  return wgrad_one(x, nullptr, dy, dw, d, dt, c_real, k_real, layout, accumulate, ws, ws_bytes, stream);
}

extern "C" int ssseg_conv_wgrad_vcat(const void* x, const ssseg_vcat* vc, const void* dy, float* dw,
                                     const ssseg_conv_desc* d, int dt, int64_t c_real, int64_t k_real, int layout,
                                     int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!vc) return SSSEG_EINVAL;
  return wgrad_one(x, vc, dy, dw, d, dt, c_real, k_real, layout, accumulate, ws, ws_bytes, stream);
}

extern "C" size_t ssseg_conv_wgrad2_workspace_bytes(const ssseg_conv_desc* d, int64_t n2, int dt) {
  ConvGeom g;
  if (!make_geom(d, g) || n2 < 1 || n2 > 0x7fffffff) return 0;
  return wgrad2_ws_bytes(g, n2, dt);
}

extern "C" int ssseg_conv_wgrad2(const void* x, const void* dy, const void* x2, const void* dy2, int64_t n2, float* dw,
                                 const ssseg_conv_desc* d, int dt, int64_t c_real, int64_t k_real, int layout,
                                 int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  return wgrad_two(x, nullptr, dy, x2, nullptr, dy2, n2, dw, d, dt, c_real, k_real, layout, accumulate, ws, ws_bytes,
                   stream);
}

extern "C" int ssseg_conv_wgrad2_vcat(const void* x, const ssseg_vcat* vc, const void* dy, const void* x2,
                                      const ssseg_vcat* vc2, const void* dy2, int64_t n2, float* dw,
                                      const ssseg_conv_desc* d, int dt, int64_t c_real, int64_t k_real, int layout,
                                      int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!vc || !vc2) return SSSEG_EINVAL;
  return wgrad_two(x, vc, dy, x2, vc2, dy2, n2, dw, d, dt, c_real, k_real, layout, accumulate, ws, ws_bytes, stream);
}

extern "C" int ssseg_wgrad_defer_reduce(int on) {
  t_defer_reduce = on != 0;
  return 0;
}

extern "C" int64_t ssseg_wgrad_reduce_pending(void) { return (int64_t)t_pending_reduce.size(); }

extern "C" int ssseg_wgrad_reduce_flush(ssseg_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  std::vector<ReduceDesc> pend;
  pend.swap(t_pending_reduce);
  for (size_t at = 0; at < pend.size(); at += RB_MAX) {
    ReduceBatch b{};
    b.n = (int)std::min<size_t>(RB_MAX, pend.size() - at);
    long long blocks = 1;
    for (int k = 0; k < b.n; ++k) {
      b.d[k] = pend[at + k];
      const long long total = (long long)b.d[k].K * b.d[k].R * b.d[k].S * b.d[k].C;
      // wide descriptors: one block per 64 outputs; plain: the plain kernel's grid over 1024-thread blocks
      const long long need = b.d[k].splits >= 64 ? (total + 63) / 64 : (long long)ssseg_grid(total, 1024);
      blocks = std::max(blocks, need);
    }
    if (blocks > 0x7fffffffLL) return SSSEG_EINVAL;
    hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3((unsigned)blocks, (unsigned)b.n), dim3(1024), 0, s, b);
    SSSEG_LAUNCH_CHECK();
  }
  return 0;
}
