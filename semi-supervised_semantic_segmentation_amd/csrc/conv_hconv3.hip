// Halo-tiled 3x3 / stride-1 / pad-1 convolution (forward, and the stride-1 input gradient, which is the same
// contraction over dY with the flipped weight pack): LDS-DMA variant 24 of the engine's autotuner (conv.hip).
//
//   y[n][y][x][k] = sum_{c, r, s} x[n][y + r - 1][x + s - 1][c] * w[k][r][s][c]
//
// The gather kernel (igemm_glds_kernel) stages, per 64-deep k-tile, a BN x 64 weight tile and a BM x 64 pixel tile
// gathered for ONE tap: every input line is fetched nine times (once per tap) and on the 64-/128-channel layers
// (K = 64 -> 64-wide n-tiles) the LDS-DMA feed, not the MFMA, bounds it (~45 flop per staged byte).  Here a block
// owns 4 output rows x 64 columns of one image (BM = 256 pixels) and 64 output channels; per 64-channel block cb of
// the input it stages the 6 x 66-pixel halo of those rows ONCE (51 KB, double-buffered across cb) and streams the
// weights of one tap row r (3 taps x 64 k x 64 c, 24 KB, double-buffered) per stage: 9.4 MFLOP per 62 KB at the
// peak stage mix, ~150 flop per staged byte.
//
// k-sequence: per cb, taps r = 0..2, s = 0..2, and the two 32-deep halves of the channel block innermost -- exactly
// the order of the gather kernel's channel-block-major k (kt = cb * RS + tap, two ks halves per k-tile), with the same
// MFMA operand roles (A = weights, B = pixels) and the same 8-channel chunk per lane group: every fp32 accumulation
// happens in the same order, so the outputs are bitwise those of the other variants (tests/test_hip_layers.py).
//
// 4 waves; wave w owns output row w of the tile (64 pixels = 4 fragments) x 64 channels (4 fragments): 16 MFMA tiles,
// 64 accumulator VGPRs.  LDS: 2 x 51,200 B halo buffers + 2 x 24,576 B weight buffers = 151,552 B (one block per CU);
// the LDS-staged epilogue (store_tile_lds, T2D row map) reuses them.
#include "conv_kernels.h"

namespace {

constexpr int HC_PX = 400;                    // halo pixels per buffer: 6 rows x 66 (+4 padding pixels)
constexpr int HC_XBUF = HC_PX * 128;          // 64 channels x 2 B per pixel
constexpr int HC_WBUF = 3 * 64 * 128;         // one tap row: 3 taps x 64 output channels x 64 input channels
constexpr int HC_SMEM = 2 * HC_XBUF + 2 * HC_WBUF;
constexpr int HC_SMEM1 = HC_XBUF + HC_WBUF;   // single-buffered form: two blocks per CU (75,776 B each)
static_assert(256 * (64 * 4 + 16) <= HC_SMEM1, "the staged epilogue tile fits the single-buffered LDS");

__device__ __forceinline__ int hc_swz(int r) { return (r >> 1) & 7; }   // 16-byte chunk swizzle of a 128-byte row

// TWO (autotuner variant 28): one halo and one weight buffer (75.8 KB), two blocks per CU -- each block loads a stage
// while the other multiplies (2 waves per SIMD); the double-buffered form (variant 24) has one 151.5 KB block per CU,
// one wave per SIMD, whose MFMA and LDS latencies do not overlap and whose prologue / epilogue latency is exposed on
// every tile
// TW: tile width (64; 32 / 16 on the 32^2 / 16^2 maps: 8 / 16 rows of 32 / 16 pixels, the same 256 pixels, a 10 x 34 /
// 18 x 18 halo in the same buffer); wave w owns tile pixels 64 w .. 64 w + 63 (row-major), fragment j = 16 of them
template <typename TO, bool STATS, bool VC, bool TWO, int TW = 64>
__global__ void __launch_bounds__(256, TWO ? 2 : 1) hconv3_kernel(const TO* __restrict__ x, const TO* __restrict__ w,
                                                                  TO* __restrict__ y, ConvGeom g, Epi<TO> ep,
                                                                  unsigned xbytes, unsigned wbytes,
                                                                  const TO* __restrict__ x2, unsigned x2bytes) {
  constexpr int TR = 256 / TW, HW = TW + 2, NPX = (TR + 2) * HW;   // tile rows, halo row width, halo pixels
  static_assert(NPX <= HC_PX && TW >= 16, "the halo fits the buffer");
  __shared__ __attribute__((aligned(1024))) char smem[TWO ? HC_SMEM1 : HC_SMEM];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nkb = g.K >> 6, nstrips = g.W / TW, nrg = g.H / TR;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);   // consecutive ids (the k-blocks of one pixel tile) share an XCD
  const int kb = tile % nkb, pt = tile / nkb;
  const int strip = pt % nstrips, q = pt / nstrips;
  const int rg = q % nrg, n = q / nrg;
  const int y0 = rg * TR, x0 = strip * TW;
  const int H = g.H, W = g.W, C = g.C, ncb = g.C >> 6;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, (int)wbytes, 0x00020000);
  __amdgpu_buffer_rsrc_t xr2 = xr;
  if constexpr (VC) xr2 = __builtin_amdgcn_make_buffer_rsrc((void*)x2, (short)0, (int)x2bytes, 0x00020000);
  char* const XB = smem;
  char* const WB = smem + (TWO ? 1 : 2) * HC_XBUF;

  // halo of channel block cb into buffer b: pixel p = 8i + lane/8 of 50 wave-instructions (row p / 66, column p % 66
  // of the 6 x 66 window whose top-left input pixel is (y0 - 1, x0 - 1)); padding / out-of-image pixels read zeros
  auto issue_x = [&](int b, int cb) {
    const bool second = VC && cb >= g.c1b;
    const int ld = second ? g.ldx2 : g.ldx, cc = (second ? cb - g.c1b : cb) * 64;
    for (int i = wave; i < HC_PX / 8; i += 4) {
      const int p = 8 * i + (lane >> 3);
      const int row = p / HW, col = p - row * HW;
      const int yy = y0 - 1 + row, xx = x0 - 1 + col;
      unsigned off = OOB;
      if (p < NPX && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
        off = (unsigned)(((n * H + yy) * W + xx) * ld + cc + 8 * ((lane & 7) ^ hc_swz(p))) * 2u;
      if (VC && second) bldslds16_nt(xr2, XB + b * HC_XBUF + i * 1024, off, 0);
      else bldslds16_nt(xr, XB + b * HC_XBUF + i * 1024, off, 0);
    }
  };
  // weights of tap row r, channel block cb into buffer b: row rho = tl * 64 + k (tl = tap s of the row), 24
  // wave-instructions, 6 per wave; packed weights [K][3][3][C] (ldw = 9 C)
  auto issue_w = [&](int b, int cb, int r) {
#pragma unroll
    for (int h = 0; h < 6; ++h) {
      const int i = wave * 6 + h;
      const int rho = 8 * i + (lane >> 3);
      const int tl = rho >> 6, k = kb * 64 + (rho & 63);
      const unsigned off = (unsigned)(k * g.ldw + (3 * r + tl) * C + cb * 64 + 8 * ((lane & 7) ^ hc_swz(rho))) * 2u;
      bldslds16_nt(wr, WB + b * HC_WBUF + i * 1024, off, 0);
    }
  };

  f32x4 acc[4][4];   // [k fragment][pixel fragment]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int li = lane & 15, lg = lane >> 4;
  auto compute = [&](int xb, int wbuf, int r) {
    const char* X = XB + xb * HC_XBUF;
    const char* Wt = WB + wbuf * HC_WBUF;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = ks * 4 + lg;
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rho = s * 64 + i * 16 + li;
          af[i] = *(const bf16x8*)(Wt + rho * 128 + ((ch ^ hc_swz(rho)) << 4));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int tp = wave * 64 + j * 16;   // first tile pixel of the fragment (16 | TW: one tile row)
          const int p = (tp / TW + r) * HW + tp % TW + li + s;
          bfr[j] = *(const bf16x8*)(X + p * 128 + ((ch ^ hc_swz(p)) << 4));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = M16<TO>::mma(af[i], bfr[j], acc[i][j]);
      }
    }
  };

  const int nst = ncb * 3;
  if constexpr (TWO) {
    // stages (cb, r) in order, each loaded into the single buffers after the previous stage's reads (the other block
    // on the CU multiplies meanwhile)
    for (int st = 0; st < nst; ++st) {
      const int cb = st / 3, r = st - cb * 3;
      if (r == 0) issue_x(0, cb);
      issue_w(0, cb, r);
      vmcnt_wait<0>();
      __builtin_amdgcn_s_barrier();   // the stage landed for every wave
      compute(0, 0, r);
      __builtin_amdgcn_s_barrier();   // every wave is done reading it
    }
  } else {
    // stages (cb, r) in order; the halo of cb + 1 is issued with stage (cb, 0) (its buffer was last read by cb - 1),
    // the weights of the next stage with every stage: one stage of prefetch, vmcnt(0) + barrier per stage
    issue_x(0, 0);
    issue_w(0, 0, 0);
    vmcnt_wait<0>();
    __builtin_amdgcn_s_barrier();
    for (int st = 0; st < nst; ++st) {
      const int cb = st / 3, r = st - cb * 3;
      if (st + 1 < nst) {
        const int cb1 = (st + 1) / 3, r1 = (st + 1) - cb1 * 3;
        if (r == 0 && cb + 1 < ncb) issue_x((cb + 1) & 1, cb + 1);
        issue_w((st + 1) & 1, cb1, r1);
      }
      compute(cb & 1, st & 1, r);
      vmcnt_wait<0>();
      __builtin_amdgcn_s_barrier();   // this stage's buffers are free, the next stage's landed for every wave
    }
  }

  // LDS-staged epilogue over the 4 x 64 pixel tile (the ring is idle: the loop ended on a barrier)
  const Tile2D t2{n, y0, x0, min(TR, H - y0), (long long)pt, TW == 64 ? 6 : (TW == 32 ? 5 : 4)};
  store_tile_lds<TO, 256, 64, 4, 4, 256, STATS, 1, true>(acc, smem, 0, kb * 64, wave * 64, 0, lane, g, y, ep,
                                                         PreRes<1>{{}, false}, t2);
}

}  // namespace

// tile width for the map: 64 (W % 64 == 0, H % 4 == 0), else 32 (W % 32, H % 8) or 16 (W % 16, H % 16); 0 = none
static int hconv3_tw(const ConvGeom& g) {
  if (g.W % 64 == 0 && g.H % 4 == 0) return 64;
  if (g_knobs[16] < 0) return 0;   // knob 16 = -1: the 64-wide tile only (A/B)
  if (g.W % 32 == 0 && g.H % 8 == 0) return 32;
  if (g.W % 16 == 0 && g.H % 16 == 0) return 16;
  return 0;
}

bool hconv3_ok(const ConvGeom& g, const PhaseTab* ph, const float* ws) {
  return g_knobs[11] >= 0 && !ws && !(ph && ph->n > 1) && g.R == 3 && g.S == 3 && g.sy == 1 && g.sx == 1 &&
         g.dy == 1 && g.dx == 1 && g.py == -1 && g.px == -1 && g.oident && g.H == g.OH && g.W == g.OW &&
         hconv3_tw(g) > 0 && g.C % 64 == 0 && g.K % 64 == 0 && g.ldw == 9 * g.C && g.ldx % 8 == 0 &&
         g.ldy % 8 == 0 && g.ldx >= g.C && g.M < 0x7fffffffLL;
}

template <typename TO, bool TWO, int TW>
static void launch_hconv3_t(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                            unsigned wb, hipStream_t s, const void* x2, unsigned x2b, long long blocks) {
  const TO* xa = (const TO*)x2;
  const dim3 grid((unsigned)blocks), blk(256);
  if (x2) {
    if (ep.stats)
      hipLaunchKernelGGL((hconv3_kernel<TO, true, true, TWO, TW>), grid, blk, 0, s, (const TO*)x, (const TO*)w, (TO*)y,
                         g, ep, xb, wb, xa, x2b);
    else
      hipLaunchKernelGGL((hconv3_kernel<TO, false, true, TWO, TW>), grid, blk, 0, s, (const TO*)x, (const TO*)w,
                         (TO*)y, g, ep, xb, wb, xa, x2b);
  } else if (ep.stats) {
    hipLaunchKernelGGL((hconv3_kernel<TO, true, false, TWO, TW>), grid, blk, 0, s, (const TO*)x, (const TO*)w, (TO*)y,
                       g, ep, xb, wb, xa, x2b);
  } else {
    hipLaunchKernelGGL((hconv3_kernel<TO, false, false, TWO, TW>), grid, blk, 0, s, (const TO*)x, (const TO*)w,
                       (TO*)y, g, ep, xb, wb, xa, x2b);
  }
}

template <typename TO, bool TWO>
static void launch_hconv3_w(int tw, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep,
                            unsigned xb, unsigned wb, hipStream_t s, const void* x2, unsigned x2b, long long blocks) {
  if (tw == 64) launch_hconv3_t<TO, TWO, 64>(x, w, y, g, ep, xb, wb, s, x2, x2b, blocks);
  else if (tw == 32) launch_hconv3_t<TO, TWO, 32>(x, w, y, g, ep, xb, wb, s, x2, x2b, blocks);
  else launch_hconv3_t<TO, TWO, 16>(x, w, y, g, ep, xb, wb, s, x2, x2b, blocks);
}

// mode 0: the double-buffered kernel (variant 24), 1: the single-buffered two-blocks-per-CU kernel (variant 28)
template <typename TO>
int launch_hconv3(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                  unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2, unsigned x2b, int mode) {
  if (!hconv3_ok(g, ph, ws) || (x2 && (g.ldx2 % 8 || g.c1b < 1 || g.c1b >= g.C / 64))) return -1;
  if (mode == 1 && g_knobs[15] < 0) return -1;   // knob 15 = -1: no variant 28 (A/B)
  const int tw = hconv3_tw(g);
  const long long blocks = (long long)g.N * (g.H / (256 / tw)) * (g.W / tw) * (g.K / 64);
  if (blocks > 0x7fffffffLL) return -1;
  if (mode == 1)
    launch_hconv3_w<TO, true>(tw, x, w, y, g, ep, xb, wb, s, x2, x2b, blocks);
  else
    launch_hconv3_w<TO, false>(tw, x, w, y, g, ep, xb, wb, s, x2, x2b, blocks);
  return 256;
}

template int launch_hconv3<bf16_t>(const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&, unsigned,
                                   unsigned, hipStream_t, float*, const PhaseTab*, const void*, unsigned, int);
template int launch_hconv3<f16_t>(const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&, unsigned,
                                  unsigned, hipStream_t, float*, const PhaseTab*, const void*, unsigned, int);
