// Halo-tiled 3x3 / stride-1 / pad-1 convolution for 32 input and 32 output channels (HRNet-W32's branch-0 basic
// blocks, config C4: 128 forward + 64 input-gradient launches per step at 16x256^2 and 16x128^2): LDS-DMA variant 25
// of the engine's autotuner (conv.hip).
//
// The gather kernel runs these layers on its general-k loader (C = 32: a 64-deep k-tile holds two taps): every input
// pixel is staged nine times (576 B per output pixel through L2 and the LDS-DMA path for 64 B of output), half of each
// 64-wide n-tile is padding, and the layer runs at ~1.3 TB/s.  Here a block owns 4 output rows x 64 columns of one
// image and all 32 output channels: the 6 x 66-pixel halo (64 B per pixel) is staged ONCE (25.6 KB), the 9 x 32 x 32
// weights live in registers (loaded once per block, L2-resident), and each wave multiplies its output row against
// the halo for the nine taps -- 96 staged bytes per output pixel.
//
// k-sequence: taps 0..8 in order, each one 32-deep MFMA step with lane group g supplying channels 8g..8g+7 -- exactly
// the general-k gather kernel's sequence for C = 32 (k = tap * 32 + c, two taps per 64-deep k-tile, ks halves in
// order; its tenth tap is a zero padding tap), with the same operand roles (A = weights, B = pixels): the outputs are
// the other variants' bit for bit (tests/test_hip_layers.py).
//
// 4 waves; wave w owns output row w of the tile: 4 pixel fragments x 2 channel fragments (32 accumulator VGPRs), its
// weights are 18 bf16x8 fragments (72 VGPRs).  Halo pixel p keeps its four 16-byte channel chunks at slots c ^ ((p >> 2)
// & 3): the 16 lanes of a fragment read 16 consecutive pixels' chunk c from four different bank groups.  The LDS-staged
// epilogue (store_tile_lds, T2D row map, fused BN statistics) reuses the tile's halo buffer.  Measured: a one-tile-per-
// block form (4096 blocks at 16x256^2) ran 32->32 @16x256^2 in 60 us (the gather kernel: 89 us); persistent below.
#include "conv_kernels.h"

#include <algorithm>

namespace {

constexpr int HS_PX = 400;                    // halo pixels: 6 rows x 66 (+4 padding pixels)
constexpr int HS_XBUF = HS_PX * 64;           // 32 channels x 2 B per pixel
constexpr int HS_EPI = 256 * (32 * 4 + 16);   // the staged 256 x 32 fp32 output tile
constexpr int HS_BUF = HS_EPI > HS_XBUF ? HS_EPI : HS_XBUF;
constexpr int HS_SMEM = 2 * HS_BUF;           // two buffers: 73,728 B, two blocks per CU

__device__ __forceinline__ int hs_swz(int p) { return (p >> 2) & 3; }

// Persistent: block b runs tiles b, b + G, b + 2G, ... (G = grid size).  Buffer (it & 1) holds tile it's halo, and
// after its MFMAs the same buffer stages its output for the epilogue; tile it + 1's halo streams into the other
// buffer meanwhile.  The halo DMA is issued from inline asm (invisible to the compiler's waitcnt bookkeeping) and
// waited for with an explicit count: at the top of iteration it, the only VM operations younger than tile it's halo
// are tile it - 1's epilogue stores -- at least 4 per thread (4 row passes x one 16-byte store; more with an aux copy,
// residual loads or the statistics row) -- so vmcnt(4) guarantees the halo landed (in-order retirement).
template <typename TO, bool STATS>
__global__ void __launch_bounds__(256, 2) hconv3s_kernel(const TO* __restrict__ x, const TO* __restrict__ w,
                                                         TO* __restrict__ y, ConvGeom g, Epi<TO> ep, unsigned xbytes,
                                                         int ntiles) {
  __shared__ __attribute__((aligned(1024))) char smem[HS_SMEM];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nstrips = g.W >> 6, nrg = g.H >> 2;
  const int H = g.H, W = g.W;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)xbytes, 0x00020000);

  // halo of tile pt into buffer b: 25 wave-instructions of 64 chunks, chunk q = 64 i + lane -> pixel p = q / 4 at
  // slot q % 4, which holds the global chunk (q % 4) ^ swz(p); padding / out-of-image pixels read zeros
  auto issue_halo = [&](int b, int pt) {
    const int strip = pt % nstrips, q = pt / nstrips;
    const int rg = q % nrg, n = q / nrg;
    const int y0 = rg * 4, x0 = strip * 64;
    for (int i = wave; i < HS_PX * 4 / 64; i += 4) {
      const int qq = 64 * i + lane, p = qq >> 2, slot = qq & 3;
      const int row = p / 66, col = p - row * 66;
      const int yy = y0 - 1 + row, xx = x0 - 1 + col;
      unsigned off = OOB;
      if (p < 396 && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
        off = (unsigned)(((n * H + yy) * W + xx) * g.ldx + 8 * (slot ^ hs_swz(p))) * 2u;
      bldslds16_nt(xr, smem + b * HS_BUF + i * 1024, off, 0u);
    }
  };

  // weights into registers once: tap t, fragment i -> output channel 16 i + (lane & 15), channels 8 (lane >> 4) .. + 7
  const int li = lane & 15, lg = lane >> 4;
  bf16x8 wf[9][2];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int i = 0; i < 2; ++i) wf[tp][i] = *(const bf16x8*)(w + (long long)(i * 16 + li) * g.ldw + tp * 32 + lg * 8);

  const int G = gridDim.x;
  int pt = blockIdx.x;
  if (pt < ntiles) issue_halo(0, pt);
  for (int it = 0; pt < ntiles; ++it, pt += G) {
    const int b = it & 1;
    if (it == 0) vmcnt_wait<0>();
    else vmcnt_wait<4>();
    __syncthreads();   // tile pt's halo landed for every wave; buffer b ^ 1 (the last epilogue's) is free
    if (pt + G < ntiles) issue_halo(b ^ 1, pt + G);
    const char* X = smem + b * HS_BUF;
    f32x4 acc[2][4];   // [channel fragment][pixel fragment]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        bf16x8 bfr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int p = (wave + r) * 66 + j * 16 + li + s;
          bfr[j] = *(const bf16x8*)(X + p * 64 + ((lg ^ hs_swz(p)) << 4));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = M16<TO>::mma(wf[r * 3 + s][i], bfr[j], acc[i][j]);
      }
    const int strip = pt % nstrips, q = pt / nstrips;
    const int rg = q % nrg, n = q / nrg;
    const Tile2D t2{n, rg * 4, strip * 64, min(4, H - rg * 4), (long long)pt};
    // staged in this tile's own buffer (store_tile_lds opens with a barrier: every wave's MFMAs are done with it)
    store_tile_lds<TO, 256, 32, 4, 2, 256, STATS, 1, true>(acc, smem + b * HS_BUF, 0, 0, wave * 64, 0, lane, g, y, ep,
                                                          PreRes<1>{{}, false}, t2);
  }
}

}  // namespace

bool hconv3s_ok(const ConvGeom& g, const PhaseTab* ph, const float* ws) {
  return g_knobs[11] >= 0 && !ws && !(ph && ph->n > 1) && g.R == 3 && g.S == 3 && g.sy == 1 && g.sx == 1 &&
         g.dy == 1 && g.dx == 1 && g.py == -1 && g.px == -1 && g.oident && g.H == g.OH && g.W == g.OW &&
         g.W % 64 == 0 && g.H % 4 == 0 && g.C == 32 && g.K == 32 && g.ldw == 9 * 32 && g.ldx >= 32 &&
         g.ldx % 8 == 0 && g.ldy % 8 == 0 && g.M < 0x7fffffffLL;
}

template <typename TO>
int launch_hconv3s(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                   hipStream_t s, float* ws, const PhaseTab* ph, const void* x2) {
  if (x2 || !hconv3s_ok(g, ph, ws)) return -1;
  const long long tiles = (long long)g.N * (g.H / 4) * (g.W / 64);
  if (tiles > 0x7fffffffLL) return -1;
  // two resident blocks per CU (73.7 KB of LDS each): a grid of 2 x 256 covers the chip once, every block then
  // loops over its tiles (the epilogue's stores must leave >= 4 VM operations per thread behind the next halo's DMA:
  // 4 row passes of the 256 x 32 tile, guaranteed by H % 4 == 0, W % 64 == 0, K == 32)
  const unsigned grid = (unsigned)std::min<long long>(tiles, 512);
  if (ep.stats)
    hipLaunchKernelGGL((hconv3s_kernel<TO, true>), dim3(grid), dim3(256), 0, s, (const TO*)x, (const TO*)w, (TO*)y, g,
                       ep, xb, (int)tiles);
  else
    hipLaunchKernelGGL((hconv3s_kernel<TO, false>), dim3(grid), dim3(256), 0, s, (const TO*)x, (const TO*)w, (TO*)y,
                       g, ep, xb, (int)tiles);
  return 256;
}

template int launch_hconv3s<bf16_t>(const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&, unsigned,
                                    hipStream_t, float*, const PhaseTab*, const void*);
template int launch_hconv3s<f16_t>(const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&, unsigned,
                                   hipStream_t, float*, const PhaseTab*, const void*);
