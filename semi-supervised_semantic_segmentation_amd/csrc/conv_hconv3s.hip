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
// epilogue (store_tile_lds, T2D row map, fused BN statistics) reuses the halo buffer.
#include "conv_kernels.h"

namespace {

constexpr int HS_PX = 400;                    // halo pixels: 6 rows x 66 (+4 padding pixels)
constexpr int HS_XBUF = HS_PX * 64;           // 32 channels x 2 B per pixel
constexpr int HS_EPI = 256 * (32 * 4 + 16);   // the staged 256 x 32 fp32 output tile
constexpr int HS_SMEM = HS_EPI > HS_XBUF ? HS_EPI : HS_XBUF;

__device__ __forceinline__ int hs_swz(int p) { return (p >> 2) & 3; }

template <typename TO, bool STATS>
__global__ void __launch_bounds__(256) hconv3s_kernel(const TO* __restrict__ x, const TO* __restrict__ w,
                                                      TO* __restrict__ y, ConvGeom g, Epi<TO> ep, unsigned xbytes) {
  __shared__ __attribute__((aligned(1024))) char smem[HS_SMEM];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nstrips = g.W >> 6, nrg = g.H >> 2;
  const int pt = xcd_tile(blockIdx.x, gridDim.x);
  const int strip = pt % nstrips, q = pt / nstrips;
  const int rg = q % nrg, n = q / nrg;
  const int y0 = rg * 4, x0 = strip * 64;
  const int H = g.H, W = g.W;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)xbytes, 0x00020000);

  // halo: 25 wave-instructions of 64 chunks, chunk q = 64 i + lane -> pixel p = q / 4 at slot q % 4, which holds the
  // global chunk (q % 4) ^ swz(p); padding / out-of-image pixels read zeros (out-of-range offset)
  for (int i = wave; i < HS_PX * 4 / 64; i += 4) {
    const int qq = 64 * i + lane, p = qq >> 2, slot = qq & 3;
    const int row = p / 66, col = p - row * 66;
    const int yy = y0 - 1 + row, xx = x0 - 1 + col;
    unsigned off = OOB;
    if (p < 396 && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
      off = (unsigned)(((n * H + yy) * W + xx) * g.ldx + 8 * (slot ^ hs_swz(p))) * 2u;
    bldslds16(xr, smem + i * 1024, off, 0u);
  }

  // weights into registers: tap t, fragment i -> output channel 16 i + (lane & 15), channels 8 (lane >> 4) .. + 7
  const int li = lane & 15, lg = lane >> 4;
  bf16x8 wf[9][2];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int i = 0; i < 2; ++i) wf[tp][i] = *(const bf16x8*)(w + (long long)(i * 16 + li) * g.ldw + tp * 32 + lg * 8);

  f32x4 acc[2][4];   // [channel fragment][pixel fragment]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  vmcnt_wait<0>();
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      bf16x8 bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = (wave + r) * 66 + j * 16 + li + s;
        bfr[j] = *(const bf16x8*)(smem + p * 64 + ((lg ^ hs_swz(p)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = M16<TO>::mma(wf[r * 3 + s][i], bfr[j], acc[i][j]);
    }

  const Tile2D t2{n, y0, x0, min(4, H - y0), (long long)pt};
  store_tile_lds<TO, 256, 32, 4, 2, 256, STATS, 1, true>(acc, smem, 0, 0, wave * 64, 0, lane, g, y, ep,
                                                        PreRes<1>{{}, false}, t2);
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
  const long long blocks = (long long)g.N * (g.H / 4) * (g.W / 64);
  if (blocks > 0x7fffffffLL) return -1;
  if (ep.stats)
    hipLaunchKernelGGL((hconv3s_kernel<TO, true>), dim3((unsigned)blocks), dim3(256), 0, s, (const TO*)x,
                       (const TO*)w, (TO*)y, g, ep, xb);
  else
    hipLaunchKernelGGL((hconv3s_kernel<TO, false>), dim3((unsigned)blocks), dim3(256), 0, s, (const TO*)x,
                       (const TO*)w, (TO*)y, g, ep, xb);
  return 256;
}

template int launch_hconv3s<bf16_t>(const void*, const void*, void*, const ConvGeom&, const Epi<bf16_t>&, unsigned,
                                    hipStream_t, float*, const PhaseTab*, const void*);
template int launch_hconv3s<f16_t>(const void*, const void*, void*, const ConvGeom&, const Epi<f16_t>&, unsigned,
                                   hipStream_t, float*, const PhaseTab*, const void*);
