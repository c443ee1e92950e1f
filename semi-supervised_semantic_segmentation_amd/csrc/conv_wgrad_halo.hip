// Weight gradient of 3x3 / stride-1 / pad-1 convolutions with halo-tiled row streaming (bf16 / fp16, gfx950).
//
//   dW[k][r][s][c] = sum_{n,y,x} dY[n][y][x][k] * X[n][y + r - 1][x + s - 1][c]
//
// The split-K weight gradient (conv_wgrad.hip) stages, for every tap, a gathered copy of the input tile: each input
// line is fetched nine times (once per tap, from L2 at best) and the 64-pixel k-tiles of a 128-wide kk-tile carry
// 24 KB for 1 MFLOP -- on the 256^2 UNet layers the LDS-DMA feed, not the MFMA, bounds it (0.16 of the layer roof,
// VERDICT r3).  Here a block walks the output rows of one 64-pixel column strip top to bottom and keeps the three
// input rows y-1, y, y+1 of the strip (66 pixels with the halo) in an LDS ring: every step fetches ONE new input row
// segment and ONE dY row segment (2 x 8 KB) and runs all nine taps on them (9 x 64 x 64 x 64 x 2 = 4.7 MFLOP),
// 290 flop per fetched byte.
//
// Block = (split, 64-channel block cb of C, 64-channel block kb of K), 4 waves; wave w owns the 16 input channels
// [16w, 16w + 16) of the block for all nine taps and all 64 output channels: 9 x 4 accumulator tiles of 16x16
// (144 VGPRs).  Per 32-pixel step a wave reads one dY fragment per 16 output channels (4, shared by the taps) and one
// X fragment per tap (9): the X fragment of tap (r, s) is the ring row of input row y + r - 1 read s pixels to the
// right.  Both operands are pixel-major in LDS and read with ds_read_b64_tr_b16 under the k-slot -> pixel map of the
// split-K kernel (wkp), so the pixel contraction is permuted identically for A and B.
//
// A split is a contiguous range of row steps t = ((n * nstrips) + strip) * H + y of one pixel segment (the merged
// supervised + consistency launch has two); a column change (new strip or image) reloads the three ring rows.  Every
// split writes its fp32 partial of the whole dW into its own slab, which wgrad_reduce sums in split order
// (deterministic), exactly like the split-K path.
#include "conv_kernels.h"

namespace {

constexpr int HX_ROWS = 72;                 // ring row: 66 pixels (64 + halo) padded to whole 8-row wave-instructions
constexpr int HX_SLOT = HX_ROWS * 128;      // one input row segment: 64 channels x 2 B per pixel
constexpr int HD_SLOT = 64 * 128;           // one dY row segment
constexpr int H_SMEM = 4 * HX_SLOT + 2 * HD_SLOT;

__device__ __forceinline__ int hswz(int r) { return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 1); }
__device__ __forceinline__ int hkp(int g, int j) { return 16 * (g >> 1) + 8 * (g & 1) + 4 * (j >> 2) + (j & 3); }

template <typename T16>
__global__ void __launch_bounds__(256, 2) wgrad_halo3_kernel(HaloArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[H_SMEM];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles = a.ncb * a.nkb;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int split = tile / tiles, rem = tile - split * tiles;
  const int cb = rem % a.ncb, kb = rem / a.ncb;
  const int sg = split >= a.s1 ? 1 : 0;
  const long long t0 = (long long)(sg ? split - a.s1 : split) * a.sps[sg];
  const long long t1 = min(t0 + a.sps[sg], a.steps[sg]);
  const HaloSeg& S = a.seg[sg];
  // the channel block's source (a virtual concat's second part is a block-uniform choice: c1 % 64 == 0)
  const bool part2 = a.c1 > 0 && cb * 64 >= a.c1;
  const char* xsrc = (const char*)(part2 ? S.x2 : S.x);
  const unsigned xbytes = part2 ? S.x2bytes : S.xbytes;
  const int ldx = part2 ? a.ldx2 : a.ldx, c0 = part2 ? cb * 64 - a.c1 : cb * 64;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)xsrc, (short)0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc((void*)S.dy, (short)0, (int)S.dbytes, 0x00020000);
  const int H = a.H, W = a.W;

  // this lane's fixed part of its LDS-DMA pieces: row-in-instruction and logical 16-byte chunk (bank swizzle applied
  // on the source side: the DMA writes lane-linearly)
  const int lrow = lane >> 3;
  auto x_chunk = [&](int row) { return ((lane & 7) ^ hswz(row)) * 16; };

  auto issue_x = [&](int slot, int n, int yy, int strip) {   // input row yy of the strip (66 pixels) -> ring slot
    char* base = smem + slot * HX_SLOT;
    const bool yok = (unsigned)yy < (unsigned)H;
    for (int i = wave; i < HX_ROWS / 8; i += 4) {
      const int row = 8 * i + lrow;
      const int xx = strip * 64 - 1 + row;
      unsigned off = OOB;
      if (yok && row < 66 && (unsigned)xx < (unsigned)W)
        off = (unsigned)(((n * H + yy) * W + xx) * ldx + c0) * 2u + (unsigned)x_chunk(row);
      bldslds16(xr, base + i * 1024, off, 0);
    }
  };
  auto issue_dy = [&](int slot, int n, int y, int strip) {   // dY row y of the strip (64 pixels) -> dy slot
    char* base = smem + 4 * HX_SLOT + slot * HD_SLOT;
#pragma unroll
    for (int i = wave; i < 8; i += 4) {
      const int row = 8 * i + lrow;
      const int xx = strip * 64 + row;
      const unsigned off = (unsigned)(((n * H + y) * W + xx) * a.ldy + kb * 64) * 2u + (unsigned)x_chunk(row);
      bldslds16(dr, base + i * 1024, off, 0);
    }
  };
  auto decode = [&](long long t, int& n, int& strip, int& y) {
    const long long q = t / H;
    y = (int)(t - q * H);
    n = (int)(q / a.nstrips);
    strip = (int)(q - (long long)n * a.nstrips);
  };

  f32x4 acc[9][4];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int gq = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  // fragment addresses inside a slot: rows (pixel) of the lane's lo / hi transposed reads, column chunk + byte
  const int xcol = 2 * wave + (p4 >> 1), dsub = 8 * (p4 & 1);

  auto compute = [&](int y, int dslot) {
    const char* D = smem + 4 * HX_SLOT + dslot * HD_SLOT;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r0 = ks * 32 + hkp(gq, q4), r1 = ks * 32 + hkp(gq, 4 + q4);
      bf16x8 bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = 2 * j + (p4 >> 1);
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(D + r0 * 128 + ((ch ^ hswz(r0)) * 16) + dsub));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(D + r1 * 128 + ((ch ^ hswz(r1)) * 16) + dsub));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const char* X = smem + ((y + r) & 3) * HX_SLOT;   // input row y + r - 1 lives in slot (y + r) & 3
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int x0 = r0 + s, x1 = r1 + s;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(X + x0 * 128 + ((xcol ^ hswz(x0)) * 16) + dsub));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(X + x1 * 128 + ((xcol ^ hswz(x1)) * 16) + dsub));
          const bf16x8 af = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[r * 3 + s][j] = M16<T16>::mma(af, bfr[j], acc[r * 3 + s][j]);
        }
      }
    }
  };

  // prologue / column change: the three ring rows of row y's taps and dY row y, then wait
  auto load_column = [&](int n, int strip, int y, int dslot) {
    issue_x((y) & 3, n, y - 1, strip);
    issue_x((y + 1) & 3, n, y, strip);
    issue_x((y + 2) & 3, n, y + 1, strip);
    issue_dy(dslot, n, y, strip);
  };

  if (t0 < t1) {
    int n, strip, y;
    decode(t0, n, strip, y);
    load_column(n, strip, y, 0);
    vmcnt_wait<0>();
    __builtin_amdgcn_s_barrier();
    int dslot = 0;
    for (long long t = t0; t < t1; ++t) {
      // prefetch the next step while this one is multiplied: within a column one new input row (y + 2) and the
      // next dY row; the slot of row y + 2 held row y - 2, last read by the previous step (behind the barrier)
      const bool more = t + 1 < t1;
      const bool same_col = more && y + 1 < H;
      if (same_col) {
        issue_x((y + 3) & 3, n, y + 2, strip);
        issue_dy(dslot ^ 1, n, y + 1, strip);
      }
      compute(y, dslot);
      if (!more) break;
      if (same_col) {
        ++y;
      } else {   // next column: every ring slot may be rewritten once all waves are done with this step
        __builtin_amdgcn_s_barrier();
        decode(t + 1, n, strip, y);
        load_column(n, strip, y, dslot ^ 1);
      }
      dslot ^= 1;
      vmcnt_wait<0>();
      __builtin_amdgcn_s_barrier();   // every wave's pieces of the next step landed; the ring slot it frees is idle
    }
  }

  // slab[split][k][tap * C + c], 4 consecutive input channels per lane (16-byte stores); splits == 1: dW directly
  const int cbase = cb * 64 + 16 * wave + 4 * gq;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = kb * 64 + 16 * j + li;
      const int kk = tap * a.C + cbase;
      if (a.dw) {
        if (k >= a.k_real) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = cbase + e;
          if (c >= a.c_real) continue;
          const long long o = a.layout == 0 ? ((long long)k * 9 + tap) * a.C + c
                                            : (((long long)k * a.c_real + c) * 3 + tap / 3) * 3 + tap % 3;
          a.dw[o] = a.accumulate ? a.dw[o] + acc[tap][j][e] : acc[tap][j][e];
        }
      } else {
        float* p = a.slab + ((long long)split * a.K + k) * (9LL * a.C) + kk;
        *(float4*)p = make_float4(acc[tap][j][0], acc[tap][j][1], acc[tap][j][2], acc[tap][j][3]);
      }
    }
}

}  // namespace

bool halo3_eligible(const ConvGeom& g, int dt) {
  if (g_knobs[11] < 0 || (dt != SSSEG_BF16 && dt != SSSEG_F16)) return false;
  return g.R == 3 && g.S == 3 && g.sy == 1 && g.sx == 1 && g.dy == 1 && g.dx == 1 && g.py == -1 && g.px == -1 &&
         g.OH == g.H && g.OW == g.W && g.W % 64 == 0 && g.C % 64 == 0 && g.K % 64 == 0 && g.ldx % 8 == 0 &&
         g.ldy % 8 == 0 && g.ldx >= g.C && g.ldy >= g.K;
}

// split plan: ~2 resident blocks per CU over the chip, slabs capped at 32 MiB (>= one block per CU), splits shared out
// between the two pixel segments in proportion to their row steps
HaloPlan halo3_plan(const ConvGeom& g, long long n1, long long n2) {
  HaloPlan p;
  p.ncb = g.C / 64;
  p.nkb = g.K / 64;
  p.nstrips = g.W / 64;
  const long long tiles = (long long)p.ncb * p.nkb;
  const long long st1 = n1 * p.nstrips * g.H, st2 = n2 * p.nstrips * g.H;
  const long long slab1 = 4LL * g.K * 9 * g.C;
  long long want = std::max<long long>(1, (512 + tiles - 1) / tiles);
  const long long cap = std::max<long long>((256 + tiles - 1) / tiles, (32LL << 20) / slab1);
  want = std::min(want, cap);
  want = std::min<long long>(want, st1 + st2);
  long long a1 = n2 > 0 ? std::max<long long>(1, std::min(want - 1, (long long)((double)want * st1 / (st1 + st2) + 0.5)))
                        : want;
  if (n2 > 0 && want < 2) a1 = 1;
  const long long a2 = n2 > 0 ? std::max<long long>(1, want - a1) : 0;
  p.steps[0] = st1;
  p.steps[1] = st2;
  p.sps[0] = (st1 + a1 - 1) / a1;
  p.sps[1] = a2 ? (st2 + a2 - 1) / a2 : 1;
  p.s1 = (int)((st1 + p.sps[0] - 1) / p.sps[0]);
  p.splits = p.s1 + (a2 ? (int)((st2 + p.sps[1] - 1) / p.sps[1]) : 0);
  return p;
}

size_t halo3_ws_bytes(const ConvGeom& g, long long n1, long long n2) {
  const HaloPlan p = halo3_plan(g, n1, n2);
  return (size_t)p.splits * g.K * 9 * g.C * sizeof(float) + 256;
}

void launch_wgrad_halo3(int dt, const HaloArgs& a, hipStream_t s) {
  const unsigned blocks = (unsigned)(a.splits * a.ncb * a.nkb);
  if (dt == SSSEG_F16)
    hipLaunchKernelGGL(wgrad_halo3_kernel<f16_t>, dim3(blocks), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(wgrad_halo3_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, a);
}
