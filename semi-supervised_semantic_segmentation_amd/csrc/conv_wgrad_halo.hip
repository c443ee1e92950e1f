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
// The ring is HD = 2 row steps deep (5 input-row slots, 3 dY slots, 69 KB: two blocks per CU): while row y is
// multiplied, the pieces of rows y + 1 and y + 2 are in flight (one block per CU and one step ahead measured latency-
// bound: 1.9 us per step for 0.5 us of MFMA work).
// A split is a contiguous range of row steps t = ((n * nstrips) + strip) * H + y of one pixel segment (the merged
// supervised + consistency launch has two); a column change (new strip or image) drains the ring and reloads the
// three rows of the first step's taps.  Every
// split writes its fp32 partial of the whole dW into its own slab, which wgrad_reduce sums in split order
// (deterministic), exactly like the split-K path.
#include "conv_kernels.h"

namespace {

constexpr int HX_ROWS = 66;                 // ring row: 64 pixels + the halo pixel on each side
constexpr int HX_SLOT = 72 * 128;           // one input row segment (64 channels x 2 B per pixel), 8-row padded
constexpr int HD_SLOT = 64 * 128;           // one dY row segment
constexpr int HD = 2;                       // row steps in flight ahead of the one being multiplied
constexpr int HXS = HD + 3;                 // input-row ring slots: rows y-1 .. y+1 in use, y+2 .. y+HD+1 landing
constexpr int HDS = HD + 1;                 // dY ring slots
constexpr int H_SMEM = HXS * HX_SLOT + HDS * HD_SLOT;
constexpr int H_NL = 5;                     // vmcnt units of one row step per wave: 3 input pieces + 2 dY pieces

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

  // LDS-DMA pieces (the DMA writes lane-linearly: 16-byte chunk (lane & 7) of row lane >> 3 of an 8-row piece; the
  // bank swizzle is applied on the source side).  An input row segment is 66 pixel rows: every wave issues two full
  // 8-row pieces (rows 16w .. 16w + 15) and a quarter piece (rows 64 + 2w, 65 + 2w: lanes 0-15, the rest masked off,
  // rows 66+ never read), so every wave counts the same 3 + 2 vmcnt units per row step.
  const int lrow = lane >> 3;
  auto chunk_of = [&](int row) { return ((lane & 7) ^ hswz(row)) * 16; };
  auto x_off = [&](int n, int yy, int row, int strip) {
    const int xx = strip * 64 - 1 + row;
    if ((unsigned)yy >= (unsigned)H || row >= HX_ROWS || (unsigned)xx >= (unsigned)W) return OOB;
    return (unsigned)(((n * H + yy) * W + xx) * ldx + c0) * 2u + (unsigned)chunk_of(row);
  };
  auto issue_x = [&](int slot, int n, int yy, int strip) {   // input row yy of the strip -> ring slot
    char* base = smem + slot * HX_SLOT;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = 2 * wave + h;
      bldslds16_nt(xr, base + i * 1024, x_off(n, yy, 8 * i + lrow, strip), 0);
    }
    if (lane < 16) bldslds16_nt(xr, base + 8 * 1024 + wave * 256, x_off(n, yy, 64 + 2 * wave + lrow, strip), 0);
  };
  auto issue_dy = [&](int slot, int n, int y, int strip) {   // dY row y of the strip (64 pixels) -> dy slot
    char* base = smem + HXS * HX_SLOT + slot * HD_SLOT;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = 2 * wave + h;
      const int row = 8 * i + lrow;
      const unsigned off =
          (unsigned)(((n * H + y) * W + strip * 64 + row) * a.ldy + kb * 64) * 2u + (unsigned)chunk_of(row);
      bldslds16_nt(dr, base + i * 1024, off, 0);
    }
  };
  auto decode = [&](long long t, int& n, int& strip, int& y) {
    const long long q = t / H;
    y = (int)(t - q * H);
    n = (int)(q / a.nstrips);
    strip = (int)(q - (long long)n * a.nstrips);
  };
  // ring slots, rebased at every column start (the ring is drained there): input row yy in slot (yy + 1) % HXS,
  // dY row y in slot y % HDS
  auto xslot = [&](int yy) { return (yy + 1) % HXS; };

  f32x4 acc[9][4];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int gq = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  // fragment addresses inside a slot: rows (pixel) of the lane's lo / hi transposed reads, column chunk + byte
  const int xcol = 2 * wave + (p4 >> 1), dsub = 8 * (p4 & 1);

  auto compute = [&](int y) {
    const char* D = smem + HXS * HX_SLOT + (y % HDS) * HD_SLOT;
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
        const char* X = smem + xslot(y + r - 1) * HX_SLOT;
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

  if (t0 < t1) {
    int n, strip, y;
    decode(t0, n, strip, y);
    long long t = t0;
    while (true) {
      // column start (the ring is idle): the three input rows of row y's taps and dY row y, then the rows of the
      // next HD - 1 steps of this column
      const int last = (int)min((long long)(H - 1), y + (t1 - 1 - t));   // last row of this column in the range
      issue_x(xslot(y - 1), n, y - 1, strip);
      issue_x(xslot(y), n, y, strip);
      issue_x(xslot(y + 1), n, y + 1, strip);
      issue_dy(y % HDS, n, y, strip);
#pragma unroll
      for (int d = 1; d < HD; ++d)
        if (y + d <= last) {
          issue_x(xslot(y + d + 1), n, y + d + 1, strip);
          issue_dy((y + d) % HDS, n, y + d, strip);
        }
      for (;; ++y, ++t) {
        // row y's pieces landed: only the later steps already issued (at most HD - 1) may stay in flight
        ring_wait<H_NL, HD + 1>(min(HD - 1, last - y));
        __builtin_amdgcn_s_barrier();   // every wave's pieces of row y landed; the slots of row y - 2 are idle
        if (y + HD <= last) {
          issue_x(xslot(y + HD + 1), n, y + HD + 1, strip);
          issue_dy((y + HD) % HDS, n, y + HD, strip);
        }
        compute(y);
        if (y == last) break;
      }
      ++t;
      if (t >= t1) break;
      lds_barrier();   // every wave is done with the ring before the next column rewrites it
      decode(t, n, strip, y);
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
         g.ldy % 8 == 0 && g.ldy >= g.K;   // ldx >= C unless a virtual concat supplies channels >= c1 (caller)
}

// split plan: 2 resident blocks per CU over the chip, slabs capped at 64 MiB (>= one block per CU), splits shared out
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
  const long long cap = std::max<long long>((256 + tiles - 1) / tiles, (64LL << 20) / slab1);
  want = std::min(want, cap);
  if (g_knobs[10] != 100 && g_knobs[10] > 0) want = std::max<long long>(1, want * g_knobs[10] / 100);   // A/B
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
