// Binary Lovász-softmax on the device (losses.binary_lovasz_loss_with_logits losses.py:239-250 ->
// lovasz.lovasz_softmax lovasz.py:155-201 with classes=[1], per_image=True; lovasz_grad lovasz.py:19-31).
//
// Per image b (a segment of HW pixels):
//   label = argmax_c target[b][c][p] (first max),  fg = [label == 1],  e = |fg - logit[b][1][p]|
//   sort e descending (stable: ties keep pixel order; the reference's torch.sort is unstable, the loss
//   is invariant to the order inside a tie), F(i) = #fg among the first i+1 sorted pixels,
//   J(i) = 1 - (gts - F(i)) / (gts + (i+1) - F(i)),  g(i) = J(i) - J(i-1) (g(0) = J(0)),  loss_b = <e, g>
//   loss = sum_b loss_b * valid_b / (sum_b valid_b + 0.001), valid_b = [gts_b > 0]
//   d loss / d logit[b][1][p] = -sign(fg - x) * g(rank(p)) * valid_b / denom  (other channels 0)
//
// The sort is an LSD radix sort over all segments at once: 4 passes of 8-bit digits on the key
// ~bits(e) (ascending key = descending e; e >= 0 so float bits are monotone), values = pixel index | fg<<31.
// Each pass: per-(segment, tile) digit histograms -> per-segment exclusive scan in (digit, tile) order
// -> stable scatter (rank inside a tile from wave ballots + per-(slot, wave) digit counts).
// Then a tile scan of fg in sorted order gives F(i); J/g follow in fp32 exactly as lovasz_grad computes
// them; the dot accumulates in fp64.  Deterministic; no atomics on data.
#include "common.h"

namespace {

constexpr int LT = 256;              // threads per block
constexpr int ITEMS = 8;             // elements per thread per tile
constexpr int TILE = LT * ITEMS;     // 2048
constexpr int NW = LT / 64;

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// keys / values from the inputs
__global__ void lovasz_prep_kernel(const float* __restrict__ logits, const float* __restrict__ target, int64_t B,
                                   int C, int64_t HW, unsigned* __restrict__ keys, unsigned* __restrict__ vals) {
  const int64_t n = B * HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / HW, p = i - b * HW;
    const float* tb = target + b * C * HW + p;
    int lab = 0;
    float best = tb[0];
    for (int c = 1; c < C; ++c) {
      const float v = tb[(int64_t)c * HW];
      if (v > best) {   // torch.argmax: first maximal index
        best = v;
        lab = c;
      }
    }
    const unsigned fg = lab == 1;
    const float x = logits[b * C * HW + HW + p];
    const float e = fabsf((float)fg - x);
    keys[i] = ~__float_as_uint(e);
    vals[i] = (unsigned)p | (fg << 31);
  }
}

// hist[b][d][t] = count of digit d in tile t of segment b; dtot[b][d] += that count (integer atomics: exact, so the
// totals do not depend on the order of the adds; dtot zeroed before the pass)
__global__ void __launch_bounds__(LT) radix_hist_kernel(const unsigned* __restrict__ keys, int64_t HW, int T, int shift,
                                                        unsigned* __restrict__ hist, unsigned* __restrict__ dtot) {
  __shared__ unsigned cnt[256];
  const int b = blockIdx.y, t = blockIdx.x;
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const unsigned* kb = keys + (int64_t)b * HW;
  const int64_t base = (int64_t)t * TILE;
#pragma unroll
  for (int s = 0; s < ITEMS; ++s) {
    const int64_t i = base + s * LT + threadIdx.x;
    if (i < HW) atomicAdd(&cnt[(kb[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  const unsigned c = cnt[threadIdx.x];
  hist[((int64_t)b * 256 + threadIdx.x) * T + t] = c;
  if (c) atomicAdd(&dtot[b * 256 + threadIdx.x], c);
}

// per segment: exclusive scan of hist[b] (digit-major) in place, one wave per (segment, digit) row: the row's base is
// the sum of the earlier digits' totals (dtot), then a carried wave scan along the T tiles.  (One 1024-thread block
// per segment walking 32 entries per thread in sequence took 52 us per pass at 16 x 512^2: a chain of dependent
// loads in 16 blocks.)
__global__ void __launch_bounds__(256) seg_rowscan_kernel(unsigned* __restrict__ hist, const unsigned* __restrict__ dtot,
                                                          int T) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.y, d = blockIdx.x * 4 + (threadIdx.x >> 6);
  const unsigned* tb = dtot + b * 256;
  unsigned base = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int dd = lane * 4 + k;
    base += dd < d ? tb[dd] : 0u;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) base += __shfl_xor(base, o, 64);
  unsigned* row = hist + ((int64_t)b * 256 + d) * T;
  unsigned carry = base;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    const unsigned v = t < T ? row[t] : 0u;
    unsigned inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (t < T) row[t] = carry + inc - v;
    carry += __shfl(inc, 63, 64);
  }
}

// stable scatter of one pass
__global__ void __launch_bounds__(LT) radix_scatter_kernel(const unsigned* __restrict__ kin, const unsigned* __restrict__ vin,
                                                           unsigned* __restrict__ kout, unsigned* __restrict__ vout,
                                                           int64_t HW, int T, int shift, const unsigned* __restrict__ off) {
  __shared__ unsigned cnt[ITEMS * NW][256];   // per (slot, wave) digit counts -> exclusive bases
  const int b = blockIdx.y, t = blockIdx.x;
  const int wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < ITEMS * NW * 256; i += LT) (&cnt[0][0])[i] = 0;
  __syncthreads();
  const int64_t seg = (int64_t)b * HW, base = (int64_t)t * TILE;
  unsigned key[ITEMS], val[ITEMS], dig[ITEMS], lrank[ITEMS];
#pragma unroll
  for (int s = 0; s < ITEMS; ++s) {
    const int64_t i = base + s * LT + threadIdx.x;
    const bool ok = i < HW;
    key[s] = ok ? kin[seg + i] : 0u;
    val[s] = ok ? vin[seg + i] : 0u;
    dig[s] = ok ? (key[s] >> shift) & 255u : 256u;
    // lanes of this wave with the same digit: AND of 9 ballots (bit 8 separates the invalid sentinel)
    unsigned long long m = ~0ull;
#pragma unroll
    for (int bit = 0; bit < 9; ++bit) {
      const unsigned long long bb = __ballot((dig[s] >> bit) & 1u);
      m &= ((dig[s] >> bit) & 1u) ? bb : ~bb;
    }
    lrank[s] = (unsigned)__popcll(m & lanemask_lt());
    if (ok && lrank[s] == 0) cnt[s * NW + wave][dig[s]] = (unsigned)__popcll(m);
  }
  __syncthreads();
  // exclusive scan over (slot, wave) per digit; thread = digit
  {
    const int d = threadIdx.x;
    unsigned run = off[((int64_t)b * 256 + d) * T + t];
    for (int q = 0; q < ITEMS * NW; ++q) {
      const unsigned v = cnt[q][d];
      cnt[q][d] = run;
      run += v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < ITEMS; ++s) {
    if (dig[s] > 255u) continue;
    const unsigned pos = cnt[s * NW + wave][dig[s]] + lrank[s];
    kout[seg + pos] = key[s];
    vout[seg + pos] = val[s];
  }
}

// fg count per (segment, tile) of the sorted order
__global__ void __launch_bounds__(LT) fg_count_kernel(const unsigned* __restrict__ vals, int64_t HW, int T,
                                                      unsigned* __restrict__ tile_fg) {
  __shared__ unsigned red[NW];
  const int b = blockIdx.y, t = blockIdx.x;
  const int64_t seg = (int64_t)b * HW, base = (int64_t)t * TILE;
  unsigned c = 0;
#pragma unroll
  for (int s = 0; s < ITEMS; ++s) {
    const int64_t i = base + s * LT + threadIdx.x;
    if (i < HW) c += vals[seg + i] >> 31;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned tot = 0;
    for (int w = 0; w < NW; ++w) tot += red[w];
    tile_fg[(int64_t)b * (T + 1) + t] = tot;
  }
}

// per segment: exclusive scan of tile_fg[b][0..T) and gts into tile_fg[b][T]
__global__ void fg_scan_kernel(unsigned* __restrict__ tile_fg, int T) {
  unsigned* d = tile_fg + (int64_t)blockIdx.x * (T + 1);
  if (threadIdx.x == 0) {
    unsigned run = 0;
    for (int i = 0; i < T; ++i) {
      const unsigned v = d[i];
      d[i] = run;
      run += v;
    }
    d[T] = run;
  }
}

__device__ __forceinline__ float jac(float gts, float F, float k1) {   // k1 = i + 1
  return 1.f - (gts - F) / (gts + (k1 - F));
}

// Lovász gradient in sorted order, scattered back to pixels (gpix[b][p]); fp64 partial dots per tile
__global__ void __launch_bounds__(LT) lovasz_grad_kernel(const unsigned* __restrict__ keys,
                                                         const unsigned* __restrict__ vals, int64_t HW, int T,
                                                         const unsigned* __restrict__ tile_fg,
                                                         float* __restrict__ gpix, double* __restrict__ dots) {
  __shared__ unsigned wsum[NW];
  __shared__ double dred[NW];
  const int b = blockIdx.y, t = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t seg = (int64_t)b * HW, base = (int64_t)t * TILE;
  const unsigned* tf = tile_fg + (int64_t)b * (T + 1);
  const float gts = (float)tf[T];
  // this thread owns ITEMS consecutive sorted positions: i = base + threadIdx.x*ITEMS + s
  unsigned fg[ITEMS], v[ITEMS];
  unsigned mine = 0;
#pragma unroll
  for (int s = 0; s < ITEMS; ++s) {
    const int64_t i = base + (int64_t)threadIdx.x * ITEMS + s;
    v[s] = i < HW ? vals[seg + i] : 0u;
    fg[s] = v[s] >> 31;
    mine += fg[s];
  }
  // block exclusive scan of per-thread fg counts
  unsigned incl = mine;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  unsigned wbase = 0;
  for (int w = 0; w < wave; ++w) wbase += wsum[w];
  unsigned F = tf[t] + wbase + incl - mine;   // fg count before this thread's first item
  double dot = 0.0;
#pragma unroll
  for (int s = 0; s < ITEMS; ++s) {
    const int64_t i = base + (int64_t)threadIdx.x * ITEMS + s;
    if (i >= HW) break;
    const float Fprev = (float)F;
    F += fg[s];
    float g = jac(gts, (float)F, (float)(i + 1));
    if (i > 0) g = g - jac(gts, Fprev, (float)i);
    const float e = __uint_as_float(~keys[seg + i]);
    dot += (double)e * (double)g;
    gpix[seg + (v[s] & 0x7fffffffu)] = g;
  }
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
  if (lane == 0) dred[wave] = dot;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < NW; ++w) s += dred[w];
    dots[(int64_t)b * T + t] = s;
  }
}

// loss and the per-image scale valid_b / denom (kept in ws for the gradient).  One wave per image sums its T tile
// dots (lane-strided, then a fixed xor tree: deterministic); lane 0 of block thread 0 combines the B images in order.
// (A single thread walking all B*T dots was a chain of dependent loads: 122 us at B=16, T=128.)
constexpr int FIN_T = 1024;
__global__ void __launch_bounds__(FIN_T) lovasz_final_kernel(const double* __restrict__ dots,
                                                             const unsigned* __restrict__ tile_fg, int B, int T,
                                                             float* __restrict__ loss_out, float* __restrict__ wscale) {
  extern __shared__ double img_dot[];   // [B] dots, then [B] valid flags
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = FIN_T / 64;
  for (int b = wv; b < B; b += nw) {
    double s = 0.0;
    for (int t = lane; t < T; t += 64) s += dots[(int64_t)b * T + t];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) {
      img_dot[b] = s;
      img_dot[B + b] = tile_fg[(int64_t)b * (T + 1) + T] > 0 ? 1.0 : 0.0;
    }
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float nvalid = 0.f;
  for (int b = 0; b < B; ++b) nvalid += (float)img_dot[B + b];
  const float denom = nvalid + 0.001f;
  float total = 0.f;
  for (int b = 0; b < B; ++b) {
    const float valid = (float)img_dot[B + b];
    total += (float)img_dot[b] * valid;   // losses.py:248: loss += lovasz_softmax(...) * mask_sample
    if (wscale) wscale[b] = valid / denom;
  }
  if (loss_out) loss_out[0] = total / denom;
}

__global__ void lovasz_bwd_kernel(const float* __restrict__ logits, const float* __restrict__ target, int64_t B, int C,
                                  int64_t HW, const float* __restrict__ gpix, const float* __restrict__ wscale,
                                  const float* __restrict__ gout, float* __restrict__ grad) {
  const int64_t n = B * HW;
  const float go = gout ? gout[0] : 1.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / HW, p = i - b * HW;
    const float* tb = target + b * C * HW + p;
    int lab = 0;
    float best = tb[0];
    for (int c = 1; c < C; ++c) {
      const float v = tb[(int64_t)c * HW];
      if (v > best) {
        best = v;
        lab = c;
      }
    }
    const float d = (lab == 1 ? 1.f : 0.f) - logits[b * C * HW + HW + p];
    const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    float* gb = grad + b * C * HW + p;
    for (int c = 0; c < C; ++c) gb[(int64_t)c * HW] = 0.f;
    gb[HW] = -sg * gpix[i] * wscale[b] * go;
  }
}

struct Ws {
  unsigned *ka, *va, *kb, *vb, *hist, *tile_fg, *dtot;
  float *gpix, *wscale;
  double* dots;
};

int64_t tiles_of(int64_t HW) { return (HW + TILE - 1) / TILE; }

size_t ws_layout(int64_t B, int64_t HW, char* p, Ws* w) {
  const int64_t n = B * HW, T = tiles_of(HW);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = p ? p + off : nullptr;
    off += (bytes + 255) / 256 * 256;
    return q;
  };
  char* ka = take(4 * n);
  char* va = take(4 * n);
  char* kb = take(4 * n);
  char* vb = take(4 * n);
  char* hist = take(4 * (size_t)B * 256 * T);
  char* tf = take(4 * (size_t)B * (T + 1));
  char* dots = take(8 * (size_t)B * T);
  char* wsc = take(4 * (size_t)B);
  char* dt = take(4 * (size_t)B * 256 * 4);   // per pass: digit totals of each segment
  if (w) {
    w->dtot = (unsigned*)dt;
    w->ka = (unsigned*)ka; w->va = (unsigned*)va; w->kb = (unsigned*)kb; w->vb = (unsigned*)vb;
    w->hist = (unsigned*)hist; w->tile_fg = (unsigned*)tf; w->dots = (double*)dots; w->wscale = (float*)wsc;
    w->gpix = (float*)kb;   // the sorted data ends in (ka, va); kb is free afterwards
  }
  return off;
}

// sort + Lovász gradient per pixel + loss (shared by fwd and bwd)
int lovasz_core(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW, float* loss_out, Ws& w,
                hipStream_t s) {
  const int64_t n = B * HW;
  const int T = (int)tiles_of(HW);
  hipLaunchKernelGGL(lovasz_prep_kernel, dim3(ssseg_grid(n, 256)), dim3(256), 0, s, logits, target, B, (int)C, HW,
                     w.ka, w.va);
  unsigned *kin = w.ka, *vin = w.va, *kout = w.kb, *vout = w.vb;
  (void)hipMemsetAsync(w.dtot, 0, sizeof(unsigned) * (size_t)B * 256 * 4, s);   // the four passes' digit totals
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    unsigned* dtot = w.dtot + (size_t)pass * B * 256;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(T, (unsigned)B), dim3(LT), 0, s, kin, HW, T, shift, w.hist, dtot);
    hipLaunchKernelGGL(seg_rowscan_kernel, dim3(64, (unsigned)B), dim3(256), 0, s, w.hist, dtot, T);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(T, (unsigned)B), dim3(LT), 0, s, kin, vin, kout, vout, HW, T, shift,
                       w.hist);
    unsigned* tk = kin; kin = kout; kout = tk;
    unsigned* tv = vin; vin = vout; vout = tv;
  }
  // 4 passes: sorted data is back in (ka, va)
  hipLaunchKernelGGL(fg_count_kernel, dim3(T, (unsigned)B), dim3(LT), 0, s, w.va, HW, T, w.tile_fg);
  hipLaunchKernelGGL(fg_scan_kernel, dim3((unsigned)B), dim3(64), 0, s, w.tile_fg, T);
  hipLaunchKernelGGL(lovasz_grad_kernel, dim3(T, (unsigned)B), dim3(LT), 0, s, w.ka, w.va, HW, T, w.tile_fg, w.gpix,
                     w.dots);
  hipLaunchKernelGGL(lovasz_final_kernel, dim3(1), dim3(FIN_T), 2 * B * sizeof(double), s, w.dots, w.tile_fg, (int)B, T, loss_out, w.wscale);
  return 0;
}

}  // namespace

extern "C" size_t ssseg_lovasz_workspace_bytes(int64_t B, int64_t HW) {
  if (B < 1 || HW < 1) return 0;
  return ws_layout(B, HW, nullptr, nullptr);
}

extern "C" int ssseg_lovasz_fwd(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW,
                                float* loss_out, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!logits || !target || !loss_out || B < 1 || B > 4096 || C < 2 || HW < 1 || HW > 0x7fffffff) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_lovasz_workspace_bytes(B, HW)) return SSSEG_EWORKSPACE;
  Ws w;
  ws_layout(B, HW, (char*)ws, &w);
  lovasz_core(logits, target, B, C, HW, loss_out, w, (hipStream_t)stream);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_lovasz_bwd(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW,
                                const float* gout, float* grad_out, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!logits || !target || !grad_out || B < 1 || B > 4096 || C < 2 || HW < 1 || HW > 0x7fffffff) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_lovasz_workspace_bytes(B, HW)) return SSSEG_EWORKSPACE;
  Ws w;
  ws_layout(B, HW, (char*)ws, &w);
  hipStream_t s = (hipStream_t)stream;
  lovasz_core(logits, target, B, C, HW, nullptr, w, s);
  hipLaunchKernelGGL(lovasz_bwd_kernel, dim3(ssseg_grid(B * HW, 256)), dim3(256), 0, s, logits, target, B, (int)C, HW,
                     w.gpix, w.wscale, gout, grad_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

// the backward of a preceding ssseg_lovasz_fwd on the same inputs and workspace: the per-pixel Lovász gradient and the
// per-image scale it left in ws are scattered into grad_out (one launch; the sort is not repeated)
extern "C" int ssseg_lovasz_bwd_from_fwd(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW,
                                         const float* gout, float* grad_out, const void* ws, size_t ws_bytes,
                                         ssseg_stream_t stream) {
  if (!logits || !target || !grad_out || B < 1 || B > 4096 || C < 2 || HW < 1 || HW > 0x7fffffff) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_lovasz_workspace_bytes(B, HW)) return SSSEG_EWORKSPACE;
  Ws w;
  ws_layout(B, HW, (char*)ws, &w);
  hipLaunchKernelGGL(lovasz_bwd_kernel, dim3(ssseg_grid(B * HW, 256)), dim3(256), 0, (hipStream_t)stream, logits,
                     target, B, (int)C, HW, w.gpix, w.wscale, gout, grad_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}
