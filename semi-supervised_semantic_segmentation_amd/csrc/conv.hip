// Implicit-GEMM convolution engine: host dispatch, variant autotune, register-staged launches, weight
// packing.  Device code: conv_kernels.h; LDS-DMA configs: conv_glds_*.hip; weight gradients: conv_wgrad.hip.
#include <mutex>
#include <algorithm>
#include <unordered_map>
#include <vector>

#include "conv_kernels.h"

int g_knobs[17] = {0, -1, 0, 0, 0, 1, 0, 0, 0, 0, 100, 0, 0, 0, 0, 0, 0};   // runtime variant switches (ssseg_set_knob)
// (knob 1, the register-staged kernel's fp32-atomic split-K, stays off: measured a net loss on the C2 step (r2u) and its
// sums are order-dependent; knob 14 is the deterministic split-K of the LDS-DMA configs)
thread_local int t_dsplit = 1;

// the ticket pool of the in-launch reductions (deterministic split-K): zero when the library loads, each ticket reset
// by the block that draws last, so a launch only needs a range no launch in flight with it uses
constexpr long long TICKET_POOL = 1 << 20;
__device__ unsigned g_ticket_pool[TICKET_POOL];

unsigned* ticket_slots(long long n) {
  static unsigned* const base = [] {
    void* p = nullptr;
    return hipGetSymbolAddress(&p, HIP_SYMBOL(g_ticket_pool)) == hipSuccess ? (unsigned*)p : nullptr;
  }();
  static std::mutex mu;
  static long long next = 0;
  if (!base || n <= 0 || n > TICKET_POOL / 16) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (next + n > TICKET_POOL) next = 0;
  unsigned* p = base + next;
  next += n;
  return p;
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

// one launch repacks many convs: blockIdx.y = descriptor, blocks along x grid-stride over its tiles.  A tile is KG
// consecutive output rows k x CC input channels x every tap: the fp32 source sub-block is read in source order
// (coalesced: [k][c][taps] runs for layout 0, [c][k][taps] runs for layout 1) into LDS, then written in packed order
// [k][rr][ss][c] with 8 channels per thread (16-byte stores for the 16-bit packs).  (The per-element gather of the
// earlier kernel -- three integer divisions and one strided 4-byte read per packed element -- took 156 us per
// C2 repack of the student's two layouts; 2 per step.)  32-bit index math: the host checks every pack < 2^31 elements.
constexpr int PK_KG = 4;
constexpr int PK_MAXD = 2048;   // descriptors per launch (the host splits larger batches)
// a / d for 0 <= a < 8192 and d >= 1 by a float reciprocal (3 VALU instead of an integer division's ~40): (a + 0.5) / d
// lies >= 0.5 / d away from every integer and the two roundings err by < 1.2e-7 relative, i.e. < (a + 0.5) * 1.2e-7 / d
// < 0.5 / d while a < 4e6: the truncation is exact
__device__ __forceinline__ int pk_div(int a, float inv_d) { return (int)(((float)a + 0.5f) * inv_d); }
// channels per tile: the largest power of two (8 .. 1024) whose PK_KG x CC x (RS | 1) floats fit the LDS tile, so a 1x1
// conv's tile holds 4096 weights (with 64 channels per tile the ResNet's 1x1 layers made ~150K tiny tiles per repack)
__device__ __forceinline__ int pk_cc(int RS) {
  int cc = 1024;
  while (cc > 8 && PK_KG * cc * (RS | 1) > PK_KG * 64 * 17) cc >>= 1;
  return cc;
}
__device__ __forceinline__ int pk_tiles(const ssseg_pack_desc& d) {
  const int RS = (int)(d.Rs * d.Ss);
  if (RS > 135) return 0;   // (host contract: filters of <= 135 taps, ssseg.h)
  return (int)((d.Kd + PK_KG - 1) / PK_KG) * (int)((d.Cp + pk_cc(RS) - 1) / pk_cc(RS));
}

template <typename T>
__global__ void __launch_bounds__(256) weight_pack_batch_kernel(const ssseg_pack_desc* __restrict__ descs, int n) {
  __shared__ float lds[PK_KG * 64 * 17];
  __shared__ int pre[PK_MAXD + 1];   // tile-count prefix sums of the descriptors (the flat tile space of the launch)
  if (threadIdx.x < 64) {
    int carry = 0;
    const int lane = threadIdx.x;
    for (int base = 0; base < n; base += 64) {
      const int d = base + lane;
      int v = d < n ? pk_tiles(descs[d]) : 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
      }
      if (d < n) pre[d + 1] = carry + v;
      carry += __shfl(v, 63, 64);
    }
    if (lane == 0) pre[0] = 0;
  }
  __syncthreads();
  const int total = pre[n];
  for (int g = blockIdx.x; g < total; g += gridDim.x) {
    int lo = 0, hi = n - 1;   // the descriptor d with pre[d] <= g < pre[d + 1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= g) lo = mid;
      else hi = mid - 1;
    }
    const ssseg_pack_desc& d = descs[lo];
    const int tile = g - pre[lo];
    const int Cp = (int)d.Cp, Sn = (int)d.Sn, Rn = (int)d.Rn, Cd = (int)d.Cd, Kr = (int)d.Kr, Kd = (int)d.Kd,
              Ss = (int)d.Ss, r0 = (int)d.r0, rstep = (int)d.rstep, s0 = (int)d.s0, sstep = (int)d.sstep;
    const int RS = (int)d.Rs * Ss, RSP = RS | 1;   // odd LDS row stride: the 8-channel reads are conflict-free
    const int CC = pk_cc(RS);
    const bool l0 = d.layout == 0;
    const float* src = d.src;
    T* dst = (T*)d.dst;
    const int ncc = (Cp + CC - 1) / CC, taps = Rn * Sn;
    const int k0 = (tile / ncc) * PK_KG, c0 = (tile % ncc) * CC;
    const float iRS = 1.f / (float)RS, iCRS = 1.f / (float)(CC * RS), iKRS = 1.f / (float)(PK_KG * RS);
    // phase 1: the source sub-block in source order; every thread's loads are issued before the first LDS write (one
    // memory round trip per tile instead of one per element row: n1 / 256 <= 17)
    const int n1 = PK_KG * CC * RS;
    constexpr int PK_IT = 17;
    float v1[PK_IT];
    int o1[PK_IT];
#pragma unroll
    for (int it = 0; it < PK_IT; ++it) {
      const int i = threadIdx.x + it * 256;
      o1[it] = -1;
      v1[it] = 0.f;
      if (i >= n1) continue;
      int kk, c, t;
      if (l0) {   // [k][c][t]: contiguous over (c, t) per k
        kk = pk_div(i, iCRS);
        const int rem = i - kk * CC * RS;
        c = pk_div(rem, iRS);
        t = rem - c * RS;
      } else {    // [c][k][t]: contiguous over (k, t) per c
        c = pk_div(i, iKRS);
        const int rem = i - c * PK_KG * RS;
        kk = pk_div(rem, iRS);
        t = rem - kk * RS;
      }
      const int k = k0 + kk, cc = c0 + c;
      o1[it] = (kk * CC + c) * RSP + t;
      if (k < Kr && cc < Cd) v1[it] = src[l0 ? (k * Cd + cc) * RS + t : (cc * Kr + k) * RS + t];
    }
#pragma unroll
    for (int it = 0; it < PK_IT; ++it)
      if (o1[it] >= 0) lds[o1[it]] = v1[it];
    __syncthreads();
    // phase 2: packed order [k][rr][ss][c], 8 channels per thread
    const int c8n = CC / 8, lc8 = __builtin_ctz((unsigned)c8n);
    const int n2 = PK_KG * taps * c8n;
    const float iTC = 1.f / (float)(taps * c8n), iSn = 1.f / (float)Sn;
    for (int j = threadIdx.x; j < n2; j += 256) {
      const int kk = pk_div(j, iTC);
      const int rem = j - kk * taps * c8n;
      const int tt = rem >> lc8, c8 = rem & (c8n - 1);
      const int k = k0 + kk, c = c0 + c8 * 8;
      if (k >= Kd || c >= Cp) continue;
      const int rr = pk_div(tt, iSn), ss = tt - rr * Sn;
      const int t = (r0 + rr * rstep) * Ss + s0 + ss * sstep;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = lds[(kk * CC + c8 * 8 + e) * RSP + t];
      const int o = (k * taps + tt) * Cp + c;
      if (c + 8 <= Cp && (Cp & 7) == 0) {
        Out8<T>::st(dst + o, v);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (c + e < Cp) io<T>::st(dst, o + e, v[e]);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
namespace {

// returns the tile height BM of the launched config (the fused BN statistics write ceil(M / BM) partial rows)
template <typename TO>
int launch_glds_cfg(int cfg, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep_in,
                    unsigned xb, unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2 = nullptr,
                    unsigned x2b = 0) {
  Epi<TO> ep = ep_in;
  ep.sdbg = g_knobs[12];
  switch (cfg) {
    case 1:
    case 2:
    case 3: return launch_glds_grp_a<TO>(cfg, x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 4:
    case 6:
    case 18:
    case 19:
    case 20: return launch_glds_grp_d<TO>(cfg, x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 21:
    case 22:
    case 23: return launch_glds_grp_e<TO>(cfg, x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    case 24: return launch_hconv3<TO>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);   // halo-tiled 3x3 (-1: n/a)
    case 28: return launch_hconv3<TO>(x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b, 1);   // its two-blocks-per-CU form
    case 25: return launch_hconv3s<TO>(x, w, y, g, ep, xb, s, ws, ph, x2);   // its 32 -> 32-channel form
    case 26: return launch_pw<TO>(4, x, w, y, g, ep, s, ws, ph, x2);   // pointwise, 64-pixel wave tiles
    case 27: return launch_pw<TO>(2, x, w, y, g, ep, s, ws, ph, x2);   // pointwise, 32-pixel wave tiles
    case 5:
    case 7:
    case 8:
    case 9:
    case 12: return launch_glds_grp_b<TO>(cfg, x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
    default: return launch_glds_grp_c<TO>(cfg, x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
  }
}

// ---- bf16 variant choice: per-geometry autotune cache ----------------------------------------
// Every variant accumulates the same 32-deep MFMA k-sequence in the same order, so the choice changes
// speed, never results (tests/test_hip_layers.py::test_conv_variants_bitwise).  Variant 0 is the
// register-staged kernel, 1..10 and 12..23 the LDS-DMA configs, 24 the halo-tiled 3x3 kernel (conv_hconv3.hip; only
// where it applies).  With knob 5 on (default) an unseen geometry is timed once over the candidates on the caller's
// stream (HIP events) and the fastest is cached.
constexpr int kCandidates[] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  10, 12, 13, 14,
                                15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28};
std::unordered_map<unsigned long long, int> g_variant;
std::mutex g_variant_mu;

static unsigned long long geom_key(const ConvGeom& g, int tag) {
  const long long v[] = {g.N, g.H, g.W, g.C, g.ldx, g.OH, g.OW, g.K, g.R, g.S, g.sy, g.sx, g.dy, g.dx, g.py, g.px,
                         g.outH, g.outW, g.osy, g.osx, g.ldy, g.ldw, g.c1b, g.ldx2, tag};
  unsigned long long h = 1469598103934665603ull;
  for (long long e : v) h = (h ^ (unsigned long long)e) * 1099511628211ull;
  return h;
}

static int heuristic_variant(const ConvGeom& g) {
  auto tiles = [&](int bm, int bn) { return ((g.M + bm - 1) / bm) * ((g.K + bn - 1) / bn); };
  if (g.KK <= 128) return 0;
  if (g.C % 64) return 5;   // general-k loader: 64-wide n-tiles only
  if (g.K > 64) return tiles(256, 128) >= 128 ? 6 : (tiles(128, 128) >= 256 ? 8 : 5);
  return tiles(64, 64) < 512 ? 10 : 0;
}

// Deterministic split-K plan (knob 14: 0 = this rule, -1 = off, 2 / 4 / 8 = forced S): a static function of the
// contraction, never of timings, so the summation order -- and with it every output bit -- is the same in every run and
// for every tile config the autotuner may pick.  Tile-starved launches with long k-loops: fewer than 512 nominal
// 128 x 64 output tiles (over all phases) and >= 64 k-tiles of 64.  Measured (tools/split_ab.py, bs 16, device time
// of graph-replayed launches): 1152->128 3x3 @32^2 78.5 -> 56.5 us (S = 2; S = 4 no better), 512->512 3x3 @16^2
// 37.9 -> 33.2, 512->512 3x3/s2 @32^2 36.9 -> 33.0, ConvTranspose2d 2048->128 @16^2 (4 phases) 63.9 -> 49.2; slower
// with S = 2 where the k-loop is short or the tiles already fill the chip (2048->512 1x1 @16^2, nk = 32: 16.7 -> 21.1;
// 256->256 3x3 @32^2, 512 tiles: 28.3 -> 35.2), and S = 4 / 8 lose everywhere but the longest contractions.
static int dsplit_plan(const ConvGeom& g, int nph) {
  const int kn = g_knobs[14];
  if (kn < 0 || g.KK == 0) return 1;
  const int nk = (g.C % 64 == 0) ? g.R * g.S * (g.C / 64) : (g.KK + 63) / 64;
  if (kn > 0) return (kn == 2 || kn == 4 || kn == 8) && nk >= kn ? kn : 1;
  const long long t = (long long)nph * ((g.M + 127) / 128) * ((g.K + 63) / 64);
  if (t < 512 && nk >= 64) return (t < 128 && nk >= 128) ? 4 : 2;
  // few tiles over a moderate contraction (HarDNet's growth layers at 8^2-32^2: 16-128 tiles, 8-63 k-tiles): the
  // largest S with at most 512 blocks and at least 4 k-tiles per slice
  if (t < 256 && nk >= 8) {
    int S = 8;
    while (S > 1 && (t * S > 512 || nk < 4 * S)) S >>= 1;
    return S;
  }
  return 1;
}

// x2: second source of a virtual concat input (LDS-DMA configs only: the register-staged kernel returns -1)
template <typename T, typename TO>
int run_variant(int v, const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph = nullptr, const void* x2 = nullptr,
                unsigned x2b = 0) {
  t_pw_rows = -1;
  // a split launch runs on the LDS-DMA configs only (the register-staged, halo and pointwise kernels do not split)
  if (t_dsplit > 1 && (v == 0 || v >= 24)) return -1;
  if constexpr (sizeof(TO) == 2) {
    if (v != 0) return launch_glds_cfg<TO>(v, x, w, y, g, ep, xb, wb, s, ws, ph, x2, x2b);
  }
  if (x2) return -1;
  ws = nullptr;   // (the register-staged kernel's fp32-atomic split-K stays off, knob 1)
  if (ph && ph->n > 1) {   // register-staged kernel: one launch per phase
    int bm = 0;
    long long rows = 0;
    for (int p = 0; p < ph->n; ++p) {
      ConvGeom gp = g;
      gp.py = ph->py[p];
      gp.px = ph->px[p];
      gp.ooy = ph->ooy[p];
      gp.oox = ph->oox[p];
      Epi<TO> ep2 = ep;
      if (ep.stats) ep2.stats = ep.stats + rows * 2 * ep.sld;
      bm = dispatch_regstaged<T, TO>(x, ph->w[p], y, gp, ep2, ws, s);
      if (bm <= 0) return bm;
      rows += (g.M + bm - 1) / bm;
    }
    return bm;
  }
  return dispatch_regstaged<T, TO>(x, w, y, g, ep, ws, s);
}

// *cache_it = false when the choice is only the heuristic's stand-in (the stream is being captured: nothing may be
// timed, and the geometry is tuned at its next eager launch)
template <typename T, typename TO>
int tune_variant(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, unsigned xb,
                 unsigned wb, hipStream_t s, float* ws, const PhaseTab* ph, const void* x2, unsigned x2b,
                 bool* cache_it) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const int heur = x2 && heuristic_variant(g) == 0 ? 5 : heuristic_variant(g);
  *cache_it = true;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
    *cache_it = false;
    return heur;
  }
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return heuristic_variant(g);
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return heuristic_variant(g);
  }
  int best = heur;
  float best_ms = 1e30f;
  static const bool log = getenv("SSSEG_TUNE_LOG") != nullptr;   // one line per tuned geometry (stderr)
  char line[512];
  int len = log ? snprintf(line, sizeof line, "tune N%d %dx%d C%d -> %dx%d K%d %dx%d s%d d%d out%dx%d/%d ep%d%d:",
                           g.N, g.H, g.W, g.C, g.OH, g.OW, g.K, g.R, g.S, g.sy, g.dy, g.outH, g.outW, g.osy,
                           ep.scale ? 1 : 0, ep.aux ? 1 : 0) : 0;
  // every variant (with the launch's split-K plan t_dsplit, where there is one: configs that cannot split are skipped)
  {
    const int split = t_dsplit > 1;
    float* wsv = ws;
    for (int v : kCandidates) {
      // a virtually padded contraction (C > ldx: the host's vpad) runs on the bounded LDS-DMA loads only
      if (g.C > g.ldx && (v == 0 || v == 24 || v == 28)) continue;
      // warm (code load, caches); a variant that cannot run this launch (-1) is skipped
      if (run_variant<T, TO>(v, x, w, y, g, ep, xb, wb, s, wsv, ph, x2, x2b) <= 0) continue;
      float ms = 1e30f;
      static const int reps = [] {   // best of `reps` timed launches (SSSEG_TUNE_REPS: A/B of the tuning depth)
        const char* e = getenv("SSSEG_TUNE_REPS");
        const int v = e ? atoi(e) : 5;
        return v >= 1 && v <= 64 ? v : 5;
      }();
      for (int rep = 0; rep < reps; ++rep) {
        (void)hipEventRecord(e0, s);
        run_variant<T, TO>(v, x, w, y, g, ep, xb, wb, s, wsv, ph, x2, x2b);
        (void)hipEventRecord(e1, s);
        float t = 1e30f;
        if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&t, e0, e1) == hipSuccess) ms = std::min(ms, t);
      }
      if (log && len > 0 && len < (int)sizeof line - 24)
        len += snprintf(line + len, sizeof line - len, " %d%s:%.0f", v, split ? "s" : "", ms * 1e3f);
      if (ms < best_ms) {
        best_ms = ms;
        best = v;
      }
    }
  }
  if (log) fprintf(stderr, "%s -> %d\n", line, best);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

// x2 (virtual concat, g.c1b / g.ldx2 set): LDS-DMA configs only; returns -1 where they cannot run the launch.
// ws (sized by ssseg_conv_igemm_workspace_bytes) enables the deterministic split-K plan of the contraction.
struct DsplitScope {   // t_dsplit for the duration of one dispatch
  explicit DsplitScope(int S) { t_dsplit = S; }
  ~DsplitScope() { t_dsplit = 1; }
};

template <typename T, typename TO>
int dispatch_igemm(const void* x, const void* w, void* y, const ConvGeom& g, const Epi<TO>& ep, float* ws,
                   hipStream_t s, const PhaseTab* ph = nullptr, const void* x2 = nullptr) {
  if constexpr (sizeof(T) == 2 && sizeof(TO) == 2) {
    const long long xb = (long long)g.N * g.H * g.W * g.ldx * 2, wb = (long long)g.K * g.ldw * 2;
    const long long x2b = x2 ? (long long)g.N * g.H * g.W * g.ldx2 * 2 : 0;
    // C % 64 != 0 (general-k loader, 64-wide n-tiles): any C % 8 == 0 (geom_ok), no virtual concat
    if (sizeof(TO) == 2 && g_knobs[3] == 0 && (g.C % 64 == 0 || !x2) && g.ldx % 8 == 0 && g.ldw % 8 == 0 && g.ldw == g.KK &&
        g.K > 16 && xb < 0x7fffffffLL && wb < 0x7fffffffLL && x2b < 0x7fffffffLL && (!x2 || g.ldx2 % 8 == 0)) {
      const int nph = ph ? ph->n : 1;
      const int S = ws ? dsplit_plan(g, nph) : 1;
      DsplitScope scope(S);
      float* wsv = S > 1 ? ws : nullptr;
      int v = g_knobs[4];
      if (v < 0) v = 0;
      if (v == 0) {
        const unsigned long long key =
            geom_key(g, (int)sizeof(TO) * 8 + (ep.stats ? 4 : 0) + (ep.res ? 2 : 0) + (ep.scale ? 1 : 0) + 16 * S +
                        256 * nph + (x2 ? 4096 * (g.c1b + 1) : 0) + (ep.y2 ? (1 << 24) : 0) + (ep.rmask ? (1 << 25) : 0) + (ep.gstat ? (1 << 26) : 0));
        std::lock_guard<std::mutex> lk(g_variant_mu);
        auto it = g_variant.find(key);
        if (it != g_variant.end()) {
          v = it->second;
        } else {
          bool cache_it = true;
          v = g_knobs[5] ? tune_variant<T, TO>(x, w, y, g, ep, (unsigned)xb, (unsigned)wb, s, wsv, ph, x2,
                                               (unsigned)x2b, &cache_it)
                         : heuristic_variant(g);
          if (x2 && v == 0) v = 5;   // the register-staged kernel has no second source
          if (g.C > g.ldx && (v == 0 || v == 24 || v == 28)) v = 14;   // (vpad: LDS-DMA only)
          if (S > 1 && (v == 0 || v >= 24)) v = 14;         // a split launch: LDS-DMA configs only
          if (cache_it) g_variant[key] = v;
        }
      } else if (g_knobs[4] == 11) {
        v = (g.C > g.ldx || S > 1) ? 14 : 0;   // forced register-staged (a vpad / split contraction runs config 14)
        if (x2 && v == 0) return -1;
      } else if ((g.C > g.ldx || S > 1) && (g_knobs[4] == 24 || g_knobs[4] == 28)) {
        v = 14;
      }
      // every variant of a split launch sums the same k-slices in the same order: forced variants stay bit-comparable
      int r = run_variant<T, TO>(v, x, w, y, g, ep, (unsigned)xb, (unsigned)wb, s, wsv, ph, x2, (unsigned)x2b);
      // a forced config that cannot run the split launch (too many fragments per wave): config 14
      if (r == -1 && S > 1 && g_knobs[4] != 0)
        return run_variant<T, TO>(14, x, w, y, g, ep, (unsigned)xb, (unsigned)wb, s, wsv, ph, x2, (unsigned)x2b);
      // a forced config without a general-k instantiation (128/256-wide n-tiles, C % 64 != 0): register-staged
      if (r == -1 && g_knobs[4] != 0 && !x2 && g.C % 64 && g.C <= g.ldx)
        return run_variant<T, TO>(0, x, w, y, g, ep, 0, 0, s, nullptr, ph);
      if (r == -1 && g_knobs[4] >= 24 && g_knobs[4] <= 28) {   // a forced halo / pointwise kernel does not apply: the heuristic's
        const int hv = x2 && heuristic_variant(g) == 0 ? 5 : heuristic_variant(g);
        return run_variant<T, TO>(hv, x, w, y, g, ep, (unsigned)xb, (unsigned)wb, s, nullptr, ph, x2, (unsigned)x2b);
      }
      return r;
    }
  }
  if (x2) return -1;
  if (g.C > g.ldx) return SSSEG_EUNSUPPORTED;   // a virtually padded contraction needs the bounded LDS-DMA loads
  return run_variant<T, TO>(0, x, w, y, g, ep, 0, 0, s, nullptr, ph);
}

bool geom_ok(const ConvGeom& g, int dt) {
  const int vec = (dt == SSSEG_F32 ? 4 : 8);
  if (g.C % vec || g.ldx % vec || g.ldw % vec) return false;
  if (g.N < 1 || g.OH < 1 || g.OW < 1 || g.K < 1 || g.C < 1) return false;
  if (g.M >= 0x7fffffffLL) return false;   // kernels decode output positions with 32-bit math
  if (g.R < 0 || g.S < 0) return false;
  return true;
}

}  // namespace

extern "C" int ssseg_set_knob(int id, int value) {
  if (id < 0 || id >= 17) return SSSEG_EINVAL;
  if (id == 6 && value) {
    std::lock_guard<std::mutex> lk(g_variant_mu);
    g_variant.clear();
    return 0;
  }
  g_knobs[id] = value;
  return 0;
}

// the variant table (geometry key -> variant): exported by one rank and imported by the others, so every rank of a
// data-parallel job launches the same kernels without tuning them itself (ssseg/tune.py)
extern "C" int64_t ssseg_tune_table_export(unsigned long long* keys_host, int32_t* variants_host, int64_t cap) {
  std::lock_guard<std::mutex> lk(g_variant_mu);
  if (cap > 0 && (!keys_host || !variants_host)) return SSSEG_EINVAL;
  std::vector<std::pair<unsigned long long, int>> rows(g_variant.begin(), g_variant.end());
  std::sort(rows.begin(), rows.end());   // a canonical order: equal tables export equal arrays
  const int64_t n = (int64_t)rows.size();
  for (int64_t i = 0; i < n && i < cap; ++i) {
    keys_host[i] = rows[i].first;
    variants_host[i] = rows[i].second;
  }
  return n;
}

extern "C" int ssseg_tune_table_import(const unsigned long long* keys_host, const int32_t* variants_host, int64_t n,
                                       int overwrite) {
  if (n < 0 || (n > 0 && (!keys_host || !variants_host))) return SSSEG_EINVAL;
  for (int64_t i = 0; i < n; ++i) {
    bool known = false;
    for (int c : kCandidates) known = known || c == variants_host[i];
    if (!known) return SSSEG_EINVAL;
  }
  std::lock_guard<std::mutex> lk(g_variant_mu);
  for (int64_t i = 0; i < n; ++i) {
    if (overwrite)
      g_variant[keys_host[i]] = variants_host[i];
    else
      g_variant.emplace(keys_host[i], variants_host[i]);
  }
  return 0;
}

// deterministic split-K workspace of the 16-bit LDS-DMA path (0: the contraction does not split)
static size_t igemm_ws_bytes(const ConvGeom& g, int dt, int nph) {
  if (dt != SSSEG_BF16 && dt != SSSEG_F16) return 0;
  return dsplit_ws_bytes(g, nph, dsplit_plan(g, nph));
}

extern "C" size_t ssseg_conv_igemm_workspace_bytes(const ssseg_conv_desc* d, int dt) {
  ConvGeom g;
  if (!make_geom(d, g)) return 0;
  return igemm_ws_bytes(g, dt, 1);
}

static int conv_igemm_epi(const void* x, const void* x2, int64_t c1, int64_t ldx2, const void* w, void* y,
                          const ssseg_conv_desc* d, int dt, int dt_out, const ssseg_conv_epilogue* epi, void* ws,
                          size_t ws_bytes, ssseg_stream_t stream, const ssseg_vcat* ysplit = nullptr,
                          int mask_act = 0, float mask_slope = 0.f) {
  ConvGeom g;
  if (!make_geom(d, g) || !y) return SSSEG_EINVAL;
  if (!geom_ok(g, dt)) return SSSEG_EINVAL;
  if (x2) {   // virtual concat: channels [0, c1) from x, [c1, C) from x2 (both whole 64-channel blocks)
    if (c1 <= 0 || c1 >= g.C || c1 % 64 || (g.C - c1) % 64 || g.ldx < c1 || ldx2 < g.C - c1 || ldx2 % 8 ||
        ldx2 > 0x7fffffff)
      return SSSEG_EINVAL;
    if (dt != dt_out || (dt != SSSEG_BF16 && dt != SSSEG_F16) || g.KK == 0) return SSSEG_EUNSUPPORTED;
    g.c1b = (int)(c1 / 64);
    g.ldx2 = (int)ldx2;
  }
  const ssseg_conv_epilogue none = {nullptr, nullptr, nullptr, 0, nullptr, 0, 0.f, nullptr, 0, nullptr};
  const ssseg_conv_epilogue& e = epi ? *epi : none;
  if (e.residual && ((!ysplit && e.ldr < g.K) || e.ldr > 0x7fffffff)) return SSSEG_EINVAL;
  if (e.stats && (!e.stats_rows_host || e.stats_ld < 1 || e.stats_ld > g.K)) return SSSEG_EINVAL;
  // fused statistics are of acc + shift: the conv feeding a training BatchNorm has no affine / residual / act (with
  // mask_act they are the gradient statistics of a BatchNorm backward instead: Epi::gstat)
  const bool gst = mask_act != 0 && e.stats != nullptr;
  if (e.stats && !gst && (e.scale || e.residual || e.relu || e.aux)) return SSSEG_EINVAL;
  if (e.stats_rows_host) *e.stats_rows_host = 0;
  if (g.M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (e.relu < 0 || e.relu > SSSEG_ACT_LEAKY) return SSSEG_EINVAL;
  Epi<float> ef{e.scale, e.shift, (const float*)e.residual, (int)e.ldr, e.relu, (float*)e.aux, e.slope,
                e.stats, (int)e.stats_ld};
  Epi<bf16_t> eb{e.scale, e.shift, (const bf16_t*)e.residual, (int)e.ldr, e.relu, (bf16_t*)e.aux, e.slope,
                 e.stats, (int)e.stats_ld};
  Epi<f16_t> eh{e.scale, e.shift, (const f16_t*)e.residual, (int)e.ldr, e.relu, (f16_t*)e.aux, e.slope,
                e.stats, (int)e.stats_ld};
  if (mask_act) {   // the residual is the input's producer's activation output: its backward applied in place
    // (a scale multiplies the masked value: the folded eval BatchNorm's backward, dconv = scale * mask(dy))
    if (ysplit || x2 || !e.residual || e.aux || e.relu || e.shift ||
        (mask_act != SSSEG_ACT_RELU && mask_act != SSSEG_ACT_LEAKY))
      return SSSEG_EINVAL;
    ef.rmask = eb.rmask = eh.rmask = mask_act;
    ef.rslope = eb.rslope = eh.rslope = mask_slope;
    ef.gstat = eb.gstat = eh.gstat = gst ? 1 : 0;
  }
  if (ysplit) {   // split output: channels [c1, K) to ysplit->x2 (pixel stride ldx2); 16-bit, plain epilogue
    const int64_t oc1 = ysplit->c1, ld2 = ysplit->ldx2;
    if (!ysplit->x2 || oc1 <= 0 || oc1 >= g.K || oc1 % 8 || g.ldy < oc1 || g.ldy % 8 || ld2 < g.K - oc1 || ld2 % 8 ||
        ld2 > 0x7fffffff)
      return SSSEG_EINVAL;
    if (dt_out != dt || (dt != SSSEG_BF16 && dt != SSSEG_F16) || e.stats || e.aux) return SSSEG_EUNSUPPORTED;
    if (e.residual && (e.ldr < oc1 || e.ldr % 8)) return SSSEG_EINVAL;
    // a residual here is the first part's ReLU mask (its producer's forward output), never an addend
    eb.rmask = eh.rmask = e.residual ? 1 : 0;
    eb.y2 = (bf16_t*)ysplit->x2;
    eh.y2 = (f16_t*)ysplit->x2;
    eb.oc1 = eh.oc1 = (int)oc1;
    eb.ldy2 = eh.ldy2 = (int)ld2;
  }
  if (g.KK == 0) {   // no taps reach this output phase: the contraction is zero
    if (e.stats) return SSSEG_EUNSUPPORTED;
    const bool v8 = g.K % 8 == 0 && g.ldy % 8 == 0 && (!e.residual || e.ldr % 8 == 0);
    if (v8 && dt_out == SSSEG_BF16) {
      hipLaunchKernelGGL(phase_zero_vec_kernel<bf16_t>, dim3(ssseg_grid(g.M * (g.K / 8), 256)), dim3(256), 0, s,
                         (bf16_t*)y, g, eb);
      SSSEG_LAUNCH_CHECK();
      return 0;
    }
    if (v8 && dt_out == SSSEG_F16) {
      hipLaunchKernelGGL(phase_zero_vec_kernel<f16_t>, dim3(ssseg_grid(g.M * (g.K / 8), 256)), dim3(256), 0, s,
                         (f16_t*)y, g, eh);
      SSSEG_LAUNCH_CHECK();
      return 0;
    }
    if (dt_out == SSSEG_F32)
      hipLaunchKernelGGL(phase_zero_kernel<float>, dim3(ssseg_grid(g.M * g.K, 256)), dim3(256), 0, s, (float*)y, g, ef);
    else if (dt_out == SSSEG_F16)
      hipLaunchKernelGGL(phase_zero_kernel<f16_t>, dim3(ssseg_grid(g.M * g.K, 256)), dim3(256), 0, s, (f16_t*)y, g,
                         eh);
    else
      hipLaunchKernelGGL(phase_zero_kernel<bf16_t>, dim3(ssseg_grid(g.M * g.K, 256)), dim3(256), 0, s, (bf16_t*)y, g,
                         eb);
    SSSEG_LAUNCH_CHECK();
    return 0;
  }
  if (!x || !w) return SSSEG_EINVAL;
  const size_t need = igemm_ws_bytes(g, dt, 1);
  // no (or a too small) workspace: no split-K
  float* wsf = (need > 0 && ws && ws_bytes >= need) ? (float*)ws : nullptr;
  int bm;
  if (x2 && dt == SSSEG_BF16)
    bm = dispatch_igemm<bf16_t, bf16_t>(x, w, y, g, eb, wsf, s, nullptr, x2);
  else if (x2)
    bm = dispatch_igemm<f16_t, f16_t>(x, w, y, g, eh, wsf, s, nullptr, x2);
  else if (dt == SSSEG_BF16 && dt_out == SSSEG_BF16)
    bm = dispatch_igemm<bf16_t, bf16_t>(x, w, y, g, eb, wsf, s);
  else if (dt == SSSEG_BF16 && dt_out == SSSEG_F32)
    bm = dispatch_igemm<bf16_t, float>(x, w, y, g, ef, wsf, s);
  else if (dt == SSSEG_F16 && dt_out == SSSEG_F16)
    bm = dispatch_igemm<f16_t, f16_t>(x, w, y, g, eh, wsf, s);
  else if (dt == SSSEG_F16 && dt_out == SSSEG_F32)
    bm = dispatch_igemm<f16_t, float>(x, w, y, g, ef, wsf, s);
  else if (dt == SSSEG_F32 && dt_out == SSSEG_F32)
    bm = dispatch_igemm<float, float>(x, w, y, g, ef, wsf, s);
  else
    return SSSEG_EUNSUPPORTED;
  if (bm <= 0) return SSSEG_EUNSUPPORTED;
  if (e.stats_rows_host && e.stats) *e.stats_rows_host = t_pw_rows >= 0 ? t_pw_rows : (g.M + bm - 1) / bm;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_conv_igemm_epi(const void* x, const void* w, void* y, const ssseg_conv_desc* d, int dt, int dt_out,
                                    const ssseg_conv_epilogue* epi, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  return conv_igemm_epi(x, nullptr, 0, 0, w, y, d, dt, dt_out, epi, ws, ws_bytes, stream);
}

extern "C" int ssseg_conv_igemm_epi_actmask(const void* x, const void* w, void* y, const ssseg_conv_desc* d, int dt,
                                            int dt_out, const ssseg_conv_epilogue* epi, int act, float slope, void* ws,
                                            size_t ws_bytes, ssseg_stream_t stream) {
  if (act != SSSEG_ACT_RELU && act != SSSEG_ACT_LEAKY) return SSSEG_EINVAL;
  return conv_igemm_epi(x, nullptr, 0, 0, w, y, d, dt, dt_out, epi, ws, ws_bytes, stream, nullptr, act, slope);
}

extern "C" int ssseg_conv_igemm_epi_vcat(const void* x, const ssseg_vcat* vc, const void* w, void* y,
                                         const ssseg_conv_desc* d, int dt, int dt_out, const ssseg_conv_epilogue* epi,
                                         void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!vc || !vc->x2) return SSSEG_EINVAL;
  return conv_igemm_epi(x, vc->x2, vc->c1, vc->ldx2, w, y, d, dt, dt_out, epi, ws, ws_bytes, stream);
}

extern "C" int ssseg_conv_igemm_epi_vsplit(const void* x, const void* w, void* y, const ssseg_vcat* ysplit,
                                           const ssseg_conv_desc* d, int dt, int dt_out, const ssseg_conv_epilogue* epi,
                                           void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!ysplit) return SSSEG_EINVAL;
  return conv_igemm_epi(x, nullptr, 0, 0, w, y, d, dt, dt_out, epi, ws, ws_bytes, stream, ysplit);
}

extern "C" int ssseg_conv_igemm(const void* x, const void* w, void* y, const ssseg_conv_desc* d, int dt, int dt_out,
                                const float* bias, int relu, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  const ssseg_conv_epilogue e = {nullptr, bias, nullptr, 0, nullptr, relu ? SSSEG_ACT_RELU : 0, 0.f, nullptr, 0, nullptr};
  return ssseg_conv_igemm_epi(x, w, y, d, dt, dt_out, &e, ws, ws_bytes, stream);
}

extern "C" int ssseg_weight_pack_batch(const ssseg_pack_desc* descs, int64_t n, int dt, ssseg_stream_t stream) {
  if (n < 0 || n > 65535 || (n > 0 && !descs)) return SSSEG_EINVAL;
  if (dt != SSSEG_BF16 && dt != SSSEG_F16 && dt != SSSEG_F32) return SSSEG_EUNSUPPORTED;
  // one block per CU slot over the launch's flat tile space; PK_MAXD descriptors per launch
  for (int64_t b = 0; b < n; b += PK_MAXD) {
    const int m = (int)std::min<int64_t>(PK_MAXD, n - b);
    const dim3 grid(2048);
    if (dt == SSSEG_BF16)
      hipLaunchKernelGGL(weight_pack_batch_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, descs + b, m);
    else if (dt == SSSEG_F16)
      hipLaunchKernelGGL(weight_pack_batch_kernel<f16_t>, grid, dim3(256), 0, (hipStream_t)stream, descs + b, m);
    else
      hipLaunchKernelGGL(weight_pack_batch_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, descs + b, m);
  }
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
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(weight_pack_kernel<f16_t>, dim3(ssseg_grid(total, 256)), dim3(256), 0, s, src, (f16_t*)dst,
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

extern "C" size_t ssseg_conv_igemm_phases_workspace_bytes(const ssseg_conv_desc* d, int64_t nphase, int dt) {
  ConvGeom g;
  if (!make_geom(d, g) || nphase < 1 || nphase > 4) return 0;
  return igemm_ws_bytes(g, dt, (int)nphase);
}

extern "C" int ssseg_conv_igemm_phases_ws(const void* x, void* y, const ssseg_conv_desc* d, int dt, int dt_out,
                                          const ssseg_conv_epilogue* epi, int64_t nphase, const int64_t* phase_geom,
                                          const void* const* w, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  ConvGeom g;
  if (!make_geom(d, g) || !x || !y || !w || !phase_geom || nphase < 1 || nphase > 4) return SSSEG_EINVAL;
  if (!geom_ok(g, dt) || g.KK == 0 || dt != dt_out || (dt != SSSEG_BF16 && dt != SSSEG_F16)) return SSSEG_EINVAL;
  const ssseg_conv_epilogue none = {nullptr, nullptr, nullptr, 0, nullptr, 0, 0.f, nullptr, 0, nullptr};
  const ssseg_conv_epilogue& e = epi ? *epi : none;
  if (e.residual && (e.ldr < g.K || e.ldr > 0x7fffffff)) return SSSEG_EINVAL;
  if (e.stats && (!e.stats_rows_host || e.stats_ld < 1 || e.stats_ld > g.K)) return SSSEG_EINVAL;
  if (e.stats && (e.scale || e.residual || e.relu || e.aux)) return SSSEG_EINVAL;
  if (e.relu < 0 || e.relu > SSSEG_ACT_LEAKY) return SSSEG_EINVAL;
  if (e.stats_rows_host) *e.stats_rows_host = 0;
  PhaseTab ph{(int)nphase, {0}, {0}, {0}, {0}, {nullptr}};
  for (int p = 0; p < (int)nphase; ++p) {
    const int64_t* q = phase_geom + 4 * p;
    for (int k = 0; k < 4; ++k)
      if (q[k] < -0x40000000LL || q[k] > 0x40000000LL) return SSSEG_EINVAL;
    if (!w[p]) return SSSEG_EINVAL;
    ph.py[p] = (int)q[0];
    ph.px[p] = (int)q[1];
    ph.ooy[p] = (int)q[2];
    ph.oox[p] = (int)q[3];
    ph.w[p] = w[p];
  }
  g.py = ph.py[0];
  g.px = ph.px[0];
  g.ooy = ph.ooy[0];
  g.oox = ph.oox[0];
  hipStream_t s = (hipStream_t)stream;
  const size_t need = igemm_ws_bytes(g, dt, (int)nphase);
  float* wsf = (need > 0 && ws && ws_bytes >= need) ? (float*)ws : nullptr;
  int bm;
  if (dt == SSSEG_BF16) {
    const Epi<bf16_t> eb{e.scale, e.shift, (const bf16_t*)e.residual, (int)e.ldr, e.relu, (bf16_t*)e.aux, e.slope,
                         e.stats, (int)e.stats_ld};
    bm = dispatch_igemm<bf16_t, bf16_t>(x, w[0], y, g, eb, wsf, s, &ph);
  } else {
    const Epi<f16_t> eh{e.scale, e.shift, (const f16_t*)e.residual, (int)e.ldr, e.relu, (f16_t*)e.aux, e.slope,
                        e.stats, (int)e.stats_ld};
    bm = dispatch_igemm<f16_t, f16_t>(x, w[0], y, g, eh, wsf, s, &ph);
  }
  if (bm <= 0) return SSSEG_EUNSUPPORTED;
  if (e.stats_rows_host && e.stats) *e.stats_rows_host = nphase * ((g.M + bm - 1) / bm);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_conv_igemm_phases(const void* x, void* y, const ssseg_conv_desc* d, int dt, int dt_out,
                                       const ssseg_conv_epilogue* epi, int64_t nphase, const int64_t* phase_geom,
                                       const void* const* w, ssseg_stream_t stream) {
  return ssseg_conv_igemm_phases_ws(x, y, d, dt, dt_out, epi, nphase, phase_geom, w, nullptr, 0, stream);
}
