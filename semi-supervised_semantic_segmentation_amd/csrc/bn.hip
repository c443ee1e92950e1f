// BatchNorm2d (training + eval) over NHWC activations, with fused ReLU and residual add, gfx950.
// Reference call sites: every ConvBlock (unet.py:9, simple_unet.py:116), the ResNet-50 encoder and
// SyncBatchNorm (distributed_trainer.py:36).  Training statistics are produced as fp64 (sum, sumsq)
// per channel so that SyncBN can all-reduce them (RCCL) before ssseg_bn_finalize.
//
//   stats:    sums[c] = sum_p x, sums[C+c] = sum_p x^2                    (2-stage, deterministic)
//   finalize: mean, invstd = 1/sqrt(var_biased + eps); running = (1-m)*running + m*{mean, var_unbiased}
//   apply:    y = act(gamma*(x-mean)*invstd + beta [+ residual])
//   bwd:      reduce  sums[c] = sum dyr, sums[C+c] = sum dyr*xhat,  dyr = dy*[y>0] (y recomputed)
//             apply   dx = gamma*invstd*(dyr - (sum_dyr + xhat*sum_dyr_xhat)/count)   (train)
//                     dx = gamma*invstd*dyr                                            (eval)
//             dres = dyr (residual branch gradient)
#include <cstdlib>
#include <initializer_list>
#include <type_traits>

#include "common.h"

namespace {

// A thread owns one chunk of V consecutive channels (16 bytes: 8 bf16 / 4 f32; 8-byte chunks when a
// leading dimension is not 16-byte aligned) for the whole kernel, so the per-channel parameters sit in
// registers; it walks pixels with U independent loads in flight.  Channels [C, rup(C, V)) of every
// output are written as 0 (the NHWC channel padding), so callers need no memset.
constexpr int U = 4;
constexpr int CH = 4;   // ABI granularity: every leading dimension is a multiple of 4 and >= rup(C, 4); C itself
                        // may be ragged (HarDNet's growth-rate widths 10, 14, 18, ..., hardnet.py:33)

static inline bool ld_bad(int64_t C, int64_t ld) { return ld % CH != 0 || ld < (C + CH - 1) / CH * CH; }

template <typename T, int V> struct Vec;
template <> struct Vec<float, 4> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[4]) {
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[4]) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
};
template <> struct Vec<float, 2> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[2]) {
    const float2 q = *(const float2*)p;
    v[0] = q.x; v[1] = q.y;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[2]) { *(float2*)p = make_float2(v[0], v[1]); }
};
__device__ __forceinline__ void unpack2(unsigned u, float& a, float& b) {
  a = __uint_as_float(u << 16);
  b = __uint_as_float(u & 0xffff0000u);
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
  return (unsigned)f32_to_bf16(a) | ((unsigned)f32_to_bf16(b) << 16);
}
template <> struct Vec<bf16_t, 8> {
  __device__ __forceinline__ static void ld(const bf16_t* p, float (&v)[8]) {
    const uint4 q = *(const uint4*)p;
    unpack2(q.x, v[0], v[1]); unpack2(q.y, v[2], v[3]); unpack2(q.z, v[4], v[5]); unpack2(q.w, v[6], v[7]);
  }
  __device__ __forceinline__ static void st(bf16_t* p, const float (&v)[8]) {
    *(uint4*)p = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
  }
};
template <> struct Vec<bf16_t, 4> {
  __device__ __forceinline__ static void ld(const bf16_t* p, float (&v)[4]) {
    const uint2 q = *(const uint2*)p;
    unpack2(q.x, v[0], v[1]); unpack2(q.y, v[2], v[3]);
  }
  __device__ __forceinline__ static void st(bf16_t* p, const float (&v)[4]) {
    *(uint2*)p = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
  }
};

template <> struct Vec<f16_t, 8> {
  __device__ __forceinline__ static void ld(const f16_t* p, float (&v)[8]) { H16::ld8(p, v); }
  __device__ __forceinline__ static void st(f16_t* p, const float (&v)[8]) { H16::st8(p, v); }
};
template <> struct Vec<f16_t, 4> {
  __device__ __forceinline__ static void ld(const f16_t* p, float (&v)[4]) { H16::ld4(p, v); }
  __device__ __forceinline__ static void st(f16_t* p, const float (&v)[4]) { H16::st4(p, v); }
};

struct Layout {
  int cpb;        // chunks per block row (<= 256)
  int ppb;        // pixel rows per block
  int cblocks;    // blocks along channels
};

static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// Small maps (P < 64K pixels: ResNet layers 3-4, 1024-2048 channels) put at most 32 chunks (256 bf16 channels) in a
// block row: 8 pixel rows per block and the channels spread over cblocks >= 4 blocks, so the grid is filled with
// few pixel blocks -- and a reduction's partial table (one row of 2C doubles per pixel block) stays small.  With
// whole 256-chunk rows a 4096 x 2048 reduction wrote a 16.8 MB table for 16.8 MB of input.  SSSEG_BN_CPB overrides
// the cap (256 = one block row spans every channel, the earlier layout).
static Layout layout_for(int64_t C, int V, int64_t P) {
  static const int small_cap = [] {
    const int v = env_int("SSSEG_BN_CPB", 32);
    return v == 8 || v == 16 || v == 32 || v == 64 || v == 128 || v == 256 ? v : 32;
  }();
  const int cap = P < 65536 ? small_cap : 256;
  Layout l;
  const int nch = (int)((C + V - 1) / V);
  l.cpb = nch < cap ? nch : cap;
  l.ppb = 256 / l.cpb;
  l.cblocks = (nch + l.cpb - 1) / l.cpb;
  return l;
}

// pixel blocks: each workgroup walks >= U*ppb pixels, grid capped at the target below
static int64_t pixel_blocks(int64_t P, const Layout& L, int64_t cap) {
  int64_t gx = (P + (int64_t)L.ppb * U - 1) / ((int64_t)L.ppb * U);
  // workgroups per launch: 512 (2 per CU, each thread looping over several chunks) measured 1.2 ms/step faster
  // over the C2 step's BN kernels than 2048 (partial / apply / bwd / eval-bwd each 10-17 % faster, smaller
  // partial tables); SSSEG_BN_WGS overrides it for sweeps
  static const int64_t target = [] {
    const char* e = getenv("SSSEG_BN_WGS");
    const long v = e ? atol(e) : 512;
    return (int64_t)(v > 0 ? v : 512);
  }();
  // (one batch of U pixels per thread on small maps, up to 2048 workgroups, measured no faster in the step)
  const int64_t want = (target + L.cblocks - 1) / L.cblocks;
  gx = gx > want ? want : gx;
  gx = gx > cap ? cap : gx;
  return gx < 1 ? 1 : gx;
}

struct ChanParams {
  const float *mean, *invstd, *gamma, *beta;
};

// V per-channel values from c0 (clamped index past C): 16-byte loads when the whole group is in range and the vector
// is 16-byte aligned (the small maps' kernels are a few round trips long, and 4-byte gathers made the parameter
// fetch one of them: 4096 x 2048 apply 14.5 -> 7.7 us)
template <int V, typename F>
__device__ __forceinline__ void ld_chan(const F* __restrict__ p, int c0, int C, F (&v)[V]) {
  constexpr int W = 16 / sizeof(F);
  if (V % W == 0 && c0 + V <= C && ((uintptr_t)p & 15) == 0) {
    typedef F F4 __attribute__((ext_vector_type(W)));
#pragma unroll
    for (int e = 0; e < V; e += W) {
      const F4 q = *(const F4*)(p + c0 + e);
#pragma unroll
      for (int k = 0; k < W; ++k) v[e + k] = q[k];
    }
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = p[min(c0 + e, C - 1)];
  }
}

template <int V>
__device__ __forceinline__ void load_params(const ChanParams& cp, int c0, int C, float (&mu)[V], float (&is)[V],
                                            float (&ga)[V], float (&be)[V], bool (&live)[V]) {
  // clamped channel indices: every load unconditional (none waits for another), dead channels zeroed after
  const uintptr_t al = (uintptr_t)cp.mean | (uintptr_t)cp.invstd | (uintptr_t)cp.gamma | (uintptr_t)cp.beta;
  if (c0 + V <= C && V % 4 == 0 && (al & 15) == 0) {   // 16-byte loads (c0 is a multiple of V)
#pragma unroll
    for (int e = 0; e < V; e += 4) {
      const float4 m = *(const float4*)(cp.mean + c0 + e), i = *(const float4*)(cp.invstd + c0 + e);
      const float4 g = cp.gamma ? *(const float4*)(cp.gamma + c0 + e) : make_float4(1.f, 1.f, 1.f, 1.f);
      const float4 b = cp.beta ? *(const float4*)(cp.beta + c0 + e) : make_float4(0.f, 0.f, 0.f, 0.f);
      mu[e] = m.x; mu[e + 1] = m.y; mu[e + 2] = m.z; mu[e + 3] = m.w;
      is[e] = i.x; is[e + 1] = i.y; is[e + 2] = i.z; is[e + 3] = i.w;
      ga[e] = g.x; ga[e + 1] = g.y; ga[e + 2] = g.z; ga[e + 3] = g.w;
      be[e] = b.x; be[e + 1] = b.y; be[e + 2] = b.z; be[e + 3] = b.w;
    }
#pragma unroll
    for (int e = 0; e < V; ++e) live[e] = true;
    return;
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int c = min(c0 + e, C - 1);
    live[e] = c0 + e < C;
    mu[e] = cp.mean[c];
    is[e] = cp.invstd[c];
    ga[e] = cp.gamma ? cp.gamma[c] : 1.f;
    be[e] = cp.beta ? cp.beta[c] : 0.f;
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    mu[e] = live[e] ? mu[e] : 0.f;
    is[e] = live[e] ? is[e] : 0.f;
    ga[e] = live[e] ? ga[e] : 0.f;
    be[e] = live[e] ? be[e] : 0.f;
  }
}

__device__ __forceinline__ int64_t clampp(int64_t p, int64_t P) { return p < P ? p : P - 1; }

constexpr int MAXG = 1024;   // partial blocks along pixels (several per CU: the partial passes are HBM-bound)

// partial blocks along pixels of a reduction: each walks >= SSSEG_BN_PMIN (64) pixels, so the fp64 partial table
// (16 C bytes per block) is <= 1/8 of the 16-bit input it summarises
static int64_t partial_cap(int64_t P) {
  static const int pmin = [] {
    const int v = env_int("SSSEG_BN_PMIN", 64);
    return v >= 0 ? v : 64;
  }();
  const int64_t c = pmin > 0 ? P / pmin : MAXG;
  return c < 1 ? 1 : (c > MAXG ? MAXG : c);
}

// per-block partial sums of 2 per-channel quantities; mode 0: (x, x^2); mode 1: (dyr, dyr*xhat)
template <typename T, int V, int MODE>
__global__ void __launch_bounds__(256) bn_partial_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         const T* __restrict__ res, int64_t P, int C, int64_t ldx,
                                                         int64_t lddy, int64_t ldr, Layout L, ChanParams prm,
                                                         int relu, double* part) {
  __shared__ double red[2][256][V];
  const int t = threadIdx.x;
  const int cl = t % L.cpb, pl = t / L.cpb;
  const int c0 = (blockIdx.y * L.cpb + cl) * V;
  const bool active = pl < L.ppb && c0 < C;
  double s1[V], s2[V];
#pragma unroll
  for (int e = 0; e < V; ++e) s1[e] = s2[e] = 0.0;
  if (active) {
    float mu[V], is[V], ga[V], be[V];
    bool live[V];
    if (MODE == 1) load_params<V>(prm, c0, C, mu, is, ga, be, live);
    using CK = Chunk<T, V>;
    const int64_t stride = (int64_t)gridDim.x * L.ppb;
    for (int64_t p0 = (int64_t)blockIdx.x * L.ppb + pl; p0 < P; p0 += stride * U) {
      typename CK::raw qx[U], qg[U], qr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = clampp(p0 + u * stride, P);
        qx[u] = CK::ld(x + p * ldx + c0);
        qg[u] = MODE == 1 ? CK::ld(dy + p * lddy + c0) : CK::zero();
        qr[u] = CK::zero();
      }
      if (MODE == 1 && res && relu)
#pragma unroll
        for (int u = 0; u < U; ++u) qr[u] = CK::ld(res + clampp(p0 + u * stride, P) * ldr + c0);
      // the U pixels of this batch are summed in fp32 (in u order: 4 terms; bf16 squares are exact in fp32), then one
      // fp64 add per chunk and batch -- the per-element fp64 converts and adds made this pass VALU-bound (3.1 TB/s)
      float f1[V], f2[V];
#pragma unroll
      for (int e = 0; e < V; ++e) f1[e] = f2[e] = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (p0 + u * stride >= P) continue;
        float v[U][V], g[U][V], r[U][V];
        CK::cvt(qx[u], v[u]);
        CK::cvt(qg[u], g[u]);
        CK::cvt(qr[u], r[u]);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          if (MODE == 0) {
            f1[e] += v[u][e];
            f2[e] = fmaf(v[u][e], v[u][e], f2[e]);
          } else {
            const float xh = (v[u][e] - mu[e]) * is[e];
            float gr = g[u][e];
            if (relu) gr = act_bwd(gr, fmaf(ga[e], xh, be[e]) + r[u][e], relu, 0.f);
            f1[e] += gr;
            f2[e] = fmaf(gr, xh, f2[e]);
          }
        }
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        s1[e] += (double)f1[e];
        s2[e] += (double)f2[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    red[0][t][e] = s1[e];
    red[1][t][e] = s2[e];
  }
  __syncthreads();
  // reduce over the ppb pixel rows: thread (chunk cl, element e) sums one column
  for (int idx = t; idx < L.cpb * V; idx += 256) {
    const int ch = idx / V, e = idx % V;
    const int c = (blockIdx.y * L.cpb + ch) * V + e;
    if (c >= C) continue;
    double a = 0, b = 0;
#pragma unroll 8
    for (int k = 0; k < L.ppb; ++k) {   // (unrolled: the LDS reads of 8 rows in flight, the adds in row order)
      a += red[0][k * L.cpb + ch][e];
      b += red[1][k * L.cpb + ch][e];
    }
    part[((int64_t)blockIdx.x * 2) * C + c] = a;
    part[((int64_t)blockIdx.x * 2 + 1) * C + c] = b;
  }
}

// optional per-channel tail of the partial reduction (saves one tiny launch per BN layer):
// 1 = training-mode finalize (mean/invstd + running stats, bn_finalize_kernel's math), 2 = param grads
struct FinalEpi {
  int mode;
  double count;
  float eps, momentum;
  float *mean_out, *invstd_out, *rmean, *rvar;
  int64_t* nbt;
  float *dgamma, *dbeta;
  const float* scale;   // mode 2, folded eval BN: dbias += scale * sums[0:C]
  float* dbias;
  // mode 3 (gradient statistics from a dgrad epilogue, rows of (sum m, sum m * y)): sum m * x_hat = (sum m * y -
  // B * sum m) * A with training: B = beta, A = 1 / gamma; folded eval (gmean set): B = mean_eff * scale + shift,
  // A = invstd / scale (A = 0 where gamma / scale is 0: x_hat is not recoverable from y there); then mode 2's tail
  const float *ggamma, *gbeta, *gmean, *ginvstd;
  // mode 3, training BN with the pre-BN input at hand (ssseg_bn_gstat_finalize_x): channels where x_hat is not
  // recoverable from y to bf16 accuracy -- gamma == 0, or |beta| >= GSTAT_COND * |gamma|, where y ~ beta and y's
  // rounding swamps gamma * x_hat -- take sum m * x_hat from the masked gradient and x instead (the unfused pass's
  // arithmetic), inside the same launch
  const void *gx_dy, *gx_x;
  int64_t gx_P, gx_ld;
  int gx_dt;
  const float *gx_mean, *gx_invstd;
};

constexpr float GSTAT_COND = 8.f;

__device__ __forceinline__ bool gstat_ill(const FinalEpi& fe, int c) {
  const float ga = fe.ggamma ? fe.ggamma[c] : 1.f, be = fe.gbeta ? fe.gbeta[c] : 0.f;
  return !(fabsf(ga) * GSTAT_COND > fabsf(be));   // (NaN gamma: ill as well)
}

template <typename T>
__device__ __forceinline__ float ld_f32(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 4) return p[i];
  else if constexpr (std::is_same<T, bf16_t>::value) return bf16_to_f32(p[i]);
  else return (float)p[i];
}

// sum_p dy[p][c] * (x[p][c] - mean) * invstd over all P pixels by the whole block (256 threads, 8 loads in flight per
// thread, fp32 per 8-pixel batch, fp64 across batches, a fixed-order butterfly + 4 wave slots): the result is returned
// on every thread.  Strided 2-byte reads (one channel of every pixel) -- the fallback of an ill-conditioned channel,
// not a fast path.
template <typename T>
__device__ double gstat_x_moment_t(const T* dy, const T* x, int64_t P, int64_t ld, int c, float mu, float is,
                                   double* red4) {
  constexpr int U = 8;
  double acc = 0.0;
  for (int64_t p0 = threadIdx.x; p0 < P; p0 += 256 * U) {
    float g[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + u * 256 < P ? p0 + u * 256 : P - 1;
      g[u] = ld_f32(dy, p * ld + c);
      v[u] = ld_f32(x, p * ld + c);
    }
    float f = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (p0 + u * 256 < P) f = fmaf(g[u], (v[u] - mu) * is, f);
    acc += (double)f;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  __syncthreads();   // red4 reuse across calls
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = acc;
  __syncthreads();
  return (red4[0] + red4[1]) + (red4[2] + red4[3]);
}

__device__ double gstat_x_moment(const FinalEpi& fe, int c, double* red4) {
  const float mu = fe.gx_mean[c], is = fe.gx_invstd[c];
  if (fe.gx_dt == SSSEG_BF16)
    return gstat_x_moment_t((const bf16_t*)fe.gx_dy, (const bf16_t*)fe.gx_x, fe.gx_P, fe.gx_ld, c, mu, is, red4);
  if (fe.gx_dt == SSSEG_F16)
    return gstat_x_moment_t((const f16_t*)fe.gx_dy, (const f16_t*)fe.gx_x, fe.gx_P, fe.gx_ld, c, mu, is, red4);
  return gstat_x_moment_t((const float*)fe.gx_dy, (const float*)fe.gx_x, fe.gx_P, fe.gx_ld, c, mu, is, red4);
}

// mode 3: the x_hat moment of channel c from the (sum m, sum m * y) moments
__device__ __forceinline__ double gstat_xhat_moment(const FinalEpi& fe, int c, double a, double b) {
  double B, A;
  if (fe.gmean) {
    const float sc = fe.ggamma[c];
    B = (double)fe.gmean[c] * sc + (fe.gbeta ? fe.gbeta[c] : 0.f);
    A = sc != 0.f ? (double)fe.ginvstd[c] / sc : 0.0;
  } else {
    const float ga = fe.ggamma ? fe.ggamma[c] : 1.f;
    B = fe.gbeta ? fe.gbeta[c] : 0.f;
    A = ga != 0.f ? 1.0 / ga : 0.0;
  }
  return (b - B * a) * A;
}

__device__ __forceinline__ void finalize_channel(double s1, double s2, int c, double count, float eps, float momentum,
                                                 float* mean_out, float* invstd_out, float* rmean, float* rvar) {
  const double mean = s1 / count;
  double var = s2 / count - mean * mean;
  var = var < 0 ? 0 : var;
  mean_out[c] = (float)mean;
  invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
  }
}

// sums over the per-block partials: block = CH channels x (256/CH) partial lanes, two accumulator chains
// per lane, then a fixed-order LDS reduction (deterministic).  Narrow channel groups (CH = 2, 4) put more
// workgroups and shorter load chains on the small-C layers, whose partial count is the largest.
// Long tables (a conv epilogue's statistics rows: one per 128-pixel tile, 8192 rows at 16x256^2) are first folded
// in place: block b sums rows [b*S, (b+1)*S) in order -- coalesced full-row reads, every thread one column of the
// [2][C] row -- and leaves the sum in row b*S; the final kernel then reads every S-th row.  (The final kernel alone
// gave such a table C/CH = 32 workgroups of strided 8-byte reads: 30 us for 8 MB.)
__global__ void __launch_bounds__(256) bn_partial_rows_kernel(double* part, int nparts, int C, int S) {
  const int r0 = blockIdx.x * S, r1 = min(nparts, r0 + S);
  for (int k = threadIdx.x; k < 2 * C; k += 256) {
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int r = r0;
    for (; r + 3 < r1; r += 4) {
      const double q0 = part[(int64_t)(2 * r) * C + k], q1 = part[(int64_t)(2 * (r + 1)) * C + k];
      const double q2 = part[(int64_t)(2 * (r + 2)) * C + k], q3 = part[(int64_t)(2 * (r + 3)) * C + k];
      a0 += q0;
      a1 += q1;
      a2 += q2;
      a3 += q3;
    }
    for (; r < r1; ++r) a0 += part[(int64_t)(2 * r) * C + k];
    part[(int64_t)(2 * r0) * C + k] = (a0 + a1) + (a2 + a3);
  }
}

// column sums of a partial table (rows 2r = first quantity, 2r + 1 = second) for channel c = blockIdx.x * CH + lane
// group: block = CH channels x (256/CH) partial lanes, four independent chains per lane, a fixed-order in-wave butterfly
// and the four waves in order (deterministic).  Every thread of the block must call it; the totals are valid on the
// threads with threadIdx.x < CH.
template <int CH>
__device__ __forceinline__ void partial_col_sums(const double* part, int nparts, int C, int rs, int cblk, double& ta,
                                                 double& tb) {
  constexpr int LN = 256 / CH;
  __shared__ double red[2][LN][CH];
  const int cl = threadIdx.x % CH, pl = threadIdx.x / CH;
  const int c = cblk * CH + cl;
  // four row pairs per iteration, all eight loads issued before the adds (independent chains)
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  if (c < C) {
    int i = pl;
    for (; i + 3 * LN < nparts; i += 4 * LN) {
      double qa[4], qb[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        qa[k] = part[(int64_t)(2 * (i + k * LN) * rs) * C + c];
        qb[k] = part[(int64_t)(2 * (i + k * LN) * rs + 1) * C + c];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] += qa[k];
        b[k] += qb[k];
      }
    }
    for (; i < nparts; i += LN) {
      a[0] += part[(int64_t)(2 * i * rs) * C + c];
      b[0] += part[(int64_t)(2 * i * rs + 1) * C + c];
    }
  }
  const double a0 = a[0] + a[2], a1 = a[1] + a[3], b0 = b[0] + b[2], b1 = b[1] + b[3];
  // the LN lanes of a channel: a butterfly over the lane bits above log2(CH) inside each wave (fixed order), then the
  // four waves' sums in order.  (One thread summing LN = 32..128 LDS slots in sequence was most of this launch's
  // ~5 us: a chain of dependent LDS reads.)
  double sa = a0 + a1, sb = b0 + b1;
#pragma unroll
  for (int o = 32; o >= CH; o >>= 1) {
    sa += __shfl_xor(sa, o, 64);
    sb += __shfl_xor(sb, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < CH) {
    red[0][wv][cl] = sa;
    red[1][wv][cl] = sb;
  }
  __syncthreads();
  ta = tb = 0;
  if (pl == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ta += red[0][k][cl];
      tb += red[1][k][cl];
    }
  }
}

template <int CH>
__global__ void __launch_bounds__(256) bn_partial_final_kernel(const double* part, int nparts, int C, double* sums,
                                                               FinalEpi fe, int rs = 1) {
  if (fe.mode == 1 && fe.nbt && blockIdx.x == 0 && threadIdx.x == 0) *fe.nbt += 1;
  double a, b;
  partial_col_sums<CH>(part, nparts, C, rs, blockIdx.x, a, b);
  const int c = blockIdx.x * CH + threadIdx.x;
  __shared__ double xfix[CH];
  __shared__ int xill[CH];
  if (fe.mode == 3 && fe.gx_x) {   // (uniform) the ill-conditioned channels of this block, recomputed from x
    __shared__ double red4[4];
    if (threadIdx.x < CH) xill[threadIdx.x] = c < C && gstat_ill(fe, c);
    __syncthreads();
    for (int k = 0; k < CH; ++k)
      if (xill[k]) {   // (uniform)
        const double v = gstat_x_moment(fe, blockIdx.x * CH + k, red4);
        if (threadIdx.x == 0) xfix[k] = v;
      }
    __syncthreads();
  }
  if (threadIdx.x < CH && c < C) {
    if (fe.mode == 3) b = (fe.gx_x && xill[threadIdx.x]) ? xfix[threadIdx.x] : gstat_xhat_moment(fe, c, a, b);
    sums[c] = a;
    sums[C + c] = b;
    if (fe.mode == 1) {
      finalize_channel(a, b, c, fe.count, fe.eps, fe.momentum, fe.mean_out, fe.invstd_out, fe.rmean, fe.rvar);
    } else if (fe.mode >= 2) {
      if (fe.dbeta) fe.dbeta[c] += (float)a;
      if (fe.dgamma) fe.dgamma[c] += (float)b;
      if (fe.dbias) fe.dbias[c] += fe.scale[c] * (float)a;
    }
  }
}

// a long deferred table (>= PG_FOLD rows: the gradient-statistics rows of a consumer's dgrad, one per output tile) is
// first folded in place to <= 256 group rows (groups of S consecutive rows, row g*S = their sum, in row order) by
// bn_pgrad_fold_kernel, so the column sums below walk <= 256 rows instead of up to 8K
constexpr int PG_FOLD = 512;
__device__ __forceinline__ int pg_fold_stride(int nparts) { return nparts >= PG_FOLD ? (nparts + 255) / 256 : 1; }

// blockIdx.y = descriptor, blockIdx.x = group
__global__ void __launch_bounds__(256) bn_pgrad_fold_kernel(const ssseg_pgrad_desc* __restrict__ descs) {
  const ssseg_pgrad_desc& d = descs[blockIdx.y];
  const int nparts = (int)d.nparts, S = pg_fold_stride(nparts);
  if (S == 1 || (int)blockIdx.x * S >= nparts) return;   // uniform per block
  const int C = (int)d.C, r0 = blockIdx.x * S, r1 = min(nparts, r0 + S);
  double* part = (double*)d.part;
  for (int k = threadIdx.x; k < 2 * C; k += 256) {   // both rows (2r, 2r + 1) of a partial: 2C contiguous values
    double a = 0.0;
    for (int r = r0; r < r1; ++r) a += part[(int64_t)(2 * r) * C + k];
    part[(int64_t)(2 * r0) * C + k] = a;
  }
}

// the deferred parameter gradients of many eval BNs in one launch (blockIdx.y = descriptor): the same column sums and
// the same mode-2 tail as bn_partial_final_kernel<8>
__global__ void __launch_bounds__(256) bn_pgrad_batch_kernel(const ssseg_pgrad_desc* __restrict__ descs) {
  const ssseg_pgrad_desc& d = descs[blockIdx.y];
  const int C = (int)d.C;
  if ((int)blockIdx.x * 8 >= C) return;   // uniform per block
  double a, b;
  const int S = pg_fold_stride((int)d.nparts);
  partial_col_sums<8>(d.part, ((int)d.nparts + S - 1) / S, C, S, blockIdx.x, a, b);
  const int c = blockIdx.x * 8 + threadIdx.x;
  if (threadIdx.x < 8 && c < C) {
    if (d.mean_eff) {   // gradient-statistics rows: (sum m, sum m * y) -> (sum m, sum m * x_hat)
      FinalEpi fe{};
      fe.ggamma = d.scale;
      fe.gbeta = d.shift;
      fe.gmean = d.mean_eff;
      fe.ginvstd = d.invstd;
      b = gstat_xhat_moment(fe, c, a, b);
    }
    if (d.dbeta) d.dbeta[c] += (float)a;
    if (d.dgamma) d.dgamma[c] += (float)b;
    if (d.dconv_bias) d.dconv_bias[c] += d.scale[c] * (float)a;
  }
}

// one launch of the partial reduction: channel group narrowed until the grid has >= 64 workgroups
// part is consumed (a long table is folded in place first)
static void launch_partial_final(const double* part, int64_t nparts, int64_t C, double* sums, hipStream_t s,
                                 FinalEpi fe = FinalEpi{}) {
  int rs = 1;
  // (folding only tables of > 64 rows per lane measured slower: the final kernels' longer walks cost more than the
  // fold launches saved, 0.80 vs 0.64 + 0.12 ms/step)
  if (nparts >= 1024) {
    rs = (int)((nparts + 255) / 256);
    const int64_t g = (nparts + rs - 1) / rs;
    hipLaunchKernelGGL(bn_partial_rows_kernel, dim3((unsigned)g), dim3(256), 0, s, (double*)part, (int)nparts, (int)C,
                       rs);
    nparts = g;
  }
  if (C >= 512 || nparts < 256)
    hipLaunchKernelGGL(bn_partial_final_kernel<8>, dim3((unsigned)((C + 7) / 8)), dim3(256), 0, s, part, (int)nparts,
                       (int)C, sums, fe, rs);
  else if (C >= 128)
    hipLaunchKernelGGL(bn_partial_final_kernel<4>, dim3((unsigned)((C + 3) / 4)), dim3(256), 0, s, part, (int)nparts,
                       (int)C, sums, fe, rs);
  else
    hipLaunchKernelGGL(bn_partial_final_kernel<2>, dim3((unsigned)((C + 1) / 2)), dim3(256), 0, s, part, (int)nparts,
                       (int)C, sums, fe, rs);
}

__global__ void bn_finalize_kernel(const double* sums, int C, double count, float eps, float momentum, float* mean_out,
                                   float* invstd_out, float* rmean, float* rvar, int64_t* nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) *nbt += 1;
  if (c >= C) return;
  finalize_channel(sums[c], sums[C + c], c, count, eps, momentum, mean_out, invstd_out, rmean, rvar);
}

__global__ void bn_eval_params_kernel(const float* rmean, const float* rvar, float eps, int C, float* mean_out,
                                      float* invstd_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean_out[c] = rmean[c];
  invstd_out[c] = 1.f / sqrtf(rvar[c] + eps);
}

// eval BN folded into a per-channel affine for a conv epilogue: scale = gamma*invstd,
// shift = beta + (conv_bias - running_mean)*scale; channels [C, Cp) get (0, 0)
__global__ void bn_fold_kernel(const float* rmean, const float* rvar, const float* gamma, const float* beta,
                               const float* bias, float eps, int C, int Cp, float* scale, float* shift,
                               float* mean_eff, float* invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= Cp) return;
  if (c >= C) {
    scale[c] = 0.f;
    shift[c] = 0.f;
    if (mean_eff) mean_eff[c] = 0.f;
    if (invstd) invstd[c] = 0.f;
    return;
  }
  const float is = 1.f / sqrtf(rvar[c] + eps);
  const float sc = (gamma ? gamma[c] : 1.f) * is;
  const float me = rmean[c] - (bias ? bias[c] : 0.f);
  scale[c] = sc;
  shift[c] = fmaf(-me, sc, beta ? beta[c] : 0.f);
  if (mean_eff) mean_eff[c] = me;
  if (invstd) invstd[c] = is;
}

__global__ void bn_fold_batch_kernel(const ssseg_fold_desc* __restrict__ descs) {
  const ssseg_fold_desc& d = descs[blockIdx.y];
  const int Cp = (int)d.Cp;
  float* scale = d.out;
  float* shift = d.out + Cp;
  float* mean_eff = d.out + 2 * Cp;
  float* invstd = d.out + 3 * Cp;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < Cp; c += gridDim.x * blockDim.x) {
    if (c >= d.C) {
      scale[c] = shift[c] = mean_eff[c] = invstd[c] = 0.f;
      continue;
    }
    const float is = 1.f / sqrtf(d.running_var[c] + (float)d.eps);
    const float sc = (d.gamma ? d.gamma[c] : 1.f) * is;
    const float me = d.running_mean[c] - (d.conv_bias ? d.conv_bias[c] : 0.f);
    scale[c] = sc;
    shift[c] = fmaf(-me, sc, d.beta ? d.beta[c] : 0.f);
    mean_eff[c] = me;
    invstd[c] = is;
  }
}

// backward of a folded eval BN: dyr = relu ? dy*[y>0] : dy, dconv = scale*dyr, dres = dyr, and per-block
// partial sums (dyr, dyr*xhat), xhat = (aux - mean_eff)*invstd.  y-mode (shift given, no aux; layers without a
// residual): wherever dyr != 0 the stored y IS the pre-activation scale*aux + shift, so xhat = (y - beta')/gamma'
// with beta' = shift + mean_eff*scale (= beta) and 1/gamma' = invstd/scale -- the raw accumulator copy is not
// needed (saves its write in the forward and its read here); a channel with scale == 0 gets xhat = 0.
template <typename T, int V>
__global__ void __launch_bounds__(256) bn_eval_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                          const T* __restrict__ aux, T* __restrict__ dconv,
                                                          T* __restrict__ dres, int64_t P, int C, int64_t ld,
                                                          Layout L, const float* scale, const float* mean_eff,
                                                          const float* invstd, int relu, double* part,
                                                          const float* shift) {
  __shared__ double red[2][256][V];
  const int t = threadIdx.x;
  const int cl = t % L.cpb, pl = t / L.cpb;
  const int c0 = (blockIdx.y * L.cpb + cl) * V;
  const bool active = pl < L.ppb && c0 < C;
  double s1[V], s2[V];
#pragma unroll
  for (int e = 0; e < V; ++e) s1[e] = s2[e] = 0.0;
  if (active) {
    float sc[V], me[V], is[V];
    bool live[V];
    ld_chan<V>(scale, c0, C, sc);
    ld_chan<V>(mean_eff, c0, C, me);
    ld_chan<V>(invstd, c0, C, is);
#pragma unroll
    for (int e = 0; e < V; ++e) live[e] = c0 + e < C;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      sc[e] = live[e] ? sc[e] : 0.f;
      me[e] = live[e] ? me[e] : 0.f;
      is[e] = live[e] ? is[e] : 0.f;
    }
    const bool ymode = shift != nullptr;
    if (ymode) {
      float sh[V];
      ld_chan<V>(shift, c0, C, sh);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        me[e] = live[e] ? fmaf(me[e], sc[e], sh[e]) : 0.f;
        is[e] = (live[e] && sc[e] != 0.f) ? is[e] / sc[e] : 0.f;
      }
    }
    const T* __restrict__ xsrc = ymode ? y : aux;   // the pre-BN value source of xhat
    using CK = Chunk<T, V>;
    const int64_t stride = (int64_t)gridDim.x * L.ppb;
    for (int64_t p0 = (int64_t)blockIdx.x * L.ppb + pl; p0 < P; p0 += stride * U) {
      typename CK::raw qg[U], qy[U], qa[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = clampp(p0 + u * stride, P);
        qg[u] = CK::ld(dy + p * ld + c0);
        qa[u] = CK::ld(xsrc + p * ld + c0);
        qy[u] = CK::zero();
      }
      if (relu && !ymode)
#pragma unroll
        for (int u = 0; u < U; ++u) qy[u] = CK::ld(y + clampp(p0 + u * stride, P) * ld + c0);
      float f1[V], f2[V];   // this batch's U pixels summed in fp32 (in u order), then one fp64 add per chunk
#pragma unroll
      for (int e = 0; e < V; ++e) f1[e] = f2[e] = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = p0 + u * stride;
        if (p >= P) continue;
        float g[U][V], yv[U][V], a[U][V];
        CK::cvt(qg[u], g[u]);
        CK::cvt(qa[u], a[u]);
        if (ymode) {
#pragma unroll
          for (int e = 0; e < V; ++e) yv[u][e] = a[u][e];
        } else {
          CK::cvt(qy[u], yv[u]);
        }
        float od[V], oc[V];
#pragma unroll
        for (int e = 0; e < V; ++e) {
          float gr = relu ? act_bwd(g[u][e], yv[u][e], relu, 0.f) : g[u][e];
          gr = live[e] ? gr : 0.f;
          od[e] = gr;
          oc[e] = sc[e] * gr;
          f1[e] += gr;
          f2[e] = fmaf(gr, (a[u][e] - me[e]) * is[e], f2[e]);
        }
        Vec<T, V>::st(dconv + p * ld + c0, oc);
        if (dres) Vec<T, V>::st(dres + p * ld + c0, od);
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        s1[e] += (double)f1[e];
        s2[e] += (double)f2[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    red[0][t][e] = s1[e];
    red[1][t][e] = s2[e];
  }
  lds_barrier();   // the dconv / dres stores keep draining
  for (int idx = t; idx < L.cpb * V; idx += 256) {
    const int ch = idx / V, e = idx % V;
    const int c = (blockIdx.y * L.cpb + ch) * V + e;
    if (c >= C) continue;
    double a = 0, b = 0;
#pragma unroll 8
    for (int k = 0; k < L.ppb; ++k) {   // (unrolled: the LDS reads of 8 rows in flight, the adds in row order)
      a += red[0][k * L.cpb + ch][e];
      b += red[1][k * L.cpb + ch][e];
    }
    part[((int64_t)blockIdx.x * 2) * C + c] = a;
    part[((int64_t)blockIdx.x * 2 + 1) * C + c] = b;
  }
}

__global__ void bn_eval_param_grad_kernel(const double* sums, int C, const float* scale, float* dgamma, float* dbeta,
                                          float* dbias) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dbeta) dbeta[c] += (float)sums[c];
  if (dgamma) dgamma[c] += (float)sums[C + c];
  if (dbias) dbias[c] += scale[c] * (float)sums[c];
}

template <typename T, int V>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                       T* __restrict__ y, int64_t P, int C, int64_t ldx, int64_t ldr,
                                                       int64_t ldy, Layout L, ChanParams prm, int relu) {
  const int t = threadIdx.x;
  const int cl = t % L.cpb, pl = t / L.cpb;
  const int c0 = (blockIdx.y * L.cpb + cl) * V;
  if (pl >= L.ppb || c0 >= C) return;
  float mu[V], is[V], ga[V], be[V];
  bool live[V];
  load_params<V>(prm, c0, C, mu, is, ga, be, live);
  const int64_t stride = (int64_t)gridDim.x * L.ppb;
  using CK = Chunk<T, V>;
  for (int64_t p0 = (int64_t)blockIdx.x * L.ppb + pl; p0 < P; p0 += stride * U) {
    typename CK::raw qx[U], qr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      qx[u] = CK::ld(x + clampp(p0 + u * stride, P) * ldx + c0);
      qr[u] = CK::zero();
    }
    if (res)
#pragma unroll
      for (int u = 0; u < U; ++u) qr[u] = CK::ld(res + clampp(p0 + u * stride, P) * ldr + c0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + u * stride;
      if (p >= P) continue;
      float v[U][V], r[U][V];
      CK::cvt(qx[u], v[u]);
      CK::cvt(qr[u], r[u]);
      float o[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float xh = (v[u][e] - mu[e]) * is[e];
        float a = fmaf(ga[e], xh, be[e]) + r[u][e];
        a = act_fwd(a, relu, 0.f);
        o[e] = live[e] ? a : 0.f;
      }
      Vec<T, V>::st(y + p * ldy + c0, o);
    }
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                           const T* __restrict__ res, T* __restrict__ dx,
                                                           T* __restrict__ dres, int64_t P, int C, int64_t ldx,
                                                           int64_t ldr, int64_t lddy, int64_t lddx, Layout L,
                                                           ChanParams prm, int relu, int train, const double* sums,
                                                           double count) {
  const int t = threadIdx.x;
  const int cl = t % L.cpb, pl = t / L.cpb;
  const int c0 = (blockIdx.y * L.cpb + cl) * V;
  if (pl >= L.ppb || c0 >= C) return;
  float mu[V], is[V], ga[V], be[V], gi[V], mdy[V], mdyx[V];
  bool live[V];
  load_params<V>(prm, c0, C, mu, is, ga, be, live);
#pragma unroll
  for (int e = 0; e < V; ++e) {
    gi[e] = ga[e] * is[e];
    mdy[e] = mdyx[e] = 0.f;
  }
  if (train) {
    double q1[V], q2[V];   // every load issued before the first division
    ld_chan<V>(sums, c0, C, q1);
    ld_chan<V>(sums + C, c0, C, q2);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float a = (float)(q1[e] / count), b = (float)(q2[e] / count);
      mdy[e] = live[e] ? a : 0.f;
      mdyx[e] = live[e] ? b : 0.f;
    }
  }
  const int64_t stride = (int64_t)gridDim.x * L.ppb;
  using CK = Chunk<T, V>;
  for (int64_t p0 = (int64_t)blockIdx.x * L.ppb + pl; p0 < P; p0 += stride * U) {
    typename CK::raw qx[U], qg[U], qr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = clampp(p0 + u * stride, P);
      qx[u] = CK::ld(x + p * ldx + c0);
      qg[u] = CK::ld(dy + p * lddy + c0);
      qr[u] = CK::zero();
    }
    if (res && relu)
#pragma unroll
      for (int u = 0; u < U; ++u) qr[u] = CK::ld(res + clampp(p0 + u * stride, P) * ldr + c0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + u * stride;
      if (p >= P) continue;
      float v[U][V], g[U][V], r[U][V];
      CK::cvt(qx[u], v[u]);
      CK::cvt(qg[u], g[u]);
      CK::cvt(qr[u], r[u]);
      float o[V], od[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float xh = (v[u][e] - mu[e]) * is[e];
        float gr = g[u][e];
        if (relu) gr = act_bwd(gr, fmaf(ga[e], xh, be[e]) + r[u][e], relu, 0.f);
        gr = live[e] ? gr : 0.f;
        od[e] = gr;
        const float d = train ? gr - mdy[e] - xh * mdyx[e] : gr;
        o[e] = gi[e] * d;
      }
      Vec<T, V>::st(dx + p * lddx + c0, o);
      if (dres) Vec<T, V>::st(dres + p * lddx + c0, od);
    }
  }
}

__global__ void bn_param_grad_kernel(const double* sums, int C, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dbeta) dbeta[c] += (float)sums[c];
  if (dgamma) dgamma[c] += (float)sums[C + c];
}

// 16-byte chunks when every leading dimension allows rup(C, V16) channels, else 8-byte chunks
template <typename T>
static bool wide_ok(int64_t C, std::initializer_list<int64_t> lds) {
  constexpr int V16 = 16 / sizeof(T);
  const int64_t cw = (C + V16 - 1) / V16 * V16;
  for (int64_t ld : lds)
    if (ld % V16 || ld < cw) return false;
  return true;
}

template <typename T, int V, int MODE>
void run_partials(const T* x, const T* dy, const T* res, int64_t P, int64_t C, int64_t ldx, int64_t lddy, int64_t ldr,
                  ChanParams prm, int relu, double* sums, void* ws, hipStream_t s, FinalEpi fe) {
  const Layout L = layout_for(C, V, P);
  const int64_t gx = pixel_blocks(P, L, partial_cap(P));
  hipLaunchKernelGGL((bn_partial_kernel<T, V, MODE>), dim3((unsigned)gx, L.cblocks), dim3(256), 0, s, x, dy, res, P,
                     (int)C, ldx, lddy, ldr, L, prm, relu, (double*)ws);
  launch_partial_final((const double*)ws, gx, C, sums, s, fe);
}

template <typename T, int MODE>
void partials(const T* x, const T* dy, const T* res, int64_t P, int64_t C, int64_t ldx, int64_t lddy, int64_t ldr,
              ChanParams prm, int relu, double* sums, void* ws, hipStream_t s, FinalEpi fe = FinalEpi{}) {
  constexpr int V16 = 16 / sizeof(T);
  if (wide_ok<T>(C, {ldx, MODE ? lddy : ldx, (MODE && res) ? ldr : ldx}))
    run_partials<T, V16, MODE>(x, dy, res, P, C, ldx, lddy, ldr, prm, relu, sums, ws, s, fe);
  else
    run_partials<T, V16 / 2, MODE>(x, dy, res, P, C, ldx, lddy, ldr, prm, relu, sums, ws, s, fe);
}

template <typename T>
void apply(const T* x, const T* res, T* y, int64_t P, int64_t C, int64_t ldx, int64_t ldr, int64_t ldy,
           ChanParams prm, int relu, hipStream_t s) {
  constexpr int V16 = 16 / sizeof(T);
  if (wide_ok<T>(C, {ldx, ldy, res ? ldr : ldx})) {
    const Layout L = layout_for(C, V16, P);
    hipLaunchKernelGGL((bn_apply_kernel<T, V16>), dim3((unsigned)pixel_blocks(P, L, 1 << 20), L.cblocks), dim3(256),
                       0, s, x, res, y, P, (int)C, ldx, ldr, ldy, L, prm, relu);
  } else {
    const Layout L = layout_for(C, V16 / 2, P);
    hipLaunchKernelGGL((bn_apply_kernel<T, V16 / 2>), dim3((unsigned)pixel_blocks(P, L, 1 << 20), L.cblocks),
                       dim3(256), 0, s, x, res, y, P, (int)C, ldx, ldr, ldy, L, prm, relu);
  }
}

template <typename T>
void bwd_apply(const T* dy, const T* x, const T* res, T* dx, T* dres, int64_t P, int64_t C, int64_t ldx, int64_t ldr,
               int64_t lddy, int64_t lddx, ChanParams prm, int relu, int train, const double* sums, double count,
               hipStream_t s) {
  constexpr int V16 = 16 / sizeof(T);
  if (wide_ok<T>(C, {ldx, lddy, lddx, (res && relu) ? ldr : ldx})) {
    const Layout L = layout_for(C, V16, P);
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, V16>), dim3((unsigned)pixel_blocks(P, L, 1 << 20), L.cblocks),
                       dim3(256), 0, s, dy, x, res, dx, dres, P, (int)C, ldx, ldr, lddy, lddx, L, prm, relu, train,
                       sums, count);
  } else {
    const Layout L = layout_for(C, V16 / 2, P);
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, V16 / 2>), dim3((unsigned)pixel_blocks(P, L, 1 << 20), L.cblocks),
                       dim3(256), 0, s, dy, x, res, dx, dres, P, (int)C, ldx, ldr, lddy, lddx, L, prm, relu, train,
                       sums, count);
  }
}

}  // namespace

extern "C" size_t ssseg_bn_workspace_bytes(int64_t C) { return sizeof(double) * 2 * MAXG * (size_t)C + 256; }

extern "C" int ssseg_bn_stats(const void* x, int64_t P, int64_t C, int64_t ldx, int dt, double* sums, void* ws,
                              size_t ws_bytes, ssseg_stream_t stream) {
  if (!x || !sums || P < 1 || C < 1 || ld_bad(C, ldx)) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_bn_workspace_bytes(C)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (dt == SSSEG_BF16)
    partials<bf16_t, 0>((const bf16_t*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s);
  else if (dt == SSSEG_F16)
    partials<f16_t, 0>((const f16_t*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s);
  else if (dt == SSSEG_F32)
    partials<float, 0>((const float*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_channel_sum_grad(const void* x, int64_t P, int64_t C, int64_t ldx, int dt, float* dsum,
                                      double* sums, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  if (!x || !dsum || !sums || P < 1 || C < 1 || ld_bad(C, ldx)) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_bn_workspace_bytes(C)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  FinalEpi fe{};
  fe.mode = 2;
  fe.dbeta = dsum;   // the mode-2 tail: dsum[c] += sums[c]
  if (dt == SSSEG_BF16)
    partials<bf16_t, 0>((const bf16_t*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s, fe);
  else if (dt == SSSEG_F16)
    partials<f16_t, 0>((const f16_t*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s, fe);
  else if (dt == SSSEG_F32)
    partials<float, 0>((const float*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s, fe);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_stats_finalize(const void* x, int64_t P, int64_t C, int64_t ldx, int dt, double* sums, void* ws,
                                       size_t ws_bytes, double count, float eps, float momentum, float* mean_out,
                                       float* invstd_out, float* running_mean, float* running_var,
                                       int64_t* num_batches_tracked, ssseg_stream_t stream) {
  if (!x || !sums || !mean_out || !invstd_out || P < 1 || C < 1 || ld_bad(C, ldx) || count <= 0) return SSSEG_EINVAL;
  if ((running_mean == nullptr) != (running_var == nullptr)) return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_bn_workspace_bytes(C)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  FinalEpi fe{};
  fe.mode = 1;
  fe.count = count;
  fe.eps = eps;
  fe.momentum = momentum;
  fe.mean_out = mean_out;
  fe.invstd_out = invstd_out;
  fe.rmean = running_mean;
  fe.rvar = running_var;
  fe.nbt = num_batches_tracked;
  if (dt == SSSEG_BF16)
    partials<bf16_t, 0>((const bf16_t*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s, fe);
  else if (dt == SSSEG_F16)
    partials<f16_t, 0>((const f16_t*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s, fe);
  else if (dt == SSSEG_F32)
    partials<float, 0>((const float*)x, nullptr, nullptr, P, C, ldx, 0, 0, ChanParams{}, 0, sums, ws, s, fe);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_partials_finalize(double* part, int64_t nparts, int64_t C, double* sums, double count,
                                          float eps, float momentum, float* mean_out, float* invstd_out,
                                          float* running_mean, float* running_var, int64_t* num_batches_tracked,
                                          ssseg_stream_t stream) {
  if (!part || !sums || nparts < 1 || C < 1 || nparts > 0x7fffffff) return SSSEG_EINVAL;
  if ((mean_out == nullptr) != (invstd_out == nullptr) || (running_mean == nullptr) != (running_var == nullptr))
    return SSSEG_EINVAL;
  if (mean_out && count <= 0) return SSSEG_EINVAL;
  FinalEpi fe{};
  if (mean_out) {
    fe.mode = 1;
    fe.count = count;
    fe.eps = eps;
    fe.momentum = momentum;
    fe.mean_out = mean_out;
    fe.invstd_out = invstd_out;
    fe.rmean = running_mean;
    fe.rvar = running_var;
    fe.nbt = num_batches_tracked;
  }
  launch_partial_final(part, nparts, C, sums, (hipStream_t)stream, fe);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_gstat_finalize(double* part, int64_t nparts, int64_t C, double* sums, const float* gamma,
                                       const float* beta, const float* mean_eff, const float* invstd, float* dgamma,
                                       float* dbeta, float* dconv_bias, ssseg_stream_t stream) {
  if (!part || !sums || nparts < 1 || C < 1 || nparts > 0x7fffffff) return SSSEG_EINVAL;
  if (mean_eff && (!gamma || !invstd)) return SSSEG_EINVAL;   // folded eval: scale, (shift,) mean_eff, invstd
  if (dconv_bias && !mean_eff) return SSSEG_EINVAL;
  FinalEpi fe{};
  fe.mode = 3;
  fe.dgamma = dgamma;
  fe.dbeta = dbeta;
  fe.scale = gamma;
  fe.dbias = dconv_bias;
  fe.ggamma = gamma;
  fe.gbeta = beta;
  fe.gmean = mean_eff;
  fe.ginvstd = invstd;
  launch_partial_final(part, nparts, C, sums, (hipStream_t)stream, fe);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_gstat_finalize_x(double* part, int64_t nparts, int64_t C, double* sums, const float* gamma,
                                         const float* beta, const void* dy, const void* x, int64_t P, int64_t ld, int dt,
                                         const float* mean, const float* invstd, float* dgamma, float* dbeta,
                                         ssseg_stream_t stream) {
  if (!part || !sums || nparts < 1 || C < 1 || nparts > 0x7fffffff) return SSSEG_EINVAL;
  if (!dy || !x || !mean || !invstd || P < 1 || ld < C) return SSSEG_EINVAL;
  if (dt != SSSEG_F32 && dt != SSSEG_BF16 && dt != SSSEG_F16) return SSSEG_EUNSUPPORTED;
  FinalEpi fe{};
  fe.mode = 3;
  fe.dgamma = dgamma;
  fe.dbeta = dbeta;
  fe.ggamma = gamma;
  fe.gbeta = beta;
  fe.gx_dy = dy;
  fe.gx_x = x;
  fe.gx_P = P;
  fe.gx_ld = ld;
  fe.gx_dt = dt;
  fe.gx_mean = mean;
  fe.gx_invstd = invstd;
  launch_partial_final(part, nparts, C, sums, (hipStream_t)stream, fe);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_finalize(const double* sums, int64_t C, double count, float eps, float momentum, float* mean_out,
                                 float* invstd_out, float* running_mean, float* running_var,
                                 int64_t* num_batches_tracked, ssseg_stream_t stream) {
  if (!sums || !mean_out || !invstd_out || C < 1 || count <= 0) return SSSEG_EINVAL;
  if ((running_mean == nullptr) != (running_var == nullptr)) return SSSEG_EINVAL;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, (int)C, count,
                     eps, momentum, mean_out, invstd_out, running_mean, running_var, num_batches_tracked);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_eval_params(const float* running_mean, const float* running_var, float eps, int64_t C,
                                    float* mean_out, float* invstd_out, ssseg_stream_t stream) {
  if (!running_mean || !running_var || !mean_out || !invstd_out || C < 1) return SSSEG_EINVAL;
  hipLaunchKernelGGL(bn_eval_params_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, running_mean,
                     running_var, eps, (int)C, mean_out, invstd_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_fold(const float* running_mean, const float* running_var, const float* gamma,
                             const float* beta, const float* conv_bias, float eps, int64_t C, int64_t Cp, float* scale,
                             float* shift, float* mean_eff, float* invstd_out, ssseg_stream_t stream) {
  if (!running_mean || !running_var || !scale || !shift || C < 1 || Cp < C) return SSSEG_EINVAL;
  hipLaunchKernelGGL(bn_fold_kernel, dim3((Cp + 255) / 256), dim3(256), 0, (hipStream_t)stream, running_mean,
                     running_var, gamma, beta, conv_bias, eps, (int)C, (int)Cp, scale, shift, mean_eff, invstd_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_fold_batch(const ssseg_fold_desc* descs, int64_t n, ssseg_stream_t stream) {
  if (n < 0 || n > 65535 || (n > 0 && !descs)) return SSSEG_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(bn_fold_batch_kernel, dim3(2, (unsigned)n), dim3(256), 0, (hipStream_t)stream, descs);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

// sums == NULL: the partial rows stay in ws (the deferred parameter gradients, ssseg_bn_eval_bwd_part); returns their count
template <typename T>
static int64_t eval_bwd(const T* dy, const T* y, const T* aux, T* dconv, T* dres, int64_t P, int64_t C, int64_t ld,
                        const float* scale, const float* mean_eff, const float* invstd, int relu, double* sums, void* ws,
                        hipStream_t s, FinalEpi fe, const float* shift) {
  constexpr int V16 = 16 / sizeof(T);
  const bool wide = wide_ok<T>(C, {ld});
  const Layout L = layout_for(C, wide ? V16 : V16 / 2, P);
  const int64_t gx = pixel_blocks(P, L, partial_cap(P));
  if (wide)
    hipLaunchKernelGGL((bn_eval_bwd_kernel<T, V16>), dim3((unsigned)gx, L.cblocks), dim3(256), 0, s, dy, y, aux, dconv,
                       dres, P, (int)C, ld, L, scale, mean_eff, invstd, relu, (double*)ws, shift);
  else
    hipLaunchKernelGGL((bn_eval_bwd_kernel<T, V16 / 2>), dim3((unsigned)gx, L.cblocks), dim3(256), 0, s, dy, y, aux,
                       dconv, dres, P, (int)C, ld, L, scale, mean_eff, invstd, relu, (double*)ws, shift);
  if (sums) launch_partial_final((const double*)ws, gx, C, sums, s, fe);
  return gx;
}

static int eval_bwd_entry(const void* dy, const void* y, const void* aux, void* dconv, void* dres, int64_t P, int64_t C,
                          int64_t ld, const float* scale, const float* mean_eff, const float* invstd, int relu, int dt,
                          double* sums, void* ws, size_t ws_bytes, ssseg_stream_t stream, FinalEpi fe,
                          const float* shift = nullptr, int64_t* nparts = nullptr);

extern "C" int ssseg_bn_eval_bwd(const void* dy, const void* y, const void* aux, void* dconv, void* dres, int64_t P,
                                 int64_t C, int64_t ld, const float* scale, const float* mean_eff, const float* invstd,
                                 int relu, int dt, double* sums, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  return eval_bwd_entry(dy, y, aux, dconv, dres, P, C, ld, scale, mean_eff, invstd, relu, dt, sums, ws, ws_bytes,
                        stream, FinalEpi{});
}

extern "C" int ssseg_bn_eval_bwd_grad(const void* dy, const void* y, const void* aux, void* dconv, void* dres,
                                      int64_t P, int64_t C, int64_t ld, const float* scale, const float* mean_eff,
                                      const float* invstd, int relu, int dt, double* sums, void* ws, size_t ws_bytes,
                                      float* dgamma, float* dbeta, float* dconv_bias, ssseg_stream_t stream) {
  FinalEpi fe{};
  fe.mode = (dgamma || dbeta || dconv_bias) ? 2 : 0;
  fe.dgamma = dgamma;
  fe.dbeta = dbeta;
  fe.scale = scale;
  fe.dbias = dconv_bias;
  return eval_bwd_entry(dy, y, aux, dconv, dres, P, C, ld, scale, mean_eff, invstd, relu, dt, sums, ws, ws_bytes,
                        stream, fe);
}

extern "C" int ssseg_bn_eval_bwd_grad_y(const void* dy, const void* y, void* dconv, void* dres, int64_t P, int64_t C,
                                        int64_t ld, const float* scale, const float* shift, const float* mean_eff,
                                        const float* invstd, int relu, int dt, double* sums, void* ws, size_t ws_bytes,
                                        float* dgamma, float* dbeta, float* dconv_bias, ssseg_stream_t stream) {
  if (!shift || !y) return SSSEG_EINVAL;
  FinalEpi fe{};
  fe.mode = (dgamma || dbeta || dconv_bias) ? 2 : 0;
  fe.dgamma = dgamma;
  fe.dbeta = dbeta;
  fe.scale = scale;
  fe.dbias = dconv_bias;
  return eval_bwd_entry(dy, y, y, dconv, dres, P, C, ld, scale, mean_eff, invstd, relu, dt, sums, ws, ws_bytes,
                        stream, fe, shift);
}

static int eval_bwd_entry(const void* dy, const void* y, const void* aux, void* dconv, void* dres, int64_t P, int64_t C,
                          int64_t ld, const float* scale, const float* mean_eff, const float* invstd, int relu, int dt,
                          double* sums, void* ws, size_t ws_bytes, ssseg_stream_t stream, FinalEpi fe,
                          const float* shift, int64_t* nparts) {
  if (!dy || !aux || !dconv || (!sums && !nparts) || !scale || !mean_eff || !invstd || (relu && !y) || P < 1 || C < 1 ||
      ld_bad(C, ld))
    return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_bn_workspace_bytes(C)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  int64_t gx = 0;
  if (dt == SSSEG_BF16)
    gx = eval_bwd<bf16_t>((const bf16_t*)dy, (const bf16_t*)y, (const bf16_t*)aux, (bf16_t*)dconv, (bf16_t*)dres, P, C, ld,
                     scale, mean_eff, invstd, relu, sums, ws, s, fe, shift);
  else if (dt == SSSEG_F16)
    gx = eval_bwd<f16_t>((const f16_t*)dy, (const f16_t*)y, (const f16_t*)aux, (f16_t*)dconv, (f16_t*)dres, P, C, ld,
                         scale, mean_eff, invstd, relu, sums, ws, s, fe, shift);
  else if (dt == SSSEG_F32)
    gx = eval_bwd<float>((const float*)dy, (const float*)y, (const float*)aux, (float*)dconv, (float*)dres, P, C, ld, scale,
                    mean_eff, invstd, relu, sums, ws, s, fe, shift);
  else
    return SSSEG_EUNSUPPORTED;
  if (nparts) *nparts = gx;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_eval_bwd_part(const void* dy, const void* y, const void* aux, void* dconv, void* dres, int64_t P,
                                      int64_t C, int64_t ld, const float* scale, const float* shift,
                                      const float* mean_eff, const float* invstd, int relu, int dt, double* part,
                                      size_t part_bytes, int64_t* nparts_host, ssseg_stream_t stream) {
  if (!nparts_host || (!aux && !shift) || (shift && !y)) return SSSEG_EINVAL;
  *nparts_host = 0;
  return eval_bwd_entry(dy, y, shift ? y : aux, dconv, dres, P, C, ld, scale, mean_eff, invstd, relu, dt, nullptr, part,
                        part_bytes, stream, FinalEpi{}, shift, nparts_host);
}

extern "C" int ssseg_bn_param_grad_batch(const ssseg_pgrad_desc* descs, int64_t n, int64_t max_c,
                                         ssseg_stream_t stream) {
  if (n < 0 || n > 65535 || (n > 0 && !descs) || max_c < 0 || max_c > 0x7fffffff) return SSSEG_EINVAL;
  if (n == 0 || max_c == 0) return 0;
  hipLaunchKernelGGL(bn_pgrad_fold_kernel, dim3(256, (unsigned)n), dim3(256), 0, (hipStream_t)stream, descs);
  hipLaunchKernelGGL(bn_pgrad_batch_kernel, dim3((unsigned)((max_c + 7) / 8), (unsigned)n), dim3(256), 0,
                     (hipStream_t)stream, descs);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_eval_param_grad(const double* sums, int64_t C, const float* scale, float* dgamma, float* dbeta,
                                        float* dconv_bias, ssseg_stream_t stream) {
  if (!sums || C < 1 || (dconv_bias && !scale)) return SSSEG_EINVAL;
  if (!dgamma && !dbeta && !dconv_bias) return 0;
  hipLaunchKernelGGL(bn_eval_param_grad_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, (int)C,
                     scale, dgamma, dbeta, dconv_bias);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_apply(const void* x, const void* residual, void* y, int64_t P, int64_t C, int64_t ldx,
                              int64_t ldr, int64_t ldy, const float* mean, const float* invstd, const float* gamma,
                              const float* beta, int relu, int dt, ssseg_stream_t stream) {
  if (!x || !y || !mean || !invstd || P < 1 || C < 1 || ld_bad(C, ldx) || ld_bad(C, ldy) ||
      (residual && ld_bad(C, ldr)))
    return SSSEG_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const ChanParams prm{mean, invstd, gamma, beta};
  if (dt == SSSEG_BF16)
    apply<bf16_t>((const bf16_t*)x, (const bf16_t*)residual, (bf16_t*)y, P, C, ldx, ldr, ldy, prm, relu, s);
  else if (dt == SSSEG_F16)
    apply<f16_t>((const f16_t*)x, (const f16_t*)residual, (f16_t*)y, P, C, ldx, ldr, ldy, prm, relu, s);
  else if (dt == SSSEG_F32)
    apply<float>((const float*)x, (const float*)residual, (float*)y, P, C, ldx, ldr, ldy, prm, relu, s);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_bwd_reduce(const void* dy, const void* x, const void* residual, int64_t P, int64_t C,
                                   int64_t ldx, int64_t ldr, int64_t lddy, const float* mean, const float* invstd,
                                   const float* gamma, const float* beta, int relu, int dt, double* sums, void* ws,
                                   size_t ws_bytes, ssseg_stream_t stream) {
  if (!dy || !x || !sums || !mean || !invstd || P < 1 || C < 1 || ld_bad(C, ldx) || ld_bad(C, lddy) ||
      (residual && ld_bad(C, ldr)))
    return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_bn_workspace_bytes(C)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (dt == SSSEG_BF16)
    partials<bf16_t, 1>((const bf16_t*)x, (const bf16_t*)dy, (const bf16_t*)residual, P, C, ldx, lddy, ldr,
                        ChanParams{mean, invstd, gamma, beta}, relu, sums, ws, s);
  else if (dt == SSSEG_F16)
    partials<f16_t, 1>((const f16_t*)x, (const f16_t*)dy, (const f16_t*)residual, P, C, ldx, lddy, ldr,
                        ChanParams{mean, invstd, gamma, beta}, relu, sums, ws, s);
  else if (dt == SSSEG_F32)
    partials<float, 1>((const float*)x, (const float*)dy, (const float*)residual, P, C, ldx, lddy, ldr,
                       ChanParams{mean, invstd, gamma, beta}, relu, sums, ws, s);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_bwd_reduce_grad(const void* dy, const void* x, const void* residual, int64_t P, int64_t C,
                                        int64_t ldx, int64_t ldr, int64_t lddy, const float* mean, const float* invstd,
                                        const float* gamma, const float* beta, int relu, int dt, double* sums,
                                        void* ws, size_t ws_bytes, float* dgamma, float* dbeta,
                                        ssseg_stream_t stream) {
  if (!dy || !x || !sums || !mean || !invstd || P < 1 || C < 1 || ld_bad(C, ldx) || ld_bad(C, lddy) ||
      (residual && ld_bad(C, ldr)))
    return SSSEG_EINVAL;
  if (!ws || ws_bytes < ssseg_bn_workspace_bytes(C)) return SSSEG_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  FinalEpi fe{};
  fe.mode = (dgamma || dbeta) ? 2 : 0;
  fe.dgamma = dgamma;
  fe.dbeta = dbeta;
  if (dt == SSSEG_BF16)
    partials<bf16_t, 1>((const bf16_t*)x, (const bf16_t*)dy, (const bf16_t*)residual, P, C, ldx, lddy, ldr,
                        ChanParams{mean, invstd, gamma, beta}, relu, sums, ws, s, fe);
  else if (dt == SSSEG_F16)
    partials<f16_t, 1>((const f16_t*)x, (const f16_t*)dy, (const f16_t*)residual, P, C, ldx, lddy, ldr,
                        ChanParams{mean, invstd, gamma, beta}, relu, sums, ws, s, fe);
  else if (dt == SSSEG_F32)
    partials<float, 1>((const float*)x, (const float*)dy, (const float*)residual, P, C, ldx, lddy, ldr,
                       ChanParams{mean, invstd, gamma, beta}, relu, sums, ws, s, fe);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_param_grad(const double* sums, int64_t C, float* dgamma, float* dbeta, ssseg_stream_t stream) {
  if (!sums || C < 1) return SSSEG_EINVAL;
  if (!dgamma && !dbeta) return 0;
  hipLaunchKernelGGL(bn_param_grad_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, (int)C,
                     dgamma, dbeta);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_bn_bwd_apply(const void* dy, const void* x, const void* residual, void* dx, void* dres, int64_t P,
                                  int64_t C, int64_t ldx, int64_t ldr, int64_t lddy, int64_t lddx, const float* mean,
                                  const float* invstd, const float* gamma, const float* beta, int relu, int train,
                                  const double* sums, double count, int dt, ssseg_stream_t stream) {
  if (!dy || !x || !dx || !mean || !invstd || P < 1 || C < 1 || ld_bad(C, ldx) || ld_bad(C, lddy) ||
      ld_bad(C, lddx) || (residual && ld_bad(C, ldr)) || (train && (!sums || count <= 0)))
    return SSSEG_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const ChanParams prm{mean, invstd, gamma, beta};
  if (dt == SSSEG_BF16)
    bwd_apply<bf16_t>((const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)residual, (bf16_t*)dx, (bf16_t*)dres, P, C,
                      ldx, ldr, lddy, lddx, prm, relu, train, sums, count, s);
  else if (dt == SSSEG_F16)
    bwd_apply<f16_t>((const f16_t*)dy, (const f16_t*)x, (const f16_t*)residual, (f16_t*)dx, (f16_t*)dres, P, C,
                      ldx, ldr, lddy, lddx, prm, relu, train, sums, count, s);
  else if (dt == SSSEG_F32)
    bwd_apply<float>((const float*)dy, (const float*)x, (const float*)residual, (float*)dx, (float*)dres, P, C, ldx,
                     ldr, lddy, lddx, prm, relu, train, sums, count, s);
  else
    return SSSEG_EUNSUPPORTED;
  SSSEG_LAUNCH_CHECK();
  return 0;
}
