// RMILoss (region mutual information, sigmoid form) on the device: reference losses.RMILoss.forward ->
// forward_sigmoid -> rmi_lower_bound (losses.py:480-592), the default-config loss (configs/default_config.py:147:
// num_classes=2, rmi_radius=3, rmi_pool='avg', rmi_pool_size=4, rmi_pool_stride=4).
//
// Per (image n, channel c) -- one "series" nc = n*C + c:
//   probs = clamp(sigmoid(x), 1e-6, 1)                                        fp32   (losses.py:515)
//   Pp, Lp = avg_pool(probs / target, k, s, pad = k/2, count_include_pad)     fp32   (losses.py:534-538)
//   vectors v_i(p) = pooled[p + shift_i], i = dy*r + dx, p over the (Hp-r+1) x (Wp-r+1) grid  (losses.py:313-355)
//   centred fp64 covariances Lc = L L^T, S = P P^T + aI, M = L P^T (a = 5e-4)                 (losses.py:553-564)
//   A = Lc - (M S^-1) M^T + aI,  rmi = 0.5 * 2 * sum log(diag(chol A) + 1e-8)                 (losses.py:571-580)
//   loss = sum_k float(mean_rows rmi.view(-1, num_classes)[:, k]) / r^2                        (losses.py:583-592)
// Backward (the reference's autograd graph, closed form): with La = chol(A), G = La^-T diag(La_ii / (La_ii + 1e-8))
// La^-1 (= d(2 sum log(diag + 1e-8)) / dA, exact including the 1e-8), K = S^-1 M^T G, Q = K M S^-1:
//   d rmi / d v^P_i(p) = sum_j Q_ij Pc_j(p) - K_ij Lc_j(p)
// scattered back through the shifted crops, the pooling window (divisor), the clamp mask and sigmoid'.
//
// Kernels: pool (one pass over logits + target, HBM-bound: 8 B read + 8 B/16 written per pixel at pool 4) ->
// means (NC x 2r^2 blocks) -> centred covariance partials (NC x r^2 x chunks blocks, fixed-order reductions) ->
// per-series 9x9 fp64 solve (one lane per series) -> loss.  Backward: per pooled cell gradient, then one pass
// over the logits writing the input gradient.  Deterministic: no atomics; every reduction has a fixed order.
#include "common.h"

#include <algorithm>

namespace {

constexpr int RT = 256;            // threads per block (reductions)
constexpr int RW = RT / 64;
constexpr double POS_ALPHA = 5e-4; // losses.py:283
constexpr int POS_PER_BLOCK = RT * 16;

struct Geo {
  int64_t NC, H, W;
  int k, s, pad, Hp, Wp, r, D, Hv, Wv, chunks, ncls;
  int64_t P;
};

__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// pooled probabilities and labels, sums in window row-major order as torch's avg_pool2d (fp32)
__global__ void rmi_pool_kernel(const float* __restrict__ x, const float* __restrict__ t, Geo g, float* __restrict__ pp,
                                float* __restrict__ lp) {
  const int64_t n = g.NC * g.Hp * g.Wp;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(q % g.Wp);
    const int oy = (int)((q / g.Wp) % g.Hp);
    const int64_t nc = q / ((int64_t)g.Wp * g.Hp);
    int h0 = oy * g.s - g.pad, w0 = ox * g.s - g.pad;
    int h1 = min(h0 + g.k, (int)g.H + g.pad), w1 = min(w0 + g.k, (int)g.W + g.pad);
    const float div = (float)((h1 - h0) * (w1 - w0));
    h0 = max(h0, 0);
    w0 = max(w0, 0);
    h1 = min(h1, (int)g.H);
    w1 = min(w1, (int)g.W);
    const float* xb = x + nc * g.H * g.W;
    const float* tb = t + nc * g.H * g.W;
    float sp = 0.f, sl = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) {
        const float pr = fminf(fmaxf(sigmoid_f(xb[(int64_t)h * g.W + w]), 1e-6f), 1.0f);
        sp += pr;
        sl += tb[(int64_t)h * g.W + w];
      }
    const bool empty = h0 >= h1 || w0 >= w1;
    pp[q] = empty ? 0.f : sp / div;
    lp[q] = empty ? 0.f : sl / div;
  }
}

// mean of each shifted crop: block (nc, v), v < D label crops, v >= D probability crops
__global__ void __launch_bounds__(RT) rmi_mean_kernel(const float* __restrict__ pp, const float* __restrict__ lp, Geo g,
                                                      double* __restrict__ mean) {
  __shared__ double red[RW];
  const int v = blockIdx.x % (2 * g.D);
  const int64_t nc = blockIdx.x / (2 * g.D);
  const int i = v % g.D;
  const float* src = (v < g.D ? lp : pp) + nc * g.Hp * g.Wp + (i / g.r) * g.Wp + (i % g.r);
  double acc = 0.0;
  for (int64_t p = threadIdx.x; p < g.P; p += RT) {
    const int py = (int)(p / g.Wv), px = (int)(p % g.Wv);
    acc += (double)src[(int64_t)py * g.Wp + px];
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < RW; ++w) s += red[w];
    mean[nc * 2 * g.D + v] = s / (double)g.P;
  }
}

// centred covariance partials: block (nc, i, chunk) accumulates row i of L L^T, P P^T and L P^T over its positions
template <int D>
__global__ void __launch_bounds__(RT) rmi_cov_kernel(const float* __restrict__ pp, const float* __restrict__ lp, Geo g,
                                                     const double* __restrict__ mean, double* __restrict__ part) {
  constexpr int R = D == 1 ? 1 : (D == 4 ? 2 : 3);
  __shared__ double red[RW][3 * D];
  const int ch = blockIdx.x % g.chunks;
  const int i = (blockIdx.x / g.chunks) % D;
  const int64_t nc = blockIdx.x / ((int64_t)g.chunks * D);
  const double* mu = mean + nc * 2 * D;
  const float* lb = lp + nc * g.Hp * g.Wp;
  const float* pb = pp + nc * g.Hp * g.Wp;
  const int64_t per = (g.P + g.chunks - 1) / g.chunks;
  const int64_t p0 = ch * per, p1 = min(g.P, p0 + per);
  double aL[D], aP[D], aM[D];
#pragma unroll
  for (int j = 0; j < D; ++j) aL[j] = aP[j] = aM[j] = 0.0;
  const int oi = (i / R) * g.Wp + (i % R);
  const double mLi = mu[i], mPi = mu[D + i];
  for (int64_t p = p0 + threadIdx.x; p < p1; p += RT) {
    const int64_t base = (p / g.Wv) * g.Wp + (p % g.Wv);
    const double li = (double)lb[base + oi] - mLi;
    const double pi = (double)pb[base + oi] - mPi;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int oj = (j / R) * g.Wp + (j % R);
      const double lj = (double)lb[base + oj] - mu[j];
      const double pj = (double)pb[base + oj] - mu[D + j];
      aL[j] = fma(li, lj, aL[j]);
      aP[j] = fma(pi, pj, aP[j]);
      aM[j] = fma(li, pj, aM[j]);
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const double sL = wave_sum(aL[j]), sP = wave_sum(aP[j]), sM = wave_sum(aM[j]);
    if (lane == 0) {
      red[wv][j] = sL;
      red[wv][D + j] = sP;
      red[wv][2 * D + j] = sM;
    }
  }
  __syncthreads();
  if (threadIdx.x < 3 * D) {
    double s = 0.0;
    for (int w = 0; w < RW; ++w) s += red[w][threadIdx.x];
    part[((nc * D + i) * g.chunks + ch) * 3 * D + threadIdx.x] = s;
  }
}

// lower Cholesky factor of the lower triangle of a (NaN on a non-positive pivot: the reference raises there)
template <int D>
__device__ void chol(const double (&a)[D][D], double (&l)[D][D]) {
  for (int j = 0; j < D; ++j) {
    double s = a[j][j];
    for (int k = 0; k < j; ++k) s -= l[j][k] * l[j][k];
    const double d = s > 0.0 ? sqrt(s) : __builtin_nan("");
    l[j][j] = d;
    for (int i = j + 1; i < D; ++i) {
      double t = a[i][j];
      for (int k = 0; k < j; ++k) t -= l[i][k] * l[j][k];
      l[i][j] = t / d;
    }
    for (int i = 0; i < j; ++i) l[i][j] = 0.0;
  }
}

// inverse of a lower-triangular matrix
template <int D>
__device__ void tri_inv(const double (&l)[D][D], double (&v)[D][D]) {
  for (int j = 0; j < D; ++j) {
    for (int i = 0; i < j; ++i) v[i][j] = 0.0;
    v[j][j] = 1.0 / l[j][j];
    for (int i = j + 1; i < D; ++i) {
      double s = 0.0;
      for (int k = j; k < i; ++k) s -= l[i][k] * v[k][j];
      v[i][j] = s / l[i][i];
    }
  }
}

// one lane per series: the D x D fp64 algebra of losses.py:553-580 (+ the backward coefficients Q, K)
template <int D>
__global__ void rmi_solve_kernel(const double* __restrict__ part, Geo g, double* __restrict__ rmi,
                                 double* __restrict__ coef, int want_grad) {
  const int64_t nc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (nc >= g.NC) return;
  double Lc[D][D], S[D][D], M[D][D];
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) Lc[i][j] = S[i][j] = M[i][j] = 0.0;
  for (int i = 0; i < D; ++i)
    for (int ch = 0; ch < g.chunks; ++ch) {
      const double* b = part + ((nc * D + i) * g.chunks + ch) * 3 * D;
      for (int j = 0; j < D; ++j) {
        Lc[i][j] += b[j];
        S[i][j] += b[D + j];
        M[i][j] += b[2 * D + j];
      }
    }
  for (int i = 0; i < D; ++i) S[i][i] += POS_ALPHA;
  double L[D][D], V[D][D], T[D][D];
  chol<D>(S, L);
  tri_inv<D>(L, V);
  // S^-1 = V^T V (into S)
  for (int a = 0; a < D; ++a)
    for (int b = 0; b < D; ++b) {
      double s = 0.0;
      for (int k = (a > b ? a : b); k < D; ++k) s += V[k][a] * V[k][b];
      S[a][b] = s;
    }
  // T = M S^-1 ; A = Lc - T M^T + aI (into Lc, lower triangle is what Cholesky reads)
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) {
      double s = 0.0;
      for (int k = 0; k < D; ++k) s += M[i][k] * S[k][j];
      T[i][j] = s;
    }
  for (int i = 0; i < D; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0.0;
      for (int k = 0; k < D; ++k) s += T[i][k] * M[j][k];
      Lc[i][j] = Lc[i][j] - s;
    }
  for (int i = 0; i < D; ++i) Lc[i][i] += POS_ALPHA;
  chol<D>(Lc, L);
  double ld = 0.0;
  for (int i = 0; i < D; ++i) ld += log(L[i][i] + 1e-8);
  rmi[nc] = 0.5 * (2.0 * ld);
  if (!want_grad) return;
  // G = V^T diag(c) V, V = L^-1, c_k = L_kk / (L_kk + 1e-8)   (into Lc)
  tri_inv<D>(L, V);
  for (int a = 0; a < D; ++a)
    for (int b = 0; b < D; ++b) {
      double s = 0.0;
      for (int k = (a > b ? a : b); k < D; ++k) s += V[k][a] * (L[k][k] / (L[k][k] + 1e-8)) * V[k][b];
      Lc[a][b] = s;
    }
  // K = T^T G (into M... M still needed for nothing else: reuse V), Q = K T
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) {
      double s = 0.0;
      for (int k = 0; k < D; ++k) s += T[k][i] * Lc[k][j];
      V[i][j] = s;
    }
  double* qo = coef + nc * 2 * D * D;
  double* ko = qo + D * D;
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) {
      double s = 0.0;
      for (int k = 0; k < D; ++k) s += V[i][k] * T[k][j];
      qo[i * D + j] = s;
      ko[i * D + j] = V[i][j];
    }
}

// loss = sum_k float(mean over rows of rmi[row * ncls + k]) / D   (losses.py:583-592)
__global__ void rmi_loss_kernel(const double* __restrict__ rmi, Geo g, float* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int64_t rows = g.NC / g.ncls;
  float tot = 0.f;
  for (int c = 0; c < g.ncls; ++c) {
    double s = 0.0;
    for (int64_t r = 0; r < rows; ++r) s += rmi[r * g.ncls + c];
    tot += (float)(s / (double)rows) / (float)g.D;
  }
  *out = tot;
}

// gradient at each pooled cell: sum over the crops that contain it (each crop's fp64 value rounded to fp32 first,
// as the reference's `.type(double)` backward does before the stack/slice gradients add up)
template <int D>
__global__ void rmi_grad_pooled_kernel(const float* __restrict__ pp, const float* __restrict__ lp, Geo g,
                                       const double* __restrict__ mean, const double* __restrict__ coef,
                                       const float* __restrict__ gout, float* __restrict__ gp) {
  constexpr int R = D == 1 ? 1 : (D == 4 ? 2 : 3);
  const int64_t n = g.NC * g.Hp * g.Wp;
  const int64_t rows = g.NC / g.ncls;
  const double scale = (double)(gout[0] / (float)D) / (double)rows;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(q % g.Wp);
    const int oy = (int)((q / g.Wp) % g.Hp);
    const int64_t nc = q / ((int64_t)g.Wp * g.Hp);
    const double* mu = mean + nc * 2 * D;
    const double* Q = coef + nc * 2 * D * D;
    const double* K = Q + D * D;
    const float* lb = lp + nc * g.Hp * g.Wp;
    const float* pb = pp + nc * g.Hp * g.Wp;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int py = oy - i / R, px = ox - i % R;
      if (py < 0 || px < 0 || py >= g.Hv || px >= g.Wv) continue;
      const int64_t base = (int64_t)py * g.Wp + px;
      double v = 0.0;
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const int64_t o = base + (j / R) * g.Wp + (j % R);
        v = fma(Q[i * D + j], (double)pb[o] - mu[D + j], v);
        v = fma(-K[i * D + j], (double)lb[o] - mu[j], v);
      }
      acc += (float)(v * scale);
    }
    gp[q] = acc;
  }
}

// input gradient: pooled-cell gradient / window divisor, clamp mask (inclusive bounds), sigmoid'
__global__ void rmi_grad_input_kernel(const float* __restrict__ x, Geo g, const float* __restrict__ gp,
                                      float* __restrict__ gx) {
  const int64_t n = g.NC * g.H * g.W;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(e % g.W);
    const int h = (int)((e / g.W) % g.H);
    const int64_t nc = e / (g.W * g.H);
    const int oy = (h + g.pad) / g.s, ox = (w + g.pad) / g.s;
    float gv = 0.f;
    if (oy < g.Hp && ox < g.Wp) {
      const int h0 = oy * g.s - g.pad, w0 = ox * g.s - g.pad;
      const int h1 = min(h0 + g.k, (int)g.H + g.pad), w1 = min(w0 + g.k, (int)g.W + g.pad);
      const float div = (float)((h1 - h0) * (w1 - w0));
      const float gpool = gp[(nc * g.Hp + oy) * g.Wp + ox] / div;
      const float y = sigmoid_f(x[e]);
      gv = (y >= 1e-6f && y <= 1.0f) ? gpool * (1.f - y) * y : 0.f;
    }
    gx[e] = gv;
  }
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

struct Ws {
  float *pp, *lp, *gp;
  double *mean, *part, *coef, *rmi;
};

size_t ws_layout(const Geo& g, char* base, Ws* w) {
  const size_t cells = (size_t)g.NC * g.Hp * g.Wp;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += align256(bytes);
    return base ? base + at : nullptr;
  };
  char* pp = take(cells * 4);
  char* lp = take(cells * 4);
  char* gp = take(cells * 4);
  char* mean = take((size_t)g.NC * 2 * g.D * 8);
  char* part = take((size_t)g.NC * g.D * g.chunks * 3 * g.D * 8);
  char* coef = take((size_t)g.NC * 2 * g.D * g.D * 8);
  char* rmi = take((size_t)g.NC * 8);
  if (w) *w = Ws{(float*)pp, (float*)lp, (float*)gp, (double*)mean, (double*)part, (double*)coef, (double*)rmi};
  return o;
}

// geometry of a call; false when the reference would fail or the kernels do not cover it
bool make_geo(int64_t N, int64_t C, int64_t H, int64_t W, int64_t ncls, int64_t radius, int64_t k, int64_t s,
              int64_t pad, Geo* g) {
  if (N < 1 || C < 1 || H < 1 || W < 1 || ncls < 1 || (N * C) % ncls) return false;
  if (radius < 1 || radius > 3 || k < 1 || s < 1 || k != s || pad < 0 || pad >= k) return false;
  if (H > (1 << 24) || W > (1 << 24) || N * C * H * W > ((int64_t)1 << 40)) return false;
  Geo r{};
  r.NC = N * C;
  r.H = H;
  r.W = W;
  r.k = (int)k;
  r.s = (int)s;
  r.pad = (int)pad;
  r.Hp = (int)((H + 2 * pad - k) / s + 1);
  r.Wp = (int)((W + 2 * pad - k) / s + 1);
  r.r = (int)radius;
  r.D = (int)(radius * radius);
  r.Hv = r.Hp - r.r + 1;
  r.Wv = r.Wp - r.r + 1;
  if (r.Hv < 1 || r.Wv < 1) return false;
  r.P = (int64_t)r.Hv * r.Wv;
  r.chunks = (int)std::min<int64_t>(64, (r.P + POS_PER_BLOCK - 1) / POS_PER_BLOCK);
  r.ncls = (int)ncls;
  *g = r;
  return true;
}

template <int D>
void launch_stats(const Geo& g, const Ws& w, int want_grad, hipStream_t st) {
  hipLaunchKernelGGL(rmi_mean_kernel, dim3((unsigned)(g.NC * 2 * D)), dim3(RT), 0, st, w.pp, w.lp, g, w.mean);
  hipLaunchKernelGGL(rmi_cov_kernel<D>, dim3((unsigned)(g.NC * D * g.chunks)), dim3(RT), 0, st, w.pp, w.lp, g, w.mean,
                     w.part);
  hipLaunchKernelGGL(rmi_solve_kernel<D>, dim3((unsigned)((g.NC + 63) / 64)), dim3(64), 0, st, w.part, g, w.rmi, w.coef,
                     want_grad);
}

}  // namespace

extern "C" size_t ssseg_rmi_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W, int64_t num_classes,
                                            int64_t radius, int64_t pool_k, int64_t pool_s, int64_t pool_pad) {
  Geo g;
  if (!make_geo(N, C, H, W, num_classes, radius, pool_k, pool_s, pool_pad, &g)) return 0;
  return ws_layout(g, nullptr, nullptr);
}

extern "C" int ssseg_rmi_fwd(const float* logits, const float* target, int64_t N, int64_t C, int64_t H, int64_t W,
                             int64_t num_classes, int64_t radius, int64_t pool_k, int64_t pool_s, int64_t pool_pad,
                             int want_grad, float* loss_out, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  Geo g;
  if (!logits || !target || !loss_out || !make_geo(N, C, H, W, num_classes, radius, pool_k, pool_s, pool_pad, &g))
    return SSSEG_EINVAL;
  if (!ws || ws_bytes < ws_layout(g, nullptr, nullptr)) return SSSEG_EWORKSPACE;
  Ws w;
  ws_layout(g, (char*)ws, &w);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(rmi_pool_kernel, dim3(ssseg_grid(g.NC * g.Hp * g.Wp, 256)), dim3(256), 0, st, logits, target, g,
                     w.pp, w.lp);
  if (g.D == 1) launch_stats<1>(g, w, want_grad, st);
  else if (g.D == 4) launch_stats<4>(g, w, want_grad, st);
  else launch_stats<9>(g, w, want_grad, st);
  hipLaunchKernelGGL(rmi_loss_kernel, dim3(1), dim3(64), 0, st, w.rmi, g, loss_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_rmi_bwd(const float* logits, int64_t N, int64_t C, int64_t H, int64_t W, int64_t num_classes,
                             int64_t radius, int64_t pool_k, int64_t pool_s, int64_t pool_pad, const float* gout,
                             float* grad_out, void* ws, size_t ws_bytes, ssseg_stream_t stream) {
  Geo g;
  if (!logits || !gout || !grad_out || !make_geo(N, C, H, W, num_classes, radius, pool_k, pool_s, pool_pad, &g))
    return SSSEG_EINVAL;
  if (!ws || ws_bytes < ws_layout(g, nullptr, nullptr)) return SSSEG_EWORKSPACE;
  Ws w;
  ws_layout(g, (char*)ws, &w);
  hipStream_t st = (hipStream_t)stream;
  const unsigned gc = ssseg_grid(g.NC * g.Hp * g.Wp, 256);
  if (g.D == 1)
    hipLaunchKernelGGL(rmi_grad_pooled_kernel<1>, dim3(gc), dim3(256), 0, st, w.pp, w.lp, g, w.mean, w.coef, gout, w.gp);
  else if (g.D == 4)
    hipLaunchKernelGGL(rmi_grad_pooled_kernel<4>, dim3(gc), dim3(256), 0, st, w.pp, w.lp, g, w.mean, w.coef, gout, w.gp);
  else
    hipLaunchKernelGGL(rmi_grad_pooled_kernel<9>, dim3(gc), dim3(256), 0, st, w.pp, w.lp, g, w.mean, w.coef, gout, w.gp);
  hipLaunchKernelGGL(rmi_grad_input_kernel, dim3(ssseg_grid(g.NC * g.H * g.W, 256)), dim3(256), 0, st, logits, g, w.gp,
                     grad_out);
  SSSEG_LAUNCH_CHECK();
  return 0;
}
