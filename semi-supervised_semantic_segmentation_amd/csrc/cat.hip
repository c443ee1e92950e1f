// n-way channel concat of same-size NHWC maps and its inverse, one launch each (torch.cat(tensors, 1) of the
// HarDNet harmonic links and outputs, hardnet.py:67,78,95; higher_hrnet.py:1033; discriminator.py:56).
//
// The concat packs each operand's REAL channels back to back (HarDNet's widths are even, not multiples of the MFMA
// vector), so operand boundaries fall inside 16-byte chunks.  One thread builds one 16-byte output chunk: it walks
// the chunk's channels across the operands (table in LDS, monotone part index), gathers the elements, and stores
// the chunk once; the channels past the operands' total are written zero in the same store (no memset before).
// The split is the gather the other way round: one thread writes one 16-byte chunk of one operand's gradient
// (padding channels zero), optionally adding a pending gradient of that operand (ssseg.nn.GradJoin: a layer output
// read by several consumers gets their gradients summed here instead of by a separate add).
#include "common.h"

namespace {

constexpr int CAT_MAXP = 16;

struct CatTab {
  const void* src[CAT_MAXP];   // cat: operand; split: unused
  void* dst[CAT_MAXP];         // split: operand gradient
  const void* add[CAT_MAXP];   // split: pending gradient (dst layout) or null
  int64_t ld[CAT_MAXP];        // operand pixel stride (physical channels)
  int c[CAT_MAXP];             // real channels
  int c0[CAT_MAXP + 1];        // channel offset in the concat (c0[n] = total)
  int q0[CAT_MAXP + 1];        // split: first chunk of the operand in the flattened chunk range
  int n;
};

// the table in LDS (same layout), copied word by word by the whole block: indexed by the data-dependent part number
// without a scratch copy of the kernel argument
__device__ __forceinline__ void load_tab(const CatTab& t, CatTab& s) {
  const unsigned* a = (const unsigned*)&t;
  unsigned* b = (unsigned*)&s;
  for (int i = threadIdx.x; i < (int)(sizeof(CatTab) / 4); i += blockDim.x) b[i] = a[i];
  __syncthreads();
}

template <typename T> struct Bits;
template <> struct Bits<bf16_t> { typedef unsigned short u; };
template <> struct Bits<f16_t> { typedef unsigned short u; };
template <> struct Bits<float> { typedef unsigned u; };

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<bf16_t>(bf16_t v) { return bf16_to_f32(v); }
template <> __device__ __forceinline__ float to_f<f16_t>(f16_t v) { return (float)v; }
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <typename T>
__device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) { return f32_to_bf16(v); }
template <> __device__ __forceinline__ f16_t from_f<f16_t>(float v) { return (f16_t)v; }
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }

// y[p][0..ldy) = concat of the operands' first c channels, zero past the total; one thread per 16-byte chunk
template <typename T>
__global__ void __launch_bounds__(256) cat_n_kernel(CatTab t, T* __restrict__ y, unsigned total, unsigned Q,
                                                    int64_t ldy) {
  constexpr int V = 16 / sizeof(T);
  typedef typename Bits<T>::u U;
  __shared__ CatTab s;
  load_tab(t, s);
  const int n = t.n, ctot = s.c0[n];
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const unsigned pix = i / Q, q = i - pix * Q;
    const int ch0 = (int)q * V;
    int k = 0;
    while (k + 1 < n && ch0 >= s.c0[k + 1]) ++k;
    U v[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int ch = ch0 + e;
      while (k + 1 < n && ch >= s.c0[k + 1]) ++k;
      v[e] = 0;
      if (ch < ctot) v[e] = ((const U*)s.src[k])[(int64_t)pix * s.ld[k] + (ch - s.c0[k])];
    }
    uint4 w;
    if constexpr (V == 8) {
      w = make_uint4(v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16), v[4] | ((unsigned)v[5] << 16),
                     v[6] | ((unsigned)v[7] << 16));
    } else {
      w = make_uint4(v[0], v[1], v[2], v[3]);
    }
    *(uint4*)(y + (int64_t)pix * ldy + ch0) = w;
  }
}

// parts[k].dst[p][j] = gy[p][c0_k + j] (+ add_k[p][j]) for j < c_k, 0 for c_k <= j < ld_k; one thread per 16-byte
// chunk of one operand's gradient (chunks of all operands flattened: q0)
template <typename T>
__global__ void __launch_bounds__(256) split_n_kernel(CatTab t, const T* __restrict__ gy, int64_t ldg, unsigned total,
                                                      unsigned Q) {
  constexpr int V = 16 / sizeof(T);
  typedef typename Bits<T>::u U;
  __shared__ CatTab s;
  load_tab(t, s);
  const int n = t.n;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const unsigned pix = i / Q, q = i - pix * Q;
    int k = 0;
    while (k + 1 < n && (int)q >= s.q0[k + 1]) ++k;
    const int j0 = ((int)q - s.q0[k]) * V, c = s.c[k];
    const U* g = (const U*)gy + (int64_t)pix * ldg + s.c0[k];
    U v[V];
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = (j0 + e < c) ? g[j0 + e] : (U)0;
    const int64_t off = (int64_t)pix * s.ld[k] + j0;
    if (s.add[k] != nullptr) {
      const uint4 a = *(const uint4*)((const T*)s.add[k] + off);
      const U* av = (const U*)&a;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const T x = __builtin_bit_cast(T, v[e]), b = __builtin_bit_cast(T, av[e]);
        v[e] = __builtin_bit_cast(U, from_f<T>(to_f<T>(x) + to_f<T>(b)));
      }
    }
    uint4 w;
    if constexpr (V == 8) {
      w = make_uint4(v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16), v[4] | ((unsigned)v[5] << 16),
                     v[6] | ((unsigned)v[7] << 16));
    } else {
      w = make_uint4(v[0], v[1], v[2], v[3]);
    }
    *(uint4*)((T*)s.dst[k] + off) = w;
  }
}

int fill_tab(const ssseg_cat_part* parts, int64_t nparts, int V, bool split, CatTab& t) {
  if (!parts || nparts < 1 || nparts > CAT_MAXP) return SSSEG_EINVAL;
  t = CatTab{};
  t.n = (int)nparts;
  int c0 = 0, q0 = 0;
  for (int k = 0; k < nparts; ++k) {
    const ssseg_cat_part& p = parts[k];
    if (p.c < 0 || p.ld < p.c || p.ld > (1 << 20)) return SSSEG_EINVAL;
    if (split) {
      if ((p.ld > 0 && !p.dst) || p.ld % V != 0 || ((uintptr_t)p.dst & 15) || ((uintptr_t)p.add & 15))
        return SSSEG_EINVAL;
    } else if (!p.src && p.c > 0) {
      return SSSEG_EINVAL;
    }
    t.src[k] = p.src;
    t.dst[k] = p.dst;
    t.add[k] = p.add;
    t.ld[k] = p.ld;
    t.c[k] = (int)p.c;
    t.c0[k] = c0;
    t.q0[k] = q0;
    c0 += (int)p.c;
    q0 += (int)(p.ld / V);
  }
  for (int k = (int)nparts; k <= CAT_MAXP; ++k) {
    t.c0[k] = c0;
    t.q0[k] = q0;
  }
  return 0;
}

}  // namespace

extern "C" int ssseg_nhwc_cat_n(const ssseg_cat_part* parts_host, int64_t nparts, void* y, int64_t npix, int64_t ldy,
                                int dt, ssseg_stream_t stream) {
  const int esz = dt == SSSEG_F32 ? 4 : 2, V = 16 / esz;
  if (dt != SSSEG_F32 && dt != SSSEG_BF16 && dt != SSSEG_F16) return SSSEG_EUNSUPPORTED;
  CatTab t;
  const int rc = fill_tab(parts_host, nparts, V, false, t);
  if (rc) return rc;
  if (!y || ((uintptr_t)y & 15) || npix < 0 || ldy % V != 0 || ldy < t.c0[CAT_MAXP]) return SSSEG_EINVAL;
  const int64_t total = npix * (ldy / V);
  if (total == 0) return 0;
  if (total >= (1LL << 32)) return SSSEG_EUNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(ssseg_grid(total, 256)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(cat_n_kernel<bf16_t>, g, b, 0, st, t, (bf16_t*)y, (unsigned)total, (unsigned)(ldy / V), ldy);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(cat_n_kernel<f16_t>, g, b, 0, st, t, (f16_t*)y, (unsigned)total, (unsigned)(ldy / V), ldy);
  else
    hipLaunchKernelGGL(cat_n_kernel<float>, g, b, 0, st, t, (float*)y, (unsigned)total, (unsigned)(ldy / V), ldy);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_nhwc_split_n(const void* gy, int64_t ldg, const ssseg_cat_part* parts_host, int64_t nparts,
                                  int64_t npix, int dt, ssseg_stream_t stream) {
  const int esz = dt == SSSEG_F32 ? 4 : 2, V = 16 / esz;
  if (dt != SSSEG_F32 && dt != SSSEG_BF16 && dt != SSSEG_F16) return SSSEG_EUNSUPPORTED;
  CatTab t;
  const int rc = fill_tab(parts_host, nparts, V, true, t);
  if (rc) return rc;
  if (!gy || npix < 0 || ldg < t.c0[CAT_MAXP]) return SSSEG_EINVAL;
  const int Q = t.q0[CAT_MAXP];
  const int64_t total = npix * Q;
  if (total == 0) return 0;
  if (total >= (1LL << 32)) return SSSEG_EUNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(ssseg_grid(total, 256)), b(256);
  if (dt == SSSEG_BF16)
    hipLaunchKernelGGL(split_n_kernel<bf16_t>, g, b, 0, st, t, (const bf16_t*)gy, ldg, (unsigned)total, (unsigned)Q);
  else if (dt == SSSEG_F16)
    hipLaunchKernelGGL(split_n_kernel<f16_t>, g, b, 0, st, t, (const f16_t*)gy, ldg, (unsigned)total, (unsigned)Q);
  else
    hipLaunchKernelGGL(split_n_kernel<float>, g, b, 0, st, t, (const float*)gy, ldg, (unsigned)total, (unsigned)Q);
  SSSEG_LAUNCH_CHECK();
  return 0;
}
