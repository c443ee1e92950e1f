// Shared device helpers for the ssseg HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "../../include/ssseg.h"

#define SSSEG_WAVE 64

// Launch-error check: every extern "C" entry returns 0 or a hipError_t / SSSEG_E* code.
#define SSSEG_LAUNCH_CHECK()                                   \
  do {                                                         \
    hipError_t _e = hipGetLastError();                         \
    if (_e != hipSuccess) return (int)_e;                      \
  } while (0)

#define SSSEG_TRY(expr)                                        \
  do {                                                         \
    hipError_t _e = (expr);                                    \
    if (_e != hipSuccess) return (int)_e;                      \
  } while (0)

typedef unsigned short bf16_t;   // raw bfloat16 bits

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN kept a NaN)
// round-to-nearest-even f32 -> bf16 in hardware (gfx950 v_cvt_pk_bf16_f32; NaN stays a quiet NaN): one
// instruction instead of the bit-twiddled rounding (~6 VALU) the epilogues and BN passes spent per value
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

// IEEE half (the fp16 compute mode, config C5): hardware round-to-nearest-even conversions
typedef _Float16 f16_t;
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

// workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global stores.
// __syncthreads() (release fence) also drains vmcnt, i.e. every store the wave issued before it: in an epilogue
// that stores its tile and then reduces statistics through LDS that is ~2 us of HBM write latency per tile,
// serialised (+60 % on the conv 1x1 expansions' fused-statistics launches).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <typename T> struct io;
template <> struct io<float> {
  __device__ __forceinline__ static float ld(const float* p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void st(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct io<bf16_t> {
  __device__ __forceinline__ static float ld(const bf16_t* p, int64_t i) { return bf16_to_f32(p[i]); }
  __device__ __forceinline__ static void st(bf16_t* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }
};
template <> struct io<f16_t> {
  __device__ __forceinline__ static float ld(const f16_t* p, int64_t i) { return (float)p[i]; }
  __device__ __forceinline__ static void st(f16_t* p, int64_t i, float v) { p[i] = (f16_t)v; }
};

// 16-byte (8 x fp16) and 8-byte (4 x fp16) vector loads/stores with fp32 values: the fp16 member of the
// per-file 16-byte chunk helpers (bf16 and fp32 have their own)
struct H16 {
  __device__ __forceinline__ static void ld8(const f16_t* p, float (&v)[8]) {
    const uint4 q = *(const uint4*)p;
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f16x2_t h = __builtin_bit_cast(f16x2_t, w[i]);
      v[2 * i] = (float)h[0];
      v[2 * i + 1] = (float)h[1];
    }
  }
  __device__ __forceinline__ static void st8(f16_t* p, const float (&v)[8]) {
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f16x2_t h = {(f16_t)v[2 * i], (f16_t)v[2 * i + 1]};
      w[i] = __builtin_bit_cast(unsigned, h);
    }
    *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ __forceinline__ static void ld4(const f16_t* p, float (&v)[4]) {
    const uint2 q = *(const uint2*)p;
    const f16x2_t a = __builtin_bit_cast(f16x2_t, q.x), b = __builtin_bit_cast(f16x2_t, q.y);
    v[0] = (float)a[0]; v[1] = (float)a[1]; v[2] = (float)b[0]; v[3] = (float)b[1];
  }
  __device__ __forceinline__ static void st4(f16_t* p, const float (&v)[4]) {
    const f16x2_t a = {(f16_t)v[0], (f16_t)v[1]}, b = {(f16_t)v[2], (f16_t)v[3]};
    *(uint2*)p = make_uint2(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b));
  }
};

// Raw V-element chunks (16 or 8 bytes): ld() moves the bits only, cvt() converts to fp32 later.  Streaming
// kernels issue every load of a batch first (clamped addresses, no branch around a load) and convert after,
// so the batch is in flight together: a conversion right behind each conditional load makes the compiler
// wait for that load (s_waitcnt vmcnt(0)) before issuing the next, serialising the memory round trips.
template <typename T, int V> struct Chunk;
template <> struct Chunk<bf16_t, 8> {
  typedef uint4 raw;
  __device__ __forceinline__ static raw ld(const bf16_t* p) { return *(const uint4*)p; }
  __device__ __forceinline__ static raw zero() { return make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ static void cvt(const raw& q, float (&v)[8]) {
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
};
template <> struct Chunk<bf16_t, 4> {
  typedef uint2 raw;
  __device__ __forceinline__ static raw ld(const bf16_t* p) { return *(const uint2*)p; }
  __device__ __forceinline__ static raw zero() { return make_uint2(0, 0); }
  __device__ __forceinline__ static void cvt(const raw& q, float (&v)[4]) {
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  }
};
template <> struct Chunk<f16_t, 8> {
  typedef uint4 raw;
  __device__ __forceinline__ static raw ld(const f16_t* p) { return *(const uint4*)p; }
  __device__ __forceinline__ static raw zero() { return make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ static void cvt(const raw& q, float (&v)[8]) {
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f16x2_t h = __builtin_bit_cast(f16x2_t, w[i]);
      v[2 * i] = (float)h[0];
      v[2 * i + 1] = (float)h[1];
    }
  }
};
template <> struct Chunk<f16_t, 4> {
  typedef uint2 raw;
  __device__ __forceinline__ static raw ld(const f16_t* p) { return *(const uint2*)p; }
  __device__ __forceinline__ static raw zero() { return make_uint2(0, 0); }
  __device__ __forceinline__ static void cvt(const raw& q, float (&v)[4]) {
    const f16x2_t a = __builtin_bit_cast(f16x2_t, q.x), b = __builtin_bit_cast(f16x2_t, q.y);
    v[0] = (float)a[0]; v[1] = (float)a[1]; v[2] = (float)b[0]; v[3] = (float)b[1];
  }
};
template <> struct Chunk<float, 4> {
  typedef float4 raw;
  __device__ __forceinline__ static raw ld(const float* p) { return *(const float4*)p; }
  __device__ __forceinline__ static raw zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ static void cvt(const raw& q, float (&v)[4]) {
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
};
template <> struct Chunk<float, 2> {
  typedef float2 raw;
  __device__ __forceinline__ static raw ld(const float* p) { return *(const float2*)p; }
  __device__ __forceinline__ static raw zero() { return make_float2(0.f, 0.f); }
  __device__ __forceinline__ static void cvt(const raw& q, float (&v)[2]) {
    v[0] = q.x; v[1] = q.y;
  }
};

// wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum; `scratch` needs blockDim.x/64 entries; result valid in every thread
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T t = 0;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

// grid-stride launch size: one thread per element up to `cap` workgroups (SSSEG_GRID_CAP overrides the default
// cap for sweeps)
static inline int ssseg_grid_cap() {
  static const int cap = [] {
    const char* e = getenv("SSSEG_GRID_CAP");
    const int v = e ? atoi(e) : 256 * 16;
    return v > 0 ? v : 256 * 16;
  }();
  return cap;
}
static inline int ssseg_grid(int64_t n, int block, int cap = -1) {
  if (cap < 0) cap = ssseg_grid_cap();
  int64_t g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

// activation codes (SSSEG_ACT_*): forward, and the derivative evaluated from the output y (sign and the
// open interval (0, 6) survive every activation here, so y decides like the pre-activation does) or from
// the pre-activation z.  PyTorch semantics: ReLU6 = hardtanh(0, 6) passes gradient for 0 < z < 6;
// LeakyReLU passes 1 for z > 0 and slope otherwise.
__device__ __forceinline__ float act_fwd(float z, int act, float slope) {
  if (act == SSSEG_ACT_RELU) return fmaxf(z, 0.f);
  if (act == SSSEG_ACT_RELU6) return fminf(fmaxf(z, 0.f), 6.f);
  if (act == SSSEG_ACT_LEAKY) return z > 0.f ? z : z * slope;
  return z;
}
// g * d act / d z with the gradient SELECTED (not multiplied) where it is cut, like threshold_backward
__device__ __forceinline__ float act_bwd(float g, float yz, int act, float slope) {
  if (act == SSSEG_ACT_RELU) return yz > 0.f ? g : 0.f;
  if (act == SSSEG_ACT_RELU6) return (yz > 0.f && yz < 6.f) ? g : 0.f;
  if (act == SSSEG_ACT_LEAKY) return yz > 0.f ? g : g * slope;
  return g;
}
