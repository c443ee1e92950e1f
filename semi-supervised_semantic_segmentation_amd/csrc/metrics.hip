// Validation metrics of train.validate (train.py:150-195): argmax of the logits -> one-hot -> nearest
// resize to the mask size -> Dice on channel 1 (metrics.dice_metric, metrics.py:1-7) and the confusion
// counts of lovasz.iou (lovasz.py:54-73, per_image=False, C=2) for mIoU.
//
// One pass over the logits (any strides: the heads return a 2-channel view of an NHWC buffer) and the
// mask; HBM-bound (8 B of mask + 8 B of logits gathered per output pixel).  Per-image integer counters
// are reduced in registers / across the wave with DPP shuffles and added with one 64-bit atomic per
// counter per workgroup, so the result is exact and order-independent.
#include "common.h"

namespace {

constexpr int MET_THREADS = 256;
constexpr int MET_PIX_PER_THREAD = 8;

// ATen nearest_idx (UpSample.h) for scale_factor=None: identity, exact 2x, else floor(o * in/out).
__device__ __forceinline__ int64_t nearest_src(int64_t o, int64_t in, int64_t out) {
  if (out == in) return o;
  if (out == 2 * in) return o >> 1;
  const float scale = (float)in / (float)out;
  const int64_t i = (int64_t)floorf((float)o * scale);
  return i < in - 1 ? i : in - 1;
}

// torch.argmax over 2 channels: first maximum wins, NaN counts as the maximum.
__device__ __forceinline__ int argmax2(float a0, float a1) {
  if (a0 != a0) return 0;
  if (a1 != a1) return 1;
  return a1 > a0 ? 1 : 0;
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
#pragma unroll
  for (int off = SSSEG_WAVE / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, SSSEG_WAVE);
  return v;
}

// counters per image: 0 sum(pred1 * t1), 1 sum(pred1), 2 sum(t1)  (t1 = mask[:,1] > 0.5, dice)
//                     3 inter0, 4 union0, 5 inter1, 6 union1         (label = argmax(mask), iou)
//                     7 pixels
__global__ void __launch_bounds__(MET_THREADS)
seg_metrics_count_kernel(const float* __restrict__ logits, int64_t lsb, int64_t lsc, int64_t lsh, int64_t lsw,
                         int64_t h, int64_t w, const float* __restrict__ mask, int64_t msb, int64_t msc,
                         int64_t msh, int64_t msw, int64_t H, int64_t W,
                         unsigned long long* __restrict__ counts) {
  const int64_t b = blockIdx.y;
  const int64_t HW = H * W;
  const float* lb = logits + b * lsb;
  const float* mb = mask + b * msb;
  unsigned c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t stride = (int64_t)gridDim.x * MET_THREADS;
  for (int64_t p = (int64_t)blockIdx.x * MET_THREADS + threadIdx.x; p < HW; p += stride) {
    const int64_t y = p / W, x = p - y * W;
    const int64_t sy = nearest_src(y, h, H), sx = nearest_src(x, w, W);
    const float* lp = lb + sy * lsh + sx * lsw;
    const int pred = argmax2(lp[0], lp[lsc]);
    const float* mp = mb + y * msh + x * msw;
    const float m0 = mp[0], m1 = mp[msc];
    const unsigned t1 = m1 > 0.5f ? 1u : 0u;
    const int label = argmax2(m0, m1);
    c[0] += (unsigned)pred & t1;
    c[1] += (unsigned)pred;
    c[2] += t1;
    c[3] += (label == 0 && pred == 0);
    c[4] += (label == 0 || pred == 0);
    c[5] += (label == 1 && pred == 1);
    c[6] += (label == 1 || pred == 1);
    c[7] += 1u;
  }
  __shared__ unsigned part[MET_THREADS / SSSEG_WAVE][8];
  const int lane = threadIdx.x & (SSSEG_WAVE - 1), wid = threadIdx.x / SSSEG_WAVE;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const unsigned v = wave_sum(c[k]);
    if (lane == 0) part[wid][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    unsigned long long s = 0;
#pragma unroll
    for (int i = 0; i < MET_THREADS / SSSEG_WAVE; ++i) s += part[i][threadIdx.x];
    if (s) atomicAdd(counts + b * 8 + threadIdx.x, s);
  }
}

// out[0] = mean_b dice_b  (dice_b = (2 I + 1) / (card + 1) in fp32, metrics.py:3-7)
// out[1], out[2] = 100 * IoU of class 0 / 1 over the batch (or the running totals), EMPTY = 1
// out[3] = mean of out[1..2] (lovasz.iou + mean, lovasz.py:54-73)
__global__ void seg_metrics_final_kernel(const unsigned long long* __restrict__ counts, int64_t B,
                                         unsigned long long* __restrict__ total, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double dice = 0.0;
  unsigned long long agg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t b = 0; b < B; ++b) {
    const unsigned long long* cb = counts + b * 8;
    const float inter = (float)cb[0];
    const float card = (float)cb[1] + (float)cb[2];
    dice += (double)((2.f * inter + 1.f) / (card + 1.f));
    for (int k = 0; k < 8; ++k) agg[k] += cb[k];
  }
  out[0] = (float)(dice / (double)B);
  if (total) {
    for (int k = 0; k < 8; ++k) {
      total[k] += agg[k];
      agg[k] = total[k];
    }
  }
  const float iou0 = agg[4] ? (float)((double)agg[3] / (double)agg[4]) : 1.f;
  const float iou1 = agg[6] ? (float)((double)agg[5] / (double)agg[6]) : 1.f;
  out[1] = 100.f * iou0;
  out[2] = 100.f * iou1;
  out[3] = 0.5f * (out[1] + out[2]);
}

// InferenceWrapper head (models/inference_wrapper.py:17-24): probabilities = sigmoid(logits) and the
// one-hot of argmax over 2 channels, for contiguous [B][2][HW] fp32 logits; 8 B read + 16 B written / px.
__global__ void prob_onehot_kernel(const float* __restrict__ logits, int64_t B, int64_t HW, float* __restrict__ prob,
                                   float* __restrict__ onehot) {
  const int64_t n = B * HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / HW, p = i - b * HW;
    const int64_t o0 = b * 2 * HW + p, o1 = o0 + HW;
    const float l0 = logits[o0], l1 = logits[o1];
    prob[o0] = 1.f / (1.f + expf(-l0));
    prob[o1] = 1.f / (1.f + expf(-l1));
    const int c = argmax2(l0, l1);
    onehot[o0] = c == 0 ? 1.f : 0.f;
    onehot[o1] = c == 1 ? 1.f : 0.f;
  }
}

}  // namespace

extern "C" int ssseg_seg_metrics(const float* logits, const int64_t* lstride, int64_t h, int64_t w,
                                 const float* mask, const int64_t* mstride, int64_t B, int64_t H, int64_t W,
                                 unsigned long long* counts, unsigned long long* total, float* out4,
                                 ssseg_stream_t stream) {
  if (!logits || !lstride || !mask || !mstride || !counts || !out4) return SSSEG_EINVAL;
  if (B <= 0 || h <= 0 || w <= 0 || H <= 0 || W <= 0) return SSSEG_EINVAL;
  if (B > 65535) return SSSEG_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  SSSEG_TRY(hipMemsetAsync(counts, 0, (size_t)B * 8 * sizeof(unsigned long long), s));
  const int64_t HW = H * W;
  int64_t bx = (HW + (int64_t)MET_THREADS * MET_PIX_PER_THREAD - 1) / ((int64_t)MET_THREADS * MET_PIX_PER_THREAD);
  if (bx < 1) bx = 1;
  if (bx > 4096) bx = 4096;
  hipLaunchKernelGGL(seg_metrics_count_kernel, dim3((unsigned)bx, (unsigned)B), dim3(MET_THREADS), 0, s, logits,
                     lstride[0], lstride[1], lstride[2], lstride[3], h, w, mask, mstride[0], mstride[1], mstride[2],
                     mstride[3], H, W, counts);
  hipLaunchKernelGGL(seg_metrics_final_kernel, dim3(1), dim3(64), 0, s, (const unsigned long long*)counts, B, total,
                     out4);
  SSSEG_LAUNCH_CHECK();
  return 0;
}

extern "C" int ssseg_prob_onehot(const float* logits, int64_t B, int64_t HW, float* prob, float* onehot,
                                 ssseg_stream_t stream) {
  if (!logits || !prob || !onehot || B <= 0 || HW <= 0) return SSSEG_EINVAL;
  const int64_t n = B * HW;
  int64_t nb = (n + 255) / 256;
  if (nb > 8192) nb = 8192;
  hipLaunchKernelGGL(prob_onehot_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, logits, B, HW, prob,
                     onehot);
  SSSEG_LAUNCH_CHECK();
  return 0;
}
