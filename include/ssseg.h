/* ssseg.h — C ABI of libssseg.so, the MI355X (gfx950) native hot path of the semi-supervised
 * segmentation trainer (drop-in for Luonic/semi-supervised_semantic_segmentation).
 *
 * The reference is pure Python; its "operator API" is a set of Python functions and nn.Module
 * constructors.  Each entry point below replaces the implicit PyTorch/cuDNN kernels
 * behind one of those reference call sites (cited per function).  The Python host layer
 * (semi-supervised_semantic_segmentation_amd/ssseg/native.py) binds these with ctypes.
 *
 * Conventions
 *   - every pointer is a DEVICE pointer unless named *_host; shapes/strides are int64_t;
 *   - every call takes the hipStream_t it runs on (PyTorch's current stream) and never
 *     synchronises, allocates or frees: callers own all buffers, workspaces included, so every
 *     call is capturable into a hipGraph;
 *   - return value: 0 on success, a hipError_t (>0) on a launch failure, or SSSEG_E* (<0) on an
 *     argument error detected on the host;
 *   - dtype codes: SSSEG_F32 = fp32, SSSEG_BF16 = bfloat16 (raw 16-bit, round-to-nearest-even).
 *   - activations inside the networks are NHWC (PyTorch channels_last); loss/CowMix tensors
 *     are NCHW-contiguous like the reference.
 */
#ifndef SSSEG_H
#define SSSEG_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* ssseg_stream_t;   /* == hipStream_t */

enum { SSSEG_F32 = 0, SSSEG_BF16 = 1 };
enum { SSSEG_OK = 0, SSSEG_EINVAL = -1, SSSEG_EUNSUPPORTED = -2, SSSEG_EWORKSPACE = -3 };

/* library identity: returns a static string "ssseg <version> gfx950" */
const char* ssseg_version(void);

/* ---------------------------------------------------------------------------------------------
 * CowMix  (reference cowmix.py)
 * ------------------------------------------------------------------------------------------- */

/* Workspace bytes for ssseg_cowmix_mask(B, H, W). */
size_t ssseg_cowmix_workspace_bytes(int64_t B, int64_t H, int64_t W);

/* Replaces generate_cowmix_masks_like's arithmetic (cowmix.py:40-69, dual_pass_gaussian_fileter2d
 * cowmix.py:27-37, generate_gaussian cowmix.py:6-11):
 *   K = 2*round(3*max(sigma))+1 (computed on device, so no host sync), per-sample Gaussian taps with
 *   the reference's +1-px offset, zero-padded vertical then horizontal pass (fp32, taps in order),
 *   per-sample mean / unbiased std, thr = erfinv(2p-1)*sqrt(2)*std + mean, mask = field > thr.
 * noise [B,H,W] f32, sigma [B] f32, p [B] f32 -> mask_out [B,H,W] f32 in {0,1}.
 * field_out (nullable) receives the filtered field; thr_out (nullable) [B] the thresholds. */
int ssseg_cowmix_mask(const float* noise, const float* sigma, const float* p, int64_t B, int64_t H,
                      int64_t W, float* mask_out, float* field_out, float* thr_out, void* workspace,
                      size_t workspace_bytes, ssseg_stream_t stream);

/* Device normal(0,1) noise for CowMix in throughput mode (counter-based Philox-4x32-10 +
 * Box-Muller): out[i] for i in [0,n).  Parity mode instead uploads the CPU generator's draws. */
int ssseg_normal_f32(float* out, int64_t n, uint64_t seed, uint64_t offset, ssseg_stream_t stream);

/* mix_with_mask (cowmix.py:72-73): out = a*m + b*(1-m), m [B,1,HW] broadcast over C.
 * a, b, out: [B,C,HW] (NCHW) of dtype `dt`; mask f32. */
int ssseg_mix(const void* a, const void* b, const float* mask, void* out, int64_t B, int64_t C,
              int64_t HW, int dt, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Layout / dtype conversion (model input/output boundary; the reference feeds NCHW fp32)
 * ------------------------------------------------------------------------------------------- */

/* x NCHW [N,C,H,W] (dtype dt_in) -> y NHWC [N,H,W,Cp] (dtype dt_out); channels C..Cp-1 zero. */
int ssseg_nchw_to_nhwc(const void* x, void* y, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Cp,
                       int dt_in, int dt_out, ssseg_stream_t stream);
/* x NHWC [N,H,W,ldc] (first C channels used) -> y NCHW [N,C,H,W]. */
int ssseg_nhwc_to_nchw(const void* x, void* y, int64_t N, int64_t C, int64_t H, int64_t W, int64_t ldc,
                       int dt_in, int dt_out, ssseg_stream_t stream);
/* elementwise dtype cast, n elements */
int ssseg_cast(const void* x, void* y, int64_t n, int dt_in, int dt_out, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Bilinear interpolation (F.interpolate mode='bilinear': losses.py:18, train.py:71,74,93,
 * unet.py:26 (align_corners=True), simple_unet.py:71)
 * Generic strides (elements) so NCHW and NHWC both work: x[n*sn + c*sc + h*sh + w*sw].
 * ------------------------------------------------------------------------------------------- */
int ssseg_bilinear_fwd(const void* x, void* y, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Ho,
                       int64_t Wo, const int64_t* x_strides4_host, const int64_t* y_strides4_host,
                       int align_corners, int dt, ssseg_stream_t stream);
/* gx = d(y)/d(x)^T gy (deterministic gather; gx overwritten, not accumulated). */
int ssseg_bilinear_bwd(const void* gy, void* gx, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Ho,
                       int64_t Wo, const int64_t* gy_strides4_host, const int64_t* gx_strides4_host,
                       int align_corners, int dt, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Losses.  Reductions are two-stage and deterministic; scalars live in device memory.
 * ------------------------------------------------------------------------------------------- */
size_t ssseg_reduce_workspace_bytes(int64_t n);

/* DenseBinaryCrossEntropyLossWithLogits(reduction='mean') (losses.py:41-48): loss_out[0] = mean. */
int ssseg_bce_logits_fwd(const float* x, const float* t, int64_t n, float* loss_out, void* ws,
                         size_t ws_bytes, ssseg_stream_t stream);
/* gx = (sigmoid(x) - t) / n * gout[0] */
int ssseg_bce_logits_bwd(const float* x, const float* t, int64_t n, const float* gout, float* gx,
                         ssseg_stream_t stream);

/* Consistency loss (inline at train.py:97-108).  s, t: [B,C,HW] f32 full-resolution logits.
 * out[0] = sum_pix(sum_c (sig(s)-sig(t))^2 * cm) / sum(cm)   (NaN when sum(cm)==0, like the ref)
 * out[1] = mean(cm) (logged confidence modulator);  out[2] = sum(cm) (kept for backward). */
int ssseg_consistency_fwd(const float* s, const float* t, int64_t B, int64_t C, int64_t HW, float thr,
                          float* out3, void* ws, size_t ws_bytes, ssseg_stream_t stream);
/* gs = 2 (sig(s)-sig(t)) sig(s)(1-sig(s)) cm / sum(cm) * gout[0]  (sum(cm) read from out3[2]) */
int ssseg_consistency_bwd(const float* s, const float* t, int64_t B, int64_t C, int64_t HW, float thr,
                          const float* out3, const float* gout, float* gs, ssseg_stream_t stream);

/* Binary Lovász (losses.binary_lovasz_loss_with_logits losses.py:239-250 -> lovasz_softmax
 * lovasz.py:155-201 with classes=[1], per_image=True).  logits, target [B,C,HW] f32.
 * Per image: labels = argmax_c target, e = |[label==1] - logit1|, sort e descending, Lovász gradient
 * (lovasz_grad lovasz.py:19-31) by a scan, loss_b = <e_sorted, grad>;
 * loss_out[0] = sum_b loss_b*valid_b / (sum valid + 0.001).  grad_out (nullable) [B,C,HW]:
 * d loss/d logits (channel 1 only, channel 0 written 0), scaled by gout[0] if gout != NULL. */
size_t ssseg_lovasz_workspace_bytes(int64_t B, int64_t HW);
int ssseg_lovasz_fwd(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW,
                     float* loss_out, void* ws, size_t ws_bytes, ssseg_stream_t stream);
int ssseg_lovasz_bwd(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW,
                     const float* gout, float* grad_out, void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Teacher EMA and optimiser over flat parameter arenas
 * ------------------------------------------------------------------------------------------- */

/* mean_teacher.update_ema_variables (mean_teacher.py:5-18), parameters only (buffers are aliased
 * on the host):  ema = fma(param, (float)(1-alpha), round(ema*alpha))  — bit-exact with torch CPU. */
int ssseg_ema_update(float* ema, const float* param, int64_t n, double alpha, ssseg_stream_t stream);

/* sum of squares of x[0,n) accumulated into out[0] (f32, caller zeroes out first: clip_grad_norm_). */
int ssseg_sqnorm_accum(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* torch.nn.utils.clip_grad_norm_ (train.py:122) + torch.optim.SGD(momentum, weight_decay) step
 * (default_config.py:151-154), fused:  coef = min(1, max_norm/(sqrt(sqnorm[0])+1e-6)) (skipped when
 * max_norm <= 0); g *= coef; d = g + wd*p; buf = first ? d : momentum*buf + d; p -= lr*buf.
 * bf16_shadow (nullable) receives bf16(p) for the compute path.  grad is left clipped. */
int ssseg_sgd_step(float* param, float* grad, float* momentum_buf, uint16_t* bf16_shadow, int64_t n,
                   float lr, float momentum, float weight_decay, float max_norm, const float* sqnorm,
                   int first_step, ssseg_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SSSEG_H */
