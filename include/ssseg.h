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
 *   - dtype codes: SSSEG_F32 = fp32, SSSEG_BF16 = bfloat16 (raw 16-bit, round-to-nearest-even),
 *     SSSEG_F16 = IEEE half (the fp16 compute mode of config C5; same storage and MFMA rate as bf16).
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

enum { SSSEG_F32 = 0, SSSEG_BF16 = 1, SSSEG_F16 = 2, SSSEG_F64 = 3 /* collectives only */ };
enum { SSSEG_OK = 0, SSSEG_EINVAL = -1, SSSEG_EUNSUPPORTED = -2, SSSEG_EWORKSPACE = -3, SSSEG_ECOMM = -4 };

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

/* Throughput-mode draws of generate_cowmix_masks_like's random inputs (cowmix.py:44-55), all on device
 * so a captured step replays fresh masks: p ~ U(prop_lo, prop_hi), sigma = exp(U(log lo, log hi)),
 * noise ~ N(0,1) [B*HW]; Philox counter = offset (+B for the noise).  Parity mode instead draws the
 * same quantities from the CPU torch generator in the reference's order and uploads them. */
int ssseg_cowmix_draw(float* p, float* sigma, float* noise, int64_t B, int64_t HW, double prop_lo, double prop_hi,
                      double sigma_lo, double sigma_hi, uint64_t seed, uint64_t offset, ssseg_stream_t stream);
/* as ssseg_cowmix_draw with the Philox counter offset read from device memory and advanced there by
 * B + ceil(B*HW/4) + 1 after the draw (the host form's sequence): a captured HIP graph replays fresh draws. */
int ssseg_cowmix_draw_dev(float* p, float* sigma, float* noise, int64_t B, int64_t HW, double prop_lo, double prop_hi,
                          double sigma_lo, double sigma_hi, uint64_t seed, unsigned long long* offset_dev,
                          ssseg_stream_t stream);

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

/* ssseg_bilinear_bwd for 16-bit NHWC tensors in two separable passes (output rows summed over their columns into an
 * fp32 workspace, then combined over the rows): bitwise the same gx, parallel over Ho x W chunks instead of walking the
 * whole output window per input chunk.  Falls back to ssseg_bilinear_bwd where the NHWC kernels do not apply. */
size_t ssseg_bilinear_bwd_workspace_bytes(int64_t N, int64_t C, int64_t W, int64_t Ho);
int ssseg_bilinear_bwd_ws(const void* gy, void* gx, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                          const int64_t* gy_strides4_host, const int64_t* gx_strides4_host, int align_corners, int dt,
                          void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* Rotation about the image centre by angle_deg (counter-clockwise, OpenCV / kornia get_rotation_matrix2d),
 * bilinear with zero padding, NCHW contiguous fp32: reversible_augmentations.Rotate.apply / reverse
 * (reference reversible_augmentations.py:5-23, kornia.rotate; kornia is unpinned and absent, parity with it is
 * unpinned).  bwd: gx = (d y / d x)^T gy (gx overwritten). */
int ssseg_rotate_fwd(const float* x, float* y, int64_t N, int64_t C, int64_t H, int64_t W, double angle_deg,
                     ssseg_stream_t stream);
int ssseg_rotate_bwd(const float* gy, float* gx, int64_t N, int64_t C, int64_t H, int64_t W, double angle_deg,
                     ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Train-time augmentations on the device (reference configs/default_config.py:179-212: the albumentations
 * ReplayCompose pipelines the reference datasets apply per sample, data/dataset.py:71-74,
 * unsupervised_dataset.py:20-21).  The host (data/device_augment.py) draws each sample's parameters in the
 * pipeline's order and uploads one record per sample; images are uint8 NHWC (3 channels) after the host's
 * LongestMaxSize + PadIfNeeded, masks uint8 NHWC.  albumentations / cv2 are absent: parity with them is unpinned.
 * ------------------------------------------------------------------------------------------- */
typedef struct ssseg_aug_warp_params {
  float a[6];        /* input-image coords = A * q, q = the crop-grid pixel after the distortion (OpenCV centres) */
  int32_t distort;   /* 0 none, 1 ElasticTransform, 2 GridDistortion, 3 OpticalDistortion */
  int32_t field;     /* ElasticTransform: index of this sample's displacement field in `fields` */
  float m[6];        /* ElasticTransform: inverse of its random affine (applied to (x + dx, y + dy)) */
  float k, cx, cy, fx, fy;   /* OpticalDistortion: radial k (k1 = k2 = k), centre, focal lengths */
  int32_t border;    /* image / mask border: 0 constant 0, 1 reflect-101 */
} ssseg_aug_warp_params;

typedef struct ssseg_aug_color_params {
  int32_t bc;    float alpha, beta;      /* RandomBrightnessContrast: floor(clip(v * alpha + beta * 255)) */
  int32_t gray;                          /* ToGray */
  int32_t rgb;   float shift[3];         /* RGBShift: floor(clip(v + shift)) */
  int32_t hsv;   float hsv_shift[3];     /* HueSaturationValue on 8-bit HSV (H in [0, 180)) */
  int32_t iso;   float iso_color_std, iso_intensity;   /* ISONoise: hue N(0, color_std), luminance Poisson */
} ssseg_aug_color_params;

/* One resampling per sample: out pixel (x, y) -> distortion -> A -> bilinear image sample (rounded to the uint8
 * grid), nearest mask sample.  gmaps: [N][Wo + Ho] GridDistortion axis maps; fields: [nf][Ho][Wo][2] elastic
 * displacements.  out_nchw01 = 0: out_img NHWC [0, 255] (feeds ssseg_aug_color); 1: NCHW [0, 1] (ToFloat).
 * out_mask: NCHW [0, 1]; mask may be NULL (unsupervised pipeline). */
int ssseg_aug_warp(const uint8_t* img, const uint8_t* mask, int64_t mask_c, int64_t N, int64_t H, int64_t W,
                   float* out_img, float* out_mask, int64_t Ho, int64_t Wo, const ssseg_aug_warp_params* params,
                   const float* gmaps, const float* fields, int out_nchw01, ssseg_stream_t stream);
/* Brightness / contrast, gray, RGB shift / HSV on an NHWC [0, 255] float batch, in place. */
int ssseg_aug_color(float* img, int64_t N, int64_t H, int64_t W, const ssseg_aug_color_params* params,
                    ssseg_stream_t stream);
/* Separable Gaussian per sample, in place (tmp: same size): radius[n] (0 = untouched), weights [N][wmax];
 * sym_border 0 = reflect-101 (cv2), 1 = symmetric (scipy 'reflect'); round_u8_out rounds to the uint8 grid. */
int ssseg_aug_blur(float* x, float* tmp, int64_t N, int64_t H, int64_t W, int64_t C, const int32_t* radius,
                   const float* weights, int64_t wmax, int sym_border, int round_u8_out, ssseg_stream_t stream);
/* ISONoise on the samples with params[n].iso (per-image luminance std from fp64 sums in stats_ws [N][2]), then
 * ToFloat: out = NCHW [0, 1]. */
int ssseg_aug_iso_finish(const float* img, float* out, int64_t N, int64_t H, int64_t W,
                         const ssseg_aug_color_params* params, double* stats_ws, uint64_t seed, ssseg_stream_t stream);
/* uniform(-1, 1) noise (Philox, key = seed) for the ElasticTransform displacement fields. */
int ssseg_aug_uniform_field(float* f, int64_t n, uint64_t seed, ssseg_stream_t stream);

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
 * lovasz.py:155-201 with classes=[1], per_image=True).  logits, target [B,C,HW] f32, 1 <= B <= 4096.
 * Per image: labels = argmax_c target, e = |[label==1] - logit1|, sort e descending, Lovász gradient
 * (lovasz_grad lovasz.py:19-31) by a scan, loss_b = <e_sorted, grad>;
 * loss_out[0] = sum_b loss_b*valid_b / (sum valid + 0.001).  grad_out (nullable) [B,C,HW]:
 * d loss/d logits (channel 1 only, channel 0 written 0), scaled by gout[0] if gout != NULL. */
size_t ssseg_lovasz_workspace_bytes(int64_t B, int64_t HW);
int ssseg_lovasz_fwd(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW,
                     float* loss_out, void* ws, size_t ws_bytes, ssseg_stream_t stream);
int ssseg_lovasz_bwd(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW,
                     const float* gout, float* grad_out, void* ws, size_t ws_bytes, ssseg_stream_t stream);
/* The backward of the immediately preceding ssseg_lovasz_fwd with the same logits, target and workspace (kept
 * unchanged in between): the forward leaves the per-pixel Lovász gradient in sorted-rank terms and the per-image scale
 * valid_b / denom in ws, so the backward is one scatter launch instead of a second sort (bitwise the same gradient as
 * ssseg_lovasz_bwd). */
int ssseg_lovasz_bwd_from_fwd(const float* logits, const float* target, int64_t B, int64_t C, int64_t HW,
                              const float* gout, float* grad_out, const void* ws, size_t ws_bytes,
                              ssseg_stream_t stream);

/* RMILoss, sigmoid form (losses.RMILoss.forward -> forward_sigmoid -> rmi_lower_bound, losses.py:480-592; the
 * default-config loss, configs/default_config.py:147).  logits, target [N,C,H,W] f32 contiguous.
 * pool (k, s, pad): avg_pool2d(k, s, pad, count_include_pad) of losses.py:534-538 (k == s, pad = k/2; (1,1,0) for
 * rmi_pool='none' or stride <= 1).  radius 1..3 (rmi_radius; D = radius^2 <= 9).  (N*C) % num_classes == 0.
 * Forward: loss_out[0] = sum_k float(mean over rows of rmi.view(-1, num_classes)[:, k]) / D, rmi per (n, c) from
 * fp64 centred covariances, inverse and Cholesky log-det.  want_grad != 0 also leaves the backward coefficients in
 * ws; ssseg_rmi_bwd (same ws, same geometry) then writes grad_out [N,C,H,W] = gout[0] * d loss / d logits.
 * A non-positive-definite matrix gives a NaN loss (the reference's torch.cholesky raises); the +5e-4*I of
 * losses.py:283,553-563 makes every covariance PD in exact arithmetic, so only degenerate fp64 input reaches it, and a
 * NaN loss is visible to the caller (the fp16 loss scaler then skips the step).  Workspace 0 = the
 * geometry is not supported. */
size_t ssseg_rmi_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W, int64_t num_classes, int64_t radius,
                                 int64_t pool_k, int64_t pool_s, int64_t pool_pad);
int ssseg_rmi_fwd(const float* logits, const float* target, int64_t N, int64_t C, int64_t H, int64_t W,
                  int64_t num_classes, int64_t radius, int64_t pool_k, int64_t pool_s, int64_t pool_pad, int want_grad,
                  float* loss_out, void* ws, size_t ws_bytes, ssseg_stream_t stream);
int ssseg_rmi_bwd(const float* logits, int64_t N, int64_t C, int64_t H, int64_t W, int64_t num_classes,
                  int64_t radius, int64_t pool_k, int64_t pool_s, int64_t pool_pad, const float* gout,
                  float* grad_out, void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Teacher EMA and optimiser over flat parameter arenas
 * ------------------------------------------------------------------------------------------- */

/* mean_teacher.update_ema_variables (mean_teacher.py:5-18), parameters only (buffers are aliased
 * on the host):  ema = fma(param, (float)(1-alpha), round(ema*alpha))  — bit-exact with torch CPU. */
int ssseg_ema_update(float* ema, const float* param, int64_t n, double alpha, ssseg_stream_t stream);

/* torch.sigmoid on contiguous fp32 (the discriminator input of the adversarial branch, configs C5):
 * y = 1/(1+exp(-x)); backward gx = gy * y * (1 - y) from the saved output. */
int ssseg_sigmoid_fwd(const float* x, float* y, int64_t n, ssseg_stream_t stream);
int ssseg_sigmoid_bwd(const float* y, const float* gy, float* gx, int64_t n, ssseg_stream_t stream);

/* out = a*x + b*y over n fp32 (y may be NULL: out = a*x; out may alias x or y): the weighted sums of the
 * loss terms (CalculateLoss weights losses.py:19, 1/virtual_batch_size_multiplier train.py:61, consistency
 * weight x float(epoch > 25) train.py:112) and their backward. */
int ssseg_axpby(const float* x, float a, const float* y, float b, float* out, int64_t n, ssseg_stream_t stream);
/* x[i] *= a (in place): the 1/world average after a SUM all-reduce on backends without AVG (gloo). */
int ssseg_scale_f32(float* x, int64_t n, float a, ssseg_stream_t stream);

/* sum of squares of x[0,n) accumulated into out[0] (f32, caller zeroes out first: clip_grad_norm_). */
int ssseg_sqnorm_accum(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* torch.nn.utils.clip_grad_norm_ (train.py:122) + torch.optim.SGD(momentum, weight_decay) step
 * (default_config.py:151-154), fused:  coef = min(1, max_norm/(sqrt(sqnorm[0])+1e-6)) (skipped when
 * max_norm <= 0); g *= coef; d = g + wd*p; buf = first ? d : momentum*buf + d; p -= lr*buf.
 * bf16_shadow (nullable) receives bf16(p) for the compute path.  grad is left clipped.
 * amp_state (nullable; the fp16 mode's dynamic loss scale [scale, tracker, found_inf, 1/scale]): the
 * gradients are loss-scaled: they are unscaled by 1/scale first, and a non-finite sqnorm (which must then be
 * given) skips the step entirely (GradScaler semantics, decided on the device: no host sync). */
int ssseg_sgd_step(float* param, float* grad, float* momentum_buf, uint16_t* bf16_shadow, int64_t n,
                   float lr, float momentum, float weight_decay, float max_norm, const float* sqnorm,
                   int first_step, const float* amp_state, ssseg_stream_t stream);
/* Dynamic loss-scale update after a step (torch.cuda.amp.GradScaler.update): non-finite sqnorm[0] ->
 * scale *= backoff, tracker = 0, found_inf = 1; else tracker += 1 and scale *= growth every `interval`
 * finite steps.  state = [scale, tracker, found_inf, 1/scale] on the device. */
int ssseg_amp_update(float* state, const float* sqnorm, float growth, float backoff, int interval,
                     ssseg_stream_t stream);
/* y = x * s[0] (s a device scalar): the loss-scaled gradient entering the backward pass (fp16 mode). */
int ssseg_scale_by(const float* x, const float* s, float* y, int64_t n, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Convolution engine (implicit GEMM on MFMA).  Replaces the cuDNN/MIOpen convolutions behind
 * nn.Conv2d / nn.ConvTranspose2d in unet.py:8,21,27,85, simple_unet.py:64,72,138, the encoders,
 * and their autograd backward (train.py:61,115).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int64_t N, H, W, C, ldx;        /* input activations NHWC; C = physical channels (multiple of 8 bf16 / 4 f32),
                                     ldx = pixel stride in elements */
  int64_t OH, OW;                 /* GEMM spatial grid (per image) */
  int64_t K;                      /* output channels (GEMM N) */
  int64_t R, S;                   /* taps */
  int64_t sy, sx, dy, dx, py, px; /* input row = oy*sy + r*dy + py (zero outside), same for columns */
  int64_t outH, outW;             /* output map; pixel written = (oy*osy + ooy, ox*osx + oox) */
  int64_t osy, osx, ooy, oox;
  int64_t ldy;                    /* output pixel stride (elements) */
  int64_t ldw;                    /* packed weight row stride (rows = K, row = [R][S][C]) */
} ssseg_conv_desc;

/* y[m][n] = act(sum_k A[m][k] * W[n][k] + bias[n]).  Used for the forward conv, the stride-1 dgrad
 * (flipped packing), every phase of a strided dgrad and of ConvTranspose2d(4,2,1) (dilation -1 and
 * strided output), and the ConvTranspose2d input gradient.  dt: input/weight dtype; dt_out: output.
 * When R*S == 0 (an output phase no tap reaches) the phase is zero-filled. */
int ssseg_conv_igemm(const void* x, const void* w, void* y, const ssseg_conv_desc* desc_host, int dt, int dt_out,
                     const float* bias, int relu, void* ws, size_t ws_bytes, ssseg_stream_t stream);
/* Activation codes of the fused epilogues, BN kernels and ssseg_act_bwd: ReLU (unet.py:10, encoders),
 * ReLU6 (MobileNetV2 ConvBNReLU, mobilenetv2.py:39), LeakyReLU(slope) (discriminator.py:16). */
#define SSSEG_ACT_NONE 0
#define SSSEG_ACT_RELU 1
#define SSSEG_ACT_RELU6 2
#define SSSEG_ACT_LEAKY 3

/* Fused conv epilogue (ssseg_conv_igemm_epi):
 *   y[m][n]   = act(acc[m][n] * scale[n] + shift[n] + residual[pixel(m)][n])
 *   aux[m][n] = acc[m][n]                          (optional; same pixel stride as y)
 * scale NULL = 1, shift NULL = 0, residual NULL = 0 (dtype dt_out, pixel stride ldr), aux NULL = not written.
 * Folds an eval-mode BatchNorm (ssseg_bn_fold) and the Bottleneck identity add + ReLU (unet.py:9-10,
 * encoder blocks) into the conv that produces them; aux keeps the pre-BN activation the BN backward
 * needs when the eval pass is differentiated (consistency pass, train.py:90-92). */
typedef struct ssseg_conv_epilogue {
  const float* scale;
  const float* shift;
  const void* residual;
  int64_t ldr;
  void* aux;
  int32_t relu;    /* activation code SSSEG_ACT_* (1 = ReLU, the historical flag) */
  float slope;     /* LeakyReLU negative slope (SSSEG_ACT_LEAKY) */
  /* Fused training-BatchNorm statistics (optional; the BN that consumes y, unet.py:9 / every encoder BN in
   * train mode): per output tile row r, stats[(2r)*stats_ld + c] = sum of y[.][c] and stats[(2r+1)*stats_ld + c]
   * = sum of y^2 over the tile's pixels (fp64, of the value as stored), c < stats_ld; *stats_rows_host receives
   * the number of rows written (<= ceil(M/64)).  Reduce them with ssseg_bn_partials_finalize: the separate
   * statistics pass over y (ssseg_bn_stats) is not needed.  Not allowed with an empty tap set (R*S == 0). */
  double* stats;
  int64_t stats_ld;
  int64_t* stats_rows_host;
} ssseg_conv_epilogue;
int ssseg_conv_igemm_epi(const void* x, const void* w, void* y, const ssseg_conv_desc* desc_host, int dt, int dt_out,
                         const ssseg_conv_epilogue* epi, void* ws, size_t ws_bytes, ssseg_stream_t stream);
/* ssseg_conv_igemm_epi for an input gradient whose input was the forward output y of an activation (act =
 * SSSEG_ACT_RELU or SSSEG_ACT_LEAKY with its slope; the discriminator's Conv4x4 + LeakyReLU(0.2) pairs,
 * discriminator.py:14-17): epi->residual is that y (not an addend), and the stored value is the activation's backward
 * applied in place, (y > 0 ? v : v * slope) -- the producer's separate activation-backward pass is not needed.
 * epi carries no shift / activation / aux.  Optional: epi->scale multiplies the masked value (a folded eval
 * BatchNorm's backward, dconv = scale * mask(dy)); epi->stats makes the rows the GRADIENT statistics of the
 * BatchNorm that produced y: per tile row r, (sum m, sum m * y) of the masked value m before the scale, rounded to
 * the output type (fp64 sums) -- reduce them with ssseg_bn_gstat_finalize instead of a ssseg_bn_bwd_reduce pass over
 * dy and x (the reference's BN backward, unet.py:9-10 / resnet Bottleneck bn1, bn2 -> ReLU -> next conv). */
int ssseg_conv_igemm_epi_actmask(const void* x, const void* w, void* y, const ssseg_conv_desc* desc_host, int dt,
                                 int dt_out, const ssseg_conv_epilogue* epi, int act, float slope, void* ws,
                                 size_t ws_bytes, ssseg_stream_t stream);
/* Virtual channel concat of a conv input (reference models/unet.py:44-45, torch.cat((x, skip), 1) feeding
 * UpBlock.conv3_0): input channels [0, c1) are read from x (pixel stride desc.ldx) and [c1, desc.C) from x2
 * (pixel stride ldx2, channel 0 of x2 = input channel c1); same N x H x W.  c1 and C - c1 are multiples of 64
 * (the LDS-DMA engine takes whole 64-channel k-blocks from one source).  The concatenated tensor is never
 * written: forward, input-gradient and weight-gradient launches read the two parts where they lie. */
typedef struct {
  const void* x2;
  int64_t c1;
  int64_t ldx2;
} ssseg_vcat;

/* ssseg_conv_igemm_epi over a virtual concat input (16-bit dt == dt_out; SSSEG_EUNSUPPORTED where the LDS-DMA
 * engine cannot run the geometry: the caller then materialises the concat).  Bit-identical to the same launch on
 * the materialised tensor. */
int ssseg_conv_igemm_epi_vcat(const void* x, const ssseg_vcat* vc, const void* w, void* y,
                              const ssseg_conv_desc* desc_host, int dt, int dt_out, const ssseg_conv_epilogue* epi,
                              void* ws, size_t ws_bytes, ssseg_stream_t stream);
/* ssseg_conv_igemm_epi with a SPLIT output: channels [0, ysplit->c1) of each output pixel go to y (pixel stride
 * desc.ldy >= c1), channels [c1, K) to ysplit->x2 at channel n - c1 (pixel stride ysplit->ldx2).  The input
 * gradient of a virtual concat (the UNet decoder's conv3_0, unet.py:44-47: dgrad of torch.cat((up, skip), 1)) is
 * written straight into the gradients of its two parts: no [up | skip] gradient tensor, no split copies.
 * c1 % 8 == 0; 16-bit dt == dt_out; the epilogue may carry scale / shift / act but no residual, aux or statistics
 * (SSSEG_EUNSUPPORTED).  Bit-identical to the unsplit launch followed by the two channel copies. */
int ssseg_conv_igemm_epi_vsplit(const void* x, const void* w, void* y, const ssseg_vcat* ysplit,
                                const ssseg_conv_desc* desc_host, int dt, int dt_out, const ssseg_conv_epilogue* epi,
                                void* ws, size_t ws_bytes, ssseg_stream_t stream);
/* The output phases of a transposed conv in ONE launch (ConvTranspose2d(4,2,1): four 2x2-tap phases over the same
 * input; on 16x16..32x32 inputs a single phase has too few tiles to fill 256 CUs).  desc describes a phase's GEMM
 * (every phase: same K, taps R x S, weight stride ldw, output sub-grid OH x OW); phase_geom[4*p .. 4*p+3] =
 * (py, px, ooy, oox) of phase p, w[p] its packed weights.  1 <= nphase <= 4; dt = dt_out = SSSEG_BF16 / SSSEG_F16.
 * Same epilogue contract as ssseg_conv_igemm_epi; fused statistics rows: phase-major, nphase x ceil(M / BM).
 * Replaces the per-phase loop of nn.ConvTranspose2d forward (unet.py:21, train_upsampling=True). */
int ssseg_conv_igemm_phases(const void* x, void* y, const ssseg_conv_desc* desc_host, int dt, int dt_out,
                            const ssseg_conv_epilogue* epi, int64_t nphase, const int64_t* phase_geom,
                            const void* const* w, ssseg_stream_t stream);
/* ssseg_conv_igemm_phases with a workspace (ssseg_conv_igemm_phases_workspace_bytes; 0 = the launch does not split):
 * the phases of a tile-starved transposed conv (e.g. ConvTranspose2d 2048 -> 128 over 16x16 maps) run the
 * deterministic split-K described at ssseg_conv_igemm_workspace_bytes. */
size_t ssseg_conv_igemm_phases_workspace_bytes(const ssseg_conv_desc* desc_host, int64_t nphase, int dt);
int ssseg_conv_igemm_phases_ws(const void* x, void* y, const ssseg_conv_desc* desc_host, int dt, int dt_out,
                               const ssseg_conv_epilogue* epi, int64_t nphase, const int64_t* phase_geom,
                               const void* const* w, void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* First conv of an encoder on a 3-channel image (<= 4 real input channels, S <= 8 taps per filter row, R in {3, 7},
 * dilation 1, stride x <= 2, OW % 128 == 0; e.g. the ResNet-50 stem 7x7/s2/p3): k = (s, c) of one filter row per
 * 32-deep MFMA step, operands from the block's image patch (channels 0..3 of each pixel; ldx % 4 == 0).  w4 = ssseg_weight_pack output
 * with Cp = 4, layout 0, full taps: [K][R][S][4].  K % 16 == 0; dt = SSSEG_BF16 or SSSEG_F16 (output dtype = dt).
 * Same epilogue contract as ssseg_conv_igemm_epi (fused BN statistics rows: ceil(M / 128)).  Replaces the
 * engine launch of the stem in Conv2d forward (reference: the encoders' first conv, e.g. SURVEY §0.4 ResNet-50). */
int ssseg_conv_stem_epi(const void* x, const void* w4, void* y, const ssseg_conv_desc* desc_host, int dt,
                        const ssseg_conv_epilogue* epi, ssseg_stream_t stream);
/* Workspace for ssseg_conv_igemm(_epi / _vcat / _vsplit): non-zero when the 16-bit launch splits K across workgroups
 * (deterministic split-K, S chosen from the geometry alone, knob 14: fewer than 512 nominal 128 x 64 output tiles and
 * >= 64 64-deep k-tiles -- ResNet layer3/4 at 32x32 / 16x16, S = 2 or 4 -- or fewer than 256 tiles and >= 8 k-tiles --
 * HarDNet's growth layers at 8x8 - 32x32, the largest S of 8 / 4 / 2 with <= 512 blocks and >= 4 k-tiles a slice).  Each slice writes fp32 partials,
 * the last-arriving slice of a tile (an agent-scope ticket) sums the S partials in slice order and runs the full fused
 * epilogue (affine, residual, activation, raw copy, BN statistics): the result is bitwise reproducible and identical
 * for every tile config.  The workspace is caller-owned scratch (no contents carried between calls); passing none
 * (or a smaller one) runs the launch unsplit. */
size_t ssseg_conv_igemm_workspace_bytes(const ssseg_conv_desc* desc_host, int dt);

/* Runtime variant switches for A/B measurement.  knob 0: register-staged pipeline depth (0 = one k-tile in
 * flight, default; 1 = two); knob 1: fp32-atomic split-K of the register-staged kernel (-1 = off, default; order-dependent sums);
 * knob 2: 64x64 small-M tiles of the register-staged kernel (0 = auto); knob 3: bf16 LDS-DMA kernel
 * (0 = on, -1 = off); knob 4: bf16 variant (0 = auto, 1..10 / 12..23 = an LDS-DMA tile config, 11 = register-staged,
 * 24 / 25 = the halo-tiled 3x3 kernels, 26 / 27 = the pointwise kernels, each where it applies);
 * knob 5: autotune unseen geometries once on the caller's stream (1 = on, default; 0 = static rule);
 * knob 6 (write 1): clear the per-geometry variant cache; knob 7: LDS-staged coalesced epilogue of the LDS-DMA
 * kernel (0 = on, default; -1 = off); knob 8: LDS-DMA weight gradient (0 = on, -1 = register-staged);
 * knob 9: LDS-DMA weight-gradient tile config (0 = the static plan, n = config n); knob 10: weight-gradient
 * split count in percent of the plan's (100 = default); knob 11: halo-tiled 3x3 kernels (0 = on, -1 = off);
 * knob 12: fused-statistics experiment switch (0 = normal); knob 13: pointwise kernels (0 = on, -1 = off);
 * knob 14: deterministic split-K of the LDS-DMA configs (0 = the geometry rule, default; -1 = off; 2 / 4 / 8 = forced S);
 * knob 15: the single-buffered two-blocks-per-CU halo conv, variant 28 (0 = on, -1 = off);
 * knob 16: the halo convs' 32- and 16-wide tiles on 32^2 / 16^2 maps (0 = on, -1 = 64-wide tiles only).
 * Forward variants never change results; the
 * weight-gradient knobs change the fp32 summation order of dW.  Not thread-safe. */
int ssseg_set_knob(int id, int value);

/* The conv engine's variant table (geometry key -> chosen variant; host memory).  export: writes min(n, cap) rows in
 * key order and returns n (cap 0: the count only).  import: adds rows (overwrite != 0: replaces existing ones); a
 * variant id the engine does not have is SSSEG_EINVAL.  Lets rank 0 of a data-parallel job tune and the other ranks
 * take its table (ssseg/tune.py), so every rank launches the same kernels and only one tunes.  Not thread-safe with
 * concurrent launches of unseen geometries. */
int64_t ssseg_tune_table_export(unsigned long long* keys_host, int32_t* variants_host, int64_t cap);
int ssseg_tune_table_import(const unsigned long long* keys_host, const int32_t* variants_host, int64_t n,
                            int overwrite);

/* dW = sum over output pixels of dY[p][k] * x_col[p][(r,s,c)] (split-K fp32 slabs + deterministic
 * reduce).  dy is [N][OH][OW] with pixel stride desc.ldy.  layout 0: dw [K][R][S][C];
 * layout 1: dw [k_real][c_real][R][S] (PyTorch OIHW / ConvTranspose2d [Cin][Cout][R][S]).
 * accumulate != 0 adds into dw (the reference accumulates the two backward passes, train.py:61,115). */
size_t ssseg_conv_wgrad_workspace_bytes(const ssseg_conv_desc* desc_host, int dt);
int ssseg_conv_wgrad(const void* x, const void* dy, float* dw, const ssseg_conv_desc* desc_host, int dt, int64_t c_real,
                     int64_t k_real, int layout, int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* Deferred split reductions: with ssseg_wgrad_defer_reduce(1) (per host thread) the weight-gradient entry points below
 * launch their split kernels but only RECORD the slab reduction each would launch (the slab workspace must then stay
 * valid until the flush); ssseg_wgrad_reduce_flush launches every recorded reduction on `stream`, up to 40 per launch
 * (descriptors in the kernel arguments: capturable), with the same per-element summation as the immediate reduction
 * (bitwise the same dW).  The training step's weight gradients, issued back to back after its two backward passes
 * join (train.py:61 and :115 accumulate into .grad before clip + SGD), become one or two reduction launches instead of
 * one per conv.  pending: the number recorded and not yet flushed. */
int ssseg_wgrad_defer_reduce(int on);
int64_t ssseg_wgrad_reduce_pending(void);
int ssseg_wgrad_reduce_flush(ssseg_stream_t stream);

/* The same weight gradient over TWO pixel sets in one launch: dw (+)= sum over (x, dy) of batch desc.N plus
 * (x2, dy2) of batch n2 (same geometry and strides otherwise).  The supervised and the consistency backward
 * of a student conv (train.py:61 and :115, accumulated into one .grad before clip + SGD) become one
 * contraction: one split plan over the union of the pixels, one deterministic reduce.  Kernels without the
 * LDS-DMA path run the two contributions one after the other. */
size_t ssseg_conv_wgrad2_workspace_bytes(const ssseg_conv_desc* desc_host, int64_t n2, int dt);
int ssseg_conv_wgrad2(const void* x, const void* dy, const void* x2, const void* dy2, int64_t n2, float* dw,
                      const ssseg_conv_desc* desc_host, int dt, int64_t c_real, int64_t k_real, int layout,
                      int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* Weight gradients over a virtual concat input (ssseg_vcat, same contract as ssseg_conv_igemm_epi_vcat; vc / vc2
 * describe the second part of x / x2, with the same c1 and ldx2).  The workspace queries above cover them.
 * SSSEG_EUNSUPPORTED where the LDS-DMA weight-gradient kernel cannot run the geometry. */
int ssseg_conv_wgrad_vcat(const void* x, const ssseg_vcat* vc, const void* dy, float* dw,
                          const ssseg_conv_desc* desc_host, int dt, int64_t c_real, int64_t k_real, int layout,
                          int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream);
int ssseg_conv_wgrad2_vcat(const void* x, const ssseg_vcat* vc, const void* dy, const void* x2, const ssseg_vcat* vc2,
                           const void* dy2, int64_t n2, float* dw, const ssseg_conv_desc* desc_host, int dt,
                           int64_t c_real, int64_t k_real, int layout, int accumulate, void* ws, size_t ws_bytes,
                           ssseg_stream_t stream);

/* Pack fp32 master weights into the engine's [Kd][Rn][Sn][Cp] layout (dtype dt; rows >= Kr and
 * channels >= Cd zero): layout 0 reads src[k][c][r][s] (src is [Kr][Cd][Rs][Ss]), layout 1 reads
 * src[c][k][r][s] (src is [Cd][Kr][Rs][Ss]); r = r0 + rr*rstep, s = s0 + ss*sstep. */
int ssseg_weight_pack(const float* src, void* dst, int64_t Kd, int64_t Kr, int64_t Cd, int64_t Rs, int64_t Ss,
                      int64_t Cp, int layout, int64_t r0, int64_t rstep, int64_t Rn, int64_t s0, int64_t sstep,
                      int64_t Sn, int dt, ssseg_stream_t stream);

/* Batched repack: every conv's packed layouts refreshed by ONE launch after the master weights change
 * (optimizer step, EMA; train.py:122-124, mean_teacher.py:10-11).  descs points to DEVICE memory
 * holding n descriptors with the ssseg_weight_pack arguments; every filter has Rs * Ss <= 135 taps
 * (larger ones: ssseg_weight_pack). */
typedef struct ssseg_pack_desc {
  const float* src;
  void* dst;
  int64_t Kd, Kr, Cd, Rs, Ss, Cp;
  int64_t layout, r0, rstep, Rn, s0, sstep, Sn;
} ssseg_pack_desc;
int ssseg_weight_pack_batch(const ssseg_pack_desc* descs, int64_t n, int dt, ssseg_stream_t stream);

/* Depthwise convolution (groups == channels; MobileNetV2 ConvBNReLU(groups=hidden), mobilenetv2.py:34-39,58).
 * The descriptor is the conv engine's with K == C and no output phases; weights packed [R*S][ldw] in the
 * compute dtype (ssseg_weight_pack layout 1, Kd = Kr = 1).  fwd takes the same fused epilogue as the conv
 * engine (folded eval BN, residual, activation, raw-accumulator copy).  wgrad writes the PyTorch layout
 * [C][1][R][S] (c < c_real), += when accumulate; deterministic (fixed-order block partials). */
int ssseg_dwconv_fwd(const void* x, const void* w, void* y, const ssseg_conv_desc* desc_host, int dt,
                     const ssseg_conv_epilogue* epi, ssseg_stream_t stream);
int ssseg_dwconv_dgrad(const void* dy, const void* w, void* dx, const ssseg_conv_desc* desc_host, int dt,
                       ssseg_stream_t stream);
size_t ssseg_dwconv_wgrad_workspace_bytes(const ssseg_conv_desc* desc_host, int dt);
int ssseg_dwconv_wgrad(const void* x, const void* dy, float* dw, const ssseg_conv_desc* desc_host, int dt,
                       int64_t c_real, int accumulate, void* ws, size_t ws_bytes, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * BatchNorm2d / SyncBatchNorm (nn.BatchNorm2d in every ConvBlock, unet.py:9; distributed_trainer.py:36)
 * NHWC [P][ld] activations, leading dimensions multiples of 4 and >= rup(C, 4) (C itself may be ragged).  Training: stats -> (all-reduce sums for SyncBN) -> finalize.
 * ------------------------------------------------------------------------------------------- */
size_t ssseg_bn_workspace_bytes(int64_t C);
/* sums[0:C] = sum_p x, sums[C:2C] = sum_p x^2 (fp64) */
int ssseg_bn_stats(const void* x, int64_t P, int64_t C, int64_t ldx, int dt, double* sums, void* ws, size_t ws_bytes,
                   ssseg_stream_t stream);
/* mean, invstd = 1/sqrt(biased var + eps) from sums over `count` pixels; running stats updated with
 * momentum and the unbiased variance when running_mean != NULL; *num_batches_tracked += 1 if non-NULL. */
int ssseg_bn_finalize(const double* sums, int64_t C, double count, float eps, float momentum, float* mean_out,
                      float* invstd_out, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                      ssseg_stream_t stream);
/* ssseg_bn_stats + ssseg_bn_finalize in one pass (the finalize runs in the reduction's tail): the
 * single-process / non-synchronised training BatchNorm (SyncBN all-reduces sums in between instead). */
int ssseg_bn_stats_finalize(const void* x, int64_t P, int64_t C, int64_t ldx, int dt, double* sums, void* ws,
                            size_t ws_bytes, double count, float eps, float momentum, float* mean_out, float* invstd_out,
                            float* running_mean, float* running_var, int64_t* num_batches_tracked,
                            ssseg_stream_t stream);
/* BatchNorm statistics from the partial rows a conv epilogue wrote (ssseg_conv_epilogue.stats): sums[0:C] /
 * sums[C:2C] = column sums over nparts rows of part[2*nparts][C] (fixed order, deterministic; part is scratch: a
 * long table is folded in place before the column reduce, so its contents are undefined afterwards); when mean_out is
 * non-NULL the training finalize of ssseg_bn_finalize runs in the same launch (the single-process path; SyncBN
 * passes mean_out = NULL, all-reduces sums, then calls ssseg_bn_finalize). */
int ssseg_bn_partials_finalize(double* part, int64_t nparts, int64_t C, double* sums, double count, float eps,
                               float momentum, float* mean_out, float* invstd_out, float* running_mean,
                               float* running_var, int64_t* num_batches_tracked, ssseg_stream_t stream);
/* A conv bias gradient (unet.py UpBlock ConvTranspose2d / 1x1 upsampler biases): dsum[c] += sum over P pixels of
 * x[p][c] (fp64 partials, fixed order), in the reduction's own tail; sums receives the fp64 column sums (sums[C:2C]
 * the sums of squares). */
int ssseg_channel_sum_grad(const void* x, int64_t P, int64_t C, int64_t ldx, int dt, float* dsum, double* sums,
                           void* ws, size_t ws_bytes, ssseg_stream_t stream);
/* The backward sums of a BatchNorm(+ReLU) from the gradient-statistics rows of its consumer's input-gradient launch
 * (ssseg_conv_igemm_epi_actmask with stats): sums[0:C] = sum m, sums[C:2C] = sum m * x_hat, with x_hat recovered from
 * y wherever m != 0 -- training BN (mean_eff NULL): x_hat = (y - beta) / gamma (gamma / beta NULL: 1 / 0); folded
 * eval BN (mean_eff non-NULL, gamma = its scale, beta = its shift): x_hat = (y - mean_eff*scale - shift) * invstd /
 * scale.  A channel whose gamma (scale) is 0 gets sum m * x_hat = 0 (y carries no x_hat there).  Then dbeta += sums[c],
 * dgamma += sums[C + c], dconv_bias += scale * sums[c] (eval only) for the non-NULL ones.  part is scratch as in
 * ssseg_bn_partials_finalize; sums feed ssseg_bn_bwd_apply (train = 1, relu = 0: dy is the masked gradient). */
int ssseg_bn_gstat_finalize(double* part, int64_t nparts, int64_t C, double* sums, const float* gamma,
                            const float* beta, const float* mean_eff, const float* invstd, float* dgamma, float* dbeta,
                            float* dconv_bias, ssseg_stream_t stream);
/* as ssseg_bn_gstat_finalize for a TRAINING BN (mean_eff NULL) whose input x [P][ld] and masked output gradient dy
 * [P][ld] (dtype dt; the consumer's dgrad applied the ReLU backward) are at hand, with mean / invstd of the forward:
 * channels where x_hat is not recoverable from the stored y -- gamma == 0, or |beta| >= 8 |gamma| (y ~ beta, its
 * rounding swamps gamma * x_hat) -- take sum dy * x_hat = sum dy * (x - mean) * invstd from dy and x (the unfused
 * reduction's arithmetic) in the same launch; the others use the rows as ssseg_bn_gstat_finalize does. */
int ssseg_bn_gstat_finalize_x(double* part, int64_t nparts, int64_t C, double* sums, const float* gamma,
                              const float* beta, const void* dy, const void* x, int64_t P, int64_t ld, int dt,
                              const float* mean, const float* invstd, float* dgamma, float* dbeta,
                              ssseg_stream_t stream);
/* eval mode: mean = running_mean, invstd = 1/sqrt(running_var + eps) */
int ssseg_bn_eval_params(const float* running_mean, const float* running_var, float eps, int64_t C, float* mean_out,
                         float* invstd_out, ssseg_stream_t stream);
/* eval BatchNorm as a per-channel affine of the producing conv's accumulator (ssseg_conv_igemm_epi):
 * scale = gamma*invstd, shift = beta + (conv_bias - running_mean)*scale, invstd = 1/sqrt(running_var + eps),
 * mean_eff = running_mean - conv_bias (so xhat = (acc - mean_eff)*invstd); channels C <= c < Cp get
 * zeros (padding stays zero).  gamma/beta/conv_bias may be NULL; mean_eff/invstd_out are optional. */
int ssseg_bn_fold(const float* running_mean, const float* running_var, const float* gamma, const float* beta,
                  const float* conv_bias, float eps, int64_t C, int64_t Cp, float* scale, float* shift,
                  float* mean_eff, float* invstd_out, ssseg_stream_t stream);
/* Batched ssseg_bn_fold: one launch folds every (conv, BN) pair of a model before an eval forward.
 * descs points to DEVICE memory; out receives [scale | shift | mean_eff | invstd], Cp floats each. */
typedef struct ssseg_fold_desc {
  const float* running_mean;
  const float* running_var;
  const float* gamma;
  const float* beta;
  const float* conv_bias;
  float* out;
  int64_t C, Cp;
  double eps;
} ssseg_fold_desc;
int ssseg_bn_fold_batch(const ssseg_fold_desc* descs, int64_t n, ssseg_stream_t stream);
/* backward of a folded eval BN (+residual, +ReLU): dyr = relu ? dy*[y > 0] : dy; dconv = scale*dyr (the
 * conv's output gradient); dres = dyr (optional); sums[0:C] = sum dyr, sums[C:2C] = sum dyr*xhat with
 * xhat = (aux - mean_eff)*invstd.  All tensors NHWC with pixel stride ld; padding channels written 0. */
int ssseg_bn_eval_bwd(const void* dy, const void* y, const void* aux, void* dconv, void* dres, int64_t P, int64_t C,
                      int64_t ld, const float* scale, const float* mean_eff, const float* invstd, int relu, int dt,
                      double* sums, void* ws, size_t ws_bytes, ssseg_stream_t stream);
/* parameter gradients of a folded eval BN: dgamma += sums[C:2C], dbeta += sums[0:C],
 * dconv_bias += scale*sums[0:C] (any pointer may be NULL) */
int ssseg_bn_eval_param_grad(const double* sums, int64_t C, const float* scale, float* dgamma, float* dbeta,
                             float* dconv_bias, ssseg_stream_t stream);
/* ssseg_bn_eval_bwd + ssseg_bn_eval_param_grad fused (the param grads run in the reduction's tail) */
int ssseg_bn_eval_bwd_grad(const void* dy, const void* y, const void* aux, void* dconv, void* dres, int64_t P, int64_t C,
                           int64_t ld, const float* scale, const float* mean_eff, const float* invstd, int relu, int dt,
                           double* sums, void* ws, size_t ws_bytes, float* dgamma, float* dbeta, float* dconv_bias,
                           ssseg_stream_t stream);
/* ssseg_bn_eval_bwd_grad without the raw accumulator copy, for a layer WITHOUT a residual: wherever the output
 * gradient survives the activation, y itself is the pre-activation scale*aux + shift, so x_hat is recovered from y
 * (x_hat = (y - (shift + mean_eff*scale)) * invstd / scale; a channel with scale == 0 gets x_hat = 0).  The
 * differentiated eval pass (train.py:90-92) then does not write aux in the forward nor read it here. */
int ssseg_bn_eval_bwd_grad_y(const void* dy, const void* y, void* dconv, void* dres, int64_t P, int64_t C, int64_t ld,
                             const float* scale, const float* shift, const float* mean_eff, const float* invstd,
                             int relu, int dt, double* sums, void* ws, size_t ws_bytes, float* dgamma, float* dbeta,
                             float* dconv_bias, ssseg_stream_t stream);
/* Deferred parameter gradients of the differentiated eval BN (the student's consistency pass, train.py:90-92, whose
 * BN/conv-bias gradients nothing reads before the optimizer step): ssseg_bn_eval_bwd(_grad_y) with the per-block
 * partial rows (sum dyr, sum dyr*xhat) left in part (>= ssseg_bn_workspace_bytes(C) bytes, caller-owned, kept until
 * ssseg_bn_param_grad_batch has run; *nparts_host = rows, < 1024) and no reduction launch.  shift != NULL: x_hat from y
 * (the _grad_y form, aux unused); shift == NULL: x_hat from aux. */
int ssseg_bn_eval_bwd_part(const void* dy, const void* y, const void* aux, void* dconv, void* dres, int64_t P, int64_t C,
                           int64_t ld, const float* scale, const float* shift, const float* mean_eff,
                           const float* invstd, int relu, int dt, double* part, size_t part_bytes, int64_t* nparts_host,
                           ssseg_stream_t stream);
/* ONE launch for many deferred reductions: per descriptor, dbeta[c] += sum of part rows 2r, dgamma[c] += sum of rows
 * 2r + 1, dconv_bias[c] += scale[c] * (the first sum) (NULL pointers skipped); fixed-order fp64 column sums.  descs
 * points to DEVICE memory; max_c >= every descriptor's C.  mean_eff non-NULL: the rows are gradient-statistics rows
 * (sum m, sum m * y) of a consumer's input-gradient launch, turned into the x_hat moment as ssseg_bn_gstat_finalize
 * does for a folded eval BN (scale, shift, mean_eff, invstd) before the same tail.  part is scratch: a table of >= 512
 * rows is first folded in place to <= 256 group sums (fixed order; a second launch in the same call). */
typedef struct ssseg_pgrad_desc {
  const double* part;
  int64_t nparts, C;
  const float* scale;
  float* dgamma;
  float* dbeta;
  float* dconv_bias;
  const float* shift;      /* gradient-statistics rows only (else NULL) */
  const float* mean_eff;
  const float* invstd;
} ssseg_pgrad_desc;
int ssseg_bn_param_grad_batch(const ssseg_pgrad_desc* descs, int64_t n, int64_t max_c, ssseg_stream_t stream);
/* y = act(gamma*(x-mean)*invstd + beta [+ residual]); channels [C, rup(C, 16 bytes)) of y are written 0; relu = 1 for ReLU (unet.py:10, Bottleneck add+relu) */
int ssseg_bn_apply(const void* x, const void* residual, void* y, int64_t P, int64_t C, int64_t ldx, int64_t ldr,
                   int64_t ldy, const float* mean, const float* invstd, const float* gamma, const float* beta, int relu,
                   int dt, ssseg_stream_t stream);
/* backward pass 1: sums[0:C] = sum dyr, sums[C:2C] = sum dyr*xhat, dyr = dy*[y>0] (y recomputed) */
int ssseg_bn_bwd_reduce(const void* dy, const void* x, const void* residual, int64_t P, int64_t C, int64_t ldx,
                        int64_t ldr, int64_t lddy, const float* mean, const float* invstd, const float* gamma,
                        const float* beta, int relu, int dt, double* sums, void* ws, size_t ws_bytes,
                        ssseg_stream_t stream);
/* dgamma += sums[C:2C], dbeta += sums[0:C] (local sums, before any SyncBN all-reduce) */
int ssseg_bn_param_grad(const double* sums, int64_t C, float* dgamma, float* dbeta, ssseg_stream_t stream);
/* ssseg_bn_bwd_reduce + ssseg_bn_param_grad fused (param grads from the local sums in the reduction's tail;
 * dgamma / dbeta may be NULL) */
int ssseg_bn_bwd_reduce_grad(const void* dy, const void* x, const void* residual, int64_t P, int64_t C, int64_t ldx,
                             int64_t ldr, int64_t lddy, const float* mean, const float* invstd, const float* gamma,
                             const float* beta, int relu, int dt, double* sums, void* ws, size_t ws_bytes,
                             float* dgamma, float* dbeta, ssseg_stream_t stream);
/* backward pass 2: dx = gamma*invstd*(dyr - [train]*(sum_dyr + xhat*sum_dyr_xhat)/count); dres = dyr;
 * padding channels of dx / dres written 0 as in ssseg_bn_apply */
int ssseg_bn_bwd_apply(const void* dy, const void* x, const void* residual, void* dx, void* dres, int64_t P, int64_t C,
                       int64_t ldx, int64_t ldr, int64_t lddy, int64_t lddx, const float* mean, const float* invstd,
                       const float* gamma, const float* beta, int relu, int train, const double* sums, double count,
                       int dt, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Pooling and NHWC window copies (torch.cat / _center_crop, unet.py:40-60)
 * ------------------------------------------------------------------------------------------- */
/* MaxPool2d(k, s, p): y and argmax idx (tap index within the window, PyTorch tie order) */
int ssseg_maxpool_fwd(const void* x, void* y, uint8_t* idx, int64_t N, int64_t H, int64_t W, int64_t C, int64_t OH,
                      int64_t OW, int64_t k, int64_t s, int64_t p, int dt, ssseg_stream_t stream);
int ssseg_maxpool_bwd(const void* gy, const uint8_t* idx, void* gx, int64_t N, int64_t H, int64_t W, int64_t C,
                      int64_t OH, int64_t OW, int64_t k, int64_t s, int64_t p, int dt, ssseg_stream_t stream);
/* as ssseg_maxpool_bwd, plus res (NHWC like gx, or NULL): gx = res + gather(gy) in one pass -- an activation read
 * by the max-pool and by another op (the UNet skip from the stem, unet.py:36-45) gets both gradients without a
 * separate add (ssseg.nn.GradJoin). */
int ssseg_maxpool_bwd_res(const void* gy, const uint8_t* idx, const void* res, void* gx, int64_t N, int64_t H,
                          int64_t W, int64_t C, int64_t OH, int64_t OW, int64_t k, int64_t s, int64_t p, int dt,
                          ssseg_stream_t stream);
/* dst[n][h+doy][w+dox][c] = src[n][h+soy][w+sox][c] for h<H, w<W, c<C (pixel strides sld/dld) */
int ssseg_nhwc_copy(const void* src, void* dst, int64_t N, int64_t H, int64_t W, int64_t C, int64_t sH, int64_t sW,
                    int64_t sld, int64_t soy, int64_t sox, int64_t dH, int64_t dW, int64_t dld, int64_t doy, int64_t dox,
                    int dt, ssseg_stream_t stream);
int ssseg_zero(void* p, size_t bytes, ssseg_stream_t stream);

/* One operand of an n-way channel concat of same-size NHWC maps (torch.cat(tensors, 1): HarDNet's harmonic links and
 * block outputs hardnet.py:67,78, TransitionUp hardnet.py:95; discriminator.py:56).  The concat packs the operands'
 * REAL channel counts back to back. */
typedef struct {
  const void* src;   /* ssseg_nhwc_cat_n: operand [npix][ld] (16-bit or fp32 like the concat) */
  void* dst;         /* ssseg_nhwc_split_n: operand gradient [npix][ld], 16-byte aligned */
  const void* add;   /* ssseg_nhwc_split_n: NULL, or a pending gradient of the operand (dst's layout) added in the
                        same pass (fp32 sum, one rounding: PyTorch's add of the two) */
  int64_t ld;        /* the operand's pixel stride (physical channels); split: a multiple of 16 bytes */
  int64_t c;         /* real channels, 0 <= c <= ld */
} ssseg_cat_part;
/* y[p][0..ldy) = parts' first c channels back to back, channels sum(c)..ldy-1 written zero: one launch for up to 16
 * operands (no separate zero fill).  y 16-byte aligned, ldy a multiple of 16 bytes, npix = N*H*W. */
int ssseg_nhwc_cat_n(const ssseg_cat_part* parts_host, int64_t nparts, void* y, int64_t npix, int64_t ldy, int dt,
                     ssseg_stream_t stream);
/* the concat's backward, one launch: parts[k].dst[p][j] = gy[p][c0_k + j] (+ parts[k].add[p][j]) for j < c_k and 0
 * for c_k <= j < ld_k, with c0_k = c_0 + ... + c_(k-1); gy [npix][ldg]. */
int ssseg_nhwc_split_n(const void* gy, int64_t ldg, const ssseg_cat_part* parts_host, int64_t nparts, int64_t npix,
                       int dt, ssseg_stream_t stream);

/* gx = gy * [y > 0]  (ReLU backward from the saved output; ConvTranspose2d+ReLU upsampler unet.py:21-22) */
/* gx = gy * d act / d z evaluated from the activation output y (SSSEG_ACT_*; the cut gradient is selected
 * to 0, not multiplied, like PyTorch's threshold_backward) */
int ssseg_act_bwd(const void* gy, const void* y, void* gx, int64_t n, int act, float slope, int dt,
                  ssseg_stream_t stream);
int ssseg_relu_bwd(const void* gy, const void* y, void* gx, int64_t n, int dt, ssseg_stream_t stream);


/* ---------------------------------------------------------------------------------------------
 * Pooling / elementwise primitives of the C3-C5 model families (csrc/pool.hip)
 * ------------------------------------------------------------------------------------------- */
/* nn.AvgPool2d(k, s, p) with PyTorch's defaults (ceil_mode False, count_include_pad True): HarDNet's
 * AvgPool2d(2, 2) (hardnet.py:157).  NHWC [N][H][W][C], C = physical channels (multiple of 8 bf16 / 4 f32). */
int ssseg_avgpool_fwd(const void* x, void* y, int64_t N, int64_t H, int64_t W, int64_t C, int64_t OH, int64_t OW,
                      int64_t k, int64_t s, int64_t p, int dt, ssseg_stream_t stream);
int ssseg_avgpool_bwd(const void* gy, void* gx, int64_t N, int64_t H, int64_t W, int64_t C, int64_t OH, int64_t OW,
                      int64_t k, int64_t s, int64_t p, int dt, ssseg_stream_t stream);
/* nn.AdaptiveAvgPool2d(1) (DeepLabV3 ASPPPooling, torchvision head behind deeplabv3.py:9,43): y[n][c] (pixel
 * stride ldy) = mean over HW pixels of x[n][p][c] (x pixel stride C).  Deterministic two-pass reduction. */
size_t ssseg_global_avgpool_workspace_bytes(int64_t N, int64_t HW, int64_t C);
int ssseg_global_avgpool_fwd(const void* x, void* y, int64_t N, int64_t HW, int64_t C, int64_t ldy, int dt, void* ws,
                             size_t ws_bytes, ssseg_stream_t stream);
/* gx[n][p][c] = gy[n][c] / HW (gx pixel stride C, gy row stride ldgy) */
int ssseg_global_avgpool_bwd(const void* gy, void* gx, int64_t N, int64_t HW, int64_t C, int64_t ldgy, int dt,
                             ssseg_stream_t stream);
/* y = act(x_0 + x_1 + ... + x_{n-1}) elementwise over numel (multiple of 8 bf16 / 4 f32, 16-byte aligned
 * operands), summed left to right in fp32: HRNet TransitionFuse's add chain ending in add_relu
 * (higher_hrnet.py:473-486).  xs_host: host array of n <= 8 device pointers. */
int ssseg_add_n(const void* const* xs_host, int n, void* y, int64_t numel, int act, float slope, int dt,
                ssseg_stream_t stream);
/* nn.Dropout(p) in training mode (DeepLabV3 ASPP projection): y = u >= p ? x/(1-p) : 0 with u a Philox-4x32-10
 * uniform of element i (counter offset + i/4, key seed).  The backward is the same call on the output gradient
 * with the same (seed, offset).  n % 4 == 0. */
int ssseg_dropout(const void* x, void* y, int64_t n, float p, uint64_t seed, uint64_t offset, int dt,
                  ssseg_stream_t stream);
/* as ssseg_dropout with the Philox counter offset read from device memory (a captured HIP graph replays fresh masks) */
int ssseg_dropout_dev(const void* x, void* y, int64_t n, float p, uint64_t seed, const unsigned long long* offset_dev,
                      int dt, ssseg_stream_t stream);
/* device-side counter reservation: snap[0] = counter[0]; counter[0] += inc (one thread, in stream order) */
int ssseg_rng_take(unsigned long long* counter, unsigned long long* snap, uint64_t inc, ssseg_stream_t stream);
/* MultiscaleAttention blend (multiscale_attention.py:52-54), fp32 [N][C][H][W] with arbitrary strides:
 * out = lo*s + hi*(1-s), s = sigmoid(att[n][0][h][w]); out contiguous NCHW. */
int ssseg_att_blend_fwd(const float* lo, const int64_t* lo_strides4_host, const float* hi,
                        const int64_t* hi_strides4_host, const float* att, const int64_t* att_strides4_host, float* out,
                        int64_t N, int64_t C, int64_t H, int64_t W, ssseg_stream_t stream);
/* glo = g*s, ghi = g*(1-s), gatt = sum_c g*(lo-hi)*s*(1-s); outputs contiguous NCHW, each may be NULL */
int ssseg_att_blend_bwd(const float* gout, const int64_t* g_strides4_host, const float* lo,
                        const int64_t* lo_strides4_host, const float* hi, const int64_t* hi_strides4_host,
                        const float* att, const int64_t* att_strides4_host, float* glo, float* ghi, float* gatt,
                        int64_t N, int64_t C, int64_t H, int64_t W, ssseg_stream_t stream);

/* Validation metrics (train.validate, train.py:150-195).  logits [B][2][h][w] f32 and mask [B][2][H][W]
 * f32, arbitrary strides (host arrays of 4 element strides).  pred = argmax(logits) (first max, NaN is
 * max), nearest-resized to HxW (ATen nearest_idx); t1 = mask[:,1] > 0.5; label = argmax(mask).
 * counts [B][8] (u64, overwritten): sum(pred1*t1), sum(pred1), sum(t1), inter0, union0, inter1, union1, pixels.
 * out4[0] = mean_b (2 I_b + 1)/(card_b + 1)            (metrics.dice_metric metrics.py:1-7 + .mean())
 * out4[1..2] = 100 * IoU of class 0/1, out4[3] = their mean (lovasz.iou lovasz.py:54-73, per_image=False)
 * total [8] (nullable): running dataset counts; when given, the batch counts are added and out4[1..3]
 * are computed from the running totals. */
int ssseg_seg_metrics(const float* logits, const int64_t* l_strides4_host, int64_t h, int64_t w, const float* mask,
                      const int64_t* m_strides4_host, int64_t B, int64_t H, int64_t W, unsigned long long* counts,
                      unsigned long long* total, float* out4, ssseg_stream_t stream);

/* InferenceWrapper head (models/inference_wrapper.py:17-24): logits contiguous [B][2][HW] f32 ->
 * prob = sigmoid(logits), onehot = one_hot(argmax_c logits) (first max, NaN is max), both [B][2][HW] f32. */
int ssseg_prob_onehot(const float* logits, int64_t B, int64_t HW, float* prob, float* onehot, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Collectives: the data-parallel gradient all-reduce and the SyncBN sums
 * (reference distributed_trainer.py:34-38 -- SyncBatchNorm.convert_sync_batchnorm + DistributedDataParallel,
 * whose reducer all-reduces gradient buckets during backward; SyncBN all-reduces per-channel sums)
 *
 * One RCCL communicator per process (one process per GPU), owned by the caller.  The all-reduce is an RCCL
 * enqueue on the caller's stream: no host synchronisation, no completion objects, so it is captured into a
 * hipGraph like a kernel (c10d's ProcessGroupNCCL keeps per-collective Work objects polled by a watchdog
 * thread, which breaks the capture of a step).  RCCL is resolved at run time (dlopen; PyTorch's already
 * loaded copy first).  Errors: SSSEG_ECOMM, message in ssseg_comm_last_error().
 * ------------------------------------------------------------------------------------------- */
typedef struct ssseg_comm_s* ssseg_comm_t;
enum { SSSEG_SUM = 0, SSSEG_AVG = 1 };

/* bytes of the unique id that rank 0 creates and every rank passes to ssseg_comm_init (128) */
size_t ssseg_comm_unique_id_bytes(void);
/* rank 0: fill uid_host (host memory, ssseg_comm_unique_id_bytes() bytes) -- replaces the c10d store rendezvous of
 * init_process_group(backend='nccl') (distributed_trainer.py:59 in this repo, utils/utils.py in the reference) */
int ssseg_comm_get_unique_id(void* uid_host);
/* collective over all `world` ranks (blocks until every rank has called it): selects `device` and creates the
 * communicator of this rank */
int ssseg_comm_init(ssseg_comm_t* comm_out, const void* uid_host, int rank, int world, int device);
int ssseg_comm_destroy(ssseg_comm_t comm);
/* 0, or SSSEG_ECOMM when RCCL reported an asynchronous error on the communicator */
int ssseg_comm_async_error(ssseg_comm_t comm);
/* static message of the last SSSEG_ECOMM */
const char* ssseg_comm_last_error(void);
/* n in-place all-reduces (ptrs_host[i]: device buffer of counts_host[i] elements of dtype dt -- SSSEG_F32 / BF16 /
 * F16 / F64) in one RCCL group on `stream`; op SSSEG_SUM or SSSEG_AVG.  Replaces DDP's bucket all-reduce
 * (torch/nn/parallel/distributed.py reducer, called from the backward of train.py:61,115) and SyncBN's
 * all_reduce of (sum x, sum x^2) / (sum dy, sum dy*x_hat) (torch/nn/modules/_functions.py, forward and backward). */
int ssseg_allreduce_buckets(ssseg_comm_t comm, void* const* ptrs_host, const int64_t* counts_host, int64_t n, int dt,
                            int op, ssseg_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Timing events for the live kernel probe (bench.py's roofline leg; csrc/probe.hip).  Created with
 * hipEventDisableSystemFence: recording one writes a timestamp without the system-scope cache writeback and
 * invalidation a default event performs, so a kernel bracketed by probe events runs with the caches its
 * predecessor left, as in the captured step.  ssseg_probe_event_elapsed waits for ev1 and returns ev1 - ev0 in ms.
 * ------------------------------------------------------------------------------------------- */
int ssseg_probe_event_create(void** ev_out);
int ssseg_probe_event_record(void* ev, ssseg_stream_t stream);
int ssseg_probe_event_elapsed(void* ev0, void* ev1, float* ms_out);
int ssseg_probe_event_destroy(void* ev);

#ifdef __cplusplus
}
#endif
#endif /* SSSEG_H */
