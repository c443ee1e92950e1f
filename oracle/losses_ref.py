"""Oracle: losses, interpolation and EMA (numpy, float32).  TEST INFRASTRUCTURE ONLY.

  bilinear / bilinear_backward   <- F.interpolate(mode='bilinear') as called at losses.py:18,
                                    train.py:71,74,93 (align_corners=False) and unet.py:26
                                    (nn.Upsample, align_corners=True)
  bce_logits_mean                <- DenseBinaryCrossEntropyLossWithLogits  losses.py:41-48
  lovasz_grad                    <- lovasz.lovasz_grad                     lovasz.py:19-31
  binary_lovasz                  <- losses.binary_lovasz_loss_with_logits  losses.py:239-250
                                    -> lovasz_softmax(classes=[1], per_image=True)  lovasz.py:155-201
  consistency                    <- inline consistency loss                train.py:97-112
  ema_update                     <- mean_teacher.update_ema_variables      mean_teacher.py:5-18
  seg_metrics                    <- train.validate Dice (train.py:171-176, metrics.py:1-7) + lovasz.iou
                                    (lovasz.py:54-73)
  inference_head                 <- models/inference_wrapper.py:14-24
"""
import numpy as np

F32 = np.float32


def _src_index(out_size, in_size, align_corners):
    d = np.arange(out_size, dtype=F32)
    if align_corners:
        scale = F32((in_size - 1) / (out_size - 1)) if out_size > 1 else F32(0.0)
        src = d * scale
    else:
        scale = F32(in_size) / F32(out_size)
        src = (d + F32(0.5)) * scale - F32(0.5)
        src = np.maximum(src, F32(0.0))
    i0 = np.minimum(src.astype(np.int64), in_size - 1)
    i1 = np.minimum(i0 + 1, in_size - 1)
    l1 = (src - i0.astype(F32)).astype(F32)
    l0 = (F32(1.0) - l1).astype(F32)
    return i0, i1, l0, l1


def bilinear(x, size, align_corners=False):
    """x: [N,C,H,W] -> [N,C,Ho,Wo]."""
    x = np.asarray(x, F32)
    Ho, Wo = size
    H, W = x.shape[2:]
    h0, h1, lh0, lh1 = _src_index(Ho, H, align_corners)
    w0, w1, lw0, lw1 = _src_index(Wo, W, align_corners)
    top = x[:, :, h0][:, :, :, w0] * lw0 + x[:, :, h0][:, :, :, w1] * lw1
    bot = x[:, :, h1][:, :, :, w0] * lw0 + x[:, :, h1][:, :, :, w1] * lw1
    return (top * lh0[:, None] + bot * lh1[:, None]).astype(F32)


def bilinear_backward(g, in_size, align_corners=False):
    g = np.asarray(g, np.float64)
    N, C, Ho, Wo = g.shape
    H, W = in_size
    h0, h1, lh0, lh1 = _src_index(Ho, H, align_corners)
    w0, w1, lw0, lw1 = _src_index(Wo, W, align_corners)
    out = np.zeros((N, C, H, W), np.float64)
    for (hi, lh) in ((h0, lh0), (h1, lh1)):
        for (wi, lw) in ((w0, lw0), (w1, lw1)):
            contrib = g * lh[:, None].astype(np.float64) * lw[None, :].astype(np.float64)
            # scatter-add rows then columns
            tmp = np.zeros((N, C, H, Wo), np.float64)
            np.add.at(tmp, (slice(None), slice(None), hi), contrib)
            np.add.at(out, (slice(None), slice(None), slice(None), wi), tmp)
    return out.astype(F32)


def sigmoid(x):
    x = np.asarray(x, F32)
    return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(F32)


def bce_logits_mean(x, t):
    """mean(max(x,0) - x*t + log(1 + exp(-|x|))) and its gradient (sigmoid(x) - t) / numel."""
    x = np.asarray(x, np.float64)
    t = np.asarray(t, np.float64)
    loss = np.maximum(x, 0) - x * t + np.log1p(np.exp(-np.abs(x)))
    n = x.size
    grad = (1.0 / (1.0 + np.exp(-x)) - t) / n
    return F32(loss.mean()), grad.astype(F32)


def lovasz_grad(gt_sorted):
    """lovasz.py:19-31: first difference of 1 - (gts - cumsum fg) / (gts + cumsum(1 - fg))."""
    gt = np.asarray(gt_sorted, F32)
    gts = gt.sum(dtype=F32)
    inter = gts - np.cumsum(gt, dtype=F32)
    union = gts + np.cumsum(F32(1.0) - gt, dtype=F32)
    jac = (F32(1.0) - inter / union).astype(F32)
    if gt.size > 1:
        jac[1:] = jac[1:] - jac[:-1]
    return jac


def binary_lovasz(logits, target):
    """losses.py:239-250 with lovasz_softmax(classes=[1], per_image=True, ignore=255).

    logits, target: [B, C, H, W] float32.  Raw logits (no sigmoid: losses.py:241 is commented out).
    Returns (loss, dloss/dlogits) — the gradient reaches channel 1 only.  Sorting is stable
    descending here; the reference's torch.sort is unstable, so on tied errors only the loss value
    (not the per-pixel gradient assignment) is comparable.
    """
    logits = np.asarray(logits, F32)
    target = np.asarray(target, F32)
    B = logits.shape[0]
    labels = np.argmax(target, axis=1).reshape(B, -1)        # losses.py:240
    x = logits[:, 1].reshape(B, -1)
    valid = (labels.sum(axis=1) > 0).astype(F32)             # losses.py:247
    denom = F32(valid.sum(dtype=F32) + F32(0.001))          # losses.py:250
    total = F32(0.0)
    grad = np.zeros_like(logits)
    for i in range(B):
        fg = (labels[i] == 1).astype(F32)
        err = np.abs(fg - x[i])
        perm = np.argsort(-err, kind='stable')
        g = lovasz_grad(fg[perm])
        li = F32(np.dot(err[perm].astype(np.float64), g.astype(np.float64)))
        total = F32(total + li * valid[i])
        d_err = np.zeros_like(err)
        d_err[perm] = g
        gi = -np.sign(fg - x[i]) * d_err * valid[i] / denom
        grad[i, 1] = gi.reshape(logits.shape[2:])
    return F32(total / denom), grad.astype(F32)


def consistency(student_logits, teacher_logits, thr):
    """train.py:97-108.  Inputs are the full-resolution (already interpolated) logits [B,C,H,W].

    L = sum_pix(sum_c (sig(s) - sig(t))^2 * cm) / sum(cm), cm = [max_c sig(t) > thr].
    Returns (L, mean(cm), dL/ds).  L is NaN when sum(cm) == 0, and so is the gradient.
    """
    ps = sigmoid(student_logits).astype(np.float64)
    pt = sigmoid(teacher_logits).astype(np.float64)
    cm = (pt.max(axis=1) > thr).astype(np.float64)
    n_cm = cm.sum()
    d = ps - pt
    with np.errstate(invalid='ignore', divide='ignore'):
        L = ((d * d).sum(axis=1) * cm).sum() / n_cm
        grad = 2.0 * d * ps * (1.0 - ps) * cm[:, None] / n_cm
    return F32(L), F32(cm.mean()), grad.astype(F32)


def ema_update(ema, param, alpha):
    """mean_teacher.py:10-11: ema.mul_(alpha).add_(param, alpha=1-alpha), float32.

    torch's CPU add-with-alpha is a fused multiply-add: t = round(ema*a); out = fma(param, 1-a, t).
    The fma is exact via float64 (24-bit x 24-bit product fits in 53 bits); pinned bit-exact by G5.
    """
    ema = np.asarray(ema, F32)
    param = np.asarray(param, F32)
    t = (ema * F32(alpha)).astype(F32)
    beta = np.float64(F32(1.0 - alpha))
    return (t.astype(np.float64) + param.astype(np.float64) * beta).astype(F32)


def _nearest_src(out_size, in_size):
    """ATen nearest_idx for scale_factor=None (the `F.interpolate(..., mode='nearest')` of
    reference/train.py:172): identity, exact 2x, else floor(o * float32(in/out)) clamped."""
    o = np.arange(out_size)
    if out_size == in_size:
        return o
    if out_size == 2 * in_size:
        return o >> 1
    scale = np.float32(in_size) / np.float32(out_size)
    return np.minimum(np.floor(o.astype(np.float32) * scale).astype(np.int64), in_size - 1)


def _argmax2(a0, a1):
    """torch.argmax over 2 channels: first maximum wins, NaN is the maximum."""
    return np.where(np.isnan(a0), 0, np.where(np.isnan(a1), 1, (a1 > a0).astype(np.int64)))


def seg_metrics(logits, mask):
    """train.validate's metric (reference/train.py:171-176 + metrics.dice_metric metrics.py:1-7) and
    lovasz.iou(pred, argmax(mask), C=2) (lovasz.py:54-73, per_image=False) on the same predictions.
    logits [B,2,h,w], mask [B,2,H,W] -> (dice [B] f32, ious [2] f64 x100, counts [B,8] int64)."""
    logits = np.asarray(logits, np.float32)
    mask = np.asarray(mask, np.float32)
    B, _, h, w = logits.shape
    H, W = mask.shape[2:]
    pred_lo = _argmax2(logits[:, 0], logits[:, 1])
    pred = pred_lo[:, _nearest_src(H, h)][:, :, _nearest_src(W, w)]
    t1 = (mask[:, 1] > 0.5).astype(np.int64)
    label = _argmax2(mask[:, 0], mask[:, 1])
    counts = np.zeros((B, 8), np.int64)
    counts[:, 0] = (pred * t1).reshape(B, -1).sum(1)
    counts[:, 1] = pred.reshape(B, -1).sum(1)
    counts[:, 2] = t1.reshape(B, -1).sum(1)
    for c in range(2):
        counts[:, 3 + 2 * c] = ((label == c) & (pred == c)).reshape(B, -1).sum(1)
        counts[:, 4 + 2 * c] = ((label == c) | (pred == c)).reshape(B, -1).sum(1)
    counts[:, 7] = H * W
    inter = counts[:, 0].astype(np.float32)
    card = counts[:, 1].astype(np.float32) + counts[:, 2].astype(np.float32)
    dice = (np.float32(2) * inter + np.float32(1)) / (card + np.float32(1))
    tot = counts.sum(0)
    ious = np.array([tot[3] / tot[4] if tot[4] else 1., tot[5] / tot[6] if tot[6] else 1.]) * 100
    return dice.astype(np.float32), ious, counts


def inference_head(logits, size):
    """models/inference_wrapper.py:14-24 on the first logit map [1,2,h,w]: bilinear (align_corners=False) to
    `size`, sigmoid probabilities, one-hot of the argmax -> (binary_mask [2,H,W], probabilities [2,H,W])."""
    hi = bilinear(logits, size, align_corners=False)
    prob = sigmoid(hi)
    cls = _argmax2(hi[:, 0], hi[:, 1])
    onehot = np.stack([(cls == 0), (cls == 1)], 1).astype(F32)
    return onehot[0], prob[0].astype(F32)
