"""Autograd-aware wrappers over libssseg.so for the loss / CowMix / EMA part of the hot path.

Each function documents the reference call site it replaces.  Inputs must be HIP tensors.
"""
import os

import torch

from . import native as N


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


# ------------------------------------------------------------------------------------------------
# CowMix (cowmix.py)
# ------------------------------------------------------------------------------------------------
def cowmix_mask(noise, sigma, p, return_field=False):
    """Mask arithmetic of generate_cowmix_masks_like (cowmix.py:40-69).

    noise [B,1,H,W] or [B,H,W] f32, sigma [B], p [B] (device tensors) -> mask [B,1,H,W] f32.
    """
    B = noise.shape[0]
    H, W = noise.shape[-2:]
    noise = _c(noise.float())
    sigma = _c(sigma.float().to(noise.device))
    p = _c(p.float().to(noise.device))
    mask = torch.empty(B, 1, H, W, device=noise.device, dtype=torch.float32)
    field = torch.empty_like(mask) if return_field else None
    thr = torch.empty(B, device=noise.device, dtype=torch.float32) if return_field else None
    nb = N.lib().ssseg_cowmix_workspace_bytes(B, H, W)
    ws = N.workspace(nb, noise.device)
    N.call('ssseg_cowmix_mask', N.dev_ptr(noise, 'noise'), N.dev_ptr(sigma), N.dev_ptr(p), B, H, W, N.dev_ptr(mask),
           N.dev_ptr(field) if field is not None else None, N.dev_ptr(thr) if thr is not None else None,
           N.dev_ptr(ws), nb, N.stream())
    if return_field:
        return mask, field, thr
    return mask


def normal_(out, seed, offset):
    N.call('ssseg_normal_f32', N.dev_ptr(out, 'out'), out.numel(), int(seed) & (2 ** 64 - 1),
           int(offset) & (2 ** 64 - 1), N.stream())
    return out


def mix(a, b, mask):
    """mix_with_mask (cowmix.py:72-73): a*m + b*(1-m), mask [B,1,H,W] broadcast over channels."""
    a, b = _c(a), _c(b)
    m = _c(mask.float())
    out = torch.empty_like(a)
    B, C = a.shape[0], a.shape[1]
    HW = a[0, 0].numel()
    N.call('ssseg_mix', N.dev_ptr(a, 'a'), N.dev_ptr(b, 'b'), N.dev_ptr(m, 'mask'), N.dev_ptr(out), B, C, HW,
           N.dt_code(a), N.stream())
    return out


# ------------------------------------------------------------------------------------------------
# Bilinear interpolation (F.interpolate mode='bilinear')
# ------------------------------------------------------------------------------------------------
def _axpby(x, a, y=None, b=0.0):
    out = torch.empty_like(x)
    N.call('ssseg_axpby', N.dev_ptr(x), float(a), N.dev_ptr(y) if y is not None else None, float(b), N.dev_ptr(out),
           x.numel(), N.stream())
    return out


class _Axpby(torch.autograd.Function):
    """a*x (+ b*y): the loss-term arithmetic on the device (no framework elementwise kernels)"""
    @staticmethod
    def forward(ctx, x, a, y, b):
        ctx.a, ctx.b, ctx.has_y = a, b, y is not None
        return _axpby(_c(x), a, _c(y) if y is not None else None, b)

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        gx = _axpby(g, ctx.a) if ctx.a != 1.0 else g
        gy = None
        if ctx.has_y:
            gy = _axpby(g, ctx.b) if ctx.b != 1.0 else g
        return gx, None, gy, None


def scale(x, a):
    """a * x for a device loss tensor (autograd)."""
    return _Axpby.apply(x, float(a), None, 0.0)


def add_scaled(x, y, b=1.0):
    """x + b * y for device loss tensors (autograd)."""
    return _Axpby.apply(x, 1.0, y, float(b))


_ONES = {}


def backward(loss):
    """loss.backward() seeded from a cached device 1.0 (autograd's own seed is a framework fill kernel)."""
    key = (loss.device, loss.dtype, tuple(loss.shape))
    one = _ONES.get(key)
    if one is None:
        one = torch.ones_like(loss)
        _ONES[key] = one
    loss.backward(one)


class _Bilinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size, align_corners):
        Nn, C, H, W = x.shape
        Ho, Wo = int(size[0]), int(size[1])
        fmt = torch.channels_last if (x.is_contiguous(memory_format=torch.channels_last) and C > 1
                                      and not x.is_contiguous()) else torch.contiguous_format
        y = torch.empty((Nn, C, Ho, Wo), device=x.device, dtype=x.dtype, memory_format=fmt)
        N.call('ssseg_bilinear_fwd', N.dev_ptr(x, 'x'), N.dev_ptr(y), Nn, C, H, W, Ho, Wo, N.strides4(x),
               N.strides4(y), int(bool(align_corners)), N.dt_code(x), N.stream())
        ctx.meta = (Nn, C, H, W, Ho, Wo, bool(align_corners), fmt)
        return y

    @staticmethod
    def backward(ctx, gy):
        Nn, C, H, W, Ho, Wo, ac, fmt = ctx.meta
        gx = torch.empty((Nn, C, H, W), device=gy.device, dtype=gy.dtype, memory_format=fmt)
        N.call('ssseg_bilinear_bwd', N.dev_ptr(gy, 'gy'), N.dev_ptr(gx), Nn, C, H, W, Ho, Wo, N.strides4(gy),
               N.strides4(gx), int(ac), N.dt_code(gy), N.stream())
        return gx, None, None


_IDENTITY_RESIZE = os.environ.get('SSSEG_BILINEAR_IDENTITY', '1') != '0'   # (A/B switch: 0 = always launch)


def interpolate_bilinear(x, size, align_corners=False):
    """F.interpolate(x, size, mode='bilinear', align_corners=...) on the device.  At the input's own size the sampling
    weights are (1, 0) for either align_corners -- the values are the input's -- and PyTorch's CPU kernels copy the
    input there ('special case: just copy'), so x itself is returned (the logits-to-mask-size resizes of the training
    step, train.py:71,74,93 and losses.py:18, are all identity-sized on the benchmark geometry) when it is dense NCHW
    or channels_last; the kernel would write the same layout."""
    size = (int(size[0]), int(size[1]))
    if _IDENTITY_RESIZE and x.dim() == 4 and tuple(x.shape[2:4]) == size and (
            x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last)):
        return x
    return _Bilinear.apply(x, size, align_corners)


class _Rotate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, angle):
        x = _c(x.float())
        y = torch.empty_like(x)
        Nn, C, H, W = x.shape
        N.call('ssseg_rotate_fwd', N.dev_ptr(x, 'x'), N.dev_ptr(y), Nn, C, H, W, float(angle), N.stream())
        ctx.meta = (Nn, C, H, W, float(angle))
        return y

    @staticmethod
    def backward(ctx, gy):
        Nn, C, H, W, angle = ctx.meta
        gy = _c(gy.float())
        gx = torch.empty_like(gy)
        N.call('ssseg_rotate_bwd', N.dev_ptr(gy), N.dev_ptr(gx), Nn, C, H, W, angle, N.stream())
        return gx, None


def rotate(x, angle_deg):
    """kornia.rotate(x, angle) for NCHW fp32 (reversible_augmentations.py:13-23): counter-clockwise degrees
    about the image centre, bilinear, zero padding; differentiable."""
    return _Rotate.apply(x, angle_deg)


class _Sigmoid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _c(x.float())
        y = torch.empty_like(x)
        N.call('ssseg_sigmoid_fwd', N.dev_ptr(x, 'x'), N.dev_ptr(y), x.numel(), N.stream())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        gy = _c(gy.float())
        gx = torch.empty_like(y)
        N.call('ssseg_sigmoid_bwd', N.dev_ptr(y), N.dev_ptr(gy), N.dev_ptr(gx), y.numel(), N.stream())
        return gx


def sigmoid(x):
    """torch.sigmoid (fp32, any layout -> contiguous): the probability map the discriminator sees."""
    return _Sigmoid.apply(x)


# ------------------------------------------------------------------------------------------------
# Losses
# ------------------------------------------------------------------------------------------------
class _BCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t):
        x, t = _c(x.float()), _c(t.float())
        out = torch.empty((), device=x.device, dtype=torch.float32)
        nb = N.lib().ssseg_reduce_workspace_bytes(x.numel())
        ws = N.workspace(nb, x.device)
        N.call('ssseg_bce_logits_fwd', N.dev_ptr(x, 'x'), N.dev_ptr(t, 'target'), x.numel(), N.dev_ptr(out),
               N.dev_ptr(ws), nb, N.stream())
        ctx.save_for_backward(x, t)
        return out

    @staticmethod
    def backward(ctx, g):
        x, t = ctx.saved_tensors
        gx = torch.empty_like(x)
        g = _c(g.float())
        N.call('ssseg_bce_logits_bwd', N.dev_ptr(x), N.dev_ptr(t), x.numel(), N.dev_ptr(g), N.dev_ptr(gx), N.stream())
        return gx, None


def bce_with_logits_mean(x, t):
    """F.binary_cross_entropy_with_logits(x, t, reduction='mean') (losses.py:47)."""
    return _BCE.apply(x, t)


class _Consistency(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t, thr):
        s, t = _c(s.float()), _c(t.float())
        B, C = s.shape[:2]
        HW = s[0, 0].numel()
        out = torch.empty(3, device=s.device, dtype=torch.float32)
        nb = N.lib().ssseg_reduce_workspace_bytes(B * HW)
        ws = N.workspace(nb, s.device)
        N.call('ssseg_consistency_fwd', N.dev_ptr(s, 'student'), N.dev_ptr(t, 'teacher'), B, C, HW, float(thr),
               N.dev_ptr(out), N.dev_ptr(ws), nb, N.stream())
        ctx.save_for_backward(s, t, out)
        ctx.meta = (B, C, HW, float(thr))
        ctx.mark_non_differentiable(out)
        ctx.set_materialize_grads(False)   # no zero-filled gradient for the cm output (a framework fill kernel)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_loss, g_cm):
        s, t, out = ctx.saved_tensors
        B, C, HW, thr = ctx.meta
        gs = torch.empty_like(s)
        g = _c(g_loss.float())
        N.call('ssseg_consistency_bwd', N.dev_ptr(s), N.dev_ptr(t), B, C, HW, thr, N.dev_ptr(out), N.dev_ptr(g),
               N.dev_ptr(gs), N.stream())
        return gs, None, None


def consistency_loss(student_logits, teacher_logits, thr):
    """train.py:97-108: returns (loss, confidence_modulator.mean()); loss is NaN when no pixel is confident."""
    return _Consistency.apply(student_logits, teacher_logits, thr)


# ------------------------------------------------------------------------------------------------
# EMA / optimiser over flat arenas
# ------------------------------------------------------------------------------------------------
def ema_update_(ema_flat, param_flat, alpha):
    """mean_teacher.update_ema_variables parameter loop (mean_teacher.py:10-11), one launch."""
    assert ema_flat.numel() == param_flat.numel() and ema_flat.dtype == torch.float32
    N.call('ssseg_ema_update', N.dev_ptr(ema_flat, 'ema'), N.dev_ptr(param_flat, 'param'), ema_flat.numel(),
           float(alpha), N.stream())


def sqnorm_(x_flat, out):
    nb = N.lib().ssseg_reduce_workspace_bytes(x_flat.numel())
    ws = N.workspace(nb, x_flat.device)
    N.call('ssseg_sqnorm_accum', N.dev_ptr(x_flat, 'x'), x_flat.numel(), N.dev_ptr(out), N.dev_ptr(ws), nb, N.stream())


def sgd_step_(param, grad, buf, shadow, lr, momentum, wd, max_norm, sqnorm, first, amp_state=None):
    N.call('ssseg_sgd_step', N.dev_ptr(param, 'param'), N.dev_ptr(grad, 'grad'),
           N.dev_ptr(buf) if buf is not None else None, N.dev_ptr(shadow) if shadow is not None else None,
           param.numel(), float(lr), float(momentum), float(wd), float(max_norm),
           N.dev_ptr(sqnorm) if sqnorm is not None else None, int(bool(first)),
           N.dev_ptr(amp_state) if amp_state is not None else None, N.stream())


# ------------------------------------------------------------------------------------------------
# Lovász (losses.py:239-250)
# ------------------------------------------------------------------------------------------------
class _Lovasz(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        logits, target = _c(logits.float()), _c(target.float())
        B, C = logits.shape[:2]
        HW = logits[0, 0].numel()
        out = torch.empty((), device=logits.device, dtype=torch.float32)
        nb = N.lib().ssseg_lovasz_workspace_bytes(B, HW)
        ws = N.workspace(nb, logits.device)
        N.call('ssseg_lovasz_fwd', N.dev_ptr(logits, 'logits'), N.dev_ptr(target, 'target'), B, C, HW,
               N.dev_ptr(out), N.dev_ptr(ws), nb, N.stream())
        ctx.save_for_backward(logits, target)
        ctx.ws, ctx.nb = ws, nb   # the forward's per-pixel gradient and image scales: the backward does not re-sort
        return out

    @staticmethod
    def backward(ctx, g):
        logits, target = ctx.saved_tensors
        B, C = logits.shape[:2]
        HW = logits[0, 0].numel()
        gx = torch.empty_like(logits)
        g = _c(g.float())
        N.call('ssseg_lovasz_bwd_from_fwd', N.dev_ptr(logits), N.dev_ptr(target), B, C, HW, N.dev_ptr(g),
               N.dev_ptr(gx), N.dev_ptr(ctx.ws), ctx.nb, N.stream())
        # (ctx.ws stays for the lifetime of ctx: a second backward through a retained graph reads it again)
        return gx, None


def lovasz_binary(logits, target, valid_weighted=True):
    """binary_lovasz_loss_with_logits (losses.py:239-250) on the device."""
    if not valid_weighted:
        raise NotImplementedError('lovasz_softmax without the valid-sample weighting')
    return _Lovasz.apply(logits, target)


# ------------------------------------------------------------------------------------------------
# RMILoss (losses.py:271-592, sigmoid form)
# ------------------------------------------------------------------------------------------------
class _RMI(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, geo):
        logits, target = _c(logits.float()), _c(target.float())
        Nn, C, H, W = logits.shape
        nb = N.lib().ssseg_rmi_workspace_bytes(Nn, C, H, W, *geo)
        if nb == 0:
            raise ValueError(f'RMILoss: geometry {tuple(logits.shape)} / (num_classes, radius, k, s, pad) = {geo} '
                             'is not supported')
        # the workspace carries the pooled maps and the backward coefficients to backward: a tensor of its own
        ws = torch.empty(nb, dtype=torch.uint8, device=logits.device)
        out = torch.empty((), device=logits.device, dtype=torch.float32)
        want = int(ctx.needs_input_grad[0])
        N.call('ssseg_rmi_fwd', N.dev_ptr(logits, 'logits'), N.dev_ptr(target, 'target'), Nn, C, H, W, *geo, want,
               N.dev_ptr(out), N.dev_ptr(ws), nb, N.stream())
        if want:
            ctx.save_for_backward(logits, ws)
        ctx.geo = geo
        return out

    @staticmethod
    def backward(ctx, g):
        logits, ws = ctx.saved_tensors
        Nn, C, H, W = logits.shape
        gx = torch.empty_like(logits)
        g = _c(g.float())
        N.call('ssseg_rmi_bwd', N.dev_ptr(logits), Nn, C, H, W, *ctx.geo, N.dev_ptr(g), N.dev_ptr(gx), N.dev_ptr(ws),
               ws.numel(), N.stream())
        return gx, None, None


def rmi_loss(logits, target, num_classes, radius, pool_k, pool_s, pool_pad):
    """RMILoss.forward (losses.py:480-592) on the device: sigmoid probabilities, avg pool (k, s, pad; (1, 1, 0) =
    none), fp64 region covariances and Cholesky log-det per (image, class), summed over classes."""
    if logits.dim() != 4 or tuple(logits.shape) != tuple(target.shape):
        raise ValueError(f'RMILoss: logits {tuple(logits.shape)} and target {tuple(target.shape)} must be the same NCHW shape')
    return _RMI.apply(logits, target, (int(num_classes), int(radius), int(pool_k), int(pool_s), int(pool_pad)))


# ------------------------------------------------------------------------------------------------
# Multi-scale attention blend (multiscale_attention.py:52-54)
# ------------------------------------------------------------------------------------------------
class _AttBlend(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lo, hi, att):
        Nn, C, H, W = hi.shape
        if tuple(lo.shape) != (Nn, C, H, W) or tuple(att.shape) != (Nn, 1, H, W):
            raise ValueError(f'att_blend: shapes {tuple(lo.shape)} {tuple(hi.shape)} {tuple(att.shape)}')
        for t, n in ((lo, 'lo'), (hi, 'hi'), (att, 'att')):
            if t.dtype != torch.float32:
                raise RuntimeError(f'att_blend: {n} must be fp32')
        out = torch.empty((Nn, C, H, W), device=hi.device, dtype=torch.float32)
        N.call('ssseg_att_blend_fwd', N.dev_ptr(lo, 'lo'), N.strides4(lo), N.dev_ptr(hi, 'hi'), N.strides4(hi),
               N.dev_ptr(att, 'att'), N.strides4(att), N.dev_ptr(out), Nn, C, H, W, N.stream())
        ctx.save_for_backward(lo, hi, att)
        return out

    @staticmethod
    def backward(ctx, g):
        lo, hi, att = ctx.saved_tensors
        Nn, C, H, W = hi.shape
        g = g.float()
        glo = torch.empty((Nn, C, H, W), device=g.device, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        ghi = torch.empty((Nn, C, H, W), device=g.device, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        gat = torch.empty((Nn, 1, H, W), device=g.device, dtype=torch.float32) if ctx.needs_input_grad[2] else None
        N.call('ssseg_att_blend_bwd', N.dev_ptr(g), N.strides4(g), N.dev_ptr(lo), N.strides4(lo), N.dev_ptr(hi),
               N.strides4(hi), N.dev_ptr(att), N.strides4(att), N.dev_ptr(glo), N.dev_ptr(ghi), N.dev_ptr(gat), Nn, C,
               H, W, N.stream())
        return glo, ghi, gat


def att_blend(lo, hi, att_logits):
    """lo*sigmoid(a) + hi*(1-sigmoid(a)) (MultiscaleAttention, multiscale_attention.py:52-54); fp32 NCHW
    tensors of any strides, att [N,1,H,W] pre-sigmoid; returns contiguous NCHW."""
    return _AttBlend.apply(lo, hi, att_logits)


# ------------------------------------------------------------------------------------------------
# Validation metrics (train.validate, train.py:150-195)
# ------------------------------------------------------------------------------------------------
class SegMetrics:
    """Dice (metrics.dice_metric on the nearest-resized argmax one-hot, train.py:178-186) and the
    confusion counts of lovasz.iou (lovasz.py:54-73, C=2, per_image=False) in one pass per batch.
    `update(logits, mask)` returns a device tensor [dice_mean, iou0, iou1, miou]; the IoUs are over every
    batch seen so far (running counts on the device)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.total = torch.zeros(8, dtype=torch.int64, device=self.device)

    def update(self, logits, mask):
        if logits.dim() != 4 or logits.shape[1] != 2 or mask.dim() != 4 or mask.shape[1] != 2:
            raise ValueError('SegMetrics: binary [B,2,h,w] logits and [B,2,H,W] mask expected')
        if logits.shape[0] != mask.shape[0]:
            raise ValueError('SegMetrics: batch size mismatch')
        logits = logits if logits.dtype == torch.float32 else logits.float()
        mask = mask if mask.dtype == torch.float32 else mask.float()
        B, _, h, w = logits.shape
        H, W = mask.shape[2:]
        counts = torch.empty(B, 8, dtype=torch.int64, device=logits.device)
        out = torch.empty(4, dtype=torch.float32, device=logits.device)
        N.call('ssseg_seg_metrics', N.dev_ptr(logits, 'logits'), N.strides4(logits), h, w, N.dev_ptr(mask, 'mask'),
               N.strides4(mask), B, H, W, N.dev_ptr(counts), N.dev_ptr(self.total), N.dev_ptr(out), N.stream())
        self.counts = counts
        return out


def prob_onehot(logits):
    """sigmoid probabilities + one-hot argmax mask of binary logits [B,2,H,W] (inference_wrapper.py:17-24)."""
    if logits.dim() != 4 or logits.shape[1] != 2:
        raise ValueError('prob_onehot: binary [B,2,H,W] logits expected')
    x = _c(logits.float())
    prob, onehot = torch.empty_like(x), torch.empty_like(x)
    B, _, H, W = x.shape
    N.call('ssseg_prob_onehot', N.dev_ptr(x, 'logits'), B, H * W, N.dev_ptr(prob), N.dev_ptr(onehot), N.stream())
    return prob, onehot
