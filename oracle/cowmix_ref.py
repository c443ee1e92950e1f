"""Oracle: CowMix mask generation and mixing (numpy).  TEST INFRASTRUCTURE ONLY.

Follows reference/cowmix.py:
  gaussian_taps          <- generate_gaussian            cowmix.py:6-11
  window_size            <- dual_pass_gaussian_fileter2d cowmix.py:30
  blur_field             <- dual_pass_gaussian_fileter2d cowmix.py:27-37 (vertical pass, then horizontal)
  threshold_masks        <- generate_cowmix_masks_like   cowmix.py:60-68
  draw_inputs            <- RNG order of                 cowmix.py:44-55 (rand B, rand B, normal B*H*W)
  mix                    <- mix_with_mask                cowmix.py:72-73
"""
import math

import numpy as np


def window_size(sigmas):
    """K = int(round(max sigma * 3) * 2) + 1  (cowmix.py:30).  Python round = banker's rounding."""
    return int(round(float(np.max(sigmas)) * 3) * 2) + 1


def gaussian_taps(K, sigma):
    """cowmix.py:6-11.  x = arange(-K//2, K//2) (+0.5 for even K); exp(-x^2 / (2 sigma^2)); normalise.

    For odd K the window is off-centre by one tap: x runs from -(K+1)/2 to (K-3)/2.
    float32 throughout, like the reference.
    """
    x = np.arange(-K // 2, K // 2, dtype=np.float32)
    if K % 2 == 0:
        x = x + np.float32(0.5)
    s = np.float32(sigma)
    denom = float(np.float32(2) * s * s)           # float(2 * sigma ** 2) on a float32 tensor
    g = np.exp(-(x * x) / np.float32(denom)).astype(np.float32)
    return (g / g.sum(dtype=np.float32)).astype(np.float32)


def blur_field(noise, sigmas):
    """Separable zero-padded Gaussian blur, vertical pass first (cowmix.py:33-36).

    noise: [B, H, W] float32.  Cross-correlation with padding K//2: out[y] = sum_k g[k] * in[y - K//2 + k].
    Accumulates in float32 in tap order k = 0..K-1.
    """
    noise = np.asarray(noise, dtype=np.float32)
    B, H, W = noise.shape
    K = window_size(sigmas)
    pad = K // 2
    out = np.empty_like(noise)
    for b in range(B):
        g = gaussian_taps(K, sigmas[b])
        src = np.zeros((H + 2 * pad, W), np.float32)
        src[pad:pad + H] = noise[b]
        v = np.zeros((H, W), np.float32)
        for k in range(K):
            v += g[k] * src[k:k + H]
        src = np.zeros((H, W + 2 * pad), np.float32)
        src[:, pad:pad + W] = v
        h = np.zeros((H, W), np.float32)
        for k in range(K):
            h += g[k] * src[:, k:k + W]
        out[b] = h
    return out


def threshold_masks(field, p):
    """Per-sample mean / unbiased std over (C,H,W), thr = erfinv(2p-1)*sqrt(2)*std + mean, mask = field > thr.

    cowmix.py:60-68.  Returns (mask float32 [B,H,W], thr [B], mean [B], std [B]).
    Statistics in float64 (the reference reduces float32 with pairwise sums; the difference only
    moves pixels inside the documented tie band).
    """
    from scipy.special import erfinv
    B = field.shape[0]
    f = field.reshape(B, -1).astype(np.float64)
    mean = f.mean(axis=1)
    std = f.std(axis=1, ddof=1)
    factor = (erfinv(2.0 * np.asarray(p, np.float32).astype(np.float64) - 1.0) * math.sqrt(2.0))
    thr = (factor * std + mean).astype(np.float32)
    mask = (field > thr.reshape(B, 1, 1)).astype(np.float32)
    return mask, thr, mean.astype(np.float32), std.astype(np.float32)


def draw_inputs(B, H, W, prop_range, sigma_range, generator=None):
    """Replay the reference's CPU-generator consumption order (cowmix.py:44-55).

    torch.distributions.Uniform(lo, hi).rsample(n) == lo + rand(n) * (hi - lo) on the default
    CPU generator; then torch.normal(0, 1, [B,1,H,W]).  Uses torch only as the RNG.
    """
    import torch
    lo, hi = torch.tensor(float(prop_range[0])), torch.tensor(float(prop_range[1]))
    p = torch.distributions.Uniform(lo, hi).rsample([B])
    slo = torch.tensor(math.log(float(sigma_range[0])))
    shi = torch.tensor(math.log(float(sigma_range[1])))
    sig = torch.exp(torch.distributions.Uniform(slo, shi).rsample([B]))
    noise = torch.normal(mean=0, std=1, size=(B, 1, H, W), dtype=torch.float32)
    return p.numpy(), sig.numpy(), noise.numpy().reshape(B, H, W)


def cowmix_masks(noise, sigmas, p):
    field = blur_field(noise, sigmas)
    mask, thr, mean, std = threshold_masks(field, p)
    return mask, field, thr, mean, std


def mix(a, b, m):
    """a * m + b * (1 - m)  (cowmix.py:72-73), m broadcast over channels."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    m = np.asarray(m, np.float32)
    return (a * m + b * (np.float32(1.0) - m)).astype(np.float32)
