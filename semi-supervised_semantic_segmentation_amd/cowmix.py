"""CowMix — drop-in for reference cowmix.py with the mask arithmetic on the MI355X kernels.

API (reference cowmix.py): generate_gaussian (:6-11), gaussian_kernel_2d_vertical (:14-24),
dual_pass_gaussian_fileter2d (:27-37), generate_cowmix_masks_like (:40-69), mix_with_mask (:72-73).

Random inputs (p, sigma, noise) come from one of two sources:
  NOISE_SOURCE = 'device' (default): Philox on the GPU (ssseg_cowmix_draw) — like the reference on a
      GPU, whose torch.normal(device=cuda) never touches the CPU generator; no host sync, capturable.
  NOISE_SOURCE = 'cpu': the CPU torch generator in the reference's order (rand B, rand B, normal B*H*W)
      — bit-identical draws to the reference's CPU path; used by the parity tests.
"""
import math

import torch

from ssseg import native as N
from ssseg import ops

NOISE_SOURCE = 'device'
_DEVICE_RNG = {'seed': None, 'ctr': {}}


def generate_gaussian(window_size, sigma):
    """Host helper (cowmix.py:6-11): normalised Gaussian window with the reference's +1 tap offset."""
    x = torch.arange(-window_size // 2, window_size // 2).float()
    if window_size % 2 == 0:
        x = x + 0.5
    g = torch.exp(-x * x / float(2 * sigma ** 2))
    return g / g.sum()


def gaussian_kernel_2d_vertical(size, sigmas):
    """Host helper (cowmix.py:14-24): [B,1,K,1] stack of per-sample windows."""
    return torch.stack([generate_gaussian(size, sigma=s) for s in sigmas], 0)[:, None, :, None]


def dual_pass_gaussian_fileter2d(input, sigmas):
    """cowmix.py:27-37 on the device: input 1xBxHxW -> blurred field 1xBxHxW (vertical, then horizontal)."""
    assert input.shape[1] == sigmas.shape[0]
    B, H, W = input.shape[1], input.shape[2], input.shape[3]
    noise = input.reshape(B, H, W)
    dummy_p = torch.full((B,), 0.5, device=input.device)
    _, field, _ = ops.cowmix_mask(noise, sigmas.to(input.device), dummy_p, return_field=True)
    return field.reshape(1, B, H, W)


def _device_seed(device):
    if _DEVICE_RNG['seed'] is None:
        _DEVICE_RNG['seed'] = int(torch.randint(0, 2 ** 62, (1,)).item())
    return _DEVICE_RNG['seed']


def draw_inputs(example_tensor, mask_proportion_range, sigma_range, source=None):
    """(p [B], sigma [B], noise [B,1,H,W]) on the example's device."""
    source = source or NOISE_SOURCE
    B, _, H, W = example_tensor.shape
    dev = example_tensor.device
    if source == 'cpu':
        p = torch.distributions.Uniform(torch.tensor(mask_proportion_range[0]),
                                        torch.tensor(mask_proportion_range[1])).rsample(sample_shape=[B])
        lo, hi = math.log(float(sigma_range[0])), math.log(float(sigma_range[1]))
        sig = torch.exp(torch.distributions.Uniform(torch.tensor(lo), torch.tensor(hi)).rsample([B]))
        noise = torch.normal(mean=0, std=1, size=(B, 1, H, W), dtype=torch.float32)
        return p.to(dev), sig.to(dev), noise.to(dev)
    p = torch.empty(B, device=dev)
    sig = torch.empty(B, device=dev)
    noise = torch.empty(B, 1, H, W, device=dev)
    seed = _device_seed(dev)
    # the Philox counter lives in device memory and the draw advances it there (ssseg_cowmix_draw_dev): the same
    # sequence as a host counter, and a captured HIP graph of the step (ssseg.graph) replays fresh draws
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ctr = _DEVICE_RNG['ctr'].get(key)
    if ctr is None:
        ctr = _DEVICE_RNG['ctr'][key] = torch.zeros(1, dtype=torch.int64, device=dev)
    N.call('ssseg_cowmix_draw_dev', N.dev_ptr(p), N.dev_ptr(sig), N.dev_ptr(noise), B, H * W,
           float(mask_proportion_range[0]), float(mask_proportion_range[1]), float(sigma_range[0]),
           float(sigma_range[1]), seed, N.dev_ptr(ctr), N.stream())
    return p, sig, noise


def generate_cowmix_masks_like(example_tensor, mask_proportion_range, sigma_range):
    """cowmix.py:40-69: B x 1 x H x W masks in {0, 1}, same dtype/device as the example."""
    with torch.no_grad():
        p, sig, noise = draw_inputs(example_tensor, mask_proportion_range, sigma_range)
        mask = ops.cowmix_mask(noise, sig, p)
        if mask.dtype != example_tensor.dtype:
            mask = mask.to(example_tensor.dtype)
        return mask


def mix_with_mask(tensor_a, tensor_b, mask):
    """cowmix.py:72-73: a*mask + b*(1-mask), mask broadcast over channels."""
    return ops.mix(tensor_a, tensor_b, mask)
