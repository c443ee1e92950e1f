"""Seeded model initialisation shared by the golden generator (tests/golden/gen_golden.py, run against the
reference) and the GPU parity tests (run against the product): the same constructor under the same seed,
then the same perturbation walk over modules() order, gives the same weights on both sides — checked by a
SHA-256 over the state_dict, so the large model fixtures store inputs/outputs and a hash, not weights."""
import hashlib

import numpy as np
import torch
import torch.nn as nn


def perturb(model, seed, conv_std=None):
    """BN affine + running stats drawn away from identity (eval mode is then a real test); with conv_std
    'he', conv weights re-drawn N(0, 2/fan_in) (HRNet's N(0, 0.001) init would make every logit ~0)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
                m.bias.copy_(torch.rand(m.bias.shape, generator=g) * 0.4 - 0.2)
                m.running_mean.copy_(torch.rand(m.running_mean.shape, generator=g) * 0.2 - 0.1)
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) * 1.5 + 0.5)
            elif conv_std == 'he' and isinstance(m, nn.Conv2d):
                fan_in = m.weight[0].numel()
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan_in) ** 0.5)
    return model


def state_sha(model):
    h = hashlib.sha256()
    for k, v in model.state_dict().items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v.detach().cpu().numpy()).tobytes())
    return h.hexdigest()


def array_sha(t):
    return hashlib.sha256(np.ascontiguousarray(t.detach().cpu().numpy()).tobytes()).hexdigest()
