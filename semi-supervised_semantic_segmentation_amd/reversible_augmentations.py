"""Reversible augmentations — drop-in for reference reversible_augmentations.py (Rotate :5-23, Rescale :26-49),
which wraps kornia.rotate / kornia.resize and is imported (never called) by train.py:5.

Same API and sampling: Rotate(max_angle) draws one angle ~ U(-|max_angle|, |max_angle|) per apply() from the
CPU generator and applies it to every tensor of the list; reverse() rotates back by -angle.  Rescale(min, max)
draws one scale per apply() and resizes to (int(H*s), int(W*s)); reverse() resizes by 1/s.  Compute runs on the
device kernels: ssseg_rotate_fwd/bwd (bilinear about the centre, zero padding, differentiable) and the bilinear
interpolation kernel (align_corners=False, kornia.resize's default).  kornia is absent here and unpinned by the
reference, so parity with kornia itself is unpinned; the kernels are checked against a torch grid_sample
restatement (tests/test_hip_losses.py)."""
import torch

from ssseg import ops


class Rotate:
    def __init__(self, max_angle):
        self.max_angle = torch.abs(torch.tensor([max_angle], dtype=torch.float32))
        self.distribution = torch.distributions.uniform.Uniform(low=-self.max_angle, high=self.max_angle)
        self.angle = None

    def apply(self, inputs):
        self.angle = self.distribution.sample()
        return [ops.rotate(t, float(self.angle)) for t in inputs]

    def reverse(self, inputs):
        return [ops.rotate(t, -float(self.angle)) for t in inputs]


class Rescale:
    def __init__(self, min_scale, max_scale):
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.distribution = torch.distributions.uniform.Uniform(low=torch.tensor([min_scale], dtype=torch.float32),
                                                                high=torch.tensor([max_scale], dtype=torch.float32))
        self.scale = None

    def apply(self, inputs):
        self.scale = self.distribution.sample().item()
        return [ops.interpolate_bilinear(t, (int(t.size(2) * self.scale), int(t.size(3) * self.scale)))
                for t in inputs]

    def reverse(self, inputs):
        return [ops.interpolate_bilinear(t, (int(t.size(2) * (1. / self.scale)), int(t.size(3) * (1. / self.scale))))
                for t in inputs]
