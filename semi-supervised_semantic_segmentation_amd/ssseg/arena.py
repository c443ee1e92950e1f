"""Flat parameter / gradient arenas.

All parameters of a model live in ONE contiguous fp32 buffer (param.data are views into it) and all
gradients in a second one (param.grad are views), in reverse registration order so that backward —
which produces the decoder's gradients first — fills the arena front to back.  That makes the EMA
update, the clip+SGD step and zero_grad single launches, and gives the DDP reducer contiguous buckets.
"""
import torch

from . import native as N


class FlatArena:
    def __init__(self, module, with_grads=True):
        params = [p for p in module.parameters()]
        params = params[::-1]
        dev = params[0].device
        sizes = [p.numel() for p in params]
        align = 4                                        # 16-byte alignment for vector kernels
        offs, total = [], 0
        for n in sizes:
            offs.append(total)
            total += (n + align - 1) // align * align
        self.numel = total
        self.params = params
        self.offsets = offs
        self.data = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev) if with_grads else None
        with torch.no_grad():
            for p, o, n in zip(params, offs, sizes):
                self.data[o:o + n].copy_(p.data.reshape(-1))
                p.data = self.data[o:o + n].view_as(p)
                if self.grad is not None and p.requires_grad:
                    p.grad = self.grad[o:o + n].view_as(p)
                p._ssseg_arena = self
        self._module_ref = module
        module._ssseg_arena = self

    def compatible(self, other):
        return self.offsets == other.offsets and [p.shape for p in self.params] == [q.shape for q in other.params]

    def slot(self, p):
        i = next(i for i, q in enumerate(self.params) if q is p)
        return self.offsets[i], p.numel()

    def zero_grad(self):
        if self.grad is not None:
            if self.grad.is_cuda:
                N.call('ssseg_zero', N.dev_ptr(self.grad), self.grad.numel() * 4, N.stream())
            else:
                self.grad.zero_()


def attach(module, with_grads=True):
    a = getattr(module, '_ssseg_arena', None)
    if a is None:
        a = FlatArena(module, with_grads)
    return a


def of(module):
    return getattr(module, '_ssseg_arena', None)
