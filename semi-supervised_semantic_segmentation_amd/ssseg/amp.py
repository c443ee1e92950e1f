"""Dynamic loss scaling for the fp16 compute mode (config C5 names fp16).

IEEE half has 5 exponent bits: the per-pixel loss gradients of a 16x2x512x512 BCE mean (~1e-7) fall below
its smallest normal (6.1e-5) and flush in the fp16 activation gradients.  The standard remedy
(torch.cuda.amp.GradScaler) scales the loss by S before backward and unscales the fp32 parameter gradients
before the optimizer step, skipping steps whose gradients overflowed and adapting S.  Here everything stays
on the device (no host sync per step): the backward's incoming gradient is multiplied by S in a native
kernel (ssseg_scale_by), the fused clip + SGD kernel unscales by 1/S and skips a non-finite step, and
ssseg_amp_update adapts S (x0.5 on overflow, floored at 1; x2 after `growth_interval` finite steps).  bf16 / fp32 modes do not
use it (bf16 keeps fp32's exponent range)."""
import torch

from . import native as N


class _ScaleGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, loss, state):
        ctx.save_for_backward(state)
        return loss.view_as(loss)

    @staticmethod
    def backward(ctx, g):
        (state,) = ctx.saved_tensors
        g = g.contiguous().float()
        out = torch.empty_like(g)
        N.call('ssseg_scale_by', N.dev_ptr(g), N.dev_ptr(state), N.dev_ptr(out), g.numel(), N.stream())
        return out, None


class GradScaler:
    def __init__(self, device, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000):
        self.state = torch.tensor([init_scale, 0.0, 0.0, 1.0 / init_scale], dtype=torch.float32, device=device)
        self.growth, self.backoff, self.interval = float(growth_factor), float(backoff_factor), int(growth_interval)

    def scale(self, loss):
        """The same loss value forward; its backward starts from S * dL."""
        return _ScaleGrad.apply(loss, self.state)

    def update(self, sqnorm):
        N.call('ssseg_amp_update', N.dev_ptr(self.state), N.dev_ptr(sqnorm), self.growth, self.backoff, self.interval,
               N.stream())

    def state_dict(self):
        """Checkpointable state (scale, growth counter, last-step overflow flag): resume continues the schedule."""
        return {'state': self.state.detach().cpu().clone(), 'growth_factor': self.growth,
                'backoff_factor': self.backoff, 'growth_interval': self.interval}

    def load_state_dict(self, sd):
        self.state.copy_(sd['state'].to(self.state.device, torch.float32))
        self.growth = float(sd.get('growth_factor', self.growth))
        self.backoff = float(sd.get('backoff_factor', self.backoff))
        self.interval = int(sd.get('growth_interval', self.interval))

    def get_scale(self):
        return float(self.state[0])

    def found_inf(self):
        return bool(self.state[2] > 0)
