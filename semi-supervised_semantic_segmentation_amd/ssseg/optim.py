"""SGD with momentum / weight decay and fused gradient clipping over a flat arena.

Replaces torch.optim.SGD (reference default_config.py:151-154) + clip_grad_norm_ (train.py:122):
one squared-norm reduction + one fused clip/weight-decay/momentum/update launch for the whole model
instead of ~4 launches per parameter tensor.  Subclasses torch.optim.Optimizer so LR schedulers and
state_dict()/load_state_dict() work (momentum buffers are exposed per parameter as views).
"""
import torch

from . import arena as _arena
from . import native as N
from . import ops


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr, momentum=0, dampening=0, weight_decay=0, nesterov=False):
        if dampening != 0 or nesterov:
            raise NotImplementedError('ssseg SGD: dampening / nesterov')
        params = list(params)
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=0, weight_decay=weight_decay,
                                      nesterov=False))
        ps = [p for g in self.param_groups for p in g['params']]
        arenas = {id(getattr(p, '_ssseg_arena', None)) for p in ps}
        a = getattr(ps[0], '_ssseg_arena', None)
        if a is None or len(arenas) != 1 or len(self.param_groups) != 1 or len(ps) != len(a.params):
            raise RuntimeError('ssseg SGD needs one param group covering a whole flat arena (ssseg.arena.attach)')
        self.arena = a
        self.buf = torch.zeros_like(a.data) if momentum else None
        self._first = True
        self._sq = torch.zeros(1, dtype=torch.float32, device=a.data.device)
        self.grad_scaler = None     # ssseg.amp.GradScaler in the fp16 compute mode (loss-scaled gradients)
        if self.buf is not None:
            for p, o in zip(a.params, a.offsets):
                self.state[p]['momentum_buffer'] = self.buf[o:o + p.numel()].view_as(p)

    def zero_grad(self, set_to_none=False):
        self.arena.zero_grad()

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict, then the loaded momentum buffers are copied into the flat
        momentum arena and the per-parameter state entries point back at its views (resume,
        distributed_trainer.py:64): the next step continues the momentum like torch.optim.SGD does."""
        super().load_state_dict(state_dict)
        loaded = False
        with torch.no_grad():
            for p, o in zip(self.arena.params, self.arena.offsets):
                st = self.state.get(p, {})
                mb = st.get('momentum_buffer') if isinstance(st, dict) else None
                if self.buf is None:
                    continue
                view = self.buf[o:o + p.numel()].view_as(p)
                if mb is not None:
                    view.copy_(mb.to(view.device, view.dtype))
                    loaded = True
                self.state[p]['momentum_buffer'] = view
        if loaded:
            self._first = False

    @torch.no_grad()
    def step(self, closure=None, max_norm=0.0):
        """max_norm > 0 clips the global gradient L2 norm first (clip_grad_norm_, train.py:122)."""
        g = self.param_groups[0]
        sc = self.grad_scaler
        if (max_norm and max_norm > 0) or sc is not None:
            N.call('ssseg_zero', N.dev_ptr(self._sq), 4, N.stream())
            ops.sqnorm_(self.arena.grad, self._sq)
        ops.sgd_step_(self.arena.data, self.arena.grad, self.buf, None, g['lr'], g['momentum'], g['weight_decay'],
                      max_norm or 0.0, self._sq if (max_norm or sc is not None) else None, self._first,
                      sc.state if sc is not None else None)
        if sc is not None:
            sc.update(self._sq)
        self._first = False
        return None


def from_config(factory, params):
    """Map a reference config's optimizer factory (functools.partial(torch.optim.SGD, ...)) to ssseg SGD."""
    fn = getattr(factory, 'func', factory)
    if fn is torch.optim.SGD or fn is SGD:
        kw = dict(getattr(factory, 'keywords', {}) or {})
        return SGD(params, **kw)
    return factory(params=params)
