"""Mean teacher — drop-in for reference mean_teacher.py (update_ema_variables :5-18,
detach_model_parameters :20-22).

ema <- alpha*ema + (1-alpha)*param, bit-exact with torch's CPU mul_().add_(alpha=) (ssseg_ema_update),
as ONE launch over the flat parameter arenas when both models have one (ssseg.arena), else one launch
per tensor.  Buffers are aliased, not averaged (mean_teacher.py:13-18)."""
import torch

from ssseg import arena as _arena
from ssseg import nn as snn
from ssseg import ops


def update_ema_variables(model, ema_model, alpha):
    with torch.no_grad():
        m = getattr(model, 'module', model)
        e = getattr(ema_model, 'module', ema_model)
        fa, ea = _arena.of(m), _arena.of(e)
        if fa is not None and ea is not None and fa.compatible(ea):
            ops.ema_update_(ea.data, fa.data, alpha)
        else:
            for ep, p in zip(e.parameters(), m.parameters()):
                ops.ema_update_(ep.data.view(-1), p.data.view(-1), alpha)
        for eb, b in zip(e.buffers(), m.buffers()):
            eb.data = b.data
        snn.invalidate_packed(e)


def detach_model_parameters(model):
    for param in model.parameters():
        param.detach_()
