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
        for ed, md, ek, mk in _buffer_slots(e, m):
            eb, b = ed[ek], md[mk]
            if eb.data_ptr() != b.data_ptr() or eb.shape != b.shape:   # already aliased: data = data is a no-op
                eb.data = b.data
        snn.invalidate_packed(e)


def _buffer_slots(e, m):
    """The zip(e.buffers(), m.buffers()) pairing of mean_teacher.py:16-18 as (ema _buffers dict, student
    _buffers dict, key, key) slots, built once per model pair: walking both module trees costs ~1 ms of host
    time per step, the slot lookups ~0.1 ms.  The dicts are the modules' own, so buffers replaced by
    .to()/load are still seen; the table is rebuilt if either tree's buffer count changes."""
    cache = e.__dict__.get('_ssseg_buf_slots')
    if cache is not None and cache[0] == id(m) and all(len(ed) == ne and len(md) == nm
                                                       for ed, md, ne, nm in cache[2]):
        return cache[1]

    def slots(mod):
        out = []
        for sub in mod.modules():
            for k, b in sub._buffers.items():
                if b is not None:
                    out.append((sub._buffers, k))
        return out

    es, ms = slots(e), slots(m)
    table = [(ed, md, ek, mk) for (ed, ek), (md, mk) in zip(es, ms)]
    dicts = {}
    for ed, md, _, _ in table:
        dicts[(id(ed), id(md))] = (ed, md, len(ed), len(md))
    e.__dict__['_ssseg_buf_slots'] = (id(m), table, list(dicts.values()))
    return table


def detach_model_parameters(model):
    for param in model.parameters():
        param.detach_()
