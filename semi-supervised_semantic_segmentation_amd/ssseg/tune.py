"""The conv engine's per-geometry variant table across the ranks of a data-parallel job.

Each process tunes an unseen conv geometry on first use (csrc/conv.hip tune_variant: every candidate timed with HIP
events; every variant gives bit-identical results, so only speed depends on the choice).  With one process per GPU all
ranks see the same geometries (same model, same per-rank batch); instead of each rank timing all of them (minutes on a
fresh, busy host, and possibly different picks per rank), rank 0 tunes and the others follow:

    tune.follow_rank0()   # before the first step: ranks > 0 take the static rule meanwhile (knob 5 = 0)
    ... eager warm-up steps ...
    tune.sync()           # collective: rank 0's table broadcast and imported (overwriting) on every rank

after which every rank holds the same table (tune.digest() compares) and a captured step launches the same kernels on
all of them.  save()/load() keep a table across processes (SSSEG_TUNE_FILE: loaded by bench.py / train.train at start).
"""
import ctypes
import hashlib
import os

import torch.distributed as dist

from . import native as N

_STATE = {'synced': False, 'following': False}


def export():
    """[(key, variant)] of this process, in key order."""
    L = N.lib()
    n = int(L.ssseg_tune_table_export(None, None, 0))
    if n <= 0:
        return []
    keys = (ctypes.c_ulonglong * n)()
    vals = (ctypes.c_int32 * n)()
    m = int(L.ssseg_tune_table_export(keys, vals, n))
    return list(zip(keys[:min(n, m)], vals[:min(n, m)]))


def import_(rows, overwrite=True):
    if not rows:
        return
    keys = (ctypes.c_ulonglong * len(rows))(*[k for k, _ in rows])
    vals = (ctypes.c_int32 * len(rows))(*[v for _, v in rows])
    rc = N.lib().ssseg_tune_table_import(keys, vals, len(rows), int(bool(overwrite)))
    if rc != 0:
        raise RuntimeError(f'ssseg: ssseg_tune_table_import failed ({rc})')


def digest(rows=None):
    rows = export() if rows is None else rows
    return hashlib.sha256(repr(rows).encode()).hexdigest()[:16]


def _multi():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def follow_rank0():
    """Ranks > 0 stop timing unseen geometries (static rule until sync()); rank 0 keeps tuning."""
    if _multi() and dist.get_rank() != 0:
        N.call('ssseg_set_knob', 5, 0)
        _STATE['following'] = True


def sync():
    """Collective: rank 0's table to every rank (imported, overwriting); afterwards the ranks tune again on their own
    only for geometries rank 0 never saw.  Returns this rank's table digest (equal on all ranks)."""
    if not _multi():
        return digest()
    box = [export() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(box, src=0)
    if dist.get_rank() != 0:
        import_(box[0], overwrite=True)
        if _STATE['following']:
            N.call('ssseg_set_knob', 5, 1)
            _STATE['following'] = False
    _STATE['synced'] = True
    return digest()


def synced():
    return _STATE['synced']


def digests():
    """Every rank's table digest (collective), rank order."""
    d = digest()
    if not _multi():
        return [d]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, d)
    return out


def save(path):
    with open(path, 'w') as f:
        f.write(f'# {N.lib().ssseg_version().decode()} conv variant table: key variant\n')
        for k, v in export():
            f.write(f'{k} {v}\n')


def load(path, overwrite=False):
    """Rows of a table saved by save() by the same library version; returns the number imported (0 if the file is
    absent or from another version)."""
    if not path or not os.path.exists(path):
        return 0
    with open(path) as f:
        lines = f.read().splitlines()
    if not lines or lines[0] != f'# {N.lib().ssseg_version().decode()} conv variant table: key variant':
        return 0
    rows = [tuple(int(t) for t in ln.split()) for ln in lines[1:] if ln.strip()]
    import_(rows, overwrite=overwrite)
    return len(rows)
