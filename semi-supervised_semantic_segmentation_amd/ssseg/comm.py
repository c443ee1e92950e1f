"""The process's RCCL communicator for the training step's collectives (libssseg ssseg_comm_* / ssseg_allreduce_buckets).

Reference: distributed_trainer.py:34-38 (SyncBatchNorm + DistributedDataParallel over NCCL).  torch.distributed stays the
rendezvous (init_process_group, the unique-id broadcast, barriers, epoch-end meters); the collectives INSIDE the step --
the gradient buckets (ssseg.ddp) and the SyncBN sums (ssseg.nn) -- go through one communicator owned by libssseg, an
RCCL enqueue on the caller's stream with no completion object.  That is what makes a DDP step capturable as one HIP graph:
c10d's ProcessGroupNCCL keeps a WorkNCCL per collective whose events its watchdog thread polls, and a poll while any
stream of the process is capturing fails the capture ('operation not permitted when stream is capturing').

SSSEG_COMM=c10d keeps every collective on torch.distributed (A/B, and the path gloo process groups always take: the CPU
tests and the one-GPU multi-rank tests, where RCCL refuses two ranks on one device).
"""
import ctypes
import os
import sys

import torch
import torch.distributed as dist

from . import native as N

_STATE = {'comm': None, 'tried': False, 'error': None}


class NativeComm:
    """One RCCL communicator over the default process group's ranks, bound to this process's current device."""

    def __init__(self):
        L = N.lib()
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.device = torch.cuda.current_device()
        nbytes = int(L.ssseg_comm_unique_id_bytes())
        box = [None]
        if self.rank == 0:
            uid = ctypes.create_string_buffer(nbytes)
            _check(L.ssseg_comm_get_unique_id(uid), 'ssseg_comm_get_unique_id')
            box = [bytes(uid.raw)]
        dist.broadcast_object_list(box, src=0)
        uid = ctypes.create_string_buffer(box[0], nbytes)
        h = ctypes.c_void_p()
        _check(L.ssseg_comm_init(ctypes.byref(h), uid, self.rank, self.world, self.device), 'ssseg_comm_init')
        self.handle = h
        self.calls = 0          # all-reduce groups issued (tests count them)

    def all_reduce(self, tensors, op='sum', stream=None):
        """In-place all-reduce of device tensors (one RCCL group) on `stream` (default: the current stream)."""
        if not tensors:
            return
        dt = _DT.get(tensors[0].dtype)
        if dt is None or any(t.dtype != tensors[0].dtype or not t.is_contiguous() for t in tensors):
            raise RuntimeError('ssseg comm: all_reduce needs contiguous tensors of one dtype (f32/bf16/f16/f64)')
        ptrs = (ctypes.c_void_p * len(tensors))(*[N.dev_ptr(t) for t in tensors])
        counts = (ctypes.c_int64 * len(tensors))(*[t.numel() for t in tensors])
        s = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        _check(N.lib().ssseg_allreduce_buckets(self.handle, ptrs, counts, len(tensors), dt,
                                               N.SSSEG_AVG if op == 'avg' else N.SSSEG_SUM, s),
               'ssseg_allreduce_buckets')
        self.calls += 1

    def destroy(self):
        if self.handle:
            _check(N.lib().ssseg_comm_destroy(self.handle), 'ssseg_comm_destroy')
            self.handle = None


_DT = {torch.float32: N.F32, torch.bfloat16: N.BF16, torch.float16: N.F16, torch.float64: N.F64}


def _check(rc, name):
    if rc != 0:
        msg = N.lib().ssseg_comm_last_error().decode(errors='replace') if rc == -4 else f'rc {rc}'
        raise RuntimeError(f'ssseg: {name} failed: {msg}')


def wanted():
    """True where the step's collectives should use the native communicator: an RCCL ('nccl') process group on a HIP
    device, unless SSSEG_COMM=c10d."""
    return (os.environ.get('SSSEG_COMM', 'native') != 'c10d' and dist.is_available() and dist.is_initialized()
            and dist.get_backend() == 'nccl' and torch.cuda.is_available())


def get(create=True):
    """The process's communicator (created on first use -- a collective call: every rank reaches it at the same point,
    the DDP wrapper's construction), or None where the step uses torch.distributed."""
    if _STATE['comm'] is not None or not wanted():
        return _STATE['comm']
    if not create or _STATE['tried']:
        return None
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError('ssseg comm: communicator created during a stream capture (construct DDP before capturing)')
    _STATE['tried'] = True
    try:
        _STATE['comm'] = NativeComm()
    except RuntimeError as exc:   # RCCL not loadable: the same library is behind c10d, say so and use it
        _STATE['error'] = repr(exc)
        print(f'[ssseg comm] native communicator unavailable ({exc}); collectives go through torch.distributed',
              file=sys.stderr, flush=True)
    return _STATE['comm']


def kind():
    """'native' / 'c10d' / None (no process group): reported by bench.py."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    return 'native' if _STATE['comm'] is not None else 'c10d'


def reset():
    """Destroy the communicator (before destroy_process_group; tests)."""
    c = _STATE['comm']
    _STATE.update(comm=None, tried=False, error=None)
    if c is not None:
        torch.cuda.synchronize()
        c.destroy()


def all_reduce_sum(t):
    """SyncBN's per-channel sums (fp64) all-reduced on the current stream: native communicator, else torch.distributed."""
    c = get()
    if c is not None and t.is_cuda:
        c.all_reduce([t], 'sum')
    else:
        dist.all_reduce(t)
