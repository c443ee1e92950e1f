"""Data-parallel gradient averaging on RCCL (torch.distributed 'nccl' backend = RCCL over xGMI).

Replaces torch.nn.parallel.DistributedDataParallel (reference distributed_trainer.py:38).  The
gradients live in the model's flat arena (ssseg.arena), cut into contiguous buckets (~25 MB).  The
native layers call mark_ready(param) every time they have added a gradient contribution to a
parameter; when every contribution of every parameter of a bucket has landed in the *armed* backward
pass, the bucket's all-reduce is launched on a side HIP stream (ordered after the compute stream by an
event), so communication overlaps the rest of the backward.  finish() joins the side stream.

Contribution counting (static graph, like DDP's static_graph=True): a parameter can receive several
contributions in one backward (MultiscaleAttention runs its base model twice per forward,
multiscale_attention.py:38-58), so "ready" means "as many mark_ready calls as the parameter receives in
an armed backward".  The first armed backward learns those counts and launches every bucket in finish()
(no early launch); later armed backwards launch a bucket as soon as its counts are reached.  A
contribution arriving after its bucket was launched means the graph changed: that raises instead of
racing with the in-flight all-reduce.

Reduction op: AVG on RCCL; SUM + a native 1/world scale on the side stream for gloo (which has no AVG).

Transport: on an RCCL process group the buckets go through the process's native communicator (ssseg.comm,
libssseg ssseg_allreduce_buckets): an RCCL enqueue on the side stream with no completion object, so a step with live
collectives captures into a HIP graph.  torch.distributed's own all_reduce (async Work objects, waited in finish()) is the
path of gloo groups and of SSSEG_COMM=c10d.

Reference semantics: DDP all-reduces after EACH of the two backward passes of a step (train.py:61,115).
Gradients accumulate between them and the all-reduce is linear, so reducing once — armed on the last
backward of the step — gives the same averaged gradient (up to fp summation order) with half the
traffic.  Documented in DESIGN.md; arm() on every backward restores the reference's pattern.
"""
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from . import arena as _arena
from . import comm as _comm

_FORCE = {'on': False}


def force_collectives(on):
    """TEST ONLY: run the reducer's bucketed all-reduces and SyncBN's statistic all-reduces even at world size 1, so a
    one-GPU box executes the RCCL code path (ReduceOp.AVG, the side-stream launch and its event join, the fp64
    SyncBN sums) whose results must then equal the non-distributed step bit for bit."""
    _FORCE['on'] = bool(on)


def forced():
    return _FORCE['on'] and dist.is_available() and dist.is_initialized()


class DistributedDataParallel(nn.Module):
    def __init__(self, module, device_ids=None, find_unused_parameters=False, bucket_cap_mb=25, broadcast_buffers=True):
        super().__init__()
        self.module = module
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self._active = self.world > 1 or forced()   # reduce at all (world 1 only under force_collectives)
        self.arena = _arena.attach(module)
        a = self.arena
        if self.world > 1:
            dist.broadcast(a.data, 0)
            for b in module.buffers():
                dist.broadcast(b, 0)
        cap = max(1, int(bucket_cap_mb * (1 << 20) // 4))
        self.buckets = []             # (start, end, [params])
        cur, start = [], 0
        for p, o in zip(a.params, a.offsets):
            end = o + p.numel()
            cur.append(p)
            if end - start >= cap:
                self.buckets.append((start, (end + 3) // 4 * 4, cur))
                cur, start = [], (end + 3) // 4 * 4
        if cur:
            self.buckets.append((start, a.numel, cur))
        self._bucket_of = {}
        for i, (_, _, ps) in enumerate(self.buckets):
            for p in ps:
                self._bucket_of[id(p)] = i
                if self._active:
                    p._ssseg_reducer = self
        self._avg = self._active and dist.get_backend() == 'nccl'
        self._expected = None         # per-param contributions of an armed backward (learned on the first)
        self._learning = True
        self._overlap = os.environ.get('SSSEG_DDP_OVERLAP', '1') != '0'   # 0: every bucket in finish() (A/B)
        self._armed = False
        self.last_early = 0
        self._launched = None
        self._works = []
        self._stream = torch.cuda.Stream() if (self._active and a.data.is_cuda) else None
        # the native communicator (created here, on every rank at the same point: a collective call)
        self._comm = _comm.get() if (self._active and a.data.is_cuda) else None
        if self.world > 1:   # rank 0 tunes the conv geometries, the others take its table (ssseg.tune.sync)
            from . import tune
            tune.follow_rank0()

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    # -- reducer protocol --------------------------------------------------------------------------
    def arm(self):
        """The next backward pass is the last one of this step: reduce buckets as they complete."""
        self._armed = self._active
        self._launched = [False] * len(self.buckets)
        self._works = []
        self._seen = {}
        self.last_early = 0          # buckets launched from inside the backward in the current armed pass
        if self._expected is not None:
            self._pending = [sum(self._expected.get(id(p), 0) for p in ps) for (_, _, ps) in self.buckets]

    def mark_ready(self, p):
        """One gradient contribution to `p` has been written (by a kernel on the current stream)."""
        if not self._armed:
            return
        i = self._bucket_of.get(id(p))
        if i is None:
            return
        k = id(p)
        self._seen[k] = self._seen.get(k, 0) + 1
        if self._learning or not self._overlap:
            return
        if self._launched[i]:
            raise RuntimeError('ssseg DDP: a gradient contribution arrived after its bucket was all-reduced '
                               '(the backward graph changed between steps; static graph required)')
        exp = self._expected.get(k, 0)
        if self._seen[k] > exp:
            raise RuntimeError('ssseg DDP: more gradient contributions than in the first armed backward '
                               '(static graph required)')
        self._pending[i] -= 1
        if self._pending[i] == 0:
            self.last_early += 1
            self._launch(i)

    def _launch(self, i):
        s, e, _ = self.buckets[i]
        view = self.arena.grad[s:e]
        self._launched[i] = True
        op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        if self._stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            with torch.cuda.stream(self._stream):
                self._stream.wait_event(ev)
                if self._comm is not None:   # RCCL enqueue on the side stream, nothing to wait on but the stream
                    self._comm.all_reduce([view], 'avg', stream=self._stream)
                else:
                    self._works.append((view, dist.all_reduce(view, op=op, async_op=True)))
        else:   # CPU tensors (gloo): synchronous
            dist.all_reduce(view, op=op)
            if not self._avg:
                view.div_(self.world)

    def finish(self):
        """Launch any bucket not yet reduced and make the current stream wait for all of them."""
        if not self._armed:
            return
        for i in range(len(self.buckets)):
            if not self._launched[i]:
                self._launch(i)
        if self._stream is not None:
            from . import native as N
            with torch.cuda.stream(self._stream):
                for view, w in self._works:
                    w.wait()
                    if not self._avg:
                        N.call('ssseg_scale_f32', N.dev_ptr(view), view.numel(), 1.0 / self.world, N.stream())
            torch.cuda.current_stream().wait_stream(self._stream)
        else:
            for _, w in self._works:
                w.wait()
        if self._learning:
            self._expected = dict(self._seen)
            self._learning = False
        self._armed = False
        self._works = []
