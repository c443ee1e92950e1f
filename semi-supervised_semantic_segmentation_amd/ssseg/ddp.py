"""Data-parallel gradient averaging on RCCL (torch.distributed 'nccl' backend = RCCL over xGMI).

Replaces torch.nn.parallel.DistributedDataParallel (reference distributed_trainer.py:38).  The
gradients live in the model's flat arena (ssseg.arena), cut into contiguous buckets (~25 MB).  The
native layers call mark_ready(param) when a parameter's gradient is final; when every parameter of a
bucket is ready in the *armed* backward pass, the bucket's all-reduce(AVG) is launched on a side HIP
stream (ordered after the compute stream by an event), so communication overlaps the rest of the
backward.  finish() joins the side stream.

Reference semantics: DDP all-reduces after EACH of the two backward passes of a step (train.py:61,115).
Gradients accumulate between them and the all-reduce is linear, so reducing once — armed on the last
backward of the step — gives the same averaged gradient (up to fp summation order) with half the
traffic.  Documented in DESIGN.md; arm() on every backward restores the reference's pattern.
"""
import torch
import torch.distributed as dist
import torch.nn as nn

from . import arena as _arena


class DistributedDataParallel(nn.Module):
    def __init__(self, module, device_ids=None, find_unused_parameters=False, bucket_cap_mb=25, broadcast_buffers=True):
        super().__init__()
        self.module = module
        self.world = dist.get_world_size() if dist.is_initialized() else 1
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
                if self.world > 1:
                    p._ssseg_reducer = self
        self._armed = False
        self._pending = None
        self._launched = None
        self._works = []
        self._stream = torch.cuda.Stream() if (self.world > 1 and a.data.is_cuda) else None

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    # -- reducer protocol --------------------------------------------------------------------------
    def arm(self):
        """The next backward pass is the last one of this step: reduce buckets as they complete."""
        self._armed = self.world > 1
        self._pending = [len(ps) for (_, _, ps) in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._works = []

    def mark_ready(self, p):
        if not self._armed:
            return
        i = self._bucket_of.get(id(p))
        if i is None or self._launched[i]:
            return
        self._pending[i] -= 1
        if self._pending[i] <= 0:
            self._launch(i)

    def _launch(self, i):
        s, e, _ = self.buckets[i]
        view = self.arena.grad[s:e]
        self._launched[i] = True
        if self._stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            with torch.cuda.stream(self._stream):
                self._stream.wait_event(ev)
                self._works.append(dist.all_reduce(view, op=dist.ReduceOp.AVG, async_op=True))
        else:   # gloo / CPU: SUM then scale
            dist.all_reduce(view, op=dist.ReduceOp.SUM)
            view.div_(self.world)

    def finish(self):
        """Launch any bucket not yet reduced and make the current stream wait for all of them."""
        if not self._armed:
            return
        for i in range(len(self.buckets)):
            if not self._launched[i]:
                self._launch(i)
        for w in self._works:
            w.wait()
        if self._stream is not None:
            torch.cuda.current_stream().wait_stream(self._stream)
        self._armed = False
        self._works = []
