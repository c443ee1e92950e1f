"""One training step captured as a HIP graph and replayed (torch.cuda.CUDAGraph is hipGraph on ROCm).

A C2 step is ~1,000 kernel launches, a C4 (MultiscaleAttention over HRNet-W32) step ~10,000 mostly small ones: issued
from Python through ctypes, the host falls behind the device on the small-map layers and the GPU idles between
launches.  Captured once, a step replays as one graph launch.

Everything the step launches is capture-safe by construction: no call allocates outside the caching allocator or
synchronises (include/ssseg.h), the conv autotuner falls back to its cached / heuristic choice while a stream is
capturing (so run at least two eager steps first: the first tunes every geometry and registers the conv/BN
pairs, the second builds the teacher's BN fold table, a host-to-device copy that cannot be captured), and the CowMix draws read and advance a
device-side Philox counter (ssseg_cowmix_draw_dev), so every replay draws fresh masks -- the same sequence the eager
steps would.  Host-side values are baked in at capture: a replay repeats the captured step's Python decisions (the
optimizer step taken or skipped, the epoch gate of the consistency weight, the learning rate), so capture a step with
step != 0 and recapture when those change.  Collectives: a DDP step captures when its gradient buckets and SyncBN sums
go through the native RCCL communicator (ssseg.comm: an enqueue on the stream, recorded like a kernel); c10d's
collectives do not (its watchdog polls their Work events, which a capture refuses -- DESIGN.md §6), and gloo runs on the
host.

    step = StepGraph(lambda img, mask, ua, ub: train.train_step(model, teacher, opt, img, mask, ua, ub, epoch, 1, cfg),
                     img, mask, ua, ub)
    cls, unsup, cm = step(img2, mask2, ua2, ub2)    # copies the inputs into the captured buffers, replays
"""
import os

import torch


def _capture_mode():
    """'thread_local' while an RCCL process group is live: its watchdog thread polls the events of earlier collectives
    during the capture, which the default 'global' mode refuses (hipErrorStreamCaptureUnsupported in the watchdog)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == 'nccl':
        return 'thread_local'
    return 'global'


class StepGraph:
    def __init__(self, fn, *example_inputs, warmup=0):
        self.static_in = [t.detach().clone() for t in example_inputs]
        for _ in range(warmup):   # eager steps first (they tune every conv geometry); callers usually ran them
            fn(*self.static_in)
        torch.cuda.synchronize()
        from . import nn as snn
        # SSSEG_GRAPH_KEEP=1 keeps the captured hipGraph_t next to its executable instance (raw_cuda_graph(), read by
        # tools/graph_dag.py)
        keep = os.environ.get('SSSEG_GRAPH_KEEP', '0') == '1'
        self.graph = torch.cuda.CUDAGraph(keep_graph=keep)
        # the descriptor tables the captured launches read by pointer stay alive as long as the graph
        with snn.graph_refs() as refs:
            with torch.cuda.graph(self.graph, capture_error_mode=_capture_mode()):
                self.static_out = fn(*self.static_in)
        self.refs = list(refs)
        if keep:
            self.graph.instantiate()

    def __call__(self, *inputs):
        for dst, src in zip(self.static_in, inputs):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out
