"""MI355X-native layers: drop-in subclasses of torch.nn's Conv2d / ConvTranspose2d / BatchNorm2d /
MaxPool2d whose forward and backward run libssseg.so kernels.

Activation convention inside a network: a 4-D tensor [N, Cp, H, W] in channels_last memory format
(physically NHWC), Cp = channels rounded up to the MFMA vector (8 for bf16, 4 for fp32), padded
channels zero.  Parameter names, shapes and layouts are PyTorch's, so reference state_dicts load.

Gradients of parameters are accumulated by the kernels directly into `param.grad` (the flat
gradient arena when one is attached, ssseg.arena) and the autograd Functions return None for them;
a registered reducer (ssseg.ddp) is told when each parameter's gradient is complete so the RCCL
all-reduce of its bucket can start during the rest of the backward pass.
"""
import contextlib
import ctypes
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from . import comm as _comm
from . import native as N

_CFG = {'act_mask': os.environ.get('SSSEG_ACT_MASK', '1') != '0',
        'grad_join': True, 'stem': os.environ.get('SSSEG_STEM', '1') != '0', 'phases': True, 'eval_bwd_y': True, 'dtype': torch.bfloat16, 'sync_bn': True,
        'fuse_stats': True, 'vcat': os.environ.get('SSSEG_VCAT', '1') != '0',
        'vpad': os.environ.get('SSSEG_VPAD', '1') != '0',
        'bn_gstat': os.environ.get('SSSEG_BN_GSTAT', '1') != '0'}


def set_bn_grad_stats(on):
    """A training BN(+ReLU) whose output feeds exactly one conv (conv_bn_act(..., single_use=True)): that conv's
    input-gradient launch applies the ReLU backward and writes the BN backward's two channel sums in its epilogue
    (ssseg_conv_igemm_epi_actmask with stats), so the BN backward skips its reduction pass over dy and x (default
    on)."""
    _CFG['bn_gstat'] = bool(on)


def set_virtual_concat(on):
    """cat_crop(lazy=True) returns a virtual concat the consuming conv reads part by part (default on); off: the
    concat is materialised by two copies."""
    _CFG['vcat'] = bool(on)


def set_eval_bwd_from_y(on):
    """Differentiated eval pass: recover the BN x_hat from y on layers without a residual (default on) instead of
    keeping the raw accumulator copy."""
    _CFG['eval_bwd_y'] = bool(on)


def set_phase_launch(on):
    """One launch over a transposed conv's output phases (ssseg_conv_igemm_phases; default on)."""
    _CFG['phases'] = bool(on)


def set_stem_kernel(on):
    """Route image-input convs to ssseg_conv_stem_epi (default on); off: the generic engine."""
    _CFG['stem'] = bool(on)


def set_grad_join(on):
    """Fuse the input gradients of mark_join'ed activations into their consumers' kernels (default on); off:
    autograd sums them (the separate add)."""
    _CFG['grad_join'] = bool(on)


def set_compute_dtype(dtype):
    assert dtype in (torch.bfloat16, torch.float16, torch.float32)
    _CFG['dtype'] = dtype


def compute_dtype():
    return _CFG['dtype']


def set_sync_bn(flag):
    _CFG['sync_bn'] = bool(flag)


_WGRAD = {'merge': os.environ.get('SSSEG_WGRAD_MERGE', '1') != '0', 'defer': False, 'pending': []}


def set_wgrad_merge(on):
    """Merge a conv's deferred weight gradient with its next one into a single launch (default on; see
    defer_wgrad).  Off: defer_wgrad is a no-op and every backward launches its own weight gradients."""
    _WGRAD['merge'] = bool(on)


@contextlib.contextmanager
def defer_wgrad():
    """Inside: conv weight gradients are not launched; each conv keeps its (input, output-gradient) pair until
    its NEXT weight gradient, which then runs as ONE launch over both pixel sets (ssseg_conv_wgrad2).  The
    training step wraps the supervised backward (reference train.py:61) in this: the consistency backward
    (train.py:115) accumulates into the same .grad before clip + SGD, so dW_sup + dW_cons is one contraction
    over the union of the two batches' pixels -- one split plan, half the launches and half the fp32 slab
    traffic per flop on the small-map layers.  Whatever is still pending when the step needs its gradients is
    launched by flush_wgrad()."""
    if not _WGRAD['merge']:
        yield
        return
    prev = _WGRAD['defer']
    _WGRAD['defer'] = True
    try:
        yield
    finally:
        _WGRAD['defer'] = prev


def flush_wgrad():
    """Launch every deferred weight gradient on its own (convs that ran no second backward)."""
    pending, _WGRAD['pending'] = _WGRAD['pending'], []
    for mod in pending:
        pair = mod.__dict__.pop('_ssseg_wg_pending', None)
        if pair is not None:
            mod._ssseg_wgrad(*pair, bias_grad=False, want=(True, False))


# ---- deferred split reductions of the weight gradients (ssseg_wgrad_defer_reduce / _flush) ---------------------------
# opt-in (SSSEG_WGRAD_BATCH_REDUCE=1): measured neutral on the C2 step -- 519.2 / 520.1 img/s on vs 520.4 / 522.9 off,
# A/B of two pairs in one call
_WRED = {'on': os.environ.get('SSSEG_WGRAD_BATCH_REDUCE', '0') == '1', 'live': False, 'keep': []}


def _wgrad_ws(nb, device):
    """The split-slab workspace of one weight-gradient launch; inside batched_wgrad_reduce() it is kept alive until the
    deferred reductions that read it have been launched."""
    ws = N.workspace(nb, device)
    if _WRED['live']:
        _WRED['keep'].append(ws)
    return ws


@contextlib.contextmanager
def batched_wgrad_reduce():
    """Inside: the weight-gradient launches record their split-slab reductions instead of launching them; on exit ONE
    flush launches all of them (up to 40 per launch) on the current stream -- the same per-element sums, so the same dW
    bit for bit.  Wraps the block of weight gradients train.train_step issues after its backward passes join (66
    reduction launches per C2 step otherwise).  Nothing inside may read a .grad those launches write."""
    if not _WRED['on'] or _WRED['live'] or _WSTREAM['on'] or not torch.cuda.is_available():
        yield
        return
    _WRED['live'] = True
    N.call('ssseg_wgrad_defer_reduce', 1)
    try:
        yield
    finally:
        N.call('ssseg_wgrad_defer_reduce', 0)
        _WRED['live'] = False
        try:
            N.call('ssseg_wgrad_reduce_flush', N.stream())
        finally:
            keep, _WRED['keep'] = _WRED['keep'], []
            del keep   # (stream-ordered frees: after the flush launch that reads them)


# ---- held weight-gradient calls: two backward passes issued on two streams, their gradient writes replayed after ------
_HOLD = {'on': False, 'tag': None, 'calls': [], 'params': False, 'adds': [], 'streams': {},
         # streams the replayed (merged) weight-gradient launches are spread over (SSSEG_WGRAD_BURST; 1 = this stream)
         'burst': max(1, int(os.environ.get('SSSEG_WGRAD_BURST', '1')))}


@contextlib.contextmanager
def hold_wgrad(tag, params=False):
    """Inside: every conv's weight (and bias) gradient call is recorded with its operands instead of launched.  The
    training step issues the consistency backward on the side stream and the supervised backward on the main stream
    under this, so the two run concurrently without touching the shared gradient arena; replay_held() then issues
    the recorded calls on the caller's stream exactly as the serial schedule would (the first pass deferred, the
    second merged with it, one launch per conv over both pixel sets).  params=True (the pass on the side stream): the
    other parameter gradients its backward adds (a standalone BatchNorm's weight / bias) go to zeroed temporaries,
    added into .grad by replay_held after the other pass's own writes -- the serial order, the same fp32 sums."""
    prev = _HOLD['on'], _HOLD['tag'], _HOLD['params']
    _HOLD['on'], _HOLD['tag'], _HOLD['params'] = True, tag, params
    try:
        yield
    finally:
        _HOLD['on'], _HOLD['tag'], _HOLD['params'] = prev


def _grad_ptrs(*params):
    """device pointers a backward kernel ADDS parameter gradients into: the params' .grad, or inside
    hold_wgrad(params=True) zeroed temporaries that replay_held adds into .grad (None for an absent parameter)."""
    if not (_HOLD['on'] and _HOLD['params']):
        return tuple(N.dev_ptr(_grad_of(p)) if p is not None else None for p in params)
    out = []
    for p in params:
        if p is None:
            out.append(None)
            continue
        tmp = torch.zeros_like(_grad_of(p))
        _HOLD['adds'].append((p, tmp))
        out.append(N.dev_ptr(tmp))
    return tuple(out)


def clear_held():
    """Drop held calls left by a backward that raised (their gradients are void with it)."""
    _HOLD['calls'] = []
    _HOLD['adds'] = []


def _held(mod, x, gy, bias_grad, want):
    if not _HOLD['on']:
        return False
    _HOLD['calls'].append((_HOLD['tag'], mod, (x, gy), {'bias_grad': bias_grad, 'want': want}))
    return True


def replay_held(order):
    """Issue the held calls: those of pass order[0] inside defer_wgrad(), then those of order[1] (each merges with its
    conv's deferred one), then flush_wgrad() -- the launches and the summation order of the serial schedule."""
    calls, _HOLD['calls'] = _HOLD['calls'], []
    adds, _HOLD['adds'] = _HOLD['adds'], []
    # the held operands and temporaries were allocated on the side stream; they are consumed here on this stream:
    # record it, so the allocator does not hand their blocks to later side-stream work while these launches read them
    cur = torch.cuda.current_stream()
    for _, tmp in adds:
        tmp.record_stream(cur)
    for _, _, args, kw in calls:
        for t in list(args) + list(kw.values()):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(cur)
    for p, tmp in adds:   # grad += tmp (tmp = the one fp32 term the kernel would have added): bitwise the same sum
        g = _grad_of(p)
        N.call('ssseg_axpby', N.dev_ptr(g), 1.0, N.dev_ptr(tmp), 1.0, N.dev_ptr(g), g.numel(), N.stream())
    nburst = _HOLD['burst'] if not _WRED['on'] else 1
    streams = [cur]
    if nburst > 1:   # the merged launches are independent (one .grad each): spread them round-robin over streams
        pool = _HOLD['streams'].setdefault(cur.device, [])
        while len(pool) < nburst - 1:
            pool.append(torch.cuda.Stream(device=cur.device))
        for sd in pool[:nburst - 1]:
            sd.wait_stream(cur)
            streams.append(sd)
    first = {}
    with batched_wgrad_reduce():
        with defer_wgrad():
            for tag, mod, args, kw in calls:
                if tag == order[0]:
                    first[id(mod)] = args
                    mod._ssseg_wgrad(*args, **kw)
        k = 0
        for tag, mod, args, kw in calls:
            if tag == order[1]:
                sd = streams[k % len(streams)]
                k += 1
                if sd is not cur:
                    for t in list(args) + list(first.get(id(mod), ())):
                        if isinstance(t, torch.Tensor) and t.is_cuda:
                            t.record_stream(sd)
                            vc = _vcat_of(t)
                            if vc is not None:
                                vc.a.record_stream(sd)
                                vc.b.record_stream(sd)
                with torch.cuda.stream(sd):
                    mod._ssseg_wgrad(*args, **kw)
        flush_wgrad()
    for sd in streams[1:]:
        cur.wait_stream(sd)


# ---- deferred BN parameter gradients of the differentiated eval pass ---------------------------------------------------
_PGRAD = {'on': os.environ.get('SSSEG_DEFER_BN_PGRAD', '1') != '0', 'live': False, 'pending': [], 'table': None}


@contextlib.contextmanager
def defer_param_grads():
    """Inside: the differentiated eval BatchNorms (the student's consistency pass, train.py:90-92) leave their
    parameter-gradient partial rows in per-layer buffers instead of reducing them right away; on exit ONE launch
    (ssseg_bn_param_grad_batch) turns all of them into the BN weight / bias (and conv bias) gradients.  Those gradients
    are read only by the optimizer step, so the ~60 small reduction launches per step (one per BN layer, ~4-5 us each,
    a launch floor) become one.  Layers whose parameters a DDP reducer watches (world > 1: their gradient marks a bucket
    ready) are reduced at once as before."""
    if not _PGRAD['on'] or _PGRAD['live'] or not torch.cuda.is_available():
        yield
        return
    _PGRAD['live'] = True
    try:
        yield
    finally:
        _PGRAD['live'] = False
        flush_param_grads()


# device tensors a launch reads through a raw pointer baked into a kernel argument (descriptor tables): while a HIP graph
# is captured (ssseg.graph.StepGraph) each one used is recorded here and the graph keeps it alive, so a later table
# replacing it (new rows) cannot free memory a cached graph still reads
_GRAPH_REFS = {'live': None}


def _graph_ref(t):
    if _GRAPH_REFS['live'] is not None and torch.cuda.is_current_stream_capturing():
        _GRAPH_REFS['live'].append(t)
    return t


@contextlib.contextmanager
def graph_refs():
    """Collect the descriptor tables the launches captured inside the block read (yields the list)."""
    prev, _GRAPH_REFS['live'] = _GRAPH_REFS['live'], []
    try:
        yield _GRAPH_REFS['live']
    finally:
        _GRAPH_REFS['live'] = prev


def flush_param_grads():
    import struct
    pend, _PGRAD['pending'] = _PGRAD['pending'], []
    if not pend:
        return
    # (gradient-statistics rows of a consumer's input-gradient launch carry their x_hat transform: shift, mean_eff,
    # invstd; ssseg_pgrad_desc)
    rows = tuple((e['part'].data_ptr(), e['nparts'], e['C'], e['scale'].data_ptr(), e['dg'], e['db'], e['dbias'])
                 + (e.get('gs') or (0, 0, 0)) for e in pend)
    ent = _PGRAD['table']
    if ent is None or ent[0] != rows:
        if torch.cuda.is_current_stream_capturing():
            # (a new descriptor table needs a host-to-device copy): reduce each layer on its own
            for e in pend:
                sums = torch.empty(2 * e['C'], dtype=torch.float64, device=e['part'].device)
                if e.get('gs'):
                    N.call('ssseg_bn_gstat_finalize', N.dev_ptr(e['part']), e['nparts'], e['C'], N.dev_ptr(sums),
                           N.dev_ptr(e['scale']), *e['gs'], e['dg'] or None, e['db'] or None, e['dbias'] or None,
                           N.stream())
                    continue
                N.call('ssseg_bn_partials_finalize', N.dev_ptr(e['part']), e['nparts'], e['C'], N.dev_ptr(sums), 0.0,
                       0.0, 0.0, None, None, None, None, None, N.stream())
                N.call('ssseg_bn_eval_param_grad', N.dev_ptr(sums), e['C'], N.dev_ptr(e['scale']), e['dg'] or None,
                       e['db'] or None, e['dbias'] or None, N.stream())
            return
        blob = b''.join(struct.pack('<10q', *r) for r in rows)
        ent = (rows, torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(pend[0]['part'].device))
        _PGRAD['table'] = ent
    N.call('ssseg_bn_param_grad_batch', N.dev_ptr(_graph_ref(ent[1])), len(rows), max(e['C'] for e in pend),
           N.stream())


def wgrad_pending():
    return sum(1 for m in _WGRAD['pending'] if '_ssseg_wg_pending' in m.__dict__)


_WSTREAM = {'on': os.environ.get('SSSEG_WGRAD_STREAM', '0') == '1', 'live': False, 'streams': {}, 'used': False}


@contextlib.contextmanager
def wgrad_side_stream():
    """Inside: every conv weight-gradient launch runs on a second HIP stream (ordered after everything issued so far
    on the compute stream, its operands kept alive for it by record_stream), so the weight gradients -- needed only by
    the optimizer step and the DDP buckets -- fill the compute units the input-gradient chain of the backward leaves
    idle.  On exit the compute stream waits for the side stream.  The training step wraps its last backward in this
    (train.train_step); outside it every launch stays on the compute stream.  Off unless SSSEG_WGRAD_STREAM=1: on the
    C2 step it measured 440.8 vs 443.9 img/s (A/B in one call; the teacher-pass overlap alone: 452.9)."""
    if not _WSTREAM['on'] or _WSTREAM['live'] or not torch.cuda.is_available():
        yield
        return
    _WSTREAM['live'] = True
    try:
        yield
    finally:
        _WSTREAM['live'] = False
        join_wgrad_stream()


def join_wgrad_stream():
    if _WSTREAM['used']:
        _WSTREAM['used'] = False
        torch.cuda.current_stream().wait_stream(_WSTREAM['streams'][torch.cuda.current_device()])


@contextlib.contextmanager
def _on_wgrad_stream(*tensors):
    """the launches inside go to the weight-gradient stream when wgrad_side_stream() is live"""
    if not _WSTREAM['live']:
        yield
        return
    dev = torch.cuda.current_device()
    s = _WSTREAM['streams'].get(dev)
    if s is None:
        s = _WSTREAM['streams'][dev] = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            t.record_stream(s)
            vc = _vcat_of(t)
            if vc is not None:
                vc.a.record_stream(s)
                vc.b.record_stream(s)
    _WSTREAM['used'] = True
    with torch.cuda.stream(s):
        yield


def set_fused_bn_stats(flag):
    """Training BatchNorm statistics from the producing conv's epilogue (default) or a separate pass."""
    _CFG['fuse_stats'] = bool(flag)


def vec(dtype=None):
    return 4 if (dtype or _CFG['dtype']) == torch.float32 else 8


def rup(c, v):
    return (c + v - 1) // v * v


def set_virtual_pad(on):
    """Virtual channel padding of the 16-bit conv engine's contraction (default on; SSSEG_VPAD=0 turns it off)."""
    _CFG['vpad'] = bool(on)


def vpad(c):
    """Contraction width the 16-bit conv engine runs for an input of c physical channels (c % 8 == 0).  A width that
    is not a multiple of 64 runs the general-k loader (per-lane tap / channel split of every 16-byte chunk); within
    12.5 % of the next multiple of 64 (HRNet-W32's 480- and 240-channel fuse / head layers) the GEMM instead runs the
    64-aligned path over rup(c, 64) "virtual" channels: the packed weights are zero for channels >= c and the
    activation keeps its physical pixel stride c, so a 16-byte chunk past channel c reads the next pixel's first
    channels (finite data times zero weights; past the end of the buffer the bounded LDS-DMA reads return 0).
    The engine then refuses its register-staged kernels (plain loads) for such a launch.  Measured (tools/conv_ab.py,
    16x256^2): 480->240 3x3 fwd 3.13 -> 2.2 ms, fwd+bwd 12.1 -> 6.7-8.3 ms.
    Caveat: a neighbouring pixel holding Inf/NaN couples in as 0 * Inf = NaN (IEEE), where the unpadded contraction
    would keep the other outputs finite.  The reference has no such coupling, but in every path that uses vpad an Inf
    activation already makes the step's loss non-finite (and the fp16 loss scaler skips the step), so no finite
    result changes; set_virtual_pad(False) gives the strictly per-pixel contraction."""
    if not _CFG['vpad'] or _CFG['dtype'] == torch.float32 or c % 64 == 0:
        return c
    p = rup(c, 64)
    return p if (p - c) * 8 <= c else c


def _zero_(t):
    N.call('ssseg_zero', N.dev_ptr(t), t.numel() * t.element_size(), N.stream())
    return t


def new_act(n, c, h, w, dtype, device, zero=False):
    t = torch.empty((n, c, h, w), dtype=dtype, device=device, memory_format=torch.channels_last)
    return _zero_(t) if zero else t


def _is_act(x, c_phys=None):
    return (x.is_cuda and x.dim() == 4 and (c_phys is None or x.shape[1] == c_phys)
            and x.dtype == _CFG['dtype'] and x.is_contiguous(memory_format=torch.channels_last))


def _need_act(x, c_phys, what):
    if not _is_act(x, c_phys):
        raise RuntimeError(f'ssseg: {what} expects a {_CFG["dtype"]} channels_last HIP activation with {c_phys} '
                           f'channels, got {tuple(x.shape)} {x.dtype} {x.device} strides {x.stride()}')


# ------------------------------------------------------------------------------------------------
# live kernel instrumentation (bench.py roofline): HIP events around every conv-engine launch
# ------------------------------------------------------------------------------------------------
_PROBE = {'on': False, 'rows': [], 'fenced': os.environ.get('SSSEG_PROBE_FENCED', '0') == '1'}


class ProbeEvent:
    """A HIP timing event without the system-scope fence (ssseg_probe_event_*, csrc/probe.hip): recording it leaves
    the caches as the previous kernel left them, so the bracketed conv runs as warm as in the captured step.  Same
    record() / elapsed_time() surface as torch.cuda.Event; recorded on torch's current stream."""
    __slots__ = ('ev',)

    def __init__(self):
        h = ctypes.c_void_p()
        N.call('ssseg_probe_event_create', ctypes.byref(h))
        self.ev = h.value

    def record(self):
        N.call('ssseg_probe_event_record', self.ev, N.stream())

    def elapsed_time(self, end):
        ms = ctypes.c_float()
        N.call('ssseg_probe_event_elapsed', self.ev, end.ev, ctypes.byref(ms))
        return ms.value

    def __del__(self):
        if self.ev and N._lib is not None:
            N._lib.ssseg_probe_event_destroy(self.ev)
            self.ev = None


def _probe_event():
    # SSSEG_PROBE_FENCED=1: torch's default events (system-scope release after every record: cold L2 per conv)
    return torch.cuda.Event(enable_timing=True) if _PROBE['fenced'] else ProbeEvent()


def probe(enable):
    """Start/stop recording (start_event, end_event, algorithmic_flops, kind) per conv-engine call."""
    _PROBE['on'] = bool(enable)
    if enable:
        _PROBE['rows'] = []
    return _PROBE['rows']


class _Timed:
    def __init__(self, flops, kind, tag=''):
        self.flops, self.kind, self.tag = flops, kind, tag

    def __enter__(self):
        if _PROBE['on']:
            self.e0 = _probe_event()
            self.e0.record()
        return self

    def __exit__(self, *a):
        if _PROBE['on']:
            e1 = _probe_event()
            e1.record()
            _PROBE['rows'].append((self.e0, e1, self.flops, self.kind, self.tag))


def _conv_flops(n, oh, ow, cout, cin, r, s):
    return 2.0 * n * oh * ow * cout * cin * r * s


def _tag(mod, n, h, w):
    return f'{type(mod).__name__} {mod.in_channels}->{mod.out_channels} k{mod.kernel_size[0]} s{mod.stride[0]} @{n}x{h}x{w}'


# ------------------------------------------------------------------------------------------------
# parameter gradient plumbing
# ------------------------------------------------------------------------------------------------
def _grad_of(p):
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


def _ready(*params):
    for p in params:
        r = getattr(p, '_ssseg_reducer', None)
        if r is not None:
            r.mark_ready(p)


# ------------------------------------------------------------------------------------------------
# model input / output boundary
# ------------------------------------------------------------------------------------------------
class _ToAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        n, c, h, w = x.shape
        cp = rup(c, vec())
        y = new_act(n, cp, h, w, _CFG['dtype'], x.device)
        xc = x if x.is_contiguous() else x.contiguous()
        N.call('ssseg_nchw_to_nhwc', N.dev_ptr(xc, 'image'), N.dev_ptr(y), n, c, h, w, cp, N.dt_code(xc),
               N.dt_code(y), N.stream())
        ctx.meta = (n, c, h, w, cp, x.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        n, c, h, w, cp, dt = ctx.meta
        gx = torch.empty((n, c, h, w), dtype=dt, device=gy.device)
        N.call('ssseg_nhwc_to_nchw', N.dev_ptr(gy), N.dev_ptr(gx), n, c, h, w, cp, N.dt_code(gy), N.dt_code(gx),
               N.stream())
        return gx


def to_act(x):
    """NCHW image batch (any float dtype the kernels take) -> compute-dtype NHWC activation."""
    if _is_act(x) and x.shape[1] % vec() == 0:
        return x
    return _ToAct.apply(x)


def to_act_cat(xs):
    """Several NCHW image batches -> ONE compute-dtype NHWC activation batch, each converted straight into its
    slice (no concat pass): an eval-mode model's passes over several batches become one forward (no autograd)."""
    n = sum(int(x.shape[0]) for x in xs)
    _, c, h, w = xs[0].shape
    cp = rup(c, vec())
    y = new_act(n, cp, h, w, _CFG['dtype'], xs[0].device)
    off = 0
    for x in xs:
        if tuple(x.shape[1:]) != (c, h, w):
            raise ValueError('to_act_cat: batches of different image shapes')
        xc = x if x.is_contiguous() else x.contiguous()
        N.call('ssseg_nchw_to_nhwc', N.dev_ptr(xc, 'image'), N.dev_ptr(y) + off * cp * h * w * y.element_size(),
               int(x.shape[0]), c, h, w, cp, N.dt_code(xc), N.dt_code(y), N.stream())
        off += int(x.shape[0])
    return y


# ------------------------------------------------------------------------------------------------
# convolution
# ------------------------------------------------------------------------------------------------
def _desc(**kw):
    d = N.ConvDesc()
    for k, v in kw.items():
        setattr(d, k, int(v))
    return d


def _phases(stride, pad, R, in_full, dil=1):
    """Output-phase decomposition of a strided transposed contraction (conv dgrad / ConvTranspose2d
    forward): map X (size in_full) gathers from map Y with x[s*q + phi] = sum_j y[q - j + delta] w[r0 + s*j].
    Returns [(phi, r0, Rn, delta, Q)]."""
    assert dil == 1, 'strided transposed contraction with dilation is not supported'
    out = []
    for phi in range(stride):
        r0 = (phi + pad) % stride
        rn = 0 if r0 >= R else (R - r0 + stride - 1) // stride
        delta = (phi + pad - r0) // stride
        q = (in_full - phi + stride - 1) // stride
        out.append((phi, r0, rn, delta, max(q, 0)))
    return out


ACT_NONE, ACT_RELU, ACT_RELU6, ACT_LEAKY = 0, 1, 2, 3


def _act(a):
    """Activation spec -> (SSSEG_ACT_* code, slope).  Accepts False/None (none), True (ReLU), a code
    (ACT_RELU6, ...) or ('leaky', slope)."""
    if a is None or a is False:
        return ACT_NONE, 0.0
    if a is True:
        return ACT_RELU, 0.0
    if isinstance(a, tuple):
        if a[0] != 'leaky':
            raise ValueError(f'unknown activation {a!r}')
        return ACT_LEAKY, float(a[1])
    code = int(a)
    if code not in (ACT_NONE, ACT_RELU, ACT_RELU6):
        raise ValueError(f'unknown activation {a!r}')
    return code, 0.0


class GradHandoff:
    """Hands the identity shortcut's gradient of a residual block to the dgrad of the block's first conv,
    which reads the same input x (Bottleneck, resnet.py): the residual-consuming BN backward (which runs
    first, it is downstream) parks dres here and returns None for it, and the conv adds it in its dgrad
    epilogue (y = acc + residual) -- dx = dgrad(conv1) + d(shortcut) in one kernel instead of autograd's
    separate accumulation add."""
    __slots__ = ('grad',)

    def __init__(self):
        self.grad = None

    def put(self, g):
        if self.grad is not None:
            raise RuntimeError('GradHandoff: gradient already pending')
        self.grad = g

    def take(self):
        g, self.grad = self.grad, None
        return g


def _take(handoff):
    return handoff.take() if handoff is not None else None


class GradJoin:
    """One activation read by several native ops whose backwards all run: a UNet skip (the decoder concat and
    the next encoder stage, unet.py:36-45), the input of a ResNet block with a projection shortcut (conv1 and
    the downsample conv).  Autograd would sum the consumers' input gradients with one separate add per extra
    consumer; instead every consumer's backward but the last parks its partial sum here and returns None, and
    the next one adds the parked gradient inside its own output kernel (the dgrad epilogue's residual, the
    max-pool backward's residual) -- whatever order autograd runs them in.  Opt-in per tensor (mark_join):
    only where the model guarantees every registered consumer contributes to the loss."""
    __slots__ = ('uses', 'left', 'pending')

    def __init__(self):
        self.uses, self.left, self.pending = 0, None, None


def mark_join(x):
    """Route the input gradients of x's native consumers through one GradJoin (call before the consumers)."""
    if torch.is_grad_enabled() and isinstance(x, torch.Tensor) and x.requires_grad and _CFG['grad_join']:
        if x.__dict__.get('_ssseg_join') is None:
            x._ssseg_join = GradJoin()
    return x


def _join_fwd(x):
    """forward of a consumer (outside Function.apply, where grad mode is live): one more use of x's join"""
    j = x.__dict__.get('_ssseg_join') if isinstance(x, torch.Tensor) else None
    if j is None or not torch.is_grad_enabled():
        return None
    j.uses += 1
    return j


def _join_take(j):
    """backward of a consumer: (parked gradient to add or None, whether this consumer is the last)"""
    if j is None:
        return None, True
    if j.left is None:
        j.left = j.uses
    j.left -= 1
    p, j.pending = j.pending, None
    last = j.left <= 0
    if last:
        j.left = None
    return p, last


def _join_give(j, last, g):
    if j is None or last:
        return g
    j.pending = g
    return None


def _sum_pending(a, b):
    """two pending input gradients (a GradHandoff's and a GradJoin's) for one fused residual: rare"""
    if a is None:
        return b
    if b is None:
        return a
    return a + b


class StatRows:
    """fp64 BatchNorm statistics partials written by a conv's epilogue (ssseg_conv_epilogue.stats): rows of
    (sum y, sum y^2) per output tile, appended launch by launch (a ConvTranspose2d writes one run per output
    phase).  The training BatchNorm that consumes y reduces them (ssseg_bn_partials_finalize) instead of
    reading y again."""
    __slots__ = ('part', 'C', 'rows', 'cap', '_out')

    def __init__(self, C, max_rows, device, part=None):
        import ctypes
        self.C, self.cap, self.rows = int(C), int(max_rows), 0
        need = 2 * self.cap * self.C
        ok = part is not None and part.numel() >= need and part.device == torch.device(device)
        self.part = part if ok else torch.empty(need, dtype=torch.float64, device=device)
        self._out = ctypes.c_int64(0)

    def launch_fields(self):
        """(stats pointer for the next launch, ld, host pointer receiving its row count)"""
        import ctypes
        if self.rows >= self.cap:
            raise RuntimeError('ssseg: BN statistics partial table full')
        return N.dev_ptr(self.part) + 2 * self.rows * self.C * 8, self.C, ctypes.addressof(self._out)

    def commit(self):
        self.rows += int(self._out.value)
        if self.rows > self.cap:
            raise RuntimeError('ssseg: BN statistics partial table overflow')


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, mod, relu, handoff=None, stats=None, join=None):
        y = mod._ssseg_forward(x, relu, stats=stats)
        ctx.mod, ctx.relu, ctx.handoff, ctx.join, ctx.vcat = mod, relu, handoff, join, _vcat_of(x)
        ctx.xmask = x.__dict__.get('_ssseg_act_out')   # x = a single-use activation output: mask in our dgrad
        ctx.xgstat = x.__dict__.get('_ssseg_gstat')   # ... of a training BN: its backward sums in our dgrad too
        ctx.save_for_backward(x, y if _act(relu)[0] else None)
        if _act(relu)[0] == ACT_RELU:
            # a ReLU output: a consumer's input-gradient launch may apply this ReLU's backward in place (the
            # gradient then carries _ssseg_premasked and backward() skips ssseg_act_bwd)
            y.__dict__['_ssseg_relu_out'] = True
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y = ctx.saved_tensors
        _vcat_restore(x, ctx.vcat)
        mod = ctx.mod
        gy = mod._grad_in(gy)
        code, slope = _act(ctx.relu)
        if code and not gy.__dict__.get('_ssseg_premasked', False):
            gm = torch.empty_like(gy)
            N.call('ssseg_act_bwd', N.dev_ptr(gy), N.dev_ptr(y), N.dev_ptr(gm), gy.numel(), code, slope, N.dt_code(gy),
                   N.stream())
            gy = gm
        # parameter gradients as autograd decided at forward time (a module frozen for this forward, e.g. the
        # discriminator under the student's adversarial term, stays frozen in its backward whatever its flag is now)
        mod._ssseg_wgrad(x, gy, want=(ctx.needs_input_grad[1], ctx.needs_input_grad[2]))
        joined, last = _join_take(ctx.join)
        pending = _sum_pending(_take(ctx.handoff), joined)
        if not ctx.needs_input_grad[0]:
            dx = None
        else:
            dx = _masked_dgrad(mod, gy, x, ctx.xmask, ctx.xgstat, pending, ctx.vcat)
            if dx is None:
                dx = _dgrad_acc(mod, gy, x.shape, pending, ctx.vcat)
        return _join_give(ctx.join, last, dx), None, None, None, None, None, None, None


def _masked_dgrad(conv, gy, x, xmask, xgstat, pending, vc):
    """The input gradient of a conv whose input x is the single-use activation output of its producer (xmask = (act,
    slope)): the producer's activation backward is applied in the epilogue (ssseg_conv_igemm_epi_actmask), and for a
    BN(+ReLU) producer (xgstat = (C, scale, bn)) that BN's backward sums are written as gradient-statistics rows and a
    folded eval BN's scale (scale not None) is applied: the producer's backward then skips its reduction (and, eval,
    its whole elementwise pass).  None where the engine cannot (the caller runs the plain dgrad)."""
    if not (xmask is not None and pending is None and vc is None and _CFG['act_mask']
            and getattr(conv, '_ssseg_mask_dgrad_ok', lambda: False)()):
        return None
    sr = scale = None
    if xgstat is not None and _CFG['bn_gstat'] and conv._ssseg_gstat_ok():
        C, scale, bn = xgstat
        n, _, H, W = x.shape
        buf = None
        if scale is not None and not any(e['bn'] is bn for e in _PGRAD['pending']):
            buf = bn.__dict__.get('_ssseg_gs_part')   # (a deferred eval BN keeps its rows until the flush)
        sr = StatRows(C, (n * H * W + 63) // 64 + 4, x.device, part=buf)
        if scale is not None:
            bn.__dict__['_ssseg_gs_part'] = sr.part
    dx = conv._ssseg_dgrad(gy, x.shape, mask=(x,) + tuple(xmask), stats=sr, scale=scale)
    dx.__dict__['_ssseg_premasked'] = True
    if sr is not None:
        dx.__dict__['_ssseg_gstats'] = sr
        dx.__dict__['_ssseg_prescaled'] = scale is not None
    return dx


def _dgrad_acc(mod, gy, xshape, pending, vc=None):
    """dx (+ a pending gradient of x): fused as the dgrad epilogue's residual where the engine supports it.
    vc: x is a virtual concat (its only consumer is this conv): the engine writes the gradients of the two parts
    where they are needed (VirtualCat.grads, taken by the concat's backward) and dx is a placeholder."""
    if pending is None and vc is not None and _CFG['vcat']:
        parts = getattr(mod, '_ssseg_dgrad_vsplit', lambda *a: None)(gy, xshape, vc)
        if parts is not None:
            vc.grads = parts
            # never read: an expanded 0-d tensor of x's shape (no memory, no kernel)
            return torch.empty((), dtype=gy.dtype, device=gy.device).expand(*xshape)
    if pending is None:
        return mod._ssseg_dgrad(gy, xshape)
    if getattr(mod, '_ssseg_res_dgrad', lambda: False)():
        return mod._ssseg_dgrad(gy, xshape, residual=pending)
    return mod._ssseg_dgrad(gy, xshape) + pending


def _bias_grad(mod, gy, want=None):
    """d bias += per-channel sum of gy (NHWC).  want: forward-time requires_grad (None: the live flag)."""
    if mod.bias is None or not (mod.bias.requires_grad if want is None else want):
        return
    n, cp, h, w = gy.shape
    C = mod.bias.numel()
    sums = torch.empty(2 * C, dtype=torch.float64, device=gy.device)
    nb = N.lib().ssseg_bn_workspace_bytes(C)
    ws = N.workspace(nb, gy.device)
    # one reduction with the gradient add in its tail (ssseg_channel_sum_grad)
    N.call('ssseg_channel_sum_grad', N.dev_ptr(gy), n * h * w, C, cp, N.dt_code(gy), N.dev_ptr(_grad_of(mod.bias)),
           N.dev_ptr(sums), N.dev_ptr(ws), nb, N.stream())


_PACK_EPOCH = [0]   # bumped whenever any conv's set of packed layouts changes (fast path of invalidate_packed)


class _ConvBase:
    """Shared host logic of Conv2d / ConvTranspose2d: packed-weight cache and launches."""
    def _wg_defer(self, a, b):
        """Inside defer_wgrad(): keep this weight gradient's operands for a merged launch later."""
        if not _WGRAD['defer']:
            return False
        if '_ssseg_wg_pending' in self.__dict__:   # a second use inside the same deferred pass: run the first
            _WGRAD['defer'] = False
            try:
                self._ssseg_wgrad(*self.__dict__.pop('_ssseg_wg_pending'), bias_grad=False, want=(True, False))
            finally:
                _WGRAD['defer'] = True
        self.__dict__['_ssseg_wg_pending'] = (a, b)
        _WGRAD['pending'].append(self)
        return True

    def _wg_take(self, a, b):
        """The deferred (input, output-gradient) pair to merge with (a, b): same spatial geometry, channel
        padding and dtype (only the batch may differ); an incompatible one is launched on its own first."""
        pend = self.__dict__.pop('_ssseg_wg_pending', None)
        if pend is None:
            return None
        a1, b1 = pend
        if (a1.shape[1:] == a.shape[1:] and b1.shape[1:] == b.shape[1:] and a1.dtype == a.dtype
                and b1.dtype == b.dtype and a1.stride()[1:] == a.stride()[1:] and b1.stride()[1:] == b.stride()[1:]):
            return pend
        self._ssseg_wgrad(a1, b1, bias_grad=False, want=(True, False))
        return None


    def _ssseg_init(self, head=False):
        self._ssseg_head = head           # writes fp32 logits with the real channel count visible
        self._ssseg_packs = {}
        self._ssseg_specs = {}

    def invalidate_packed(self):
        self._ssseg_packs = {}
        self._ssseg_specs = {}
        _PACK_EPOCH[0] += 1

    def _pack(self, key, Kd, Kr, Cd, Cp, layout, r0, rstep, Rn, s0, sstep, Sn):
        key = (key, _CFG['dtype'], Cp)
        t = self._ssseg_packs.get(key)
        if t is None:
            w = self.weight.detach()
            w = w if w.is_contiguous() else w.contiguous()
            Rs, Ss = self.weight.shape[2], self.weight.shape[3]
            t = torch.empty(max(Kd * Rn * Sn * Cp, 1), dtype=_CFG['dtype'], device=w.device)
            N.call('ssseg_weight_pack', N.dev_ptr(w, 'weight'), N.dev_ptr(t), Kd, Kr, Cd, Rs, Ss, Cp, layout, r0,
                   rstep, Rn, s0, sstep, Sn, N.dt_code(t), N.stream())
            self._ssseg_packs[key] = t
            self._ssseg_specs[key] = (Kd, Kr, Cd, Rs, Ss, Cp, layout, r0, rstep, Rn, s0, sstep, Sn)
            _PACK_EPOCH[0] += 1
        return t

    def _igemm(self, x, w, y, desc, out_dt, bias=None, relu=False, fold=None, stats=None, stem=False, mask=None):
        """One engine launch; epilogue y = act(acc*scale + shift + residual) with shift = bias, or
        fold = (scale, shift, residual, aux) from a folded eval BatchNorm (conv_bn_act); aux, when given,
        receives the raw accumulator (the pre-BN activation the differentiated eval pass needs).
        stem: the image-input kernel (ssseg_conv_stem_epi, w = the Cp-4 pack)."""
        dref = ctypes_ref(desc)
        nb = N.lib().ssseg_conv_igemm_workspace_bytes(dref, N.dt_code(x)) if (w is not None and not stem) else 0
        ws = N.workspace(nb, x.device) if nb else None
        scale, shift, res, aux = fold if fold is not None else (None, bias, None, None)
        if mask is not None:
            res = mask[0]
        sf = stats.launch_fields() if stats is not None else (None, 0, None)
        ep = N.ConvEpilogue(N.dev_ptr(scale) if scale is not None else None,
                            N.dev_ptr(shift) if shift is not None else None,
                            N.dev_ptr(res) if res is not None else None, res.shape[1] if res is not None else 0,
                            N.dev_ptr(aux) if aux is not None else None, *_act(relu), *sf)
        vc = _vcat_of(x)
        if mask is not None:
            if vc is not None:
                materialize(x)
            N.call('ssseg_conv_igemm_epi_actmask', N.dev_ptr(x), N.dev_ptr(w) if w is not None else None,
                   N.dev_ptr(y), dref, N.dt_code(x), out_dt, ctypes_ref(ep), int(mask[1]), float(mask[2]),
                   N.dev_ptr(ws) if ws is not None else None, nb, N.stream())
        elif stem:
            N.call('ssseg_conv_stem_epi', N.dev_ptr(x), N.dev_ptr(w), N.dev_ptr(y), dref, N.dt_code(x),
                   ctypes_ref(ep), N.stream())
        elif vc is not None and vc.ready(desc) and N.call_or_unsupported(
                'ssseg_conv_igemm_epi_vcat', N.dev_ptr(vc.a), ctypes_ref(vc.desc2()), N.dev_ptr(w), N.dev_ptr(y),
                ctypes_ref(vc.desc_for(desc)), N.dt_code(x), out_dt, ctypes_ref(ep),
                N.dev_ptr(ws) if ws is not None else None, nb, N.stream()):
            pass   # read the two parts of the virtual concat where they lie
        else:
            if vc is not None:
                materialize(x)
            N.call('ssseg_conv_igemm_epi', N.dev_ptr(x), N.dev_ptr(w) if w is not None else None, N.dev_ptr(y), dref,
                   N.dt_code(x), out_dt, ctypes_ref(ep), N.dev_ptr(ws) if ws is not None else None, nb, N.stream())
        if stats is not None:
            stats.commit()

    def _fold(self, bn, residual, cout, aux=None):
        """Eval BatchNorm (+ this conv's bias) as the epilogue's per-channel affine.  Returns the epilogue
        tuple and the (scale, mean_eff, invstd, shift) vectors the backward of a differentiated pass uses.
        Inside `folded(model)` the vectors come from that context's single batched launch."""
        if bn.num_features != self.out_channels:
            raise ValueError('conv_bn_act: BatchNorm width != conv out_channels')
        bn.__dict__['_ssseg_fold_conv'] = self      # remembered for folded(): the pair is fixed by the model
        pre = bn.__dict__.get('_ssseg_fold_live')
        if pre is not None and pre[0] is self and pre[1].numel() == 4 * cout:
            v = pre[1]
            return ((v[:cout], v[cout:2 * cout], residual, aux),
                    (v[:cout], v[2 * cout:3 * cout], v[3 * cout:], v[cout:2 * cout]))
        dev = self.weight.device
        v = torch.empty(4 * cout, dtype=torch.float32, device=dev)
        scale, shift, mean_eff, invstd = v[:cout], v[cout:2 * cout], v[2 * cout:3 * cout], v[3 * cout:]
        opt = lambda t: N.dev_ptr(t.detach()) if t is not None else None  # noqa: E731
        N.call('ssseg_bn_fold', N.dev_ptr(bn.running_mean), N.dev_ptr(bn.running_var), opt(bn.weight), opt(bn.bias),
               opt(self.bias), float(bn.eps), bn.num_features, cout, N.dev_ptr(scale), N.dev_ptr(shift),
               N.dev_ptr(mean_eff), N.dev_ptr(invstd), N.stream())
        return (scale, shift, residual, aux), (scale, mean_eff, invstd, shift)


def ctypes_ref(d):
    import ctypes
    return ctypes.byref(d)


class Conv2d(nn.Conv2d, _ConvBase):
    """nn.Conv2d on the implicit-GEMM engine (groups == 1)."""

    def __init__(self, *args, head=False, **kw):
        super().__init__(*args, **kw)
        self._ssseg_dw = self.groups != 1
        if self._ssseg_dw and not (self.groups == self.in_channels == self.out_channels):
            raise NotImplementedError('ssseg.nn.Conv2d: grouped convolution other than depthwise is not implemented')
        if self._ssseg_dw and head:
            raise NotImplementedError('ssseg.nn.Conv2d: depthwise head')
        if self.padding_mode != 'zeros':
            raise NotImplementedError('ssseg.nn.Conv2d: only zero padding')
        self._ssseg_init(head)

    # geometry helpers
    def _dims(self):
        v = vec()
        return rup(self.in_channels, v), rup(self.out_channels, v)

    def _out_hw(self, H, W):
        (R, S), (sh, sw), (ph, pw), (dh, dw) = self.kernel_size, self.stride, self.padding, self.dilation
        return (H + 2 * ph - dh * (R - 1) - 1) // sh + 1, (W + 2 * pw - dw * (S - 1) - 1) // sw + 1

    def _vpad_ok(self):
        return not (self._ssseg_dw or self._ssseg_head)

    def _fwd_desc(self, n, H, W):
        cin, cout = self._dims()
        (R, S), (sh, sw), (ph, pw), (dh, dw) = self.kernel_size, self.stride, self.padding, self.dilation
        OH, OW = self._out_hw(H, W)
        ce = vpad(cin) if self._vpad_ok() else cin
        return _desc(N=n, H=H, W=W, C=ce, ldx=cin, OH=OH, OW=OW, K=cout, R=R, S=S, sy=sh, sx=sw, dy=dh, dx=dw,
                     py=-ph, px=-pw, outH=OH, outW=OW, osy=1, osx=1, ooy=0, oox=0, ldy=cout, ldw=R * S * ce)

    def _ssseg_res_dgrad(self):
        return not self._ssseg_dw

    def forward(self, x, handoff=None, stats=None):
        if not _is_act(x):
            x = to_act(x)
        return _ConvFn.apply(x, self.weight, self.bias, self, False, handoff, stats, _join_fwd(x))

    def stat_rows_cap(self, n, H, W):
        """Upper bound of the statistics partial rows one forward writes (None: not fusable here)."""
        if self._ssseg_dw or self._ssseg_head:
            return None
        OH, OW = self._out_hw(H, W)
        return (n * OH * OW + 63) // 64

    def forward_relu(self, x):
        """Conv2d followed by ReLU, fused into the GEMM epilogue (unet.py:27-28 with no norm)."""
        return self.forward_act(x, True)

    def forward_act(self, x, act, single_use=False):
        """Conv2d followed by an activation (True = ReLU, ACT_RELU6, ('leaky', slope)) in the epilogue
        (discriminator.py:15-16 Conv + LeakyReLU(0.2)).  single_use: the caller guarantees the output feeds exactly
        one ssseg conv, whose input-gradient launch then applies this activation's backward in place
        (ssseg_conv_igemm_epi_actmask) instead of a separate pass here."""
        if not _is_act(x):
            x = to_act(x)
        y = _ConvFn.apply(x, self.weight, self.bias, self, act, None, None, _join_fwd(x))
        code, slope = _act(act)
        if single_use and code in (ACT_RELU, ACT_LEAKY) and torch.is_grad_enabled() and y.requires_grad:
            y.__dict__['_ssseg_act_out'] = (code, slope)
        return y

    # ---- depthwise (groups == channels): ssseg_dwconv_* (MobileNetV2, mobilenetv2.py:58) ----
    def _dw_desc(self, n, H, W):
        d = self._fwd_desc(n, H, W)
        d.ldw = d.C
        return d

    def _dw_pack(self):
        cin = self._dims()[0]
        R, S = self.kernel_size
        return self._pack('dw', 1, 1, self.in_channels, cin, 1, 0, 1, R, 0, 1, S)

    def _dw_forward(self, x, relu, bn, residual, keep_pre, aux_copy=True):
        cin, cout = self._dims()
        n, _, H, W = x.shape
        d = self._dw_desc(n, H, W)
        y = new_act(n, cout, d.OH, d.OW, _CFG['dtype'], x.device)
        aux = bwd = None
        if bn is not None:
            _need_res(residual, y)
            aux = torch.empty_like(y) if keep_pre and aux_copy else None
            fold, bwd = self._fold(bn, residual, cout, aux)
        else:
            fold = (None, self.bias, None, None)
        scale, shift, res, aux_t = fold
        code, slope = _act(relu)
        ep = N.ConvEpilogue(N.dev_ptr(scale) if scale is not None else None,
                            N.dev_ptr(shift.detach() if shift is not None else None) if shift is not None else None,
                            N.dev_ptr(res) if res is not None else None, res.shape[1] if res is not None else 0,
                            N.dev_ptr(aux_t) if aux_t is not None else None, code, slope)
        R, S = self.kernel_size
        with _Timed(2.0 * n * d.OH * d.OW * self.in_channels * R * S, 'fwd', _tag(self, n, H, W)):
            N.call('ssseg_dwconv_fwd', N.dev_ptr(x), N.dev_ptr(self._dw_pack()), N.dev_ptr(y), ctypes_ref(d),
                   N.dt_code(x), ctypes_ref(ep), N.stream())
        return (y, aux, bwd) if keep_pre else y

    def _ssseg_forward(self, x, relu, bn=None, residual=None, keep_pre=False, stats=None, aux_copy=True):
        cin, cout = self._dims()
        _need_act(x, cin, 'Conv2d')
        if self._ssseg_dw:
            if stats is not None:
                raise NotImplementedError('ssseg: fused BN statistics on a depthwise conv')
            return self._dw_forward(x, relu, bn, residual, keep_pre, aux_copy)
        n, _, H, W = x.shape
        d = self._fwd_desc(n, H, W)
        R, S = self.kernel_size
        stem = self._stem_ok(cout, d.OW)
        if stem:   # image-input kernel: weights [K][R][S][4]
            w = self._pack('stem', cout, self.out_channels, self.in_channels, 4, 0, 0, 1, R, 0, 1, S)
        else:
            w = self._pack('fwd', cout, self.out_channels, self.in_channels, d.C, 0, 0, 1, R, 0, 1, S)
        fl = _conv_flops(n, d.OH, d.OW, self.out_channels, self.in_channels, R, S)
        tg = _tag(self, n, H, W)
        if bn is not None:
            y = new_act(n, cout, d.OH, d.OW, _CFG['dtype'], x.device)
            _need_res(residual, y)
            aux = torch.empty_like(y) if keep_pre and aux_copy else None
            fold, bwd = self._fold(bn, residual, cout, aux)
            with _Timed(fl, 'fwd', tg):
                self._igemm(x, w, y, d, N.dt_code(y), relu=relu, fold=fold, stem=stem)
            return (y, aux, bwd) if keep_pre else y
        if self._ssseg_head:
            y = torch.empty((n, cout, d.OH, d.OW), dtype=torch.float32, device=x.device,
                            memory_format=torch.channels_last)
            with _Timed(fl, 'fwd', tg):
                self._igemm(x, w, y, d, N.F32, self.bias, relu)
            return y[:, :self.out_channels]
        y = new_act(n, cout, d.OH, d.OW, _CFG['dtype'], x.device)
        with _Timed(fl, 'fwd', tg):
            self._igemm(x, w, y, d, N.dt_code(y), self.bias, relu, stats=stats, stem=stem)
        return y

    def _stem_ok(self, cout, ow=None):
        """The image-input conv kernel (ssseg_conv_stem_epi) covers this layer: <= 4 input channels, R in {3, 7},
        S <= 8, dilation 1, stride <= 2, output width % 128 == 0, 16-bit compute, Cout % 16 == 0 (the ResNet /
        DeepLab 7x7 stems, 3x3 image convs)."""
        R, S = self.kernel_size
        return (_CFG['stem'] and not self._ssseg_head and not self._ssseg_dw and self.in_channels <= 4
                and R in (3, 7) and S <= 8 and self.dilation == (1, 1) and self.stride[1] <= 2 and cout % 16 == 0
                and _CFG['dtype'] in (torch.bfloat16, torch.float16) and ow is not None and ow % 128 == 0)

    def _grad_in(self, gy):
        """Incoming output gradient -> physical NHWC compute-dtype tensor."""
        cin, cout = self._dims()
        if self._ssseg_head:
            n, c, h, w = gy.shape
            g = new_act(n, cout, h, w, _CFG['dtype'], gy.device)
            gc = gy if gy.is_contiguous() else gy.contiguous()
            N.call('ssseg_nchw_to_nhwc', N.dev_ptr(gc), N.dev_ptr(g), n, c, h, w, cout, N.dt_code(gc), N.dt_code(g),
                   N.stream())
            return g
        _need_act(gy, cout, 'Conv2d backward')
        return gy

    def _ssseg_wgrad(self, x, gy, bias_grad=True, want=None):
        """dW (+ db) of this conv; want = (weight, bias) requires_grad as captured at forward time (None: live)."""
        if _held(self, x, gy, bias_grad, want):
            return
        ww = self.weight.requires_grad if want is None else want[0]
        if bias_grad:
            _bias_grad(self, gy, None if want is None else want[1])
        if not ww:
            if self.bias is not None and (self.bias.requires_grad if want is None else want[1]):
                _ready(self.bias)
            return
        n, _, H, W = x.shape
        if self._ssseg_dw:
            d = self._dw_desc(n, H, W)
            nb = N.lib().ssseg_dwconv_wgrad_workspace_bytes(ctypes_ref(d), N.dt_code(x))
            ws = N.workspace(nb, x.device)
            R, S = self.kernel_size
            with _Timed(2.0 * n * d.OH * d.OW * self.in_channels * R * S, 'wgrad', _tag(self, n, H, W)):
                N.call('ssseg_dwconv_wgrad', N.dev_ptr(x), N.dev_ptr(gy), N.dev_ptr(_grad_of(self.weight)),
                       ctypes_ref(d), N.dt_code(x), self.in_channels, 1, N.dev_ptr(ws), nb, N.stream())
            _ready(*[p for p in (self.weight, self.bias) if p is not None])
            return
        if self._wg_defer(x, gy):
            return
        pend = self._wg_take(x, gy)
        with _on_wgrad_stream(x, gy, *(pend or ())):
            self._wgrad_launch(x, gy, pend)

    def _wgrad_launch(self, x, gy, pend):
        n, _, H, W = x.shape
        R, S = self.kernel_size
        if pend is None:
            d = self._fwd_desc(n, H, W)
            nb = N.lib().ssseg_conv_wgrad_workspace_bytes(ctypes_ref(d), N.dt_code(x))
            ws = _wgrad_ws(nb, x.device)
            vc = _vcat_of(x)
            with _Timed(_conv_flops(n, d.OH, d.OW, self.out_channels, self.in_channels, R, S), 'wgrad',
                        _tag(self, n, H, W)):
                if not (vc is not None and vc.ready(d) and N.call_or_unsupported(
                        'ssseg_conv_wgrad_vcat', N.dev_ptr(vc.a), ctypes_ref(vc.desc2()), N.dev_ptr(gy),
                        N.dev_ptr(_grad_of(self.weight)), ctypes_ref(vc.desc_for(d)), N.dt_code(x), self.in_channels,
                        self.out_channels, 1, 1, N.dev_ptr(ws), nb, N.stream())):
                    if vc is not None:
                        materialize(x)
                    N.call('ssseg_conv_wgrad', N.dev_ptr(x), N.dev_ptr(gy), N.dev_ptr(_grad_of(self.weight)),
                           ctypes_ref(d), N.dt_code(x), self.in_channels, self.out_channels, 1, 1, N.dev_ptr(ws), nb,
                           N.stream())
        else:   # the deferred pass and this one: one launch over both pixel sets
            x1, gy1 = pend
            n1 = x1.shape[0]
            d = self._fwd_desc(n1, H, W)
            nb = N.lib().ssseg_conv_wgrad2_workspace_bytes(ctypes_ref(d), n, N.dt_code(x))
            ws = _wgrad_ws(nb, x.device)
            v1, v2 = _vcat_of(x1), _vcat_of(x)
            with _Timed(_conv_flops(n1 + n, d.OH, d.OW, self.out_channels, self.in_channels, R, S), 'wgrad',
                        _tag(self, n1 + n, H, W)):
                both = v1 is not None and v2 is not None and v1.same_split(v2) and v1.ready(d)
                if not (both and N.call_or_unsupported(
                        'ssseg_conv_wgrad2_vcat', N.dev_ptr(v1.a), ctypes_ref(v1.desc2()), N.dev_ptr(gy1),
                        N.dev_ptr(v2.a), ctypes_ref(v2.desc2()), N.dev_ptr(gy), n, N.dev_ptr(_grad_of(self.weight)),
                        ctypes_ref(v1.desc_for(d)), N.dt_code(x), self.in_channels, self.out_channels, 1, 1,
                        N.dev_ptr(ws), nb, N.stream())):
                    for t in (x1, x):
                        if _vcat_of(t) is not None:
                            materialize(t)
                    N.call('ssseg_conv_wgrad2', N.dev_ptr(x1), N.dev_ptr(gy1), N.dev_ptr(x), N.dev_ptr(gy), n,
                           N.dev_ptr(_grad_of(self.weight)), ctypes_ref(d), N.dt_code(x), self.in_channels,
                           self.out_channels, 1, 1, N.dev_ptr(ws), nb, N.stream())
        if self.bias is not None:
            _ready(self.weight, self.bias)
        else:
            _ready(self.weight)

    def _ssseg_mask_dgrad_ok(self):
        return not self._ssseg_dw and _CFG['dtype'] in (torch.bfloat16, torch.float16, torch.float32)

    def _ssseg_gstat_ok(self):
        """Gradient statistics in the masked dgrad: every output phase has taps (an empty phase's zero launch
        writes no statistics rows)."""
        (R, S), (sh, sw) = self.kernel_size, self.stride
        # (at most 4 output phases: _masked_dgrad sizes the statistics table for that many phase tails)
        return (sh == 1 and sw == 1) or (R >= sh and S >= sw and sh * sw <= 4 and self.dilation in (1, (1, 1)))

    def _ssseg_dgrad(self, gy, xshape, residual=None, mask=None, stats=None, scale=None):
        """dx of the conv; `residual` (a pending gradient of x, GradHandoff) is added in the epilogue; `mask` = (y,
        act, slope): x was the activation output y of its producer, whose backward the epilogue applies in place;
        `stats` (with mask, a StatRows): the epilogue also writes that producer BN's backward sums (gradient
        statistics rows, ssseg_conv_igemm_epi_actmask); `scale` (with mask): per-channel factor of the stored value
        (a folded eval BN producer's scale: dx is that producer's conv-output gradient)."""
        if (stats is not None or scale is not None) and (mask is None or residual is not None):
            raise ValueError('ssseg.nn.Conv2d: gradient statistics / scale need the masked input gradient')
        fold = (None, None, residual, None) if residual is not None else (
            (scale, None, None, None) if scale is not None else None)
        cin, cout = self._dims()
        n, _, H, W = xshape
        (R, S), (sh, sw), (ph, pw), (dh, dw) = self.kernel_size, self.stride, self.padding, self.dilation
        OH, OW = gy.shape[2], gy.shape[3]
        dx = new_act(n, cin, H, W, _CFG['dtype'], gy.device)
        if residual is not None:
            _need_res(residual, dx)
            if self._ssseg_dw:
                raise NotImplementedError('ssseg.nn.Conv2d: fused input-gradient accumulation needs a dense conv')
        if self._ssseg_dw:
            d = self._dw_desc(n, H, W)
            with _Timed(2.0 * n * OH * OW * self.in_channels * R * S, 'dgrad', _tag(self, n, H, W)):
                N.call('ssseg_dwconv_dgrad', N.dev_ptr(gy), N.dev_ptr(self._dw_pack()), N.dev_ptr(dx), ctypes_ref(d),
                       N.dt_code(gy), N.stream())
            return dx
        timer = _Timed(_conv_flops(n, OH, OW, self.out_channels, self.in_channels, R, S), 'dgrad', _tag(self, n, H, W))
        ce = vpad(cout) if self._vpad_ok() else cout   # the dgrad contracts over the output channels
        if sh == 1 and sw == 1:
            w = self._pack('dgrad', cin, self.in_channels, self.out_channels, ce, 1, R - 1, -1, R, S - 1, -1, S)
            d = _desc(N=n, H=OH, W=OW, C=ce, ldx=cout, OH=H, OW=W, K=cin, R=R, S=S, sy=1, sx=1, dy=dh, dx=dw,
                      py=ph - (R - 1) * dh, px=pw - (S - 1) * dw, outH=H, outW=W, osy=1, osx=1, ooy=0, oox=0,
                      ldy=cin, ldw=R * S * ce)
            with timer:
                self._igemm(gy, w, dx, d, N.dt_code(dx), fold=fold, mask=mask, stats=stats)
            return dx
        timer.__enter__()
        for (phy, ry0, rny, dly, qy) in _phases(sh, ph, R, H, dh):
            for (phx, rx0, rnx, dlx, qx) in _phases(sw, pw, S, W, dw):
                if qy == 0 or qx == 0:
                    continue
                rr, ss = (rny, rnx) if rny * rnx > 0 else (0, 0)
                w = self._pack(('dgrad', phy, phx), cin, self.in_channels, self.out_channels, ce, 1, ry0, sh,
                               rny, rx0, sw, rnx) if rr else None
                d = _desc(N=n, H=OH, W=OW, C=ce, ldx=cout, OH=qy, OW=qx, K=cin, R=rr, S=ss, sy=1, sx=1, dy=-1,
                          dx=-1, py=dly, px=dlx, outH=H, outW=W, osy=sh, osx=sw, ooy=phy, oox=phx, ldy=cin,
                          ldw=max(rr * ss * ce, ce))
                # each phase adds the pending gradient at its own output pixels (the residual is indexed by
                # the output pixel, so the phases together cover it exactly once)
                self._igemm(gy, w, dx, d, N.dt_code(dx), fold=fold, mask=mask, stats=stats)
        timer.__exit__()
        return dx


    def _ssseg_dgrad_vsplit(self, gy, xshape, vc):
        """dx of a virtual concat input [a | b] written straight into (da, db), the gradients of its parts
        (ssseg_conv_igemm_epi_vsplit: channels [0, ca) to da, [ca, ca + cb) to db).  None where the engine cannot
        (the caller runs the ordinary dgrad and the concat's backward splits it)."""
        cin, cout = self._dims()
        n, cp, H, W = xshape
        if (self._ssseg_dw or self.stride != (1, 1) or cp != vc.ca + vc.cb or cin != cp
                or _CFG['dtype'] not in (torch.bfloat16, torch.float16)):
            return None
        (R, S), (ph, pw), (dh, dw) = self.kernel_size, self.padding, self.dilation
        OH, OW = gy.shape[2], gy.shape[3]
        da = new_act(n, vc.ca, H, W, _CFG['dtype'], gy.device)
        db = new_act(n, vc.cb, H, W, _CFG['dtype'], gy.device)
        w = self._pack('dgrad', cin, self.in_channels, self.out_channels, cout, 1, R - 1, -1, R, S - 1, -1, S)
        d = _desc(N=n, H=OH, W=OW, C=cout, ldx=cout, OH=H, OW=W, K=cin, R=R, S=S, sy=1, sx=1, dy=dh, dx=dw,
                  py=ph - (R - 1) * dh, px=pw - (S - 1) * dw, outH=H, outW=W, osy=1, osx=1, ooy=0, oox=0,
                  ldy=vc.ca, ldw=R * S * cout)
        dref = ctypes_ref(d)
        nb = N.lib().ssseg_conv_igemm_workspace_bytes(dref, N.dt_code(gy))
        ws = N.workspace(nb, gy.device) if nb else None
        mask = vc.a if vc.mask_a else None   # the first part's ReLU mask (its forward output)
        ep = N.ConvEpilogue(None, None, N.dev_ptr(mask) if mask is not None else None, vc.ca if mask is not None else 0,
                            None, 0, 0.0, None, 0, None)
        split = N.VCat(N.dev_ptr(db), vc.ca, vc.cb)
        with _Timed(_conv_flops(n, OH, OW, self.out_channels, self.in_channels, R, S), 'dgrad', _tag(self, n, H, W)):
            ok = N.call_or_unsupported('ssseg_conv_igemm_epi_vsplit', N.dev_ptr(gy), N.dev_ptr(w), N.dev_ptr(da),
                                       ctypes_ref(split), dref, N.dt_code(gy), N.dt_code(gy), ctypes_ref(ep),
                                       N.dev_ptr(ws) if ws is not None else None, nb, N.stream())
        if not ok:
            return None
        if mask is not None:
            da.__dict__['_ssseg_premasked'] = True
        return da, db


class ConvTranspose2d(nn.ConvTranspose2d, _ConvBase):
    """nn.ConvTranspose2d (output_padding 0, groups 1, dilation 1) with an optional fused ReLU."""

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if self.groups != 1 or self.dilation != (1, 1) or self.output_padding != (0, 0):
            raise NotImplementedError('ssseg.nn.ConvTranspose2d: groups/dilation/output_padding not implemented')
        self._ssseg_init(False)
        self._fuse_relu = False

    def _dims(self):
        v = vec()
        return rup(self.in_channels, v), rup(self.out_channels, v)

    def forward(self, x, output_size=None, stats=None):
        if output_size is not None:
            raise NotImplementedError('ssseg.nn.ConvTranspose2d: output_size')
        if not _is_act(x):
            x = to_act(x)
        return _ConvFn.apply(x, self.weight, self.bias, self, self._fuse_relu, None, stats, _join_fwd(x))

    def stat_rows_cap(self, n, H, W):
        (R, S), (sh, sw), (ph, pw) = self.kernel_size, self.stride, self.padding
        OH, OW = self._out_hw(H, W)
        rows = 0
        for (_, _, rny, _, qy) in _phases(sh, ph, R, OH):
            for (_, _, rnx, _, qx) in _phases(sw, pw, S, OW):
                if qy == 0 or qx == 0:
                    continue
                if rny * rnx == 0:
                    return None     # an empty tap set is zero-filled by a kernel without the statistics
                rows += (n * qy * qx + 63) // 64
        return rows

    def forward_relu(self, x):
        """ConvTranspose2d followed by ReLU, fused into the epilogue (unet.py:20-23)."""
        return self.forward_act(x, True)

    def forward_act(self, x, act):
        if not _is_act(x):
            x = to_act(x)
        return _ConvFn.apply(x, self.weight, self.bias, self, act, None, None, _join_fwd(x))

    def _out_hw(self, H, W):
        (R, S), (sh, sw), (ph, pw) = self.kernel_size, self.stride, self.padding
        return (H - 1) * sh - 2 * ph + R, (W - 1) * sw - 2 * pw + S

    def _ssseg_forward(self, x, relu, bn=None, residual=None, keep_pre=False, stats=None, aux_copy=True):
        cin, cout = self._dims()
        _need_act(x, cin, 'ConvTranspose2d')
        n, _, H, W = x.shape
        (R, S), (sh, sw), (ph, pw) = self.kernel_size, self.stride, self.padding
        OH, OW = self._out_hw(H, W)
        y = new_act(n, cout, OH, OW, _CFG['dtype'], x.device)
        fold = aux = bwd = None
        if bn is not None:
            _need_res(residual, y)
            aux = torch.empty_like(y) if keep_pre and aux_copy else None
            fold, bwd = self._fold(bn, residual, cout, aux)
        timer = _Timed(_conv_flops(n, H, W, self.out_channels, self.in_channels, R, S), 'fwd', _tag(self, n, H, W))
        timer.__enter__()
        phases = []
        for (phy, ry0, rny, dly, qy) in _phases(sh, ph, R, OH):
            for (phx, rx0, rnx, dlx, qx) in _phases(sw, pw, S, OW):
                if qy == 0 or qx == 0:
                    continue
                rr, ss = (rny, rnx) if rny * rnx > 0 else (0, 0)
                w = self._pack(('fwd', phy, phx), cout, self.out_channels, self.in_channels, cin, 1, ry0, sh, rny,
                               rx0, sw, rnx) if rr else None
                d = _desc(N=n, H=H, W=W, C=cin, ldx=cin, OH=qy, OW=qx, K=cout, R=rr, S=ss, sy=1, sx=1, dy=-1, dx=-1,
                          py=dly, px=dlx, outH=OH, outW=OW, osy=sh, osx=sw, ooy=phy, oox=phx, ldy=cout,
                          ldw=max(rr * ss * cin, cin))
                phases.append((w, d, (rr, ss, qy, qx), (dly, dlx, phy, phx)))
        shapes = {p[2] for p in phases}
        if (_CFG['phases'] and 1 < len(phases) <= 4 and len(shapes) == 1 and phases[0][0] is not None
                and _CFG['dtype'] in (torch.bfloat16, torch.float16)):
            # every phase has the same taps and sub-grid: one launch over all of them (ssseg_conv_igemm_phases)
            self._igemm_phases(x, [p[0] for p in phases], y, phases[0][1], [p[3] for p in phases], self.bias, relu,
                               fold, stats)
        else:
            for w, d, _, _ in phases:
                self._igemm(x, w, y, d, N.dt_code(y), self.bias, relu, fold, stats=stats)
        timer.__exit__()
        return (y, aux, bwd) if keep_pre else y

    def _igemm_phases(self, x, ws, y, desc, geoms, bias, relu, fold, stats):
        import ctypes
        scale, shift, res, aux = fold if fold is not None else (None, bias, None, None)
        sf = stats.launch_fields() if stats is not None else (None, 0, None)
        ep = N.ConvEpilogue(N.dev_ptr(scale) if scale is not None else None,
                            N.dev_ptr(shift) if shift is not None else None,
                            N.dev_ptr(res) if res is not None else None, res.shape[1] if res is not None else 0,
                            N.dev_ptr(aux) if aux is not None else None, *_act(relu), *sf)
        geo = (ctypes.c_int64 * (4 * len(geoms)))(*[v for g4 in geoms for v in g4])
        wp = (ctypes.c_void_p * len(ws))(*[N.dev_ptr(w) for w in ws])
        # deterministic split-K scratch where the phases are tile-starved (16x16 inputs)
        nb = N.lib().ssseg_conv_igemm_phases_workspace_bytes(ctypes_ref(desc), len(ws), N.dt_code(x))
        scratch = N.workspace(nb, x.device) if nb else None
        N.call('ssseg_conv_igemm_phases_ws', N.dev_ptr(x), N.dev_ptr(y), ctypes_ref(desc), N.dt_code(x), N.dt_code(y),
               ctypes_ref(ep), len(ws), ctypes.addressof(geo), ctypes.addressof(wp),
               N.dev_ptr(scratch) if scratch is not None else None, nb, N.stream())
        if stats is not None:
            stats.commit()

    def _grad_in(self, gy):
        _need_act(gy, self._dims()[1], 'ConvTranspose2d backward')
        return gy

    def _ssseg_wgrad(self, x, gy, bias_grad=True, want=None):
        if _held(self, x, gy, bias_grad, want):
            return
        ww = self.weight.requires_grad if want is None else want[0]
        if bias_grad:
            _bias_grad(self, gy, None if want is None else want[1])
        if ww:
            if self._wg_defer(x, gy):
                return
            pend = self._wg_take(x, gy)
            with _on_wgrad_stream(x, gy, *(pend or ())):
                self._wgrad_launch(x, gy, pend, want)
            return
        wb = self.bias is not None and (self.bias.requires_grad if want is None else want[1])
        _ready(*[p for p, on in ((self.bias, wb),) if on])

    def _wgrad_launch(self, x, gy, pend, want):
        cin, cout = self._dims()
        n, _, H, W = x.shape
        (R, S), (sh, sw), (ph, pw) = self.kernel_size, self.stride, self.padding
        OH, OW = gy.shape[2], gy.shape[3]
        n1 = pend[0].shape[0] if pend is not None else n
        # dW[ci][co][r][s] = sum_p x[p][ci] * gy[p*s - pad + r][co]: a conv over gy with x as its output grad
        d = _desc(N=n1, H=OH, W=OW, C=cout, ldx=cout, OH=H, OW=W, K=cin, R=R, S=S, sy=sh, sx=sw, dy=1, dx=1,
                  py=-ph, px=-pw, outH=H, outW=W, osy=1, osx=1, ooy=0, oox=0, ldy=cin, ldw=R * S * cout)
        if pend is None:
            nb = N.lib().ssseg_conv_wgrad_workspace_bytes(ctypes_ref(d), N.dt_code(x))
            ws = _wgrad_ws(nb, x.device)
            with _Timed(_conv_flops(n, H, W, self.out_channels, self.in_channels, R, S), 'wgrad',
                        _tag(self, n, H, W)):
                N.call('ssseg_conv_wgrad', N.dev_ptr(gy), N.dev_ptr(x), N.dev_ptr(_grad_of(self.weight)),
                       ctypes_ref(d), N.dt_code(x), self.out_channels, self.in_channels, 1, 1, N.dev_ptr(ws), nb,
                       N.stream())
        else:   # the deferred pass and this one: one launch over both pixel sets (operands in (gy, x) order)
            x1, gy1 = pend
            nb = N.lib().ssseg_conv_wgrad2_workspace_bytes(ctypes_ref(d), n, N.dt_code(x))
            ws = _wgrad_ws(nb, x.device)
            with _Timed(_conv_flops(n1 + n, H, W, self.out_channels, self.in_channels, R, S), 'wgrad',
                        _tag(self, n1 + n, H, W)):
                N.call('ssseg_conv_wgrad2', N.dev_ptr(gy1), N.dev_ptr(x1), N.dev_ptr(gy), N.dev_ptr(x), n,
                       N.dev_ptr(_grad_of(self.weight)), ctypes_ref(d), N.dt_code(x), self.out_channels,
                       self.in_channels, 1, 1, N.dev_ptr(ws), nb, N.stream())
        wb = self.bias is not None and (self.bias.requires_grad if want is None else want[1])
        _ready(*[p for p, on in ((self.weight, True), (self.bias, wb)) if on])

    def _ssseg_mask_dgrad_ok(self):
        return _CFG['dtype'] in (torch.bfloat16, torch.float16, torch.float32)

    def _ssseg_gstat_ok(self):
        return True   # one strided launch over every input pixel

    def _ssseg_dgrad(self, gy, xshape, mask=None, stats=None, scale=None):
        """dx of the transposed conv (a strided conv of gy); mask / stats / scale as Conv2d._ssseg_dgrad (x was the
        single-use BN+ReLU output of UpBlock.conv3_1)."""
        if (stats is not None or scale is not None) and mask is None:
            raise ValueError('ssseg.nn.ConvTranspose2d: gradient statistics / scale need the masked input gradient')
        cin, cout = self._dims()
        n, _, H, W = xshape
        (R, S), (sh, sw), (ph, pw) = self.kernel_size, self.stride, self.padding
        OH, OW = gy.shape[2], gy.shape[3]
        dx = new_act(n, cin, H, W, _CFG['dtype'], gy.device)
        w = self._pack('dgrad', cin, self.in_channels, self.out_channels, cout, 0, 0, 1, R, 0, 1, S)
        d = _desc(N=n, H=OH, W=OW, C=cout, ldx=cout, OH=H, OW=W, K=cin, R=R, S=S, sy=sh, sx=sw, dy=1, dx=1, py=-ph,
                  px=-pw, outH=H, outW=W, osy=1, osx=1, ooy=0, oox=0, ldy=cin, ldw=R * S * cout)
        with _Timed(_conv_flops(n, H, W, self.out_channels, self.in_channels, R, S), 'dgrad', _tag(self, n, H, W)):
            self._igemm(gy, w, dx, d, N.dt_code(dx), fold=(scale, None, None, None) if scale is not None else None,
                        mask=mask, stats=stats)
        return dx


# ------------------------------------------------------------------------------------------------
# batch norm (+ReLU, +residual)
# ------------------------------------------------------------------------------------------------
def _sync_group(training):
    if not (training and _CFG['sync_bn'] and dist.is_available() and dist.is_initialized()):
        return False
    from .ddp import forced
    return dist.get_world_size() > 1 or forced()


def _pad16(C, dtype):
    """Channels the BN kernels write (padding zeros included): C rounded up to a 16-byte chunk."""
    v = 16 // torch.empty((), dtype=dtype).element_size()
    return (C + v - 1) // v * v


class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, mod, relu, handoff=None, pre=None, single_use=False):
        C = mod.num_features
        n, cp, h, w = x.shape
        P = n * h * w
        dev = x.device
        mean = torch.empty(C, dtype=torch.float32, device=dev)
        invstd = torch.empty(C, dtype=torch.float32, device=dev)
        training = mod.training or not mod.track_running_stats
        count = float(P)
        if training:
            sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
            nb = N.lib().ssseg_bn_workspace_bytes(C)
            ws = N.workspace(nb, dev)
            track = mod.track_running_stats and mod.training
            if track and mod.momentum is None:
                raise NotImplementedError('ssseg BatchNorm2d: momentum=None (cumulative average)')
            fin = (C, count, float(mod.eps), float(mod.momentum if mod.momentum is not None else 0.0),
                   N.dev_ptr(mean), N.dev_ptr(invstd), N.dev_ptr(mod.running_mean) if track else None,
                   N.dev_ptr(mod.running_var) if track else None,
                   N.dev_ptr(mod.num_batches_tracked) if track else None)
            if pre is not None and pre.rows > 0:
                # statistics partials from the producing conv's epilogue: no pass over x here
                if pre.C != C:
                    raise ValueError('ssseg BatchNorm2d: fused statistics width mismatch')
                if _sync_group(True):
                    N.call('ssseg_bn_partials_finalize', N.dev_ptr(pre.part), pre.rows, C, N.dev_ptr(sums), 0.0, 0.0,
                           0.0, None, None, None, None, None, N.stream())
                    _comm.all_reduce_sum(sums)
                    count = float(P * dist.get_world_size())
                    N.call('ssseg_bn_finalize', N.dev_ptr(sums), C, count, *fin[2:], N.stream())
                else:
                    N.call('ssseg_bn_partials_finalize', N.dev_ptr(pre.part), pre.rows, C, N.dev_ptr(sums), count,
                           *fin[2:], N.stream())
            elif _sync_group(True):
                N.call('ssseg_bn_stats', N.dev_ptr(x), P, C, cp, N.dt_code(x), N.dev_ptr(sums), N.dev_ptr(ws), nb,
                       N.stream())
                _comm.all_reduce_sum(sums)
                count = float(P * dist.get_world_size())
                N.call('ssseg_bn_finalize', N.dev_ptr(sums), C, count, *fin[2:], N.stream())
            else:   # one launch: the finalize runs in the reduction's tail
                N.call('ssseg_bn_stats_finalize', N.dev_ptr(x), P, C, cp, N.dt_code(x), N.dev_ptr(sums),
                       N.dev_ptr(ws), nb, count, *fin[2:], N.stream())
        else:
            N.call('ssseg_bn_eval_params', N.dev_ptr(mod.running_mean), N.dev_ptr(mod.running_var), float(mod.eps), C,
                   N.dev_ptr(mean), N.dev_ptr(invstd), N.stream())
        y = new_act(n, cp, h, w, x.dtype, dev, zero=cp > _pad16(C, x.dtype))
        wt = weight.detach() if weight is not None else None
        bs = bias.detach() if bias is not None else None
        N.call('ssseg_bn_apply', N.dev_ptr(x), N.dev_ptr(residual) if residual is not None else None, N.dev_ptr(y),
               P, C, cp, cp, cp, N.dev_ptr(mean), N.dev_ptr(invstd), N.dev_ptr(wt) if wt is not None else None,
               N.dev_ptr(bs) if bs is not None else None, _act(relu)[0], N.dt_code(x), N.stream())
        ctx.save_for_backward(x, residual, mean, invstd)
        ctx.mod, ctx.relu, ctx.training, ctx.count, ctx.handoff = mod, relu, training, count, handoff
        if single_use and training and residual is None and _act(relu)[0] == ACT_RELU and _CFG['bn_gstat']:
            # y feeds exactly one conv (the caller's guarantee): that conv's input-gradient launch applies this
            # ReLU's backward and writes this BN's backward sums (_ConvFn.backward); backward() then skips its
            # reduction pass
            y.__dict__['_ssseg_act_out'] = (ACT_RELU, 0.0)
            y.__dict__['_ssseg_gstat'] = (C, None, mod)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, residual, mean, invstd = ctx.saved_tensors
        mod = ctx.mod
        C = mod.num_features
        n, cp, h, w = x.shape
        P = n * h * w
        _need_act(gy, cp, 'BatchNorm2d backward')
        dev = x.device
        wt = mod.weight.detach() if mod.weight is not None else None
        bs = mod.bias.detach() if mod.bias is not None else None
        sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
        nb = N.lib().ssseg_bn_workspace_bytes(C)
        ws = N.workspace(nb, dev)
        res_p = N.dev_ptr(residual) if residual is not None else None
        pgrad = mod.weight is not None and ctx.needs_input_grad[1]   # forward-time requires_grad
        # the consumer's input-gradient launch applied the ReLU backward already (and may have written our sums)
        act = 0 if gy.__dict__.get('_ssseg_premasked', False) else _act(ctx.relu)[0]
        gs = gy.__dict__.get('_ssseg_gstats')
        if gs is not None and ctx.training and gs.rows > 0 and gs.C == C and residual is None and act == 0:
            # (sum dy, sum dy * y) rows from that epilogue -> (sum dy, sum dy * x_hat) + (dgamma, dbeta); channels
            # whose x_hat y cannot resolve (gamma == 0, |beta| >= 8 |gamma|) are summed from gy (premasked) and x
            N.call('ssseg_bn_gstat_finalize_x', N.dev_ptr(gs.part), gs.rows, C, N.dev_ptr(sums),
                   N.dev_ptr(wt) if wt is not None else None, N.dev_ptr(bs) if bs is not None else None,
                   N.dev_ptr(gy), N.dev_ptr(x), P, cp, N.dt_code(x), N.dev_ptr(mean), N.dev_ptr(invstd),
                   *(_grad_ptrs(mod.weight, mod.bias) if pgrad else (None, None)), N.stream())
        else:
            # reduction + (dgamma, dbeta) from the local sums in one launch (ssseg_bn_bwd_reduce_grad)
            N.call('ssseg_bn_bwd_reduce_grad', N.dev_ptr(gy), N.dev_ptr(x), res_p, P, C, cp, cp, cp, N.dev_ptr(mean),
                   N.dev_ptr(invstd), N.dev_ptr(wt) if wt is not None else None,
                   N.dev_ptr(bs) if bs is not None else None, act, N.dt_code(x), N.dev_ptr(sums),
                   N.dev_ptr(ws), nb, *(_grad_ptrs(mod.weight, mod.bias) if pgrad else (None, None)), N.stream())
        if pgrad:
            _ready(mod.weight, mod.bias)
        count = ctx.count
        if ctx.training and _sync_group(True):
            _comm.all_reduce_sum(sums)
        dx = new_act(n, cp, h, w, x.dtype, dev, zero=cp > _pad16(C, x.dtype))
        want_res = residual is not None and ctx.needs_input_grad[3]
        dres = new_act(n, cp, h, w, x.dtype, dev, zero=cp > _pad16(C, x.dtype)) if want_res else None
        N.call('ssseg_bn_bwd_apply', N.dev_ptr(gy), N.dev_ptr(x), res_p, N.dev_ptr(dx),
               N.dev_ptr(dres) if dres is not None else None, P, C, cp, cp, cp, cp, N.dev_ptr(mean),
               N.dev_ptr(invstd), N.dev_ptr(wt) if wt is not None else None,
               N.dev_ptr(bs) if bs is not None else None, act, int(bool(ctx.training)),
               N.dev_ptr(sums), float(count), N.dt_code(x), N.stream())
        if dres is not None and ctx.handoff is not None:
            ctx.handoff.put(dres)
            dres = None
        return dx, None, None, dres, None, None, None, None, None


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d (acts as SyncBatchNorm across the process group when one is initialised)."""

    def forward(self, x, residual=None, relu=False):
        _need_act(x, rup(self.num_features, vec()), 'BatchNorm2d')
        return _BNFn.apply(x, self.weight, self.bias, residual, self, relu)


def _need_res(residual, y):
    if residual is not None and (residual.shape != y.shape or residual.dtype != y.dtype or not _is_act(residual)):
        raise ValueError(f'fused residual must match the output activation: {tuple(residual.shape)} vs {tuple(y.shape)}')


def _no_grad(*ts):
    return not torch.is_grad_enabled() or not any(t is not None and t.requires_grad for t in ts)


class _ConvBNEvalFn(torch.autograd.Function):
    """Differentiated conv -> eval BatchNorm (-> + residual) (-> ReLU), the student's consistency pass
    (reference train.py:90-92 runs model.eval() with autograd on).  Forward: one engine launch writes
    y and the raw accumulator aux.  Backward: ssseg_bn_eval_bwd turns dy into the conv's output gradient
    (and the residual's) plus the BN parameter sums in one pass; then the ordinary conv backward."""

    @staticmethod
    def forward(ctx, x, cweight, cbias, gamma, beta, residual, conv, bn, relu, grad_in=None, grad_out=None, join=None,
                single_use=False):
        # without a residual, y itself carries the pre-activation wherever the gradient survives the activation:
        # no raw accumulator copy (ssseg_bn_eval_bwd_grad_y recovers x_hat from y)
        ycopy = residual is None and _CFG['eval_bwd_y']
        y, aux, (scale, mean_eff, invstd, shift) = conv._ssseg_forward(x, relu, bn=bn, residual=residual,
                                                                       keep_pre=True, aux_copy=not ycopy)
        ctx.save_for_backward(x, y, aux, scale, mean_eff, invstd, shift)
        ctx.conv, ctx.bn, ctx.relu, ctx.has_res = conv, bn, relu, residual is not None
        ctx.grad_in, ctx.grad_out, ctx.join, ctx.vcat = grad_in, grad_out, join, _vcat_of(x)
        ctx.xmask = x.__dict__.get('_ssseg_act_out')   # x = a single-use BN+ReLU output: its backward in our dgrad
        ctx.xgstat = x.__dict__.get('_ssseg_gstat')
        if (single_use and aux is None and residual is None and _act(relu)[0] == ACT_RELU and _CFG['bn_gstat']
                and shift is not None):
            # y feeds exactly one conv: that conv's input-gradient launch applies this ReLU's backward and this BN's
            # scale and writes its backward sums (_masked_dgrad), so backward() gets dconv itself
            y.__dict__['_ssseg_act_out'] = (ACT_RELU, 0.0)
            y.__dict__['_ssseg_gstat'] = (bn.num_features, scale, bn)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, aux, scale, mean_eff, invstd, shift = ctx.saved_tensors
        _vcat_restore(x, ctx.vcat)
        conv, bn = ctx.conv, ctx.bn
        n, cp, h, w = y.shape
        C = bn.num_features
        _need_act(gy, cp, 'conv_bn_act backward')
        dev = y.device
        gs = gy.__dict__.get('_ssseg_gstats')
        # the consumer's input-gradient launch wrote dconv (ReLU backward and BN scale applied) and this BN's backward
        # sums (gradient-statistics rows, x_hat from y)
        pre = (gs is not None and gy.__dict__.get('_ssseg_prescaled', False) and aux is None and not ctx.has_res
               and gs.rows > 0 and gs.C == C)
        act = 0 if gy.__dict__.get('_ssseg_premasked', False) else _act(ctx.relu)[0]
        dconv = gy if pre else new_act(n, cp, h, w, y.dtype, dev, zero=cp > _pad16(C, y.dtype))
        want_res = ctx.has_res and ctx.needs_input_grad[5]
        dres = new_act(n, cp, h, w, y.dtype, dev, zero=cp > _pad16(C, y.dtype)) if want_res else None
        sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
        nb = N.lib().ssseg_bn_workspace_bytes(C)
        ws = N.workspace(nb, dev)
        # parameter gradients as autograd decided at forward time (inputs 1-4: conv.weight, conv.bias, bn.weight,
        # bn.bias)
        fw = {id(p): ctx.needs_input_grad[i] for i, p in ((1, conv.weight), (2, conv.bias), (3, bn.weight),
                                                           (4, bn.bias)) if p is not None}
        want = lambda p: p is not None and fw.get(id(p), False)  # noqa: E731
        # dconv/dres + the BN (and conv-bias) parameter grads in one reduction (ssseg_bn_eval_bwd_grad)
        grads = (N.dev_ptr(_grad_of(bn.weight)) if want(bn.weight) else None,
                 N.dev_ptr(_grad_of(bn.bias)) if want(bn.bias) else None,
                 N.dev_ptr(_grad_of(conv.bias)) if want(conv.bias) else None)
        defer = (_PGRAD['live'] and any(g is not None for g in grads)
                 and not any(getattr(p, '_ssseg_reducer', None) is not None for p in (bn.weight, bn.bias, conv.bias)
                             if want(p)))
        if pre and defer:   # the gradient-statistics rows wait for defer_param_grads()' one launch
            _PGRAD['pending'].append({'bn': bn, 'part': gs.part, 'nparts': gs.rows, 'C': C, 'scale': scale,
                                      'dg': grads[0] or 0, 'db': grads[1] or 0, 'dbias': grads[2] or 0,
                                      'gs': (N.dev_ptr(shift), N.dev_ptr(mean_eff), N.dev_ptr(invstd))})
        elif pre:
            grads = _grad_ptrs(*[p if want(p) else None for p in (bn.weight, bn.bias, conv.bias)])
            N.call('ssseg_bn_gstat_finalize', N.dev_ptr(gs.part), gs.rows, C, N.dev_ptr(sums), N.dev_ptr(scale),
                   N.dev_ptr(shift), N.dev_ptr(mean_eff), N.dev_ptr(invstd), *grads, N.stream())
        elif defer:   # partial rows only; defer_param_grads() reduces every layer's in one launch
            import ctypes
            parts = bn.__dict__.setdefault('_ssseg_pg_parts', [])
            k = sum(1 for e in _PGRAD['pending'] if e['bn'] is bn)   # a module run twice in the pass (MSA)
            if k >= len(parts) or parts[k].numel() < nb or parts[k].device != dev:
                buf = torch.empty(nb, dtype=torch.uint8, device=dev)
                if k >= len(parts):
                    parts.append(buf)
                else:
                    parts[k] = buf
            part = parts[k]
            rows = ctypes.c_int64(0)
            N.call('ssseg_bn_eval_bwd_part', N.dev_ptr(gy), N.dev_ptr(y), N.dev_ptr(aux) if aux is not None else None,
                   N.dev_ptr(dconv), N.dev_ptr(dres) if dres is not None else None, n * h * w, C, cp, N.dev_ptr(scale),
                   N.dev_ptr(shift) if aux is None else None, N.dev_ptr(mean_eff), N.dev_ptr(invstd),
                   act, N.dt_code(y), N.dev_ptr(part), nb, ctypes.byref(rows), N.stream())
            _PGRAD['pending'].append({'bn': bn, 'part': part, 'nparts': rows.value, 'C': C, 'scale': scale,
                                      'dg': grads[0] or 0, 'db': grads[1] or 0, 'dbias': grads[2] or 0})
        else:   # immediate parameter gradients (temporaries inside hold_wgrad(params=True))
            grads = _grad_ptrs(*[p if want(p) else None for p in (bn.weight, bn.bias, conv.bias)])
        if defer or pre:
            pass
        elif aux is None:   # x_hat from y (no residual): ssseg_bn_eval_bwd_grad_y
            N.call('ssseg_bn_eval_bwd_grad_y', N.dev_ptr(gy), N.dev_ptr(y), N.dev_ptr(dconv),
                   N.dev_ptr(dres) if dres is not None else None, n * h * w, C, cp, N.dev_ptr(scale), N.dev_ptr(shift),
                   N.dev_ptr(mean_eff), N.dev_ptr(invstd), act, N.dt_code(y), N.dev_ptr(sums),
                   N.dev_ptr(ws), nb, *grads, N.stream())
        else:
            N.call('ssseg_bn_eval_bwd_grad', N.dev_ptr(gy), N.dev_ptr(y), N.dev_ptr(aux), N.dev_ptr(dconv),
                   N.dev_ptr(dres) if dres is not None else None, n * h * w, C, cp, N.dev_ptr(scale),
                   N.dev_ptr(mean_eff), N.dev_ptr(invstd), act, N.dt_code(y), N.dev_ptr(sums),
                   N.dev_ptr(ws), nb, *grads, N.stream())
        if want(bn.weight) or want(bn.bias):
            _ready(*[p for p in (bn.weight, bn.bias) if want(p)])
        conv._ssseg_wgrad(x, dconv, bias_grad=False, want=(ctx.needs_input_grad[1], False))
        joined, last = _join_take(ctx.join)
        pending = _sum_pending(_take(ctx.grad_in), joined)
        if not ctx.needs_input_grad[0]:
            dx = None
        else:
            dx = _masked_dgrad(conv, dconv, x, ctx.xmask, ctx.xgstat, pending, ctx.vcat)
            if dx is None:
                dx = _dgrad_acc(conv, dconv, x.shape, pending, ctx.vcat)
        if dres is not None and ctx.grad_out is not None:
            ctx.grad_out.put(dres)
            dres = None
        return _join_give(ctx.join, last, dx), None, None, None, None, dres, None, None, None, None, None, None, None


def conv_bn_act(conv, x, bn, relu=True, residual=None, grad_in=None, grad_out=None, single_use=False):
    """act(bn(conv(x)) [+ residual]).  With an eval-mode BatchNorm the BN, residual add and ReLU run in
    the conv's epilogue (ssseg_bn_fold + ssseg_conv_igemm_epi): one kernel, each activation written once.
    Without gradients (the teacher forwards, reference train.py:69-94) that is all; when the eval pass
    is differentiated (the consistency pass) the epilogue also keeps the raw accumulator and
    _ConvBNEvalFn's backward runs the fused BN backward.  Training-mode BN needs the batch statistics
    of the conv output first, so it runs as conv, then bn_act.  grad_in / grad_out (a GradHandoff shared by
    a block's first conv and its residual join) fuse the shortcut gradient into the first conv's dgrad.
    single_use: the caller guarantees the output feeds exactly one ssseg conv (Bottleneck bn1 -> conv2, bn2 -> conv3;
    a ConvBlock's first BN+ReLU): that conv's input gradient carries this BN's backward sums (training BN) or is
    this conv's output gradient itself (differentiated eval BN: ReLU backward and BN scale applied in its epilogue)."""
    fusable = (isinstance(conv, (Conv2d, ConvTranspose2d)) and not conv._ssseg_head and isinstance(bn, BatchNorm2d)
               and not bn.training and bn.track_running_stats)
    if fusable:
        if not _is_act(x):
            x = to_act(x)
        if _no_grad(x, conv.weight, conv.bias, bn.weight, bn.bias, residual):
            return conv._ssseg_forward(x, relu, bn=bn, residual=residual)
        return _ConvBNEvalFn.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, residual, conv, bn, relu, grad_in,
                                   grad_out, _join_fwd(x), bool(single_use))
    stats = None
    if (_CFG['fuse_stats'] and isinstance(conv, (Conv2d, ConvTranspose2d)) and isinstance(bn, BatchNorm2d)
            and (bn.training or not bn.track_running_stats) and bn.num_features == conv.out_channels and x.dim() == 4):
        cap = conv.stat_rows_cap(x.shape[0], x.shape[2], x.shape[3])
        if cap:
            stats = StatRows(bn.num_features, cap, x.device)
    if type(conv) is Conv2d:
        y = conv(x, handoff=grad_in, stats=stats)
    else:
        y = conv(x, stats=stats) if stats is not None else conv(x)
    return bn_act(y, bn, relu=relu, residual=residual, grad_out=grad_out, pre=stats, single_use=single_use)


def bn_act(x, bn, relu=True, residual=None, grad_out=None, pre=None, single_use=False):
    """act(bn(x) [+ residual]) in one pass: ConvBlock's BN+ReLU (unet.py:9-10), Bottleneck's bn3+add+relu.
    pre: StatRows the producing conv's epilogue filled (fused training statistics)."""
    if not isinstance(bn, BatchNorm2d):
        raise TypeError('ssseg.nn.bn_act needs an ssseg BatchNorm2d')
    _need_act(x, rup(bn.num_features, vec()), 'BatchNorm2d')
    return _BNFn.apply(x, bn.weight, bn.bias, residual, bn, relu, grad_out, pre, bool(single_use))


# ------------------------------------------------------------------------------------------------
# pooling, upsampling, concat / crop
# ------------------------------------------------------------------------------------------------
class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil_mode, join=None):
        n, c, h, w = x.shape
        ctx.join = join

        def osz(L):
            o = (L + 2 * p - k + (s - 1 if ceil_mode else 0)) // s + 1
            if ceil_mode and (o - 1) * s >= L + p:
                o -= 1
            return o
        oh, ow = osz(h), osz(w)
        y = new_act(n, c, oh, ow, x.dtype, x.device)
        idx = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
        N.call('ssseg_maxpool_fwd', N.dev_ptr(x), N.dev_ptr(y), N.dev_ptr(idx), n, h, w, c, oh, ow, k, s, p,
               N.dt_code(x), N.stream())
        ctx.save_for_backward(idx)
        ctx.meta = (n, c, h, w, oh, ow, k, s, p, x.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        n, c, h, w, oh, ow, k, s, p, dt = ctx.meta
        _need_act(gy, c, 'MaxPool2d backward')
        gx = new_act(n, c, h, w, dt, gy.device)
        joined, last = _join_take(ctx.join)
        if joined is not None:
            _need_res(joined, gx)
        # gx = gather of the selected taps' gradients (+ the parked gradient of x, in the same pass)
        N.call('ssseg_maxpool_bwd_res', N.dev_ptr(gy), N.dev_ptr(idx), N.dev_ptr(joined) if joined is not None else None,
               N.dev_ptr(gx), n, h, w, c, oh, ow, k, s, p, N.dt_code(gy), N.stream())
        return _join_give(ctx.join, last, gx), None, None, None, None, None


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        k, s, p = (self.kernel_size, self.stride, self.padding)
        k = k if isinstance(k, int) else k[0]
        s = s if isinstance(s, int) else s[0]
        p = p if isinstance(p, int) else p[0]
        if self.dilation not in (1, (1, 1)) or self.return_indices:
            raise NotImplementedError('ssseg MaxPool2d: dilation / return_indices')
        _need_act(x, None, 'MaxPool2d')
        return _MaxPoolFn.apply(x, k, s, p, bool(self.ceil_mode), _join_fwd(x))


class Upsample(nn.Upsample):
    """nn.Upsample(scale_factor, mode='bilinear') on NHWC activations (unet.py:26, simple_unet.py:71)."""

    def forward(self, x):
        if self.mode != 'bilinear' or self.size is not None:
            raise NotImplementedError('ssseg Upsample: bilinear with scale_factor only')
        from .ops import interpolate_bilinear
        sf = self.scale_factor if isinstance(self.scale_factor, (tuple, list)) else (self.scale_factor,) * 2
        oh, ow = int(x.shape[2] * sf[0]), int(x.shape[3] * sf[1])
        return interpolate_bilinear(x, (oh, ow), align_corners=bool(self.align_corners))


class VirtualCat:
    """The two parts of a virtual channel concat (cat_crop(lazy=True)): the consuming conv's kernels read channels
    [0, ca) from a and [ca, ca + cb) from b where they lie (ssseg_vcat); the concat tensor itself is allocated but
    not written unless materialize() runs (a consumer that cannot read it part by part)."""
    __slots__ = ('a', 'b', 'ca', 'cb', '_d2', 'grads', 'mask_a', 'versions')

    def __init__(self, a, b, ca, cb):
        self.a, self.b, self.ca, self.cb = a, b, ca, cb
        self._d2 = None
        # the parts are held here, not by save_for_backward: autograd's version check cannot see an in-place change
        # to them between the forward and the consumer's backward, so the backward checks these itself
        self.versions = (a._version, b._version)
        self.grads = None   # (da, db) from the consumer's split-output dgrad, taken by the concat's backward
        # a is the output of a fused conv+ReLU (the UpBlock upsampler): da can be written with that ReLU's
        # backward already applied (ssseg_conv_igemm_epi_vsplit's mask), which removes its ssseg_act_bwd pass
        self.mask_a = bool(a.__dict__.get('_ssseg_relu_out', False))

    def desc2(self):
        if self._d2 is None:
            self._d2 = N.VCat(N.dev_ptr(self.b), self.ca, self.b.shape[1])
        return self._d2

    def ready(self, desc):
        """the engine reads x as [a | b]: desc.C is the concat's width"""
        return int(desc.C) == self.ca + self.cb

    def desc_for(self, desc):
        """the launch descriptor with x = a (its own pixel stride)"""
        d = N.ConvDesc.from_buffer_copy(desc)
        d.ldx = self.a.shape[1]
        return d

    def same_split(self, other):
        return self.ca == other.ca and self.b.shape[1] == other.b.shape[1]

    def check_versions(self):
        if (self.a._version, self.b._version) != self.versions:
            raise RuntimeError('ssseg: a part of a virtual concat was modified in place between its consumer\'s '
                               'forward and backward (the gradient would be computed from the modified values)')


def _vcat_of(x):
    return x.__dict__.get('_ssseg_vcat') if isinstance(x, torch.Tensor) else None


def _vcat_restore(x, vc):
    if vc is not None:
        vc.check_versions()
    if vc is not None and '_ssseg_vcat' not in x.__dict__ and not getattr(x, '_ssseg_materialized', False):
        x.__dict__['_ssseg_vcat'] = vc


def materialize(x):
    """Write a virtual concat's two parts into its own tensor (the copy path); afterwards x is an ordinary
    activation."""
    vc = x.__dict__.pop('_ssseg_vcat', None)
    if vc is None:
        return x
    n, cp, H, W = x.shape
    for t, c, c0 in ((vc.a, vc.ca, 0), (vc.b, vc.cb, vc.ca)):
        N.call('ssseg_nhwc_copy', N.dev_ptr(t), N.dev_ptr(x) + c0 * x.element_size(), n, H, W, c, H, W, t.shape[1],
               0, 0, H, W, cp, 0, 0, N.dt_code(t), N.stream())
    x.__dict__['_ssseg_materialized'] = True
    return x


class _CatFn(torch.autograd.Function):
    """torch.cat((a, b), 1) with a center-crop of whichever map is larger (unet.py:40-45)."""

    @staticmethod
    def forward(ctx, a, b, ca, cb, ja=None, jb=None, virtual=False, vc=None):
        ctx.joins = (ja, jb)
        ctx.vc = vc
        n = a.shape[0]
        H, W = min(a.shape[2], b.shape[2]), min(a.shape[3], b.shape[3])
        v = vec()
        cp = rup(ca + cb, v)
        y = new_act(n, cp, H, W, a.dtype, a.device, zero=cp != ca + cb and not virtual)
        offs = []
        for t, c, c0 in ((a, ca, 0), (b, cb, ca)):
            oy, ox = (t.shape[2] - H) // 2, (t.shape[3] - W) // 2
            offs.append((oy, ox))
            if not virtual:
                N.call('ssseg_nhwc_copy', N.dev_ptr(t), N.dev_ptr(y) + c0 * y.element_size(), n, H, W, c, t.shape[2],
                       t.shape[3], t.shape[1], oy, ox, H, W, cp, 0, 0, N.dt_code(t), N.stream())
        ctx.meta = (a.shape, b.shape, ca, cb, offs, H, W, cp)
        return y

    @staticmethod
    def backward(ctx, gy):
        ash, bsh, ca, cb, offs, H, W, cp = ctx.meta
        n = gy.shape[0]
        grads = []
        split = ctx.vc.grads if ctx.vc is not None else None   # the consumer wrote the parts' gradients itself
        if split is not None:
            ctx.vc.grads = None
            if any(st != 0 for st in gy.stride()):
                # the consumer returned the never-written placeholder (all strides 0) as its input gradient: any
                # other gradient summed into it by autograd means a second consumer, whose contribution is lost
                raise RuntimeError('ssseg: a virtual concat (cat_crop(lazy=True)) has more than one consumer; '
                                   'use cat_crop(lazy=False) where the concat is read twice')
        for k, (sh, c, c0, (oy, ox), j) in enumerate(((ash, ca, 0, offs[0], ctx.joins[0]),
                                                        (bsh, cb, ca, offs[1], ctx.joins[1]))):
            if split is not None:
                g = split[k]
            else:
                cropped = (sh[2], sh[3]) != (H, W)
                g = new_act(n, sh[1], sh[2], sh[3], gy.dtype, gy.device, zero=cropped or sh[1] != c)
                N.call('ssseg_nhwc_copy', N.dev_ptr(gy) + c0 * gy.element_size(), N.dev_ptr(g), n, H, W, c, H, W, cp,
                       0, 0, sh[2], sh[3], sh[1], oy, ox, N.dt_code(gy), N.stream())
            joined, last = _join_take(j)
            if joined is not None:   # the concat usually runs first (it is downstream): rare
                g = g + joined
            grads.append(_join_give(j, last, g))
        return grads[0], grads[1], None, None, None, None, None, None


def _vcat_eligible(a, b, ca, cb):
    return (_CFG['vcat'] and _CFG['dtype'] in (torch.bfloat16, torch.float16) and ca % 64 == 0 and cb % 64 == 0
            and a.shape[1] == ca and b.shape[1] == cb and tuple(a.shape[2:]) == tuple(b.shape[2:])
            and a.shape[0] == b.shape[0] and a.dtype == b.dtype and _is_act(a) and _is_act(b))


def cat_crop(a, b, ca, cb, lazy=False):
    """Concatenate NHWC activations a (ca real channels) and b (cb) along channels; the larger map is
    center-cropped to the smaller (unet.py:40-45 compares dim 2; both dims are cropped to match here).
    lazy=True: the caller's only consumer is a conv that reads a virtual concat (UpBlock.conv3_0); where the parts
    qualify (16-bit, whole 64-channel parts, no crop) nothing is copied and the returned tensor carries the parts."""
    virtual = lazy and _vcat_eligible(a, b, ca, cb)
    vc = VirtualCat(a, b, ca, cb) if virtual else None
    y = _CatFn.apply(a, b, ca, cb, _join_fwd(a), _join_fwd(b), virtual, vc)
    if virtual:
        y.__dict__['_ssseg_vcat'] = vc
    return y


@contextlib.contextmanager
def folded(model):
    """Fold every eval BatchNorm of `model` that follows a conv (pairs seen by earlier conv_bn_act calls)
    with ONE ssseg_bn_fold_batch launch, and let conv_bn_act use those vectors inside the block.  Wrap an
    eval forward in it (teacher forwards, the consistency pass: train.py:69-94); the running statistics and
    parameters must not change inside the block.  Pairs not seen yet fold per layer as usual."""
    bns = [m for m in model.modules() if isinstance(m, BatchNorm2d) and '_ssseg_fold_conv' in m.__dict__
           and not m.training and m.track_running_stats]
    rows = []
    for bn in bns:
        conv = bn.__dict__['_ssseg_fold_conv']
        cout = conv._dims()[1]
        buf = bn.__dict__.get('_ssseg_fold_buf')
        if buf is None or buf.numel() != 4 * cout or buf.device != bn.running_mean.device:
            buf = torch.empty(4 * cout, dtype=torch.float32, device=bn.running_mean.device)
            bn.__dict__['_ssseg_fold_buf'] = buf
        opt = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        rows.append((bn, conv, buf, (bn.running_mean.data_ptr(), bn.running_var.data_ptr(), opt(bn.weight),
                                     opt(bn.bias), opt(conv.bias), buf.data_ptr(), bn.num_features, cout)))
    if rows:
        sig = tuple(r[3] + (float(r[0].eps),) for r in rows)
        cache = model.__dict__.setdefault('_ssseg_fold_table', [None, None])
        if cache[0] != sig:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError('ssseg.nn.folded: the BN fold table changed while a HIP graph is being captured; '
                                   'run eager steps until every conv/BN pair has been seen (two steps) before capturing')
            import struct
            blob = b''.join(struct.pack('<6q2qd', *r[3], float(r[0].eps)) for r in rows)
            dev = rows[0][2].device
            cache[0], cache[1] = sig, torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
        N.call('ssseg_bn_fold_batch', N.dev_ptr(_graph_ref(cache[1])), len(rows), N.stream())
    try:
        for bn, conv, buf, _ in rows:
            bn.__dict__['_ssseg_fold_live'] = (conv, buf)
        yield
    finally:
        for bn, _, _, _ in rows:
            bn.__dict__.pop('_ssseg_fold_live', None)


def invalidate_packed(model):
    """The master weights changed (optimizer step, EMA, load): refresh every cached packed layout of the
    model with ONE ssseg_weight_pack_batch launch per dtype (layouts not packed yet stay lazy).  The
    device descriptor table is cached on the model and rebuilt only when the set of packs changes; while
    no conv gained or dropped a pack (_PACK_EPOCH) and every master weight still has the same storage, the
    cached tables are relaunched without walking the module tree (the walk cost ~0.2 ms of host time per
    model per step)."""
    fast = model.__dict__.get('_ssseg_pack_fast')
    if fast is not None and fast[0] == _PACK_EPOCH[0] and all(
            m.weight is w and w.data_ptr() == ptr for m, w, ptr in fast[1]):
        for dtc, n, table in fast[2]:
            N.call('ssseg_weight_pack_batch', N.dev_ptr(table), n, dtc, N.stream())
        return
    rows = {}
    mods = []
    for m in model.modules():
        if not isinstance(m, _ConvBase):
            continue
        w = m.weight
        if not m._ssseg_packs:
            continue
        if not (w.is_cuda and w.is_contiguous()):
            m.invalidate_packed()
            continue
        if w.numel() >= 2 ** 31:
            m.invalidate_packed()
            continue
        if w.shape[2] * w.shape[3] > 135:   # the batched repack's tile holds filters of <= 135 taps
            m.invalidate_packed()
            continue
        for key, t in m._ssseg_packs.items():
            if t.numel() >= 2 ** 31:
                raise RuntimeError('ssseg: packed weight too large for the batched repack')
            rows.setdefault(key[1], []).append((w.data_ptr(), t.data_ptr()) + m._ssseg_specs[key])
        mods.append((m, w, w.data_ptr()))
    cache = model.__dict__.setdefault('_ssseg_pack_tables', {})
    launches = []
    for dt, rr in rows.items():
        sig = tuple(rr)
        ent = cache.get(dt)
        if ent is None or ent[0] != sig:
            dev = torch.device('cuda', torch.cuda.current_device())
            ent = (sig, torch.tensor(rr, dtype=torch.int64).to(dev))
            cache[dt] = ent
        launches.append((N.dt_code(torch.empty((), dtype=dt)), len(rr), ent[1]))
        N.call('ssseg_weight_pack_batch', N.dev_ptr(ent[1]), len(rr), launches[-1][0], N.stream())
    model.__dict__['_ssseg_pack_fast'] = (_PACK_EPOCH[0], mods, launches)


# ------------------------------------------------------------------------------------------------
# primitives of the C3-C5 model families: n-way concat, average pooling, activation-layout bilinear
# resize, n-ary add(+act), dropout (HarDNet, DeepLabV3, HRNet / MultiscaleAttention)
# ------------------------------------------------------------------------------------------------
class _CatNFn(torch.autograd.Function):
    """torch.cat(tensors, 1) of same-size NHWC activations with REAL channel counts `chans` (hardnet.py:67,78,
    95; higher_hrnet.py:1033; discriminator.py:56): the result packs the real channels densely, padding to the
    MFMA vector is zero.  One ssseg_nhwc_cat_n launch (the padding written in the same pass); the backward is one
    ssseg_nhwc_split_n launch that writes every operand's gradient (zero padding) and adds the pending gradient of
    operands whose consumers share a GradJoin (HarDNet's layer outputs feed up to four concats and a conv)."""

    @staticmethod
    def forward(ctx, chans, joins, *ts):
        n, _, H, W = ts[0].shape
        for t in ts:
            if t.shape[0] != n or t.shape[2] != H or t.shape[3] != W:
                raise ValueError(f'cat_n: spatial shapes differ: {[tuple(t.shape) for t in ts]}')
            if t.stride(1) != 1 or t.dtype != ts[0].dtype:
                raise ValueError('cat_n: operands must be NHWC activations of one dtype')
        if len(ts) > 16:
            raise ValueError('cat_n: more than 16 operands')
        cp = rup(sum(chans), vec())
        y = new_act(n, cp, H, W, ts[0].dtype, ts[0].device)
        tab = N.cat_parts([(N.dev_ptr(t), None, None, t.shape[1], c) for t, c in zip(ts, chans)])
        N.call('ssseg_nhwc_cat_n', ctypes.addressof(tab), len(ts), N.dev_ptr(y), n * H * W, cp, N.dt_code(y),
               N.stream())
        ctx.meta = (tuple(t.shape[1] for t in ts), tuple(chans), cp)
        ctx.joins = joins
        return y

    @staticmethod
    def backward(ctx, gy):
        phys, chans, cp = ctx.meta
        n, _, H, W = gy.shape
        if not _is_act(gy, cp):
            gy = gy.contiguous(memory_format=torch.channels_last)
        gs, rows, takes = [], [], []
        for k, (pc, c) in enumerate(zip(phys, chans)):
            j = ctx.joins[k] if ctx.joins is not None else None
            pending, last = _join_take(j)
            g = new_act(n, pc, H, W, gy.dtype, gy.device)
            late = None
            if pending is not None and (pending.shape != g.shape or pending.stride() != g.stride()
                                        or pending.dtype != g.dtype):
                pending, late = None, pending    # (not in the concat's layout: added after the split)
            gs.append(g)
            takes.append((j, last, late, pending))
            rows.append((None, N.dev_ptr(g), N.dev_ptr(pending) if pending is not None else None, pc, c))
        tab = N.cat_parts(rows)
        N.call('ssseg_nhwc_split_n', N.dev_ptr(gy), cp, ctypes.addressof(tab), len(rows), n * H * W, N.dt_code(gy),
               N.stream())
        out = []
        for (j, last, late, _), g in zip(takes, gs):
            if late is not None:
                g = g + late
            out.append(_join_give(j, last, g))
        return (None, None) + tuple(out)


class _ResizeCatFn(torch.autograd.Function):
    """cat_n([resize_act(t, size) for t in ts], chans) with every resize written straight into its channel slice of the
    concat (the NHWC bilinear kernels take output strides), and in the backward read straight from the slice of the
    concat's gradient: the resized maps are never materialised (HRNet's multi-resolution aggregation,
    higher_hrnet.py:1020-1034).  Same-size inputs are copied, like cat_n.  Results are bitwise those of
    resize_act + cat_n (the same kernels on the same values)."""

    @staticmethod
    def forward(ctx, size, align_corners, chans, *ts):
        n = ts[0].shape[0]
        H, W = size
        total = sum(chans)
        cp = rup(total, vec())
        y = new_act(n, cp, H, W, ts[0].dtype, ts[0].device, zero=cp != total)
        ys = y.stride()
        c0 = 0
        for t, c in zip(ts, chans):
            _, pc, h, w = t.shape
            if (h, w) == (H, W):
                N.call('ssseg_nhwc_copy', N.dev_ptr(t), N.dev_ptr(y) + c0 * y.element_size(), n, H, W, c, H, W, pc,
                       0, 0, H, W, cp, 0, 0, N.dt_code(t), N.stream())
            else:
                N.call('ssseg_bilinear_fwd', N.dev_ptr(t), N.dev_ptr(y) + c0 * y.element_size(), n, c, h, w, H, W,
                       N.strides4(t), _strides4(ys), int(align_corners), N.dt_code(t), N.stream())
            c0 += c
        ctx.meta = (tuple(tuple(t.shape) for t in ts), tuple(chans), cp, bool(align_corners), ts[0].dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        shapes, chans, cp, ac, dt = ctx.meta
        n, _, H, W = gy.shape
        gs = gy.stride()
        out, c0 = [None, None, None], 0
        for (_, pc, h, w), c in zip(shapes, chans):
            g = new_act(n, pc, h, w, dt, gy.device, zero=pc != c)
            if (h, w) == (H, W):
                N.call('ssseg_nhwc_copy', N.dev_ptr(gy) + c0 * gy.element_size(), N.dev_ptr(g), n, H, W, c, H, W, cp,
                       0, 0, H, W, pc, 0, 0, N.dt_code(gy), N.stream())
            else:
                _bilinear_bwd(gy, g, n, c, h, w, H, W, _strides4(gs), N.strides4(g), ac,
                              gy_ptr=N.dev_ptr(gy) + c0 * gy.element_size())
            out.append(g)
            c0 += c
        return tuple(out)


def _strides4(st):
    import ctypes
    return (ctypes.c_int64 * 4)(*st)


def resize_cat(tensors, chans, size, align_corners=False):
    """cat_n of the bilinear resizes of `tensors` to `size` (NHWC activations, real channel counts `chans`) without
    materialising the resized maps.  Falls back to resize_act + cat_n where the slice writes cannot be 16-byte
    vectors (a channel offset not a multiple of 8)."""
    for t in tensors:
        _need_act(t, None, 'resize_cat')
    offs = [sum(chans[:i]) for i in range(len(chans))]
    if len(tensors) == 1 or any(o % 8 for o in offs) or any(c % 8 for c in chans):
        return cat_n([resize_act(t, size, align_corners) for t in tensors], chans)
    return _ResizeCatFn.apply((int(size[0]), int(size[1])), bool(align_corners), tuple(int(c) for c in chans),
                              *tensors)


def cat_n(tensors, chans):
    """Concatenate NHWC activations along channels; chans[i] = real channel count of tensors[i]."""
    for t in tensors:
        _need_act(t, None, 'cat_n')
    if len(tensors) == 1:
        return tensors[0]
    joins = None
    if torch.is_grad_enabled() and len({id(t) for t in tensors}) == len(tensors):
        joins = tuple(_join_fwd(t) for t in tensors)
        if all(j is None for j in joins):
            joins = None
    return _CatNFn.apply(tuple(int(c) for c in chans), joins, *tensors)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        n, c, h, w = x.shape
        oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        y = new_act(n, c, oh, ow, x.dtype, x.device)
        N.call('ssseg_avgpool_fwd', N.dev_ptr(x), N.dev_ptr(y), n, h, w, c, oh, ow, k, s, p, N.dt_code(x), N.stream())
        ctx.meta = (n, c, h, w, oh, ow, k, s, p, x.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        n, c, h, w, oh, ow, k, s, p, dt = ctx.meta
        _need_act(gy, c, 'AvgPool2d backward')
        gx = new_act(n, c, h, w, dt, gy.device)
        N.call('ssseg_avgpool_bwd', N.dev_ptr(gy), N.dev_ptr(gx), n, h, w, c, oh, ow, k, s, p, N.dt_code(gy),
               N.stream())
        return gx, None, None, None


def _int1(v):
    return v if isinstance(v, int) else v[0]


class AvgPool2d(nn.AvgPool2d):
    """nn.AvgPool2d (HarDNet's AvgPool2d(2, 2), hardnet.py:157) on NHWC activations."""

    def forward(self, x):
        if self.ceil_mode or not self.count_include_pad or self.divisor_override is not None:
            raise NotImplementedError('ssseg AvgPool2d: ceil_mode / count_include_pad=False / divisor_override')
        k, s, p = _int1(self.kernel_size), _int1(self.stride if self.stride is not None else self.kernel_size), \
            _int1(self.padding)
        _need_act(x, None, 'AvgPool2d')
        return _AvgPoolFn.apply(x, k, s, p)


class _GAPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        n, c, h, w = x.shape
        y = new_act(n, c, 1, 1, x.dtype, x.device)
        nb = N.lib().ssseg_global_avgpool_workspace_bytes(n, h * w, c)
        ws = N.workspace(nb, x.device)
        N.call('ssseg_global_avgpool_fwd', N.dev_ptr(x), N.dev_ptr(y), n, h * w, c, c, N.dt_code(x), N.dev_ptr(ws), nb,
               N.stream())
        ctx.meta = (n, c, h, w, x.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        n, c, h, w, dt = ctx.meta
        gx = new_act(n, c, h, w, dt, gy.device)
        gyc = gy if gy.is_contiguous(memory_format=torch.channels_last) else gy.contiguous(memory_format=torch.channels_last)
        N.call('ssseg_global_avgpool_bwd', N.dev_ptr(gyc), N.dev_ptr(gx), n, h * w, c, c, N.dt_code(gy), N.stream())
        return gx


def global_avgpool(x):
    """nn.AdaptiveAvgPool2d(1) on an NHWC activation -> [N, Cp, 1, 1] activation (ASPPPooling)."""
    _need_act(x, None, 'AdaptiveAvgPool2d(1)')
    return _GAPFn.apply(x)


class AdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    def forward(self, x):
        if self.output_size not in (1, (1, 1)):
            raise NotImplementedError('ssseg AdaptiveAvgPool2d: output size 1 only')
        return global_avgpool(x)


def _bilinear_bwd(gy, gx, n, c, h, w, oh, ow, gys4, gxs4, ac, gy_ptr=None):
    """gx = bilinear backward of gy (ssseg_bilinear_bwd_ws: two separable passes through an fp32 workspace)."""
    nb = N.lib().ssseg_bilinear_bwd_workspace_bytes(n, c, w, oh)
    ws = N.workspace(nb, gy.device)
    N.call('ssseg_bilinear_bwd_ws', gy_ptr if gy_ptr is not None else N.dev_ptr(gy), N.dev_ptr(gx), n, c, h, w, oh, ow,
           gys4, gxs4, int(ac), N.dt_code(gy), N.dev_ptr(ws), nb, N.stream())


class _ActBilinear(torch.autograd.Function):
    """F.interpolate(mode='bilinear') between NHWC activations (always channels_last in and out, including
    1x1 maps): HarDNet TransitionUp (hardnet.py:88), HRNet fuse / aggregation (higher_hrnet.py:454,1030),
    ASPPPooling's broadcast back to the feature size."""

    @staticmethod
    def forward(ctx, x, size, align_corners):
        n, c, h, w = x.shape
        oh, ow = int(size[0]), int(size[1])
        y = new_act(n, c, oh, ow, x.dtype, x.device)
        N.call('ssseg_bilinear_fwd', N.dev_ptr(x), N.dev_ptr(y), n, c, h, w, oh, ow, N.strides4(x), N.strides4(y),
               int(bool(align_corners)), N.dt_code(x), N.stream())
        ctx.meta = (n, c, h, w, oh, ow, bool(align_corners), x.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        n, c, h, w, oh, ow, ac, dt = ctx.meta
        gx = new_act(n, c, h, w, dt, gy.device)
        _bilinear_bwd(gy, gx, n, c, h, w, oh, ow, N.strides4(gy), N.strides4(gx), ac)
        return gx, None, None


def resize_act(x, size, align_corners=False):
    """Bilinear resize of an NHWC activation; same-size resizes are the identity (PyTorch's kernel copies)."""
    _need_act(x, None, 'bilinear resize')
    if (x.shape[2], x.shape[3]) == (int(size[0]), int(size[1])):
        return x
    return _ActBilinear.apply(x, tuple(int(v) for v in size), bool(align_corners))


class _AddNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, act, *ts):
        import ctypes
        code, slope = _act(act)
        y = torch.empty_like(ts[0])
        ptrs = (ctypes.c_void_p * len(ts))(*[N.dev_ptr(t) for t in ts])
        N.call('ssseg_add_n', ptrs, len(ts), N.dev_ptr(y), y.numel(), code, slope, N.dt_code(y), N.stream())
        ctx.code, ctx.slope, ctx.n = code, slope, len(ts)
        ctx.save_for_backward(y if code else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        if ctx.code:
            g = torch.empty_like(gy)
            N.call('ssseg_act_bwd', N.dev_ptr(gy), N.dev_ptr(y), N.dev_ptr(g), gy.numel(), ctx.code, ctx.slope,
                   N.dt_code(gy), N.stream())
        else:
            g = gy
        return (None,) + (g,) * ctx.n


def add_act(tensors, act=False):
    """act(t0 + t1 + ... ) over same-shape NHWC activations in one pass (higher_hrnet.py:473-486)."""
    if len(tensors) > 8:
        return add_act([add_act(tensors[:8], False)] + list(tensors[8:]), act)
    for t in tensors:
        if not _is_act(t) or t.shape != tensors[0].shape:
            raise ValueError(f'add_act: operands must be matching activations: {[tuple(t.shape) for t in tensors]}')
    if len(tensors) == 1 and not _act(act)[0]:
        return tensors[0]
    return _AddNFn.apply(act, *tensors)


# Philox key drawn once per process; the counter lives on the device (one int64 per device) and each dropout launch
# reserves its range with ssseg_rng_take, so a captured HIP graph draws fresh masks on every replay.  Same counter
# sequence as a host offset starting at 0: the forward of a call uses [ctr, ctr + ceil(n/4)], its backward the same.
_DROP = {'seed': None, 'ctr': {}}


def dropout_counter(device):
    c = _DROP['ctr'].get(device)
    if c is None:
        c = _DROP['ctr'][device] = torch.zeros(1, dtype=torch.int64, device=device)
    return c


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        if _DROP['seed'] is None:
            _DROP['seed'] = int(torch.randint(0, 2 ** 62, (1,)).item())
        seed = _DROP['seed']
        snap = torch.empty(1, dtype=torch.int64, device=x.device)
        N.call('ssseg_rng_take', N.dev_ptr(dropout_counter(x.device)), N.dev_ptr(snap), (x.numel() + 3) // 4 + 1,
               N.stream())
        y = torch.empty_like(x)
        N.call('ssseg_dropout_dev', N.dev_ptr(x), N.dev_ptr(y), x.numel(), float(p), seed, N.dev_ptr(snap),
               N.dt_code(x), N.stream())
        ctx.meta = (float(p), seed)
        ctx.save_for_backward(snap)
        return y

    @staticmethod
    def backward(ctx, gy):
        p, seed = ctx.meta
        snap, = ctx.saved_tensors
        gyc = gy if gy.is_contiguous(memory_format=torch.channels_last) else gy.contiguous(memory_format=torch.channels_last)
        gx = torch.empty_like(gyc)
        N.call('ssseg_dropout_dev', N.dev_ptr(gyc), N.dev_ptr(gx), gyc.numel(), p, seed, N.dev_ptr(snap),
               N.dt_code(gy), N.stream())
        return gx, None


class Dropout(nn.Dropout):
    """nn.Dropout on NHWC activations (DeepLabV3 ASPP projection, torchvision): a counter-based Philox mask
    regenerated in backward (nothing stored).  Identity in eval mode or with p == 0, like PyTorch."""

    def forward(self, x):
        if not self.training or self.p == 0:
            return x
        _need_act(x, None, 'Dropout')
        if x.numel() % 4:
            raise ValueError('ssseg Dropout: element count must be a multiple of 4')
        return _DropoutFn.apply(x, self.p)
