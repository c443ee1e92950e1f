"""World-size-2 data-parallel training step of the PRODUCT path on the GPU (reference
distributed_trainer.py:33-44: DDP + SyncBatchNorm, train.py:41-130 on every rank).

Two processes share the one MI355X of the test box and talk over gloo on HIP tensors (RCCL cannot put
two ranks on one device; on an 8-GPU node bench.py runs the same code over RCCL).  Each rank runs
train.train_step on its own half of the batch through ssseg.nn (SyncBN: the fp64 statistic sums are
all-reduced in forward and backward) and ssseg.ddp (bucketed all-reduce on the side HIP stream, buckets
launched from inside the backward once their gradient contributions have landed).  The oracle
(oracle/train_ref.train_epoch_dp) runs the same steps in one process on the concatenated batch.
Checked: per-rank losses, the averaged gradients after step 0 (no optimizer step there, train.py:121),
BN running statistics, student and teacher parameters after 3 steps, and that buckets were really
launched early from the side stream in the steps after the first (learning) one."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, H, STEPS, WORLD = 2, 32, 3, int(os.environ.get('SSSEG_DDP_WORLD', '2'))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(world=WORLD):
    g = torch.Generator().manual_seed(11)
    imgs = torch.rand(STEPS, world, B, 3, H, H, generator=g)
    fg = (torch.rand(STEPS, world, B, 1, H, H, generator=g) > 0.5).float()
    masks = torch.cat([1 - fg, fg], 3)
    unl = torch.rand(STEPS, world, 2, B, 3, H, H, generator=g)
    if 'same' in os.environ.get('SSSEG_DDP_DIAG', ''):
        imgs[:] = imgs[0].clone()
        masks[:] = masks[0].clone()
    return imgs, masks, unl


def _model():
    from models import simple_unet
    from models.adapters import ListOutput
    torch.manual_seed(0)
    return ListOutput(simple_unet.UNet(2, num_blocks=3, first_channels=8, max_width=32))


def _cfg(semi=True):
    import losses
    return dict(loss=losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits('mean'),
                                           'weight': [0.5]}]),
                virtual_batch_size_multiplier=1, use_semi_supervised=semi, mask_proportion_range=(0.45, 0.55),
                sigma_range=(2, 4), confidence_threshold=0.5, consistency_loss_weight=10, ema_model_alpha=0.99,
                print_freq=1, gradient_clip_value=5.0)


class _CollectiveLog:
    """Counts every torch.distributed.all_reduce of the step (ssseg.ddp's gradient buckets, ssseg.nn's SyncBN
    statistic sums, utils.reduce_tensor): (tensor dtype, bytes) per call."""
    def __init__(self, dist):
        from ssseg import comm
        self.calls, self._orig, self._dist = [], dist.all_reduce, dist
        self._comm_cls, self._orig_native = comm.NativeComm, comm.NativeComm.all_reduce

        def wrapped(tensor, *a, **k):
            self.calls.append((str(tensor.dtype), tensor.numel() * tensor.element_size()))
            return self._orig(tensor, *a, **k)
        dist.all_reduce = wrapped

        def wrapped_native(comm_self, tensors, *a, **k):   # the native communicator (RCCL groups): one row per tensor
            for t in tensors:
                self.calls.append((str(t.dtype), t.numel() * t.element_size()))
            return self._orig_native(comm_self, tensors, *a, **k)
        comm.NativeComm.all_reduce = wrapped_native

    def restore(self):
        self._dist.all_reduce = self._orig
        self._comm_cls.all_reduce = self._orig_native

    def take(self):
        c, self.calls = self.calls, []
        return c


def _worker(rank, port, q, semi, world=WORLD):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import cowmix
        import train
        from ssseg import arena, optim
        from ssseg import nn as snn
        from ssseg.ddp import DistributedDataParallel
        dev = torch.device('cuda:0')
        snn.set_compute_dtype(torch.float32)
        diag = os.environ.get('SSSEG_DDP_DIAG', '')
        if 'notune' in diag:
            from ssseg import native as N
            N.call('ssseg_set_knob', 5, 0)
        if 'nofuse' in diag:
            snn.set_fused_bn_stats(False)
        student = _model().to(dev)
        teacher = _model().to(dev)
        for p in teacher.parameters():
            p.detach_()
        teacher.eval()
        model = DistributedDataParallel(student, bucket_cap_mb=0.02)
        arena.attach(teacher, with_grads=False)
        opt = optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
        imgs, masks, unl = _data(world)
        cowmix.NOISE_SOURCE = 'cpu'
        import utils.utils as utils
        log = _CollectiveLog(dist)
        collectives, reduced = [], []
        torch.manual_seed(3)
        model.train()
        opt.zero_grad()
        early, losses, grads = [], [], []
        orig_step = opt.step

        def step_and_record(*a, **k):     # the averaged gradients each optimizer step consumes
            grads.append({n: p.grad.detach().cpu().numpy().copy() for n, p in student.named_parameters()})
            return orig_step(*a, **k)
        opt.step = step_and_record
        for step in range(STEPS):
            c, u, _ = train.train_step(model, teacher, opt, imgs[step, rank].to(dev), masks[step, rank].to(dev),
                                       unl[step, rank, 0].to(dev), unl[step, rank, 1].to(dev), 30, step,
                                       {'train': _cfg(semi)})
            torch.cuda.synchronize()
            collectives.append(log.take())
            # the reference's logging reduction (utils.py:43-54) on the device loss scalars: sum over ranks
            red = utils.reduce_tensor(c.clone())
            reduced.append((str(red.device), float(red) / world))
            losses.append((float(c), float(u) if u is not None else 0.0))
            early.append(model.last_early)
            if step == 0:    # no optimizer step at step 0 (train.py:121): its gradients stay accumulated
                grads.append({n: p.grad.detach().cpu().numpy().copy() for n, p in student.named_parameters()})
                if os.environ.get('SSSEG_DDP_DIAG') == 'zero':
                    opt.zero_grad()
        # numpy (pickled by value): torch CPU tensors would travel as shared-memory fds that die with this process
        n_bn = sum(1 for m in student.modules() if isinstance(m, snn.BatchNorm2d))
        out = dict(losses=losses, early=early, nbuckets=len(model.buckets), grads=grads, collectives=collectives,
                   reduced=reduced, n_bn=n_bn, bn_channels=[m.num_features for m in student.modules()
                                                             if isinstance(m, snn.BatchNorm2d)],
                   bucket_bytes=[4 * (e - s0) for s0, e, _ in model.buckets],
                   student={k: v.detach().cpu().numpy().copy() for k, v in student.state_dict().items()},
                   teacher={k: v.detach().cpu().numpy().copy() for k, v in teacher.state_dict().items()})
        q.put((rank, out))
    except Exception as exc:   # report to the parent instead of hanging it
        import traceback
        q.put((rank, 'ERROR ' + repr(exc) + '\n' + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _oracle(dt=torch.float32, semi=True, pert=0.0, world=WORLD):
    from oracle import models_ref, train_ref
    torch.manual_seed(0)
    s = models_ref.ListOutput(models_ref.SimpleUNet(2, 3, 8, 32))
    t = models_ref.ListOutput(models_ref.SimpleUNet(2, 3, 8, 32))
    t.load_state_dict(_model().state_dict())
    s.load_state_dict(_model().state_dict())
    s, t = s.to(dt), t.to(dt)
    for p in t.parameters():
        p.detach_()
    t.eval()
    opt = torch.optim.SGD(s.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    imgs, masks, unl = (v.to(dt) for v in _data(world))
    if pert:    # the step's own sensitivity: inputs moved by ~fp32 rounding after a few layers
        g = torch.Generator().manual_seed(99)
        imgs = imgs * (1 + pert * torch.randn(imgs.shape, generator=g, dtype=dt))
        unl = unl * (1 + pert * torch.randn(unl.shape, generator=g, dtype=dt))
    cfg = train_ref.default_cfg(sigma_range=(2, 4), confidence_threshold=0.5, use_semi_supervised=semi)
    grads = []

    def on_step(step, rec):
        grads.append({n: p.grad.detach().clone() for n, p in s.named_parameters()})
        if step == 0 and os.environ.get('SSSEG_DDP_DIAG') == 'zero':
            opt.zero_grad()
    torch.manual_seed(3)
    logs = train_ref.train_epoch_dp(s, t, opt, [[(imgs[k, r], masks[k, r]) for r in range(world)] for k in range(STEPS)],
                                    [[(unl[k, r, 0], unl[k, r, 1]) for r in range(world)] for k in range(STEPS)], 30,
                                    cfg, on_step=on_step)
    return logs, grads, s.state_dict(), t.state_dict()


@pytest.mark.parametrize('semi,world', [(False, WORLD), (True, WORLD), (True, 4)])
@pytest.mark.timeout(400)
def test_ddp_syncbn_product_path(hip_device, semi, world):
    """world 2 (both step kinds) and world 4 (semi-supervised): 4 ranks share the one GPU over gloo -- the same
    product code an 8-GPU node runs over RCCL."""
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, semi, world)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, out = q.get(timeout=300)
            res[r] = out
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    _check_collectives(res, world)
    failures = []
    logs, g_ref, s_ref, t_ref = _oracle(semi=semi, world=world)
    logs64, g64, s64, t64 = _oracle(torch.float64, semi=semi, world=world)
    # ReLU / max-pool switches sit within ~1e-6 of these tiny-batch activations: a 1e-6 relative input
    # perturbation moves the fp64 oracle's step-1 gradients by ~1 % (measured).  After step 0 the bound is
    # therefore 2x the larger of the fp32 oracle's drift and this perturbation drift (tests/parity.py's rule).
    _, gp, sp, tp = _oracle(torch.float64, semi=semi, pert=1e-6, world=world)
    for r in range(world):
        out = res[r]
        for k, (c, u) in enumerate(out['losses']):
            np.testing.assert_allclose(c, logs[k]['sup_loss'][r], rtol=1e-4)
            if semi:   # tests/parity.py's loss rule: within max(1e-3 rel, 2x the fp32 oracle's own drift) of fp64
                u64, u32 = logs64[k]['unsup_loss'][r], logs[k]['unsup_loss'][r]
                assert abs(u - u64) <= max(1e-3 * abs(u64), 2 * abs(u32 - u64)) + 1e-9, (k, r, u, u32, u64)
        assert out['nbuckets'] > 2
        assert out['early'][0] == 0                       # first armed backward learns the counts
        if os.environ.get('SSSEG_DDP_OVERLAP', '1') != '0' and world > 1:
            assert all(e > 0 for e in out['early'][1:]), out['early']   # later ones launch from the backward
        # averaged gradients of every step vs fp64: per tensor within max(1e-3, 2x the fp32 oracle's own drift)
        # of the tensor's scale, floored at 1e-3 of the model's largest gradient (a conv bias feeding a
        # BatchNorm has a mathematically zero gradient: rounding noise on every side)
        gbad = []
        for k in range(STEPS):
            gmax = max(float(g.abs().max()) for g in g64[k].values())
            for n, g in g64[k].items():
                b = g.numpy()
                a, c, d = out['grads'][k][n], g_ref[k][n].numpy(), gp[k][n].numpy()
                scale = max(np.abs(b).max(), 1e-3 * gmax)
                e_hip, e_32 = float(np.abs(a - b).max()) / scale, float(np.abs(c - b).max()) / scale
                e_p = float(np.abs(d - b).max()) / scale if k > 0 else 0.0
                if e_hip > max(1e-3, 2 * e_32, 2 * e_p):
                    gbad.append((k, n, e_hip, e_32, e_p))
        print('rank', r, 'gradient outliers (step, tensor, hip vs fp64, ref32 vs fp64):', gbad[:8])
        for k in range(STEPS):
            gmax = max(float(g.abs().max()) for g in g64[k].values())
            worst = max((float(np.abs(out['grads'][k][n] - g.numpy()).max()) / max(float(g.abs().max()), 1e-3 * gmax), n)
                        for n, g in g64[k].items())
            print(f'rank {r} step {k} worst grad err vs fp64 {worst}')
        if r == 1 and world == 2:
            for k in range(STEPS):
                d = max(float(np.abs(res[0]['grads'][k][n] - res[1]['grads'][k][n]).max()) for n in g64[k])
                print(f'step {k} max |grad rank0 - grad rank1| = {d}')
        if gbad:
            failures.append(gbad[:8])
        # parameters / buffers after 3 steps vs an fp64 oracle run: within max(1e-3, 2x the fp32 oracle's own
        # drift) of each tensor's scale (tests/parity.py's rule)
        bad = []
        for name, got, ref, ref64, refp in (('student', out['student'], s_ref, s64, sp),
                                            ('teacher', out['teacher'], t_ref, t64, tp)):
            for k, v in ref.items():
                a, b, c, d = got[k], ref64[k].numpy(), v.numpy(), refp[k].numpy()
                if not np.issubdtype(b.dtype, np.floating):
                    assert np.array_equal(a, c), (name, k)
                    continue
                scale = np.abs(b).max() + 1e-6
                e_hip = float(np.abs(a - b).max()) / scale
                e_32 = float(np.abs(c - b).max()) / scale
                e_p = float(np.abs(d - b).max()) / scale
                if e_hip > max(1e-3, 2 * e_32, 2 * e_p):
                    bad.append((r, name, k, e_hip, e_32, e_p))
        print('rank', r, 'worst tensors (hip vs fp64, ref32 vs fp64):', sorted(bad, key=lambda x: -x[3])[:5])
        if bad:
            failures.append(bad[:5])
    assert not failures, failures
    # both ranks hold identical weights (averaged gradients, broadcast init)
    for k in res[0]['student']:
        assert np.array_equal(res[0]['student'][k], res[world - 1]['student'][k]), k
    # utils.reduce_tensor on the device loss scalars (reference utils.py:43-54, dist.reduce SUM to rank 0): rank 0
    # holds the mean of every rank's supervised loss
    for k in range(STEPS):
        dev, mean = res[0]['reduced'][k]
        assert dev.startswith('cuda'), dev
        np.testing.assert_allclose(mean, np.mean([res[r]['losses'][k][0] for r in range(world)]), rtol=1e-6)


def _check_collectives(res, world):
    """Per-step collective count and bytes on every rank: one all-reduce per gradient bucket (fp32,
    together exactly the flat gradient arena) + 2 SyncBN all-reduces per training BatchNorm (forward (sum, sum^2)
    and backward (sum dy, sum dy*xhat), fp64 [2C] each) -- the eval-mode consistency pass and the teacher run none."""
    for r in range(world):
        out = res[r]
        n_bn, bn_c = out['n_bn'], out['bn_channels']
        for k, calls in enumerate(out['collectives']):
            f64 = [b for d, b in calls if d == 'torch.float64']
            f32 = [b for d, b in calls if d == 'torch.float32']
            assert len(calls) == len(f64) + len(f32), calls
            assert len(f64) == 2 * n_bn, (r, k, len(f64), n_bn)
            assert sum(f64) == 2 * sum(2 * c * 8 for c in bn_c), (r, k, sum(f64))
            assert len(f32) == out['nbuckets'], (r, k, len(f32), out['nbuckets'])
            assert sum(f32) == sum(out['bucket_bytes']), (r, k, sum(f32))


def _worker_rccl(port, q):
    """world-1 RCCL process group with the collectives forced on (ssseg.ddp.force_collectives): the bucketed
    ReduceOp.AVG all-reduces on the side HIP stream, their event join and SyncBN's fp64 all-reduces all execute on
    RCCL; the same steps without DDP / process group must give bit-identical gradients and parameters."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    try:
        import cowmix
        import train
        from ssseg import arena, ddp, optim
        from ssseg import native as N
        from ssseg import nn as snn
        dev = torch.device('cuda:0')
        torch.cuda.set_device(dev)
        N.call('ssseg_set_knob', 5, 0)          # static variants: both runs launch the same kernels
        snn.set_compute_dtype(torch.bfloat16)
        cowmix.NOISE_SOURCE = 'cpu'
        imgs, masks, unl = _data(1)

        def run(distributed):
            student, teacher = _model().to(dev), _model().to(dev)
            for p in teacher.parameters():
                p.detach_()
            teacher.eval()
            model = ddp.DistributedDataParallel(student, bucket_cap_mb=0.02) if distributed else student
            if not distributed:
                arena.attach(student)
            arena.attach(teacher, with_grads=False)
            opt = optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
            grads, early, calls = [], [], []
            orig_step = opt.step

            def rec(*a, **k):
                grads.append([p.grad.detach().clone() for p in student.parameters()])
                return orig_step(*a, **k)
            opt.step = rec
            log = _CollectiveLog(dist) if distributed else None
            torch.manual_seed(3)
            model.train()
            opt.zero_grad()
            for step in range(STEPS):
                train.train_step(model, teacher, opt, imgs[step, 0].to(dev), masks[step, 0].to(dev),
                                 unl[step, 0, 0].to(dev), unl[step, 0, 1].to(dev), 30, step, {'train': _cfg(True)})
                torch.cuda.synchronize()
                if step == 0:
                    grads.append([p.grad.detach().clone() for p in student.parameters()])
                if distributed:
                    early.append(model.last_early)
                    calls.append(log.take())
            if log is not None:
                log.restore()
            n_bn = sum(1 for m in student.modules() if isinstance(m, snn.BatchNorm2d))
            return (grads, [v.detach().clone() for v in student.state_dict().values()],
                    [v.detach().clone() for v in teacher.state_dict().values()], early, calls, n_bn,
                    len(model.buckets) if distributed else 0)

        dist.init_process_group('nccl', rank=0, world_size=1)
        ddp.force_collectives(True)
        got = run(True)
        ddp.force_collectives(False)
        ref = run(False)
        from ssseg import comm
        out = {'backend': dist.get_backend(), 'transport': comm.kind(), 'early': got[3], 'nbuckets': got[6],
               'n_bn': got[5],
               'ncalls': [len(c) for c in got[4]], 'mismatch': []}
        for k, (ga, gb) in enumerate(zip(got[0], ref[0])):
            for i, (a, b) in enumerate(zip(ga, gb)):
                if not torch.equal(a, b):
                    out['mismatch'].append(('grad', k, i, float((a.float() - b.float()).abs().max())))
        for name, xa, xb in (('student', got[1], ref[1]), ('teacher', got[2], ref[2])):
            for i, (a, b) in enumerate(zip(xa, xb)):
                if not torch.equal(a, b):
                    out['mismatch'].append((name, i))
        out['ngrads'] = len(got[0])
        q.put(out)
    except Exception as exc:
        import traceback
        q.put('ERROR ' + repr(exc) + '\n' + traceback.format_exc())
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_rccl_world1_forced_collectives_bitwise(hip_device):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_worker_rccl, args=(_free_port(), q))
    p.start()
    try:
        out = q.get(timeout=300)
    finally:
        p.join(30)
        if p.is_alive():
            p.kill()
    assert not isinstance(out, str), out
    assert out['backend'] == 'nccl'
    assert out['transport'] == 'native'     # the step's collectives went through libssseg's RCCL communicator
    assert out['ngrads'] == STEPS
    # the learning backward launches every bucket in finish(); later armed backwards launch from inside the backward
    assert out['early'][0] == 0 and all(e > 0 for e in out['early'][1:]), out['early']
    # per step: one AVG all-reduce per bucket + (sum, sum^2) and (sum dy, sum dy*xhat) per training BatchNorm
    assert all(n == out['nbuckets'] + 2 * out['n_bn'] for n in out['ncalls']), out['ncalls']
    assert not out['mismatch'], out['mismatch'][:10]



def _worker_rccl_graph(port, q):
    """world-1 RCCL process group, collectives forced on, on the native communicator (ssseg.comm): the C2 step (UNet-R50
    at 64², bs 2, bench.build: DDP + SyncBN, teacher pass and consistency forward on the side stream) run eagerly and
    replayed from a captured HIP graph must give bit-identical losses, parameters, running statistics and teacher
    weights -- and equal the same steps without any collective."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    try:
        import bench
        import cowmix
        import train
        from ssseg import comm, ddp
        from ssseg import native as N
        from ssseg import nn as snn
        from ssseg.graph import StepGraph
        dev = torch.device('cuda:0')
        torch.cuda.set_device(dev)
        N.call('ssseg_set_knob', 5, 0)          # static variants: every run launches the same kernels
        snn.set_compute_dtype(torch.bfloat16)
        cowmix.NOISE_SOURCE = 'device'
        dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
        steps, size, batch = 3, 64, 2

        def run(mode):
            ddp.force_collectives(mode != 'plain')
            model, teacher, opt, cfg = bench.build(batch, size, dev)
            data = bench.synthetic_batches(steps + 2, batch, size, dev, 0)
            for c in cowmix._DEVICE_RNG['ctr'].values():
                c.zero_()
            model.train()
            opt.zero_grad()
            log = _CollectiveLog(dist)
            losses = [train.train_step(model, teacher, opt, *data[k], 30, k, cfg) for k in range(2)]
            torch.cuda.synchronize()
            eager_calls = len(log.take())
            replays = 0
            if mode == 'graph':
                g = StepGraph(lambda i, m, a, b: train.train_step(model, teacher, opt, i, m, a, b, 30, 2, cfg),
                              *data[2])
                capture_calls = len(log.take())
                for k in range(2, steps + 2):
                    losses.append(tuple(t.clone() for t in g(*data[k])))
                    replays += 1
                replay_calls = len(log.take())     # a replay issues nothing from Python
            else:
                for k in range(2, steps + 2):
                    losses.append(train.train_step(model, teacher, opt, *data[k], 30, k, cfg))
                capture_calls = replay_calls = None
            torch.cuda.synchronize()
            log.restore()
            ddp.force_collectives(False)
            state = {**{'s.' + k: v.detach().clone() for k, v in model.state_dict().items()},
                     **{'t.' + k: v.detach().clone() for k, v in teacher.state_dict().items()}}
            n_bn = sum(1 for m in model.modules() if isinstance(m, snn.BatchNorm2d))
            nb = len(model.buckets) if getattr(model, '_active', False) else 0
            return dict(losses=[tuple(float(t) for t in l) for l in losses], state=state, eager_calls=eager_calls,
                        capture_calls=capture_calls, replay_calls=replay_calls, replays=replays, n_bn=n_bn, nb=nb)

        eager = run('eager')
        graph = run('graph')
        plain = run('plain')
        out = {'transport': comm.kind(), 'losses': (eager['losses'], graph['losses'], plain['losses']),
               'eager_calls': eager['eager_calls'], 'capture_calls': graph['capture_calls'],
               'replay_calls': graph['replay_calls'], 'replays': graph['replays'], 'n_bn': eager['n_bn'],
               'nb': eager['nb'], 'plain_calls': plain['eager_calls'], 'mismatch': []}
        for name, other in (('graph', graph), ('plain', plain)):
            for k in eager['state']:
                if not torch.equal(eager['state'][k], other['state'][k]):
                    out['mismatch'].append((name, k))
        out['finite'] = all(np.isfinite(v).all() for v in eager['losses'])
        q.put(out)
    except Exception as exc:
        import traceback
        q.put('ERROR ' + repr(exc) + '\n' + traceback.format_exc())
    finally:
        if dist.is_initialized():
            from ssseg import comm
            comm.reset()
            dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_rccl_world1_captured_step_bitwise(hip_device):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_worker_rccl_graph, args=(_free_port(), q))
    p.start()
    try:
        out = q.get(timeout=300)
    finally:
        p.join(30)
        if p.is_alive():
            p.kill()
    assert not isinstance(out, str), out
    assert out['transport'] == 'native'
    e, g, pl = out['losses']
    assert out['finite'], e
    assert e == g, (e, g)              # captured replay == eager, bitwise
    assert e == pl, (e, pl)            # world-1 collectives change nothing
    assert not out['mismatch'], out['mismatch'][:10]
    # two eager steps: one AVG bucket group per gradient bucket + 2 SyncBN sums per training BatchNorm, each step;
    # the capture records one step's worth, a replay issues none from Python
    per_step = out['nb'] + 2 * out['n_bn']
    assert out['nb'] >= 1 and out['n_bn'] > 0
    assert out['eager_calls'] == 2 * per_step, (out['eager_calls'], per_step)
    assert out['capture_calls'] == per_step, (out['capture_calls'], per_step)
    assert out['replays'] == 3 and out['replay_calls'] == 0, out
    assert out['plain_calls'] == 0
