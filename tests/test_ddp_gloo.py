"""World-size-2 gloo (CPU) test of the data-parallel gradient reducer (ssseg/ddp.py): buckets over the
flat gradient arena, readiness-triggered launches, finish() joins, result = average over ranks."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from ssseg.ddp import DistributedDataParallel
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(64, 300), torch.nn.Linear(300, 70), torch.nn.Linear(70, 5))
        if rank == 1:        # different init on rank 1: the constructor must broadcast rank 0's weights
            with torch.no_grad():
                for p in model.parameters():
                    p.add_(1.0)
        ddp = DistributedDataParallel(model, bucket_cap_mb=0.05)
        assert len(ddp.buckets) > 1
        params = list(model.parameters())
        ref0 = [p.detach().clone() for p in params]
        # weights equal across ranks after the broadcast
        g = [torch.zeros_like(t) for t in range(world) for t in [ref0[0]]]
        dist.all_gather(g, ref0[0])
        assert torch.equal(g[0], g[1])
        # each rank's gradient = (rank + 1) * index pattern; the average is 1.5 * pattern
        for i, p in enumerate(params):
            p.grad.copy_(torch.arange(p.numel(), dtype=torch.float32).view_as(p) * (rank + 1) + i)
        ddp.arm()
        for p in reversed(params):        # readiness in backward order
            ddp.mark_ready(p)
        ddp.finish()
        ok = all(torch.allclose(p.grad, torch.arange(p.numel(), dtype=torch.float32).view_as(p) * 1.5 + i)
                 for i, p in enumerate(params))
        # an unarmed backward must not reduce
        for p in params:
            p.grad.fill_(float(rank))
            ddp.mark_ready(p)
        ok = ok and all(torch.all(p.grad == rank) for p in params)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_ddp_reducer_gloo_world2():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: True, 1: True}


def _worker_reuse(rank, world, port, q):
    """A parameter used twice per forward (MultiscaleAttention runs its base model twice,
    multiscale_attention.py:38-58) gets two gradient contributions per backward: its bucket must not be
    all-reduced before the second one lands."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from ssseg.ddp import DistributedDataParallel
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(64, 300), torch.nn.Linear(300, 70), torch.nn.Linear(70, 5))
        ddp = DistributedDataParallel(model, bucket_cap_mb=0.05)
        params = list(model.parameters())
        ok = True
        for step in range(3):
            for i, p in enumerate(params):
                p.grad.copy_(torch.arange(p.numel(), dtype=torch.float32).view_as(p) * (rank + 1) + i + step)
            ddp.arm()
            for p in reversed(params):          # first contribution (hi-res pass)
                ddp.mark_ready(p)
            ok = ok and not any(ddp._launched)   # nothing may be reduced yet
            for p in reversed(params):          # second contribution (lo-res pass)
                ddp.mark_ready(p)
            if step > 0:                        # counts learned on step 0: every bucket launched in backward
                ok = ok and all(ddp._launched) and ddp.last_early == len(ddp.buckets)
            ddp.finish()
            ok = ok and all(torch.allclose(p.grad, torch.arange(p.numel(), dtype=torch.float32).view_as(p) * 1.5
                                           + i + step) for i, p in enumerate(params))
        # a graph change (a third contribution after the bucket was launched) raises instead of racing
        ddp.arm()
        for _ in range(2):
            for p in reversed(params):
                ddp.mark_ready(p)
        try:
            ddp.mark_ready(params[-1])
            ok = False
        except RuntimeError:
            pass
        ddp.finish()
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_ddp_reducer_gloo_world2_reused_params():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_reuse, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: True, 1: True}


def _meters_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import train
        from utils import utils
        # reduce_tensor (reference utils/utils.py:43-54): SUM onto rank 0 in place, others untouched
        t = torch.tensor([float(rank + 1), 10.0 * (rank + 1)])
        out = utils.reduce_tensor(t.clone())
        # epoch-end meter reduction (train._reduce_meters): one all-reduce of the stacked sums / world
        meters = {'a': utils.AverageMeter(), 'b': utils.AverageMeter()}
        meters['a'].update(torch.tensor(2.0 * (rank + 1)))
        meters['b'].update(torch.tensor(-1.0 * (rank + 1)), 3)
        train._reduce_meters(meters, ['a', 'b'], world)
        q.put((rank, out.tolist(), float(meters['a'].sum), float(meters['b'].sum)))
    finally:
        dist.destroy_process_group()


def test_reduce_tensor_and_meters_gloo_world2():
    """utils.reduce_tensor and the epoch-end meter all-reduce at world size 2 (reference utils/utils.py:43-54,
    train.py:53-59,109-114)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_meters_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == [3.0, 30.0]          # rank 0 holds the sum
    assert res[1][0] == [2.0, 20.0]          # rank 1's tensor is not the destination
    assert res[0][1] == res[1][1] == 3.0     # (2 + 4) / 2
    assert res[0][2] == res[1][2] == -4.5    # (-3 + -6) / 2


def _tune_worker(rank, world, port, q):
    """rank 0's conv variant table reaches every rank (ssseg.tune): the ranks > 0 stop tuning (knob 5 = 0) until
    sync(), which imports rank 0's rows over their own (static-rule) picks; afterwards every digest is equal."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from ssseg import tune
        tune.follow_rank0()
        # a table as each rank would have it after the warm-up: rank 0's tuned picks, the others' static rule (and
        # rank 1 saw one geometry rank 0 keeps too)
        rows0 = [(11, 3), (12, 14), (13, 26), (99, 6)]
        rows1 = [(11, 0), (12, 5), (13, 5)]
        tune.import_(rows0 if rank == 0 else rows1, overwrite=True)
        before = tune.digest()
        tune.sync()
        got = dict(tune.export())
        q.put((rank, before, tune.digests(), got, tune.synced()))
    finally:
        dist.destroy_process_group()


def test_tune_table_sync_gloo_world2():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_tune_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(30)
    (b0, d0, t0, s0), (b1, d1, t1, s1) = res[0], res[1]
    assert b0 != b1                       # the ranks disagreed before the sync
    assert d0 == d1 and len(set(d0)) == 1  # ... and agree after it
    assert t1[11] == 3 and t1[12] == 14 and t1[13] == 26 and t1[99] == 6 and t0 == t1
    assert s0 and s1


def _comm_worker(rank, world, port, q):
    """ssseg.comm on a gloo group: no native communicator (RCCL needs the nccl backend and GPU tensors), the SyncBN sum
    helper falls through to torch.distributed and sums across ranks; kind() reports the transport bench.py prints."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from ssseg import comm
        t = torch.full((4,), float(rank + 1), dtype=torch.float64)
        comm.all_reduce_sum(t)
        q.put((rank, comm.wanted(), comm.get(), comm.kind(), t.tolist()))
    finally:
        dist.destroy_process_group()


def test_comm_falls_back_to_c10d_on_gloo():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(30)
    for r in range(2):
        wanted, c, kind, vals = res[r]
        assert wanted is False and c is None and kind == 'c10d'
        assert vals == [3.0] * 4
