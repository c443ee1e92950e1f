"""Benchmark: semi-supervised training throughput of UNet-ResNet50 512x512 (BASELINE.json config C2).

One "step" = one full reference training step (reference train.py:44-130) on one batch per GPU:
student forward + BCE loss + backward, two teacher forwards + resize, CowMix mask + mixing, student
consistency forward (eval BN) + consistency loss + backward, clip + SGD step, EMA update — all on the
libssseg.so kernels, bf16 activations/weights with fp32 accumulation, fp32 master weights and EMA.
Inputs are synthetic and pre-generated in HBM (8 batches cycled); weights random-init.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--size S] [--no-cpu-baseline]

N>1: when WORLD_SIZE is not set, bench.py itself starts torch.distributed.run as a child process
(before any GPU call) with one rank per GPU on RCCL; under an external launcher it joins as a rank.
value = images/sec of the whole job (labeled images, N*B*K / max-over-ranks time).  Rank 0 prints
ONE JSON line.

Liveness: the timed steps run the reference arithmetic with confidence_threshold 0.5 (stated in the
JSON): at the reference default 0.97 a random-init teacher has no confident pixel, so the consistency
loss is 0/0 = NaN and the weights turn NaN; the threshold does not change the work a step
does.  Every timed step's losses are checked finite after the timed region and cm_mean is reported.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd')
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BF16_DENSE_PEAK = 2.5e15        # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
FWD_GFLOP_PER_IMAGE = 95.94     # UNet-R50 mw128 ConvT @512 (verified by tests/test_models_host.py)
# conv-engine HBM bytes of one step from rocprofv3 PMC (tools/pmc_step.py; FETCH_SIZE x2 + WRITE_SIZE, the
# MI355X_MICROARCH.md gfx950 correction).  PMC cannot run inside the timed process, so the committed
# measurement of the same workload is reported next to the live flop rate.
THRESHOLD = 0.5                 # see the module docstring (liveness)
PROBE_HOLD_CYCLES = int(3e8)    # spin of the instrumented step's head (~0.12 s at the shader clock; see timed_run)
PMC_PROFILE = os.path.join(ROOT, 'profiles', 'r6_pmc_traffic.json')
# MFMA utilisation of the same workload from rocprofv3 PMC (tools/pmc_step.py --mfma: SQ_VALU_MFMA_BUSY_CYCLES over
# 1024 SIMDs x GRBM_GUI_ACTIVE / 8), committed next to the traffic; like the traffic it cannot be collected inside
# the timed process
PMC_MFMA = os.path.join(ROOT, 'profiles', 'r6_pmc_mfma.json')


def pmc_traffic():
    try:
        with open(PMC_PROFILE) as fh:
            return int(json.load(fh)['traffic_bytes'])
    except (OSError, KeyError, ValueError):
        return None


def pmc_mfma():
    try:
        with open(PMC_MFMA) as fh:
            d = json.load(fh)
        return {'conv_engine_mfma_util': d['conv_engine']['mfma_util'],
                'conv_engine_counted_gflop': d['conv_engine']['implied_gflop'],
                'whole_step_mfma_util': d['whole_step']['mfma_util'],
                'source': os.path.relpath(PMC_MFMA, ROOT) + ' (rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES '
                                                          'GRBM_GUI_ACTIVE; util = busy SIMD-cycles / (1024 x active '
                                                          'cycles))'}
    except (OSError, KeyError, ValueError, TypeError):
        return None


def build(batch, size, device):
    import losses
    from models import unet
    from models.adapters import ListOutput
    from models.encoders import resnet
    from ssseg import arena, optim
    from ssseg.ddp import DistributedDataParallel
    torch.manual_seed(0)
    student = ListOutput(unet.UNet(2, resnet.resnet50_encoder(), max_width=128, train_upsampling=True)).to(device)
    teacher = ListOutput(unet.UNet(2, resnet.resnet50_encoder(), max_width=128, train_upsampling=True)).to(device)
    for p in teacher.parameters():
        p.detach_()
    teacher.eval()
    model = DistributedDataParallel(student)
    arena.attach(teacher, with_grads=False)
    opt = optim.SGD(model.parameters(), lr=0.0001 * 9 / 4, momentum=0.9, weight_decay=0.0005)
    cfg = {'train': dict(
        loss=losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits('mean'), 'weight': [0.5]}]),
        virtual_batch_size_multiplier=1, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
        sigma_range=(8, 32), consistency_loss_weight=10, ema_model_alpha=0.99, confidence_threshold=THRESHOLD,
        gradient_clip_value=5.0, print_freq=10 ** 9)}
    return model, teacher, opt, cfg


def synthetic_batches(n_batches, batch, size, device, rank):
    """images U[0,1); masks = one-hot of smoothed-noise blobs (sigma 16, p 0.4)."""
    from ssseg import ops
    g = torch.Generator().manual_seed(1000 + rank)
    data = []
    for _ in range(n_batches):
        img = torch.rand(batch, 3, size, size, generator=g).to(device)
        noise = torch.randn(batch, 1, size, size, generator=g).to(device)
        fg = ops.cowmix_mask(noise, torch.full((batch,), 16.0, device=device), torch.full((batch,), 0.6, device=device))
        mask = torch.cat([1 - fg, fg], 1)
        ua = torch.rand(batch, 3, size, size, generator=g).to(device)
        ub = torch.rand(batch, 3, size, size, generator=g).to(device)
        data.append((img, mask.contiguous(), ua, ub))
    return data


def _cpu_threads():
    """the node's host cores (sched_getaffinity), capped by OMP_NUM_THREADS when the launcher
    sets it (the GPU box gives each GPU a share of the host: 16 threads, set there)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get('OMP_NUM_THREADS')
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(size, batch=2, steps=3):
    """The oracle's torch-CPU restatement of the same step (oracle/train_ref.py), bounded sample: batch 2,
    1 warm-up + `steps` timed steps on the host's cores.  tests/golden/time_cpu_baseline.py
    shows, in the build container, that this restatement runs at the reference train.train's own speed
    (profiles/r3_cpu_baseline_check.json)."""
    from oracle import models_ref, train_ref
    threads = _cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(0)
        s = models_ref.ListOutput(models_ref.UNet(2, models_ref.resnet50_encoder(), 128, train_upsampling=True))
        t = models_ref.ListOutput(models_ref.UNet(2, models_ref.resnet50_encoder(), 128, train_upsampling=True))
        t.load_state_dict(s.state_dict())
        for p in t.parameters():
            p.detach_()
        t.eval()
        opt = torch.optim.SGD(s.parameters(), lr=0.0001 * 9 / 4, momentum=0.9, weight_decay=0.0005)
        g = torch.Generator().manual_seed(7)
        n = steps + 1
        imgs = torch.rand(n, batch, 3, size, size, generator=g)
        fg = (torch.rand(n, batch, 1, size, size, generator=g) > 0.5).float()
        masks = torch.cat([1 - fg, fg], 2)
        unl = torch.rand(2 * n, batch, 3, size, size, generator=g)
        cfg = train_ref.default_cfg(confidence_threshold=THRESHOLD)
        times = []
        t0 = time.perf_counter()
        train_ref.train_epoch(s, t, opt, list(zip(imgs, masks)), iter(unl), 30, cfg,
                              on_step=lambda step, rec: times.append(time.perf_counter()))
        dt = (times[-1] - times[0]) / steps     # the first step is the warm-up
        return {'value': round(batch / dt, 4), 'unit': 'images/sec', 'cores': threads, 'kind': 'port',
                'sample': f'oracle/train_ref.py torch-CPU fp32 semi-supervised step (the same C2 step), UNet-R50 '
                          f'{size}x{size}, batch {batch}, {steps} timed steps after 1 warm-up '
                          f'({time.perf_counter() - t0:.1f} s total)'}
    finally:
        torch.set_num_threads(prev)


def parity_leg(student, size, device, n_img=4):
    """mIoU / Dice parity (BASELINE.json metric '...; mIoU parity'): the benched student (after
    its timed steps, running BN statistics included) validated on the same synthetic validation images by the
    HIP path (ssseg_seg_metrics: argmax -> nearest resize -> Dice counts + lovasz.iou confusion counts,
    train.validate) in the fp32 parity mode and in the bf16 throughput mode, and by the oracle (torch-CPU fp32
    restatement of the network, numpy restatement of the metrics, reference train.py:171-176, metrics.py:1-7,
    lovasz.py:54-73) on the same weights.  Part of the CPU-baseline leg (the oracle is the checker)."""
    from oracle import losses_ref, models_ref
    from ssseg import nn as snn
    from ssseg import ops
    import numpy as np
    g = torch.Generator().manual_seed(4242)
    imgs = torch.rand(n_img, 3, size, size, generator=g)
    noise = torch.randn(n_img, 1, size, size, generator=g).to(device)
    fg = ops.cowmix_mask(noise, torch.full((n_img,), 16.0, device=device), torch.full((n_img,), 0.6, device=device))
    mask = torch.cat([1 - fg, fg], 1).contiguous()
    inner = student.module if hasattr(student, 'module') else student
    sd = {k: v.detach().float().cpu() for k, v in inner.state_dict().items()}
    inner.eval()
    out = {}
    logits = {}
    try:
        for name, dt in (('hip_fp32', torch.float32), ('hip_bf16', torch.bfloat16)):
            snn.set_compute_dtype(dt)
            seg = ops.SegMetrics(device)
            with torch.no_grad():
                lg = inner(imgs.to(device))[-1][-1].float()
                res = seg.update(lg, mask)
            r = res.cpu().double().numpy()
            out[name] = {'dice': round(float(r[0]), 6), 'miou': round(float(r[3]), 6)}
            logits[name] = lg.cpu()
    finally:
        snn.set_compute_dtype(torch.bfloat16)
        inner.train()
    prev = torch.get_num_threads()
    torch.set_num_threads(_cpu_threads())
    try:
        ref = models_ref.ListOutput(models_ref.UNet(2, models_ref.resnet50_encoder(), 128, train_upsampling=True))
        ref.load_state_dict(sd)
        ref.eval()
        with torch.no_grad():
            rl = ref(imgs)[-1][-1].float()
    finally:
        torch.set_num_threads(prev)
    dice, ious, _ = losses_ref.seg_metrics(rl.numpy(), mask.cpu().numpy())
    out['oracle_fp32'] = {'dice': round(float(np.mean(dice)), 6), 'miou': round(float(np.mean(ious)), 6)}
    scale = float(rl.abs().max()) or 1.0
    # north_star: argmax labels bit-exact, logits within 1e-3 relative -- a label may flip only where the oracle's two
    # logits are closer than that tolerance (|l1 - l0| < 1e-3 * max|l|, the tie band); bf16 is judged against its own
    # 3e-2 logits bound the same way
    margin = (rl[:, 1] - rl[:, 0]).abs()
    for name, tol in (('hip_fp32', 1e-3), ('hip_bf16', 3e-2)):
        d = (logits[name] - rl).abs()
        lab = (logits[name][:, 1] > logits[name][:, 0]) != (rl[:, 1] > rl[:, 0])
        out[name]['logits_max_err_rel'] = float(d.max()) / scale
        out[name]['argmax_mismatch_frac'] = float(lab.float().mean())
        out[name]['argmax_mismatch'] = int(lab.sum())
        out[name]['tie_band_rel'] = tol
        out[name]['argmax_mismatch_outside_band'] = int((lab & (margin >= tol * scale)).sum())
        out[name]['flip_margin_max_rel'] = float(margin[lab].max()) / scale if bool(lab.any()) else 0.0
    out['argmax_mismatch_outside_band'] = out['hip_fp32']['argmax_mismatch_outside_band']
    out['data'] = (f'{n_img} synthetic {size}x{size} validation images (U[0,1)), blob masks (CowMix kernel, sigma 16, '
                   f'p 0.6); student weights after the timed steps')
    out['miou_abs_diff_fp32'] = abs(out['hip_fp32']['miou'] - out['oracle_fp32']['miou'])
    out['dice_abs_diff_fp32'] = abs(out['hip_fp32']['dice'] - out['oracle_fp32']['dice'])
    return out


def _spawn_ranks(n):
    """`bench.py --gpus N` without an external launcher: run torch.distributed.run as a CHILD process (no
    exec, and nothing has touched the GPU yet) with one rank per GPU, and exit with its code."""
    import socket
    import subprocess
    sock = socket.socket()
    sock.bind(('127.0.0.1', 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr=127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '0'))
    return subprocess.call(cmd, env=env)


def timed_run(args, world, rank, device, dtype, probe=True, eager_n1=False):
    """Build, warm up, time args.steps steps; returns (elapsed_s, conv probe rows, per-step loss records)."""
    import train
    from ssseg import nn as snn
    snn.set_compute_dtype(dtype)
    model, teacher, opt, cfg = build(args.batch, args.size, device)
    data = synthetic_batches(8, args.batch, args.size, device, rank)
    step_idx = [0]
    recs = []

    def one_step():
        img, mask, ua, ub = data[step_idx[0] % len(data)]
        rec = train.train_step(model, teacher, opt, img, mask, ua, ub, 30, step_idx[0], cfg)
        step_idx[0] += 1
        return rec

    model.train()
    opt.zero_grad()
    for _ in range(max(args.warmup, 2)):
        one_step()
    torch.cuda.synchronize()
    # N > 1: rank 0 tuned the conv geometries in the warm-up, the other ranks ran the static rule and now take its
    # table (ssseg.tune); every rank's table must be the same
    from ssseg import tune
    tune.sync()
    tune_digests = tune.digests()
    if len(set(tune_digests)) != 1:
        raise RuntimeError(f'bench: conv variant tables differ across ranks: {tune_digests}')
    rows = []
    if probe:   # instrumented step: HIP events around every conv-engine launch (dominant kernel family)
        # serial schedule for this one step: with the teacher pass overlapping the supervised backward on a side
        # stream (train.train_step), concurrent kernels would stretch each other's event intervals
        overlap = train._OVERLAP['teacher']
        train._OVERLAP['teacher'] = False
        rows = snn.probe(True)
        # the device held by a spin kernel while the host enqueues the instrumented step: every conv launch then
        # starts right behind its predecessor, so an event interval is the launch's device time, not host issue gaps
        # (the eager step issues ~1,000 launches + ~800 events from Python).  The events are fence-free
        # (snn.ProbeEvent, csrc/probe.hip): a default event's system-scope release writes back and invalidates the L2
        # after every record, which starts each bracketed conv colder than in the captured step.
        torch.cuda.synchronize()
        torch.cuda._sleep(PROBE_HOLD_CYCLES)
        one_step()
        snn.probe(False)
        torch.cuda.synchronize()
        train._OVERLAP['teacher'] = overlap
    graph = None
    # the step captured as a HIP graph and replayed, at N = 1 and at N > 1 on an RCCL group: the gradient buckets and the
    # SyncBN sums are enqueued on the native communicator (ssseg.comm), which a capture records like a kernel.  Eager
    # launches only where the collectives run on torch.distributed (gloo, SSSEG_COMM=c10d: DESIGN.md §6).  The N = 1
    # record also carries the eager rate ('eager_n1').
    from ssseg import comm as scomm
    capture_error = [None]
    if args.graph and (world == 1 or scomm.kind() == 'native'):
        # the step captured once as a HIP graph (ssseg.graph.StepGraph) and replayed: each replay copies the next
        # batch into the captured input buffers and runs the whole step (fresh CowMix draws from the device counter)
        from ssseg.graph import StepGraph
        # the replay repeats the captured step's host decisions: the optimizer step (step 2 % 1 == 0) and the epoch gate
        # (epoch 30 > 25) are the same for every timed step only with no gradient accumulation
        assert cfg['train']['virtual_batch_size_multiplier'] == 1, 'graph replay needs an optimizer step every step'
        try:
            graph = StepGraph(lambda img, mask, ua, ub: train.train_step(model, teacher, opt, img, mask, ua, ub, 30, 2,
                                                                         cfg), *data[0])
        except RuntimeError as exc:
            if world == 1:
                raise
            # N > 1: the native communicator's collectives inside a capture run here for the first time at this world
            # size (the one-GPU test box covers world 1 only); report and time the eager step rather than nothing
            graph = None
            capture_error[0] = repr(exc)[:300]
            print(f'[bench rank {rank}] step capture failed, timing eager steps: {exc}', file=sys.stderr, flush=True)
            torch.cuda.synchronize()

        if graph is not None:
            def one_step():
                out = graph(*data[step_idx[0] % len(data)])
                step_idx[0] += 1
                return tuple(t.clone() for t in out)

    def timed_steps(step_fn, n):
        # the timed region: barrier + device sync on both sides, MAX of the elapsed time over ranks
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            recs.append(step_fn())
        e1.record()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        el = max(wall, e0.elapsed_time(e1) / 1e3)
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t)
        return el

    elapsed = timed_steps(one_step, args.steps)
    eager = None
    if graph is not None and world == 1 and eager_n1:
        # the same model continued for the same number of steps with every launch issued from Python
        def eager_step():
            img, mask, ua, ub = data[step_idx[0] % len(data)]
            rec = train.train_step(model, teacher, opt, img, mask, ua, ub, 30, 2, cfg)
            step_idx[0] += 1
            return tuple(t.clone() for t in rec)
        eager = timed_steps(eager_step, args.steps)
    live = torch.stack([torch.stack([c.float(), u.float(), m.float()]) for c, u, m in recs]).cpu()
    snn.set_compute_dtype(torch.bfloat16)
    return elapsed, rows, live, model, (graph is not None, capture_error[0]), eager, tune_digests


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--size', type=int, default=512)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-fp32', action='store_true', help='skip the secondary fp32 (parity-mode) record')
    ap.add_argument('--no-graph', dest='graph', action='store_false',
                    help='issue every launch from Python each step instead of replaying the captured HIP graph')
    args = ap.parse_args()

    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(_spawn_ranks(args.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # one rank per GPU (LOCAL_RANK); SSSEG_BENCH_BACKEND=gloo and more ranks than GPUs are for the one-GPU test of this
    # branch (tests/test_bench_ddp.py): RCCL needs one GPU per rank
    dev_idx = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        backend = os.environ.get('SSSEG_BENCH_BACKEND', 'nccl')
        torch.cuda.set_device(dev_idx)
        kw = {'device_id': torch.device('cuda', dev_idx)} if backend == 'nccl' else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        print(f'[bench rank {rank}] process group: world {dist.get_world_size()}, backend '
              f'{dist.get_backend()}, device cuda:{dev_idx}', file=sys.stderr, flush=True)
    device = torch.device('cuda', dev_idx)

    from ssseg import comm as scomm
    from ssseg import tune
    elapsed, rows, live, model, graphed, eager, tune_digests = timed_run(args, world, rank, device, torch.bfloat16,
                                                                         eager_n1=(world == 1))
    finite = bool(torch.isfinite(live).all())
    if not finite:
        raise RuntimeError(f'bench: non-finite loss in the timed steps (rank {rank}): {live.tolist()}')
    conv_ms = sum(r[0].elapsed_time(r[1]) for r in rows)
    conv_flops = sum(r[2] for r in rows)
    images = world * args.batch * args.steps
    value = images / elapsed
    achieved = conv_flops / (conv_ms / 1e3)
    result = {
        'metric': 'images/sec (UNet-R50 512x512 bs=16/GPU, mean-teacher + CowMix semi-supervised training step)',
        'value': round(value, 3), 'unit': 'images/sec', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'bf16', 'data': 'synthetic (SURVEY §8d), random-init weights',
        'config': {'workload': 'C2: UNet(ResNet-50 encoder, max_width=128, ConvT up) 512x512, semi-supervised '
                               'mean-teacher + CowMix step (BCE sup loss w=0.5, consistency w=10, SGD m=0.9)',
                   'global_batch': world * args.batch, 'per_gpu_batch': args.batch, 'image_size': args.size,
                   'parallelism': f'dp{world}', 'confidence_threshold': THRESHOLD},
        'roofline': {'bound': 'mfma', 'kernel': 'conv engine (igemm fwd/dgrad/ConvT + wgrad), all launches of one step',
                     'achieved': round(achieved / 1e12, 2), 'peak': BF16_DENSE_PEAK / 1e12, 'unit': 'TFLOP/s',
                     'frac': round(achieved / BF16_DENSE_PEAK, 4), 'traffic': pmc_traffic(),
                     'traffic_unit': 'HBM bytes per step, conv engine (rocprofv3 PMC, ' + os.path.relpath(PMC_PROFILE, ROOT) + ')',
                     'conv_ms_per_step': round(conv_ms, 3), 'conv_gflop_per_step': round(conv_flops / 1e9, 1),
                     'launches_per_step': len(rows), 'mfma_pmc': pmc_mfma()},
        'execution': ('HIP graph replay of the captured step (ssseg.graph.StepGraph), one per step' if graphed[0]
                      else 'eager launches from Python (the host reducer issues the bucket all-reduces)'
                      + (f'; capture failed: {graphed[1]}' if graphed[1] else '')),
        'conv_variant_table': {'rows': len(tune.export()),
                               'digest_per_rank': tune_digests,
                               'note': 'rank 0 tunes, the other ranks import its table (ssseg.tune.sync)'},
        'collectives': (None if world == 1 else
                        {'transport': scomm.kind(), 'backend': dist.get_backend(),
                         'note': 'native = libssseg RCCL communicator (ssseg_allreduce_buckets), gradient buckets on a '
                                 'side stream + SyncBN sums, inside the captured step'}),
        'step_tflops': round(8 * FWD_GFLOP_PER_IMAGE * args.batch * world / (elapsed / args.steps) / 1e3, 2),
        'liveness': {'losses_finite': finite, 'sup_loss_last': round(float(live[-1, 0]), 6),
                     'unsup_loss_last': round(float(live[-1, 1]), 6),
                     'cm_mean_avg': round(float(live[:, 2].mean()), 4)},
    }
    if eager is not None:
        result['eager_n1'] = {'value': round(world * args.batch * args.steps / eager, 3), 'unit': 'images/sec',
                              'ms_per_step': round(eager / args.steps * 1e3, 3), 'steps': args.steps,
                              'note': 'the same N=1 workload, every launch issued from Python instead of the '
                                      'captured-step replay'}
    if rank == 0 and world == 1 and not args.no_fp32:
        try:
            f_el, _, f_live, _, _, _, _ = timed_run(argparse.Namespace(**dict(vars(args), steps=min(args.steps, 5), warmup=2)),
                                        world, rank, device, torch.float32, probe=False)
            n = min(args.steps, 5)
            result['fp32_mode'] = {'value': round(args.batch * n / f_el, 3), 'unit': 'images/sec',
                                   'ms_per_step': round(f_el / n * 1e3, 3), 'steps': n,
                                   'losses_finite': bool(torch.isfinite(f_live).all()),
                                   'note': 'same C2 step in the fp32 parity mode (the reference arithmetic)'}
        except Exception as exc:  # report, never hide
            result['fp32_mode'] = {'error': repr(exc)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result['cpu_baseline'] = cpu_baseline(args.size)
        except Exception as exc:  # report, never hide
            result['cpu_baseline'] = {'error': repr(exc)}
        try:
            result['parity'] = parity_leg(model, args.size, device)
        except Exception as exc:  # report, never hide
            result['parity'] = {'error': repr(exc)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import gc
        gc.collect()               # the captured step (its RCCL persistent plans) goes before the communicator
        torch.cuda.synchronize()
        scomm.reset()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
