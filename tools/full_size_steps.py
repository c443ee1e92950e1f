"""Full-size smoke of the BASELINE configs C3-C5 on ONE GPU (world 1): the model, teacher, optimizer and (C5) the
discriminator built exactly as distributed_trainer.distributed_train builds them, synthetic batches at the config's
image size and per-worker batch, three train_step calls (epoch 30: the consistency term is live).  Checks memory fit
and 32-bit offsets at the real geometries (every kernel entry validates its offsets) and prints per config: losses,
finiteness of losses and parameters, ms/step of the last two steps, peak device memory.

    python tools/full_size_steps.py [--configs c3,c4,c5] > gpurun_out/full_size.log
Teacher liveness: a random-init network normalised with the init running statistics (mean 0, var 1) is
degenerate in eval mode (HRNet-MSA's eval logits are ~1e-14: tools/diag_c4.py), so at any threshold >= 0.5 no
pixel is confident and the consistency loss is the reference's own 0/0 NaN.  Before the timed steps
the student's BatchNorm running statistics are therefore calibrated by ONE train-mode forward (no grad) with
momentum 1 (running stats = that batch's statistics; the teacher's buffers alias the student's, mean_teacher.py:
13-18), which is what training does to them anyway, and the teacher starts from the student's weights (the shared
pretrained checkpoint of distributed_trainer.py:56-61); the steps then run at confidence threshold 0.5 and the record
carries cm_mean (the confident-pixel fraction) so a degenerate mean-teacher path is visible.  --threshold 0 and
--no-calibrate restore the round-2 smoke.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd')
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# semi-supervised step GFLOP per labelled image (3F sup fwd+bwd + 2F teacher + 3F consistency fwd+bwd)
STEP_GFLOP_PER_IMAGE = {'c2': 765.1, 'c3': 3855.8, 'c4': 3904.2, 'c5': 85.2}
PEAK = {'bfloat16': 2.5e15, 'float16': 2.5e15, 'float32': 0.16e15}   # dense MFMA (MI355X_MICROARCH.md)
CFGS = {'c2': 'configs/c2_unet_r50.py', 'c3': 'configs/c3_deeplabv3_r101.py', 'c4': 'configs/c4_msa_hrnet.py',
        'c5': 'configs/c5_hardnet_disc.py'}


def train_loop(name, path, dev, threshold, calibrate, n_warm=4, n_timed=10):
    """The reference entry point (train.train, reference train.py:25-147) over in-HBM batches: a first call of n_warm
    steps (two eager tuning steps, the first optimizer step, then the step captured as a HIP graph), a second call whose
    step 0 (no optimizer step) captures its own graph, then a timed call of n_timed steps, every one replayed.  Returns
    (ms per step of the timed call, captures, replays)."""
    import train
    model, ema, opt, cfg, tc, (img, mask, ua, ub), _, _ = build(name, path, dev, threshold, calibrate)
    loader = lambda n: [{'image': img, 'semantic_mask': mask} for _ in range(n)]  # noqa: E731
    unl = iter(lambda: {'image': ua}, None)
    c0, r0 = train._GRAPH['captures'], train._GRAPH['replays']
    train.train(model, ema, opt, loader(n_warm), unl, 30, 0, None, cfg, dev)
    # (an epoch's step 0 takes no optimizer step, train.py:121: its own graph, captured by this second warm-up call)
    train.train(model, ema, opt, loader(2), unl, 30, n_warm, None, cfg, dev)
    torch.cuda.synchronize()
    t0 = time.time()
    train.train(model, ema, opt, loader(n_timed), unl, 30, n_warm, None, cfg, dev)
    torch.cuda.synchronize()
    ms = 1e3 * (time.time() - t0) / n_timed
    train.release_graphs()
    return ms, train._GRAPH['captures'] - c0, train._GRAPH['replays'] - r0


def rescale_heads(model, ncls=2):
    """Re-initialise the class-logit convs (out_channels == ncls) with a unit-gain fan-in normal init: the configs'
    own inits leave a random network's logits at ~0 (C4 MSA-HRNet and C5 HarDNet: sup loss exactly ln2 / 2 at step 0),
    so p = 0.5 everywhere and no pixel is confident at any threshold.  A synthetic-data stand-in for a trained head."""
    import math
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.Conv2d) and m.out_channels == ncls:
                fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1] // m.groups
                m.weight.normal_(0.0, 1.0 / math.sqrt(fan_in))
                if m.bias is not None:
                    m.bias.zero_()
                if hasattr(m, 'invalidate_packed'):
                    m.invalidate_packed()


def calibrate_bn(model, x):
    """One train-mode forward with BN momentum 1: running statistics := this batch's statistics."""
    from ssseg import nn as snn
    bns = [m for m in model.modules() if isinstance(m, (snn.BatchNorm2d, torch.nn.BatchNorm2d))]
    saved = [m.momentum for m in bns]
    for m in bns:
        m.momentum = 1.0
    model.train()
    with torch.no_grad():
        model(x)
    for m, mo in zip(bns, saved):
        m.momentum = mo


def build(name, path, dev, threshold=0.5, calibrate=True):
    """model / teacher / optimizer / config / synthetic batch of config `name`, deterministic (seed 0)"""
    import config
    import cowmix
    import mean_teacher
    from ssseg import amp, arena
    from ssseg import nn as snn
    from ssseg import optim as soptim
    from ssseg.ddp import DistributedDataParallel
    import train
    torch.manual_seed(0)
    for c in cowmix._DEVICE_RNG['ctr'].values():   # the CowMix Philox counter restarts with every build
        c.zero_()
    train._OVERLAP['seen'].clear()   # and so does the step schedule (the first serial_steps steps run without overlap)
    for c in snn._DROP['ctr'].values():   # and the dropout Philox counter
        c.zero_()
    cfg = config.fromfile(os.path.join(PKG, path))
    snn.set_compute_dtype({'fp32': torch.float32, 'fp16': torch.float16}.get(cfg['common'].get('compute_dtype'),
                                                                             torch.bfloat16))
    model = DistributedDataParallel(cfg['model']['model_fn']().to(dev))
    if calibrate:
        rescale_heads(model.module)
    ema = cfg['model']['model_fn']().to(dev)
    # the teacher starts from the student's weights: the stand-in for the pretrained checkpoint both models load in
    # the reference (distributed_trainer.py:56-61); two independent random inits give a teacher whose eval logits do
    # not match the (student-calibrated, aliased) BN statistics and are degenerate (C4: cm_mean 0, 0/0 NaN)
    mean_teacher.detach_model_parameters(ema)
    arena.attach(ema, with_grads=False)
    ema.eval()
    opt = soptim.from_config(cfg['train']['optimizer'], [p for p in model.parameters() if p.requires_grad])
    if snn.compute_dtype() == torch.float16:
        opt.grad_scaler = amp.GradScaler(dev)
    tc = cfg['train']
    tc['confidence_threshold'] = threshold
    tc['print_freq'] = 10 ** 9
    if cfg['model'].get('discriminator') is not None and tc.get('adversarial_loss_weight'):
        disc = DistributedDataParallel(cfg['model']['discriminator']().to(dev))
        dopt = soptim.from_config(tc['discriminator_optimizer'], disc.parameters())
        if snn.compute_dtype() == torch.float16:
            dopt.grad_scaler = amp.GradScaler(dev)
        tc['adversarial'] = dict(discriminator=disc, optimizer=dopt, weight=float(tc['adversarial_loss_weight']))
    b, s = tc['batch_size_per_worker'], cfg['common']['image_size']
    g = torch.Generator().manual_seed(5)
    img = torch.rand(b, 3, s, s, generator=g).to(dev)
    fg = (torch.rand(b, 1, s, s, generator=g) > 0.5).float().to(dev)
    mask = torch.cat([1 - fg, fg], 1).contiguous()
    ua = torch.rand(b, 3, s, s, generator=g).to(dev)
    ub = torch.rand(b, 3, s, s, generator=g).to(dev)
    if calibrate:
        calibrate_bn(model.module, ua)
    with torch.no_grad():   # after the calibration: the teacher's own BN buffers are used until the first EMA update
        ema.load_state_dict(model.module.state_dict())
    return model, ema, opt, cfg, tc, (img, mask, ua, ub), b, s


def graph_steps(name, path, dev, threshold, calibrate, eager_losses, n_eager=3, n_replay=5):
    """Rebuild the config, run the same first n_eager eager steps, capture step n_eager as a HIP graph
    (ssseg.graph.StepGraph) and replay it: the replayed steps' losses must equal the eager run's bit for bit; returns
    (ms per replayed step, bitwise flag, replayed losses)."""
    import train
    from ssseg.graph import StepGraph
    model, ema, opt, cfg, tc, data, _, _ = build(name, path, dev, threshold, calibrate)
    rerun = []
    for step in range(n_eager):
        r = train.train_step(model, ema, opt, *data, 30, step, cfg)
        rerun.append(tuple(None if t is None else float(t) for t in r))
    g = StepGraph(lambda i, m, a, b: train.train_step(model, ema, opt, i, m, a, b, 30, n_eager, cfg), *data)
    out = []
    for _ in range(2):
        out.append(tuple(None if t is None else float(t) for t in g(*data)))
    same = out == [tuple(v for v in row) for row in eager_losses[n_eager:n_eager + 2]]
    same_eager = rerun == [tuple(v for v in row) for row in eager_losses[:n_eager]]   # the rebuild's eager steps
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(n_replay):
        g(*data)
    torch.cuda.synchronize()
    ms = 1e3 * (time.time() - t0) / n_replay
    del g, model, ema, opt
    return ms, same, out, same_eager


def run(name, path, dev, threshold=0.5, calibrate=True, layers=False, graph=False, loop=False):
    import train
    from ssseg import nn as snn
    model, ema, opt, cfg, tc, (img, mask, ua, ub), b, s = build(name, path, dev, threshold, calibrate)
    torch.cuda.reset_peak_memory_stats(dev)
    times, out = [], []
    for step in range(5 if graph else 3):
        torch.cuda.synchronize()
        t0 = time.time()
        cls, unsup, cm = train.train_step(model, ema, opt, img, mask, ua, ub, 30, step, cfg)
        torch.cuda.synchronize()
        times.append(time.time() - t0)
        out.append((float(cls), float(unsup) if unsup is not None else None, float(cm) if cm is not None else None))
    conv = None
    if layers:   # one more step with HIP events around every conv-engine launch (tools/layer_report.py format)
        sys.path.insert(0, os.path.join(ROOT, 'tools'))
        import layer_report
        overlap, train._OVERLAP['teacher'] = train._OVERLAP['teacher'], False   # serial schedule for the probe
        rows = snn.probe(True)
        train.train_step(model, ema, opt, img, mask, ua, ub, 30, 3, cfg)
        snn.probe(False)
        torch.cuda.synchronize()
        train._OVERLAP['teacher'] = overlap
        print(f'== {name} conv layers', file=sys.stderr)
        stdout, sys.stdout = sys.stdout, sys.stderr
        try:
            conv = layer_report.report(rows, 40)
        finally:
            sys.stdout = stdout
    params_finite = all(bool(torch.isfinite(p).all()) for p in model.parameters())
    losses_finite = all(v is None or v == v and abs(v) != float('inf') for row in out for v in row)
    rec = {'config': name, 'image_size': s, 'batch': b, 'dtype': str(snn.compute_dtype()).replace('torch.', ''),
           'confidence_threshold': threshold, 'bn_calibrated': calibrate,
           'cm_mean': [row[2] for row in out], 'losses': out, 'losses_finite': losses_finite, 'params_finite': params_finite,
           'ms_per_step_last2': round(1e3 * sum(times[-2:]) / 2, 1), 'first_step_s': round(times[0], 1),
           'peak_mem_GB': round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1),
           'collectives': getattr(model, '_active', False) and __import__('ssseg.comm', fromlist=['kind']).kind()}
    step_s = sum(times[-2:]) / 2
    tf = STEP_GFLOP_PER_IMAGE[name] * b / step_s / 1e3
    rec['conv_tflops'] = round(tf, 1)
    rec['frac_of_dense_peak'] = round(tf * 1e12 / PEAK[rec['dtype']], 4)
    if conv:   # the conv engine of the extra probed step: MFMA and bytes rooflines (algorithmic flops / bytes)
        rec['conv_engine'] = conv
    if 'adversarial' in tc:
        rec['loss_d'] = float(tc['adversarial']['last_loss_d'])
    if graph:   # the same steps replayed from a captured HIP graph (fresh build, same seeds)
        del model, ema, opt
        torch.cuda.empty_cache()
        gms, same, gl, same_eager = graph_steps(name, path, dev, threshold, calibrate, out)
        rec['graph'] = {'ms_per_step': round(gms, 1), 'losses_bitwise_equal_eager': same, 'losses_steps_3_4': gl,
                        'rebuild_eager_steps_bitwise_equal': same_eager,
                        'frac_of_dense_peak': round(STEP_GFLOP_PER_IMAGE[name] * b / (gms / 1e3) / 1e3 * 1e12 /
                                                    PEAK[rec['dtype']], 4)}
    if loop:   # the same config through the reference entry point train.train (captured-step replay inside)
        torch.cuda.empty_cache()
        lms, caps, reps = train_loop(name, path, dev, threshold, calibrate)
        rec['train_train'] = {'ms_per_step': round(lms, 1), 'captures': caps, 'replays': reps,
                              'note': 'train.train over in-HBM batches: 10 timed steps (one epoch call) after 4 + 2 warm-up steps'}
    print(json.dumps(rec), flush=True)
    return rec['losses_finite'] and rec['params_finite']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='c3,c4,c5')
    ap.add_argument('--threshold', type=float, default=0.5)
    ap.add_argument('--no-calibrate', action='store_true')
    ap.add_argument('--layers', action='store_true', help='per-layer conv report of one extra step (stderr)')
    ap.add_argument('--graph', action='store_true', help='also replay a captured HIP graph of the step (5 eager steps '
                    'first; graph losses checked bitwise against eager steps 3 and 4)')
    ap.add_argument('--train-loop', action='store_true', help='also time the config through train.train (the reference '
                    'entry point, captured-step replay inside)')
    ap.add_argument('--collectives', action='store_true', help='world 1 with the DDP bucket all-reduces and SyncBN sums '
                    'forced on (ssseg.ddp.force_collectives): the multi-GPU step\'s collectives on the native RCCL '
                    'communicator, eager and captured')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:29533', rank=0, world_size=1)
    if a.collectives:
        from ssseg import ddp
        ddp.force_collectives(True)
    ok = True
    for name in a.configs.split(','):
        ok &= run(name, CFGS[name], dev, a.threshold, not a.no_calibrate, a.layers, a.graph, a.train_loop)
        torch.cuda.empty_cache()
    from ssseg import comm
    comm.reset()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
