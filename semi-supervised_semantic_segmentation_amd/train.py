"""Training / validation loop — drop-in for reference train.py (train :25-147, validate :150-195).

Same signatures and the same step semantics: supervised forward + CalculateLoss +
backward; mean-teacher forwards (no_grad, eval) + bilinear resize; CowMix mask + mixing; the student's
consistency forward in eval() with grads on; consistency loss gated by float(epoch > 25) (NaN when no
pixel is confident, like the reference); clip_grad_norm_ + optimizer step skipped at step 0;
EMA update every step.  Every tensor op of the step runs on the MI355X kernels.

Deliberate differences: loss scalars stay on the device and are reduced / synced only on
print steps (the reference syncs 4x per step for logging only); the DDP gradient all-reduce runs once
per step, armed on the last backward pass (linear, so the averaged gradient is the same).
"""
import contextlib
import os
import time

import torch

import cowmix
import mean_teacher
import metrics
import utils.utils as utils
from ssseg import nn as snn
from ssseg import ops
from ssseg.ddp import DistributedDataParallel as _DDP
from ssseg.optim import SGD as _SGD


def _inner(model):
    return model.module if hasattr(model, 'module') else model


def _batched_eval_ok(ema_model, a, b):
    """The teacher takes an NHWC activation batch and is per-sample in eval mode (models that declare
    ssseg_batched_eval), and both unlabelled batches have the same image shape."""
    m = _inner(ema_model)
    return (getattr(m, 'ssseg_batched_eval', False) and tuple(a.shape[1:]) == tuple(b.shape[1:])
            and a.dtype == b.dtype)


def _world():
    return torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1


_TARGETS = {}


def _target(ref, value):
    """Constant real/fake label maps of the discriminator losses, allocated once per shape."""
    key = (tuple(ref.shape), ref.device, value)
    t = _TARGETS.get(key)
    if t is None:
        t = torch.full(tuple(ref.shape), float(value), device=ref.device, dtype=torch.float32)
        _TARGETS[key] = t
    return t


def _set_requires_grad(module, flag):
    for p in module.parameters():
        p.requires_grad_(flag)


def adversarial_terms(pred_maps, mask, adv):
    """Adversarial semi-supervised branch of config C5 (build-defined: the reference constructs
    models/discriminator.py's Discriminator from its config, default_config.py:116-120, but its trainer never
    calls it; the formulation follows Hung et al. 2018, "Adversarial Learning for Semi-Supervised Semantic
    Segmentation").  The discriminator sees the student's probability map p = sigmoid(up(logits)) at the mask
    resolution (the reference's BCE treats each of the 2 channels as an independent sigmoid, losses.py:41-48).
    Student term: weight * BCE(D(p), 1) with D frozen: D's parameters are built with requires_grad off for this
    forward, and the native layers take their parameter-gradient decision from forward time (ctx.needs_input_grad),
    so the student's backward never writes D's gradient arena.  D stays frozen until the caller has run that
    backward (train_step re-enables it right before discriminator_step).
    Returns (student adversarial loss, detached p for the discriminator update)."""
    D = adv['discriminator']
    logits = pred_maps[-1]
    if tuple(logits.shape[2:]) != tuple(mask.shape[2:]):
        logits = ops.interpolate_bilinear(logits, mask.shape[2:4], align_corners=False)
    prob = ops.sigmoid(logits)
    _set_requires_grad(D, False)
    d_fake = D(prob)
    adv_loss = ops.scale(ops.bce_with_logits_mean(d_fake, _target(d_fake, 1.0)), adv['weight'])
    return adv_loss, prob.detach()


def discriminator_step(mask, prob, adv):
    """Discriminator update of the adversarial branch: BCE(D(mask), 1) + BCE(D(p), 0) on the labelled
    batch, backward into D's own gradient arena (all-reduced by its own DDP reducer at world > 1), SGD step
    (every step: the student's step-0 skip, train.py:121, is a property of the student's accumulation).
    Returns the device scalar discriminator loss."""
    D, opt = adv['discriminator'], adv['optimizer']
    ddp = D if isinstance(D, _DDP) else None
    d_real = D(mask)
    d_fake = D(prob)
    loss_d = ops.add_scaled(ops.bce_with_logits_mean(d_real, _target(d_real, 1.0)),
                            ops.bce_with_logits_mean(d_fake, _target(d_fake, 0.0)))
    if ddp is not None:
        ddp.arm()
    ops.backward(_scaled(loss_d, opt))
    if ddp is not None:
        ddp.finish()
    opt.step()
    opt.zero_grad()
    snn.invalidate_packed(_inner(D))
    return loss_d.detach()


def _scaled(loss, optimizer):
    """fp16 mode: the loss whose backward starts from S*dL (ssseg.amp.GradScaler attached to the optimizer;
    the optimizer step unscales and skips overflowed steps on the device).  Identity otherwise."""
    sc = getattr(optimizer, 'grad_scaler', None)
    return sc.scale(loss) if sc is not None else loss


# the first `serial_steps` steps of every (student, teacher, input geometry, compute dtype) run serially: the engine
# autotunes every new conv geometry on first use (HIP-event timings, conv.hip tune_variant), and a teacher pass running
# concurrently on the side stream would skew those timings -- and with them the variant choices kept for the rest of
# the run.  Counted per step key (a second model, a new batch size or dtype in the same process tunes serially too).
_OVERLAP = {'teacher': os.environ.get('SSSEG_OVERLAP_TEACHER', '1') != '0', 'streams': {}, 'steps': 0,
            'serial_steps': 2, 'seen': {},
            'consistency': os.environ.get('SSSEG_OVERLAP_CONSISTENCY', '1') != '0',
            'consistency_bwd': os.environ.get('SSSEG_OVERLAP_CONSISTENCY_BWD', '1') != '0',
            'merge_wgrad': os.environ.get('SSSEG_MERGE_WGRAD', '1') != '0'}


def _step_key(model, ema_model, image, unsup_a):
    return (id(_inner(model)), id(_inner(ema_model)) if ema_model is not None else None, tuple(image.shape),
            image.dtype, tuple(unsup_a.shape) if unsup_a is not None else None, snn.compute_dtype())


def _teacher_targets(ema_model, unsup_a, unsup_b, tc):
    """train.py:66-85: the teacher's predictions on both unlabelled batches (no grad, eval), resized to the image size,
    the CowMix mask and the two mixes.  Returns (mixed teacher logits, mixed images)."""
    size = unsup_a.shape[2:4]
    with torch.no_grad(), snn.folded(_inner(ema_model)):   # one batched BN fold for both teacher passes
        if _batched_eval_ok(ema_model, unsup_a, unsup_b):
            # train.py:69-75 runs the teacher twice; in eval mode every output depends on its own sample
            # only, so ONE forward over [unsup_a; unsup_b] gives the same logits (the conv variants
            # accumulate the same k-sequence at any batch) with half the launches and twice the tiles on
            # the small-map layers
            b = unsup_a.shape[0]
            ema_logits = ema_model(snn.to_act_cat([unsup_a, unsup_b]))[-1][-1]
            ema_pred_a = ops.interpolate_bilinear(ema_logits[:b], size, align_corners=False)
            ema_pred_b = ops.interpolate_bilinear(ema_logits[b:], size, align_corners=False)
            del ema_logits
        else:
            ema_pred_a = ops.interpolate_bilinear(ema_model(unsup_a)[-1][-1], size, align_corners=False)
            ema_pred_b = ops.interpolate_bilinear(ema_model(unsup_b)[-1][-1], size, align_corners=False)
        cmask = cowmix.generate_cowmix_masks_like(unsup_a, mask_proportion_range=tc['mask_proportion_range'],
                                                  sigma_range=tc['sigma_range'])
        mixed_ema_pred = cowmix.mix_with_mask(ema_pred_a, ema_pred_b, cmask)
        mixed_images = cowmix.mix_with_mask(unsup_a, unsup_b, cmask)
    return mixed_ema_pred, mixed_images


def _consistency_forward(model, targets, tc, epoch):
    """train.py:87-112: the student's eval-mode forward on the mixed images (with grad), resized, and the weighted
    consistency loss.  Returns (unsup_loss, cm_mean)."""
    mixed_ema_pred, mixed_images = targets
    model.eval()
    with snn.folded(_inner(model)):
        student_pred = model(mixed_images)[-1][-1]
    model.train()
    student_pred = ops.interpolate_bilinear(student_pred, mixed_images.shape[2:4], align_corners=False)
    consistency, cm_mean = ops.consistency_loss(student_pred, mixed_ema_pred, tc['confidence_threshold'])
    # consistency * weight * float(epoch > 25) (train.py:112; a 0/0 NaN survives the 0.0 gate, as there)
    return ops.scale(consistency, float(tc['consistency_loss_weight']) * float(epoch > 25)), cm_mean


def _side_stream(device):
    s = _OVERLAP['streams'].get(device)
    if s is None:
        s = _OVERLAP['streams'][device] = torch.cuda.Stream(device=device)
    return s


def train_step(model, ema_model, optimizer, image, mask, unsup_a, unsup_b, epoch, step, config):
    """One step of train.py:44-130.  Returns device scalars (classification loss, unsup loss, cm mean).
    With config['train']['adversarial'] = dict(discriminator=D, optimizer=opt_D, weight=w) the student's
    supervised loss gets the adversarial term and D is updated after the supervised backward (C5).

    Stream schedule (same arithmetic as the reference order): the teacher pass (train.py:66-85) depends on the
    supervised forward only -- the running statistics its eval BatchNorms read are the ones that forward updated
    (the teacher's BN buffers alias the student's, mean_teacher.py:13-18), and the supervised backward neither
    changes them nor draws random numbers -- so it is issued on a side HIP stream right after the supervised forward
    and runs concurrently with the supervised backward (and, in C5, the discriminator step).  The consistency forward
    (train.py:87-112) reads the same weights and statistics, so it follows the teacher on the side stream; its
    backward runs after the supervised backward's gradient writes (autograd runs it on the side stream, its forward's:
    explicit waits on both sides).  The consistency backward can put its (merged) weight gradients on a side stream too
    (ssseg.nn.wgrad_side_stream; off by default, measured neutral).  Measured (A/B in one call): C2 443.9 img/s serial,
    452.9 with the teacher overlap (round 4); 499.7 / 501.9 -> 512.9 / 514.8 with the consistency forward on the side
    stream too; C5 25.5 -> 21.9 ms (the overlap was off for the adversarial config before)."""
    tc = config['train']
    ddp = model if isinstance(model, _DDP) else None
    semi = tc['use_semi_supervised']
    adv = tc.get('adversarial')
    features, pred_maps = model(image)
    classification_loss = tc['loss'](pred_maps, mask)
    sup_loss = classification_loss
    prob = None
    if adv is not None:
        adv_loss, prob = adversarial_terms(pred_maps, mask, adv)
        sup_loss = ops.add_scaled(sup_loss, adv_loss)
    key = _step_key(model, ema_model, image, unsup_a)
    seen = _OVERLAP['seen'].get(key, 0)
    overlap = (semi and _OVERLAP['teacher'] and image.is_cuda and unsup_a.is_cuda
               and seen >= _OVERLAP['serial_steps'])
    _OVERLAP['seen'][key] = seen + 1
    _OVERLAP['steps'] += 1
    targets = cons = None
    # the consistency backward too, when no DDP reducer needs its gradients as they are written: both backward passes
    # then run concurrently, their weight / bias gradients held (snn.hold_wgrad) and replayed after both
    side_bwd = overlap and ddp is None and _OVERLAP['consistency'] and _OVERLAP['consistency_bwd']
    pgrad_ctx = contextlib.ExitStack()
    with pgrad_ctx:   # (closed early on the normal path; on an exception it leaves defer_param_grads too)
        if overlap:
            main = torch.cuda.current_stream()
            side = _side_stream(image.device)
            side.wait_stream(main)                # the supervised forward (and its running statistics) first
            for t in (unsup_a, unsup_b):
                t.record_stream(side)
            with torch.cuda.stream(side):
                targets = _teacher_targets(ema_model, unsup_a, unsup_b, tc)
                if _OVERLAP['consistency']:
                    # the consistency forward needs the student's weights and running statistics as the supervised
                    # forward left them -- the supervised backward changes neither -- so it runs on the side stream
                    # too, concurrently with that backward
                    cons = _consistency_forward(model, targets, tc, epoch)
                if side_bwd:
                    # its backward writes no gradient now: the eval BNs' parameter gradients are reduced after the join
                    # (defer_param_grads, left open until then) and the conv weight / bias gradients are held
                    snn.clear_held()
                    pgrad_ctx.enter_context(snn.defer_param_grads())
                    with snn.hold_wgrad('cons', params=True):
                        ops.backward(_scaled(cons[0], optimizer))
            for t in targets:
                t.record_stream(main)
        if ddp is not None and not semi:
            ddp.arm()
        # with a consistency backward to follow, each conv's supervised weight gradient is merged into that pass's
        # (one launch over both batches' pixels; ssseg.nn.defer_wgrad) -- the .grad sum is the same
        # (merge_wgrad off: the supervised weight gradients are launched in its backward -- written into .grad while
        # the side stream still runs the teacher and consistency passes -- and the consistency pass's add to them)
        merge = _OVERLAP['merge_wgrad']
        with (snn.hold_wgrad('sup') if side_bwd and merge else snn.defer_wgrad() if semi and merge
              else contextlib.nullcontext()):
            vbm = tc['virtual_batch_size_multiplier']
            ops.backward(_scaled(ops.scale(sup_loss, 1.0 / vbm) if vbm != 1 else sup_loss, optimizer))
        del pred_maps, features
        if adv is not None:
            # frozen since adversarial_terms; the student backward is done
            _set_requires_grad(adv['discriminator'], True)
            adv['last_loss_d'] = discriminator_step(mask, prob, adv)
            adv['last_loss_adv'] = adv_loss.detach()
            del prob
        unsup_loss = cm_mean = None
        if side_bwd:
            torch.cuda.current_stream().wait_stream(_side_stream(image.device))
            unsup_loss, cm_mean = cons
            del targets, cons
            snn.replay_held(('sup', 'cons'))   # the serial schedule's weight-gradient launches, on this stream
            pgrad_ctx.close()                  # the eval BNs' parameter gradients: one batched reduction
            semi_rest = False
        else:
            semi_rest = semi
    with snn.wgrad_side_stream():
        if semi_rest:
            if overlap:
                torch.cuda.current_stream().wait_stream(_side_stream(image.device))
            else:
                targets = _teacher_targets(ema_model, unsup_a, unsup_b, tc)
            side_fwd = cons is not None
            unsup_loss, cm_mean = cons if side_fwd else _consistency_forward(model, targets, tc, epoch)
            del targets, cons
            if ddp is not None:
                ddp.arm()
            with snn.defer_param_grads():   # the eval BNs' parameter gradients: one batched reduction at the end
                if side_fwd:
                    # autograd runs each backward node on its forward's stream: the consistency backward runs on the
                    # side stream, after the supervised backward's gradient writes (main) and before what follows
                    side = _side_stream(image.device)
                    side.wait_stream(torch.cuda.current_stream())
                ops.backward(_scaled(unsup_loss, optimizer))
                if side_fwd:
                    torch.cuda.current_stream().wait_stream(side)
        snn.flush_wgrad()
    if ddp is not None:
        ddp.finish()
    if step % tc['virtual_batch_size_multiplier'] == 0 and step != 0:
        clip = tc['gradient_clip_value']
        if isinstance(optimizer, _SGD):
            optimizer.step(max_norm=clip)
        else:
            torch.nn.utils.clip_grad_norm_(_inner(model).parameters(), clip)
            optimizer.step()
        optimizer.zero_grad()
        snn.invalidate_packed(_inner(model))
    if semi:
        mean_teacher.update_ema_variables(model, ema_model, alpha=tc['ema_model_alpha'])
    return classification_loss.detach(), (unsup_loss.detach() if unsup_loss is not None else None), \
        (cm_mean.detach() if cm_mean is not None else None)


# ---- captured-step execution of train.train --------------------------------------------------------------------------
# After the eager steps that tune every conv geometry and build the teacher's BN fold table, train() captures one step
# of each kind as a HIP graph (ssseg.graph.StepGraph) and replays it for the following steps, the way bench.py runs
# the benchmark: C5 (HarDNet + discriminator, ~660 small launches) 63.6 -> 33.5 ms/step, C4 213 -> 195 ms.  A replay
# repeats the Python decisions of its capture, so the graph is keyed on every one of them: the optimizer step taken
# or skipped (train.py:121, step % virtual_batch_size_multiplier), the epoch gate of the consistency weight
# (train.py:112), every learning rate, the input geometry and compute dtype -- a new key captures a new graph (the two
# most recent are kept).  Not captured (eager steps instead): CowMix drawn from the CPU generator (parity mode), steps
# with collectives on torch.distributed (gloo, or SSSEG_COMM=c10d: the native RCCL communicator's steps ARE captured),
# the first optimizer step (SGD's momentum buffer starts from it),
# and SSSEG_TRAIN_GRAPH=0.
_GRAPH = {'on': os.environ.get('SSSEG_TRAIN_GRAPH', '1') != '0', 'cache': {}, 'eager_steps': 2, 'max_graphs': 2,
          'captures': 0, 'replays': 0}


_TUNE = {'steps': 0}


def _optimizers(optimizer, config):
    adv = config['train'].get('adversarial')
    return [optimizer] + ([adv['optimizer']] if adv is not None else [])


def _graph_key(model, ema_model, optimizer, image, mask, unsup_a, unsup_b, epoch, step, config):
    """None where the step must run eagerly, else the key of its captured graph."""
    tc = config['train']
    if not (_GRAPH['on'] and image.is_cuda and torch.cuda.is_available()):
        return None
    if tc['use_semi_supervised'] and cowmix.NOISE_SOURCE != 'device':
        return None
    if torch.distributed.is_initialized() and (_world() > 1 or getattr(model, '_active', False)):
        # collectives in the step (DDP buckets, SyncBN): capturable only on the native communicator (ssseg.comm; c10d's
        # Work objects and watchdog break a capture, gloo runs on the host) -- DESIGN.md §6
        from ssseg import comm as scomm
        if scomm.kind() != 'native':
            return None
    opts = _optimizers(optimizer, config)
    opt_step = step % tc['virtual_batch_size_multiplier'] == 0 and step != 0
    # the first SGD step initialises the momentum buffer (a different kernel argument): run it eagerly (the
    # discriminator of C5 steps every step)
    if (opt_step and getattr(optimizer, '_first', False)) or any(getattr(o, '_first', False) for o in opts[1:]):
        return None
    step_key = _step_key(model, ema_model, image, unsup_a)
    if _OVERLAP['seen'].get(step_key, 0) < _GRAPH['eager_steps']:
        return None
    lrs = tuple(float(g['lr']) for o in opts for g in o.param_groups)
    shapes = tuple((tuple(t.shape), t.dtype) if t is not None else None for t in (image, mask, unsup_a, unsup_b))
    return step_key + (id(optimizer), opt_step, float(epoch > 25), lrs, shapes, id(config))


def _graph_step(key, model, ema_model, optimizer, image, mask, unsup_a, unsup_b, epoch, step, config):
    """One step replayed from the captured graph of `key` (captured from this step's inputs on first use)."""
    from ssseg.graph import StepGraph
    g = _GRAPH['cache'].pop(key, None)
    if g is None:
        while len(_GRAPH['cache']) >= _GRAPH['max_graphs']:
            _GRAPH['cache'].pop(next(iter(_GRAPH['cache'])))
        ins = (image, mask, unsup_a, unsup_b)
        live = [i for i, t in enumerate(ins) if t is not None]

        def fn(*xs):
            full = [None] * 4
            for i, t in zip(live, xs):
                full[i] = t
            out = train_step(model, ema_model, optimizer, *full, epoch, step, config)
            return tuple(t for t in out if t is not None)
        g = StepGraph(fn, *[ins[i] for i in live])
        g.live = live
        _GRAPH['captures'] += 1
    _GRAPH['cache'][key] = g   # most recent last
    ins = (image, mask, unsup_a, unsup_b)
    outs = iter(t.clone() for t in g(*[ins[i] for i in g.live]))
    _GRAPH['replays'] += 1
    semi = config['train']['use_semi_supervised']
    cls = next(outs)
    unsup = next(outs) if semi else None
    cm = next(outs) if semi else None
    return cls, unsup, cm


def run_step(model, ema_model, optimizer, image, mask, unsup_a, unsup_b, epoch, step, config):
    """train_step, replayed from a captured HIP graph where the step's key allows it (see _GRAPH)."""
    if _world() > 1 and image.is_cuda:
        # rank 0's conv variant table to every rank once the eager tuning steps are done (ssseg.tune: ranks > 0 ran
        # the static rule meanwhile), before any capture -- the same kernels on every rank
        from ssseg import tune
        _TUNE['steps'] += 1
        if not tune.synced() and _TUNE['steps'] > _GRAPH['eager_steps']:
            tune.sync()
    key = _graph_key(model, ema_model, optimizer, image, mask, unsup_a, unsup_b, epoch, step, config)
    if key is None:
        return train_step(model, ema_model, optimizer, image, mask, unsup_a, unsup_b, epoch, step, config)
    return _graph_step(key, model, ema_model, optimizer, image, mask, unsup_a, unsup_b, epoch, step, config)


def release_graphs():
    """Drop the captured steps (their private memory pools) -- e.g. before the parameters are reallocated."""
    _GRAPH['cache'].clear()


def _reduce_meters(meters, keys, world):
    """Epoch-end average of the loss meters over ranks (the reference logs rank-reduced losses divided by
    world, train.py:53-59,109-114): one all-reduce of the stacked sums instead of one per step."""
    if world < 2:
        return
    live = [k for k in keys if meters[k].initialized]
    if not live:
        return
    dev = next((meters[k].sum.device for k in live if isinstance(meters[k].sum, torch.Tensor)), None)
    sums = torch.stack([torch.as_tensor(meters[k].sum, dtype=torch.float32, device=dev).reshape(()) for k in live])
    torch.distributed.all_reduce(sums)
    sums = sums / world
    for i, k in enumerate(live):
        meters[k].sum = sums[i]


def train(model, ema_model, optimizer, dataloader, unsupervised_dataloader, epoch, initial_step, summary_writer,
          config, device):
    model.train()
    meters = {k: utils.AverageMeter() for k in ('cls', 'sup', 'unsup', 'cm', 'time')}
    rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
    world = _world()
    optimizer.zero_grad()
    tc = config['train']
    # the reference's per-sample albumentations pipelines (dataset.py:70-74, default_config.py:179-212) as batched device
    # kernels: the loaders then deliver the host-only transforms' uint8 output (data.device_augment)
    aug = tc.get('device_augment')
    for step, sample in enumerate(dataloader):
        tic = time.time()
        global_step = initial_step + step
        if aug is not None:
            sample = aug.train_batch(sample)
        image = sample['image'].to(device, non_blocking=True)
        mask = sample['semantic_mask'].to(device, non_blocking=True)
        ua = ub = None
        if tc['use_semi_supervised']:
            us = [next(unsupervised_dataloader) for _ in range(2)]
            if aug is not None:
                us = [aug.unsupervised_batch(u) for u in us]
            ua = us[0]['image'].to(device, non_blocking=True)
            ub = us[1]['image'].to(device, non_blocking=True)
        cls, unsup, cm = run_step(model, ema_model, optimizer, image, mask, ua, ub, epoch, step, config)
        meters['cls'].update(cls)
        meters['sup'].update(cls)
        meters['unsup'].update(unsup if unsup is not None else 0.)
        meters['cm'].update(cm if cm is not None else 0.)
        meters['time'].update(time.time() - tic)
        if step % tc['print_freq'] == 0:
            red_cls = utils.reduce_tensor(cls.clone()) / world
            red_uns = utils.reduce_tensor(unsup.clone()) / world if unsup is not None else torch.zeros(())
            if rank == 0:
                print(f'Epoch: {epoch} Step: {step} Batch time: {meters["time"].average()} '
                      f'Loss: {meters["cls"].average()}')
                if summary_writer is not None:
                    summary_writer.add_scalar('train_classification_loss', float(red_cls), global_step)
                    summary_writer.add_scalar('train_unsupervised_loss', float(red_uns), global_step)
    _reduce_meters(meters, ('cls', 'sup', 'unsup', 'cm'), world)
    if rank == 0 and summary_writer is not None and meters['sup'].initialized:
        summary_writer.add_scalar('batch_time', meters['time'].average(), global_step)
        summary_writer.add_scalar('train_loss_avg', meters['sup'].average() + meters['unsup'].average(), global_step)
        summary_writer.add_scalar('train_supervised_loss_avg', meters['sup'].average(), global_step)
        summary_writer.add_scalar('train_unsupervised_loss_avg', meters['unsup'].average(), global_step)
        summary_writer.add_scalar('train_classification_loss', meters['cls'].average(), global_step)
        summary_writer.add_scalar('train_confidence_modulator', meters['cm'].average(), global_step)


def validate(model, dataloader, epoch, initial_step, summary_writer, config, device):
    """train.py:150-195: Dice on the nearest-resized argmax one-hot (the reference metric) plus mIoU over the
    whole validation set (lovasz.iou, lovasz.py:54-73) from the same device pass (ssseg_seg_metrics)."""
    model.eval()
    avg_loss, avg_metric = utils.AverageMeter(), utils.AverageMeter()
    rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
    world = _world()
    seg = None
    with torch.no_grad():
        for sample in dataloader:
            if seg is None:
                seg = ops.SegMetrics(device)
            image = sample['image'].to(device)
            mask = sample['semantic_mask'].to(device)
            features, pred_maps = model(image)
            loss = config['train']['loss'](pred_maps, mask)
            # argmax -> one-hot -> nearest resize -> dice (train.py:178-186) + lovasz.iou counts: one kernel
            res = seg.update(pred_maps[-1], mask)
            metric = res[0:1].clone()[0]
            avg_loss.update(utils.reduce_tensor(loss.clone()) / world)
            avg_metric.update(utils.reduce_tensor(metric) / world)
    miou = None
    if seg is not None:
        total = seg.total.clone()
        if world > 1:
            torch.distributed.all_reduce(total)
        t = total.double()
        ious = [float(t[3] / t[4]) if t[4] else 1., float(t[5] / t[6]) if t[6] else 1.]
        miou = 100. * sum(ious) / 2
    if rank == 0:
        print(f'Eval: Epoch: {epoch} Val loss: {avg_loss.average()} Val metric: {avg_metric.average()} mIoU: {miou}')
        if summary_writer is not None:
            summary_writer.add_scalar('val_loss_avg', avg_loss.average(), initial_step)
            summary_writer.add_scalar('val_dice', avg_metric.average(), initial_step)
            if miou is not None:
                summary_writer.add_scalar('val_miou', miou, initial_step)
    model.train()
    return avg_loss.average(), avg_metric.average()
