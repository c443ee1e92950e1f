"""Oracle: the mean-teacher + CowMix training step on torch-CPU fp32.  TEST INFRASTRUCTURE ONLY.

Restates reference/train.py:41-130 (one epoch of steps) for plain torch.nn models on the CPU:
  supervised forward + CalculateLoss (interp -> BCE * weight)         train.py:47-61, losses.py:15-22
  teacher forwards (no_grad, eval) + interp to the image size         train.py:69-75
  CowMix mask (oracle.cowmix_ref, RNG order of cowmix.py:44-55) + mix train.py:77-86
  student consistency forward in eval() with grads on                 train.py:90-94
  consistency loss + gate float(epoch > 25) + backward                train.py:97-115
  optimizer step skipped at step 0; clip_grad_norm_ before SGD         train.py:121-124
  EMA of parameters, buffers aliased                                  train.py:130, mean_teacher.py:5-18
It is pinned by tests/golden trainsteps.npz (G7) and consistency_*.npz (G3).
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import cowmix_ref


class _Lovasz(torch.autograd.Function):
    """binary_lovasz_loss_with_logits (losses.py:239-250) on the CPU through the numpy restatement
    (losses_ref.binary_lovasz, pinned by golden G4)."""

    @staticmethod
    def forward(ctx, logits, target):
        from . import losses_ref
        loss, grad = losses_ref.binary_lovasz(logits.detach().numpy(), target.detach().numpy())
        ctx.save_for_backward(torch.from_numpy(grad))
        return torch.tensor(float(loss), dtype=torch.float32)

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g, None


def lovasz_loss(pred, target):
    return _Lovasz.apply(pred, target)


def bce_loss(pred, target):
    return F.binary_cross_entropy_with_logits(pred, target, reduction='mean')


def calculate_loss(pred_list, target, weights=(0.5,), loss_fn=None):
    """CalculateLoss([{'loss_fn': f, 'weight': weights}]) (losses.py:15-22); f = BCE-with-logits by default."""
    loss_fn = loss_fn or bce_loss
    loss = 0
    for i, p in enumerate(pred_list):
        p = F.interpolate(p, size=(target.size(2), target.size(3)), mode='bilinear', align_corners=False)
        loss = loss + loss_fn(p, target) * weights[i]
    return loss


def cowmix_mask_like(example, prop_range, sigma_range):
    B, _, H, W = example.shape
    p, sig, noise = cowmix_ref.draw_inputs(B, H, W, prop_range, sigma_range)
    m, *_ = cowmix_ref.cowmix_masks(noise, sig, p)
    return torch.from_numpy(m).view(B, 1, H, W).to(example.dtype)


def consistency_loss(student_up, teacher_mixed, thr):
    pt = torch.sigmoid(teacher_mixed)
    ps = torch.sigmoid(student_up)
    cm = (pt.max(dim=1).values > thr).to(pt)
    loss = ((ps - pt).pow(2.0).sum(dim=1) * cm).sum() / cm.sum()
    return loss.mean(), cm.mean()


@torch.no_grad()
def ema_update(model, ema_model, alpha):
    for e, p in zip(ema_model.parameters(), model.parameters()):
        e.mul_(alpha).add_(p, alpha=1.0 - alpha)
    for eb, b in zip(ema_model.buffers(), model.buffers()):
        eb.data = b.data


def adversarial_terms(preds, mask, adv):
    """Build-defined adversarial branch of config C5 (train.adversarial_terms): D frozen, student term
    weight * BCE(D(sigmoid(up(logits))), 1) (Hung et al. 2018; the reference only constructs D,
    default_config.py:116-120)."""
    D = adv['D']
    logits = preds[-1]
    if tuple(logits.shape[2:]) != tuple(mask.shape[2:]):
        logits = F.interpolate(logits, size=mask.shape[2:], mode='bilinear', align_corners=False)
    prob = torch.sigmoid(logits)
    for p in D.parameters():
        p.requires_grad_(False)
    d = D(prob)
    loss = F.binary_cross_entropy_with_logits(d, torch.ones_like(d)) * adv['weight']
    for p in D.parameters():
        p.requires_grad_(True)
    return loss, prob.detach()


def discriminator_step(mask, prob, adv):
    """D update: BCE(D(mask), 1) + BCE(D(p), 0), SGD step every step (train.discriminator_step)."""
    D, opt = adv['D'], adv['opt']
    d_real, d_fake = D(mask), D(prob)
    loss = F.binary_cross_entropy_with_logits(d_real, torch.ones_like(d_real)) + \
        F.binary_cross_entropy_with_logits(d_fake, torch.zeros_like(d_fake))
    loss.backward()
    opt.step()
    opt.zero_grad()
    return float(loss.detach())


def train_epoch(model, ema_model, optimizer, batches, unsup_iter, epoch, cfg, loss_weights=(0.5,),
                on_step=None, loss_fn=None, adv=None):
    """Run len(batches) steps; returns per-step dict(sup_loss, unsup_loss, cm_mean) (+ adv_loss, d_loss with
    the adversarial branch adv = dict(D, opt, weight))."""
    tc = cfg
    model.train()
    optimizer.zero_grad()
    logs = []
    for step, (image, mask) in enumerate(batches):
        _, preds = model(image)
        sup = calculate_loss(preds, mask, loss_weights, loss_fn)
        rec = dict(sup_loss=float(sup.detach()))
        total = sup
        if adv is not None:
            adv_loss, prob = adversarial_terms(preds, mask, adv)
            total = sup + adv_loss
            rec['adv_loss'] = float(adv_loss.detach())
        (total / tc['virtual_batch_size_multiplier']).backward()
        if adv is not None:
            rec['d_loss'] = discriminator_step(mask, prob, adv)
        if tc['use_semi_supervised']:
            ua = next(unsup_iter)
            ub = next(unsup_iter)
            with torch.no_grad():
                ta = F.interpolate(ema_model(ua)[-1][-1], ua.shape[2:4], mode='bilinear', align_corners=False)
                tb = F.interpolate(ema_model(ub)[-1][-1], ua.shape[2:4], mode='bilinear', align_corners=False)
                m = cowmix_mask_like(ua, tc['mask_proportion_range'], tc['sigma_range'])
                t_mix = ta * m + tb * (1. - m)
                x_mix = ua * m + ub * (1. - m)
            model.eval()
            s = model(x_mix)[-1][-1]
            model.train()
            s = F.interpolate(s, x_mix.shape[2:4], mode='bilinear', align_corners=False)
            cons, cm_mean = consistency_loss(s, t_mix, tc['confidence_threshold'])
            unsup = cons * tc['consistency_loss_weight'] * float(epoch > 25)
            unsup.backward()
            rec.update(unsup_loss=float(unsup.detach()), cm_mean=float(cm_mean))
        if step % tc['virtual_batch_size_multiplier'] == 0 and step != 0:
            torch.nn.utils.clip_grad_norm_(model.parameters(), tc['gradient_clip_value'])
            optimizer.step()
            optimizer.zero_grad()
        if tc['use_semi_supervised']:
            ema_update(model, ema_model, tc['ema_model_alpha'])
        logs.append(rec)
        if on_step is not None:
            on_step(step, rec)
    return logs


def train_epoch_dp(model, ema_model, optimizer, rank_batches, rank_unsup, epoch, cfg, loss_weights=(0.5,),
                   on_step=None):
    """The same steps as train_epoch for a data-parallel job of `world` ranks (distributed_trainer.py:33-44:
    DDP + SyncBatchNorm, train.py:41-130 on every rank), restated in ONE process on the concatenated batch:
      - SyncBN training statistics over the global batch == BatchNorm over the concatenation;
      - every rank's loss is a mean over its own slice; DDP averages the ranks' gradients, i.e. the gradient
        of mean_r loss_r (SyncBN's backward all-reduce makes each rank's gradient that of sum_r loss_r
        through the shared statistics, DDP divides by world);
      - every rank seeds the same generator (distributed_trainer.py:17), so each rank draws the SAME CowMix
        p, sigma and noise for its own slice: the draw is replayed per rank from one generator state.
    rank_batches[step] = [(image_r, mask_r) per rank]; rank_unsup[step] = [(ua_r, ub_r) per rank].
    Returns per-step dicts with per-rank sup/unsup losses."""
    tc = cfg
    model.train()
    optimizer.zero_grad()
    logs = []
    for step, ranks in enumerate(rank_batches):
        world = len(ranks)
        sizes = [im.shape[0] for im, _ in ranks]
        image = torch.cat([im for im, _ in ranks])
        _, preds = model(image)
        sups = []
        o = 0
        for (im, mk), n in zip(ranks, sizes):
            sups.append(calculate_loss([p[o:o + n] for p in preds], mk, loss_weights))
            o += n
        sup = sum(sups) / world
        (sup / tc['virtual_batch_size_multiplier']).backward()
        rec = dict(sup_loss=[float(s.detach()) for s in sups])
        if tc['use_semi_supervised']:
            uas = [u[0] for u in rank_unsup[step]]
            ubs = [u[1] for u in rank_unsup[step]]
            ua, ub = torch.cat(uas), torch.cat(ubs)
            with torch.no_grad():
                ta = F.interpolate(ema_model(ua)[-1][-1], ua.shape[2:4], mode='bilinear', align_corners=False)
                tb = F.interpolate(ema_model(ub)[-1][-1], ua.shape[2:4], mode='bilinear', align_corners=False)
                state = torch.get_rng_state()
                ms = []
                for u in uas:
                    torch.set_rng_state(state)
                    ms.append(cowmix_mask_like(u, tc['mask_proportion_range'], tc['sigma_range']))
                m = torch.cat(ms)
                t_mix = ta * m + tb * (1. - m)
                x_mix = ua * m + ub * (1. - m)
            model.eval()
            s = model(x_mix)[-1][-1]
            model.train()
            s = F.interpolate(s, x_mix.shape[2:4], mode='bilinear', align_corners=False)
            cons, o = [], 0
            for n in sizes:
                c, _ = consistency_loss(s[o:o + n], t_mix[o:o + n], tc['confidence_threshold'])
                cons.append(c * tc['consistency_loss_weight'] * float(epoch > 25))
                o += n
            unsup = sum(cons) / world
            unsup.backward()
            rec.update(unsup_loss=[float(c.detach()) for c in cons])
        if on_step is not None:
            on_step(step, rec)     # before the optimizer step: grads are the step's averaged gradients
        if step % tc['virtual_batch_size_multiplier'] == 0 and step != 0:
            torch.nn.utils.clip_grad_norm_(model.parameters(), tc['gradient_clip_value'])
            optimizer.step()
            optimizer.zero_grad()
        if tc['use_semi_supervised']:
            ema_update(model, ema_model, tc['ema_model_alpha'])
        logs.append(rec)
    return logs


def default_cfg(**over):
    cfg = dict(virtual_batch_size_multiplier=1, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
               sigma_range=(8, 32), consistency_loss_weight=10, ema_model_alpha=0.99,
               confidence_threshold=0.97, gradient_clip_value=5.0)
    cfg.update(over)
    return cfg


def as_np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
