"""The adversarial semi-supervised branch of config C5 (build-defined: the reference builds models/
discriminator.py's Discriminator from default_config.py:116-120 but its trainer never calls it; formulation
after Hung et al. 2018, train.adversarial_terms / discriminator_step) on the GPU vs the oracle restatement
(oracle/train_ref.py adversarial_terms / discriminator_step), fp32 mode: two full semi-supervised steps with
the adversarial term on the student and a discriminator SGD step per step.  Losses (classification,
adversarial, discriminator, consistency) and the student's and the discriminator's parameters are compared
against fp32 and fp64 oracle runs (tests/parity.py)."""
import copy

import numpy as np
import pytest
import torch

from oracle import models_ref, train_ref

pytestmark = pytest.mark.gpu

B, H, STEPS = 2, 64, 2


def _data():
    g = torch.Generator().manual_seed(21)
    imgs = torch.rand(STEPS, B, 3, H, H, generator=g)
    fg = (torch.rand(STEPS, B, 1, H, H, generator=g) > 0.5).float()
    masks = torch.cat([1 - fg, fg], 2)
    unl = torch.rand(2 * STEPS, B, 3, H, H, generator=g)
    return imgs, masks, unl


def _oracle(s0, t0, d0, dt, pert=0.0):
    s, t, d = (copy.deepcopy(m).to(dt) for m in (s0, t0, d0))
    opt = torch.optim.SGD(s.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    optd = torch.optim.SGD(d.parameters(), lr=0.01, momentum=0.9)
    imgs, masks, unl = (v.to(dt) for v in _data())
    if pert:
        g = torch.Generator().manual_seed(99)
        imgs = imgs * (1 + pert * torch.randn(imgs.shape, generator=g, dtype=dt))
    torch.manual_seed(3)
    logs = train_ref.train_epoch(s, t, opt, list(zip(imgs, masks)), iter(unl), 30,
                                 train_ref.default_cfg(sigma_range=(4, 8), confidence_threshold=0.5),
                                 adv=dict(D=d, opt=optd, weight=0.01))
    return logs, s, d


def test_adversarial_branch_vs_oracle(hip_device):
    import cowmix
    import losses
    import train
    from models import simple_unet
    from models.adapters import ListOutput
    from models.discriminator import Discriminator
    from parity import check_losses, tensor_outliers
    from ssseg import arena, optim
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.float32)
    try:
        torch.manual_seed(0)
        s_ref = models_ref.ListOutput(models_ref.SimpleUNet(2, 3, 8, 32))
        t_ref = copy.deepcopy(s_ref)
        d_ref = models_ref.Discriminator(5, 2, 64, 512, 1)
        for p in t_ref.parameters():
            p.detach_()
        t_ref.eval()
        student = ListOutput(simple_unet.UNet(2, 3, 8, 32))
        teacher = ListOutput(simple_unet.UNet(2, 3, 8, 32))
        D = Discriminator(5, 2, 64, 512, 1)
        student.load_state_dict(s_ref.state_dict())
        teacher.load_state_dict(s_ref.state_dict())
        D.load_state_dict(d_ref.state_dict())
        student, teacher, D = student.to(hip_device), teacher.to(hip_device), D.to(hip_device)
        for p in teacher.parameters():
            p.detach_()
        teacher.eval()
        arena.attach(student)
        arena.attach(teacher, with_grads=False)
        arena.attach(D)
        opt = optim.SGD(student.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
        optd = optim.SGD(D.parameters(), lr=0.01, momentum=0.9)
        adv = dict(discriminator=D, optimizer=optd, weight=0.01)
        tcfg = dict(loss=losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits('mean'),
                                                'weight': [0.5]}]),
                    virtual_batch_size_multiplier=1, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
                    sigma_range=(4, 8), confidence_threshold=0.5, consistency_loss_weight=10, ema_model_alpha=0.99,
                    print_freq=1, gradient_clip_value=5.0, adversarial=adv)
        r32, s32, d32 = _oracle(s_ref, t_ref, d_ref, torch.float32)
        r64, s64, d64 = _oracle(s_ref, t_ref, d_ref, torch.float64)
        _, sp, dp = _oracle(s_ref, t_ref, d_ref, torch.float64, pert=1e-6)
        imgs, masks, unl = _data()
        old = cowmix.NOISE_SOURCE
        cowmix.NOISE_SOURCE = 'cpu'
        try:
            torch.manual_seed(3)
            student.train()
            opt.zero_grad()
            logs = []
            for k in range(STEPS):
                c, u, _ = train.train_step(student, teacher, opt, imgs[k].to(hip_device), masks[k].to(hip_device),
                                           unl[2 * k].to(hip_device), unl[2 * k + 1].to(hip_device), 30, k,
                                           {'train': tcfg})
                logs.append((float(c), float(adv['last_loss_adv']), float(adv['last_loss_d']), float(u)))
        finally:
            cowmix.NOISE_SOURCE = old
        keys = ('sup_loss', 'adv_loss', 'd_loss', 'unsup_loss')
        check_losses(logs, [tuple(r[k] for k in keys) for r in r32], [tuple(r[k] for k in keys) for r in r64],
                     names=('sup', 'adv', 'disc', 'unsup'))
        np_sd = lambda m: {k: v.detach().cpu().double().numpy() for k, v in m.state_dict().items()}  # noqa: E731
        bad_s = tensor_outliers(np_sd(student), np_sd(s32), np_sd(s64), np_sd(sp))
        bad_d = tensor_outliers(np_sd(D), np_sd(d32), np_sd(d64), np_sd(dp))
        print('student outliers', bad_s[:5], 'discriminator outliers', bad_d[:5])
        assert not bad_s and not bad_d, (bad_s[:5], bad_d[:5])
    finally:
        snn.set_compute_dtype(torch.bfloat16)


def test_frozen_discriminator_gets_no_student_gradient(hip_device):
    """The student's adversarial term weight*BCE(D(p), 1) must not reach D's parameters: after the student's
    supervised backward (the adversarial term included, weight gradients deferred as in train_step) and a flush
    of every deferred weight gradient, D's whole gradient arena is exactly zero -- whatever D's requires_grad
    flags are by the time the backward runs (train.adversarial_terms freezes D for its forward only)."""
    import losses
    import train
    from models import simple_unet
    from models.adapters import ListOutput
    from models.discriminator import Discriminator
    from ssseg import arena, ops
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.float32)
    try:
        torch.manual_seed(0)
        student = ListOutput(simple_unet.UNet(2, 3, 8, 32)).to(hip_device)
        D = Discriminator(5, 2, 64, 512, 1).to(hip_device)
        sa = arena.attach(student)
        da = arena.attach(D)
        imgs, masks, _ = _data()
        image, mask = imgs[0].to(hip_device), masks[0].to(hip_device)
        loss_fn = losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits('mean'),
                                         'weight': [0.5]}])
        adv = dict(discriminator=D, optimizer=None, weight=0.01)
        student.train()
        _, pred_maps = student(image)
        sup = loss_fn(pred_maps, mask)
        adv_loss, _ = train.adversarial_terms(pred_maps, mask, adv)
        train._set_requires_grad(D, True)      # live flags back on BEFORE the backward: must not matter
        with snn.defer_wgrad():
            ops.backward(ops.add_scaled(sup, adv_loss))
        snn.flush_wgrad()
        torch.cuda.synchronize()
        assert float(da.grad.abs().max()) == 0.0
        assert float(sa.grad.abs().max()) > 0.0     # the student did get its gradients
    finally:
        snn.set_compute_dtype(torch.bfloat16)
