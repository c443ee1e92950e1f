"""C5 fp16 diagnosis: the student's step-0 gradients (no optimizer step yet, train.py:121) of FC-HarDNet + the adversarial
branch at 128^2, bs 2, from the HIP path in fp32 and fp16 (unscaled by the loss scale) against the oracle in fp64, fp32
and fp16 -- per tensor rel-RMS and max error against fp64, the worst tensors first.

    python tools/diag_c5.py > gpurun_out/diag_c5.log
"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'), os.path.join(ROOT, 'tests')]

import numpy as np  # noqa: E402
import torch  # noqa: E402

B, H = 2, 128


def main(variant='full'):
    import cowmix
    import losses
    import train
    from models.adapters import ListOutput
    from models.discriminator import Discriminator
    from models.hardnet import HarDNet
    from oracle import hardnet_ref, models_ref, train_ref
    from ssseg import amp, arena, optim
    from ssseg import nn as snn
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    s_ref = models_ref.ListOutput(hardnet_ref.HarDNet(2))
    torch.manual_seed(1)
    t_ref = models_ref.ListOutput(hardnet_ref.HarDNet(2))
    d_ref = models_ref.Discriminator(5, 2, 64, 512, 1)
    for p in t_ref.parameters():
        p.detach_()
    g = torch.Generator().manual_seed(4)
    imgs = torch.rand(1, B, 3, H, H, generator=g)
    fg = (torch.rand(1, B, 1, H, H, generator=g) > 0.5).float()
    masks = torch.cat([1 - fg, fg], 2)
    unl = torch.rand(2, B, 3, H, H, generator=g)
    cfg = dict(sigma_range=(4, 8), confidence_threshold=0.0)
    semi = variant != 'sup'
    use_adv = variant == 'full'
    if not semi:
        cfg['use_semi_supervised'] = False
    grads = {}
    for dt in (torch.float64, torch.float32, torch.float16):
        s, t, d = (copy.deepcopy(m).to(dt) for m in (s_ref, t_ref, d_ref))
        t.eval()
        opt = torch.optim.SGD(s.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
        optd = torch.optim.SGD(d.parameters(), lr=0.01, momentum=0.9)
        torch.manual_seed(3)
        train_ref.train_epoch(s, t, opt, list(zip(imgs.to(dt), masks.to(dt))), iter(unl.to(dt)), 30,
                              train_ref.default_cfg(**cfg), adv=dict(D=d, opt=optd, weight=0.01) if use_adv else None)
        grads['o' + str(dt)[-2:]] = {n: p.grad.detach().double() for n, p in s.named_parameters()}
    for name, dt in (('hip32', torch.float32), ('hip16', torch.float16)):
        snn.set_compute_dtype(dt)
        student, teacher = ListOutput(HarDNet(n_classes=2)), ListOutput(HarDNet(n_classes=2))
        D = Discriminator(5, 2, 64, 512, 1)
        student.load_state_dict(s_ref.state_dict())
        teacher.load_state_dict(t_ref.state_dict())
        D.load_state_dict(d_ref.state_dict())
        student, teacher, D = student.to(dev), teacher.to(dev), D.to(dev)
        for p in teacher.parameters():
            p.detach_()
        teacher.eval()
        arena.attach(student)
        arena.attach(teacher, with_grads=False)
        arena.attach(D)
        opt = optim.SGD(student.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
        optd = optim.SGD(D.parameters(), lr=0.01, momentum=0.9)
        S = 1.0
        if dt == torch.float16:
            opt.grad_scaler = amp.GradScaler(dev, init_scale=2.0 ** 12)
            optd.grad_scaler = amp.GradScaler(dev, init_scale=2.0 ** 12)
            S = 2.0 ** 12
        adv = dict(discriminator=D, optimizer=optd, weight=0.01)
        tcfg = dict(loss=losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits('mean'),
                                                'weight': [0.5]}]),
                    virtual_batch_size_multiplier=1, use_semi_supervised=semi, mask_proportion_range=(0.45, 0.55),
                    consistency_loss_weight=10, ema_model_alpha=0.99, print_freq=1, gradient_clip_value=5.0,
                    **{k: v for k, v in cfg.items() if k != 'use_semi_supervised'})
        if use_adv:
            tcfg['adversarial'] = adv
        cowmix.NOISE_SOURCE = 'cpu'
        torch.manual_seed(3)
        student.train()
        opt.zero_grad()
        train.train_step(student, teacher, opt, imgs[0].to(dev), masks[0].to(dev), unl[0].to(dev) if semi else None,
                         unl[1].to(dev) if semi else None, 30, 0, {'train': tcfg})
        torch.cuda.synchronize()
        grads[name] = {n: p.grad.detach().double().cpu() / S for n, p in student.named_parameters()}
        snn.set_compute_dtype(torch.bfloat16)
    ref = grads['o64']
    rows = []
    for n, r in ref.items():
        nr = float(r.pow(2).mean().sqrt()) + 1e-30
        mx = float(r.abs().max()) + 1e-30
        e = {k: (float((grads[k][n] - r).pow(2).mean().sqrt()) / nr, float((grads[k][n] - r).abs().max()) / mx)
             for k in ('o32', 'o16', 'hip32', 'hip16')}
        rows.append((e['hip16'][0], n, e, mx))
    rows.sort(reverse=True)
    print(f'== variant {variant}')
    watch = [r for r in rows if 'denseBlocksUp.4' in r[1] or 'conv1x1_up.4' in r[1] or 'finalConv' in r[1]]
    print('the last decoder stage (the r6 C5 test outliers):')
    for _, n, e, mx in sorted(watch, key=lambda r: r[1]):
        print('%-48s %10.3g %s' % (n[:48], mx, ' '.join('%9.2e(%8.1e)' % e[k] for k in ('o32', 'o16', 'hip32', 'hip16'))))
    print('step-0 student gradients vs oracle fp64: rel-RMS (rel-max) per tensor, worst hip16 first')
    print('%-48s %10s %19s %19s %19s %19s' % ('tensor', 'max|g64|', 'oracle32', 'oracle16', 'hip32', 'hip16'))
    for _, n, e, mx in rows[:15]:
        print('%-48s %10.3g %s' % (n[:48], mx, ' '.join('%9.2e(%8.1e)' % e[k] for k in ('o32', 'o16', 'hip32', 'hip16'))))
    agg = {k: np.median([r[2][k][0] for r in rows]) for k in ('o32', 'o16', 'hip32', 'hip16')}
    print('median rel-RMS:', agg)


if __name__ == '__main__':
    for v in (sys.argv[1:] or ['full']):
        main(v)
