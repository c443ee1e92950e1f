"""Diagnose the unsupervised (consistency) loss deviation HIP vs oracle on the G7 golden setup, step 0:
compares every intermediate of train.py:66-115 (teacher logits, CowMix mask, mixed inputs, student
logits, confidence mask, loss) and attributes the loss error by swapping one operand at a time.

    python tools/diag_unsup.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conftest import golden  # noqa: E402
from oracle import cowmix_ref, models_ref, train_ref  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def main():
    import losses
    from models import simple_unet
    from models.adapters import ListOutput
    from ssseg import arena, ops
    from ssseg import nn as snn
    dev = torch.device('cuda:0')
    snn.set_compute_dtype(torch.float32)
    g = golden('trainsteps.npz')

    def load(m):
        sd = {k[5:]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith('init.')}
        m.load_state_dict(sd, strict=True)
        return m
    s = load(ListOutput(simple_unet.UNet(2, num_blocks=2, first_channels=4, max_width=8))).to(dev)
    t = load(ListOutput(simple_unet.UNet(2, num_blocks=2, first_channels=4, max_width=8))).to(dev)
    for p in t.parameters():
        p.detach_()
    t.eval()
    arena.attach(s)
    arena.attach(t, with_grads=False)
    rs = models_ref.load_state(models_ref.ListOutput(models_ref.SimpleUNet(2, 2, 4, 8)), g, 'init.')
    rt = models_ref.load_state(models_ref.ListOutput(models_ref.SimpleUNet(2, 2, 4, 8)), g, 'init.')
    for p in rt.parameters():
        p.detach_()
    rt.eval()
    imgs, masks, unl = (torch.from_numpy(g[k]) for k in ('imgs', 'masks', 'unl'))
    loss = losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits('mean'), 'weight': [0.5]}])
    # supervised pass (train mode: BN running stats move)
    s.train()
    rs.train()
    _, pm = s(imgs[0].to(dev))
    sup = loss(pm, masks[0].to(dev))
    sup.backward()
    _, rpm = rs(imgs[0])
    rsup = train_ref.calculate_loss(rpm, masks[0])
    rsup.backward()
    print(f'sup loss hip {float(sup):.9g} ref {float(rsup):.9g} rel {abs(float(sup) - float(rsup)) / float(rsup):.2e}')
    ua, ub = unl[0], unl[1]
    with torch.no_grad(), snn.folded(t):
        ta = ops.interpolate_bilinear(t(ua.to(dev))[-1][-1], ua.shape[2:4]).cpu()
        tb = ops.interpolate_bilinear(t(ub.to(dev))[-1][-1], ua.shape[2:4]).cpu()
    with torch.no_grad():
        rta = F.interpolate(rt(ua)[-1][-1], ua.shape[2:4], mode='bilinear', align_corners=False)
        rtb = F.interpolate(rt(ub)[-1][-1], ua.shape[2:4], mode='bilinear', align_corners=False)
    print(f'teacher logits rel err a {rel(ta, rta):.2e} b {rel(tb, rtb):.2e}')
    torch.manual_seed(int(g['rng_seed']))
    B, _, H, W = ua.shape
    pp, sig, noise = cowmix_ref.draw_inputs(B, H, W, (0.45, 0.55), (2, 4))
    rm, *_ = cowmix_ref.cowmix_masks(noise, sig, pp)
    rm = torch.from_numpy(rm).view(B, 1, H, W).float()
    hm = ops.cowmix_mask(torch.from_numpy(noise).to(dev), torch.from_numpy(sig).to(dev),
                         torch.from_numpy(pp).to(dev)).cpu()
    print(f'cowmix mask flips {int((hm != rm).sum())} of {rm.numel()}')
    for name, m in (('hip-mask', hm), ('ref-mask', rm)):
        x_mix = ua * m + ub * (1 - m)
        t_mix_h = ta * m + tb * (1 - m)
        t_mix_r = rta * m + rtb * (1 - m)
        s.eval()
        with snn.folded(s):
            sh = s(x_mix.to(dev))[-1][-1]
        s.train()
        sh = ops.interpolate_bilinear(sh, x_mix.shape[2:4])
        rs.eval()
        sr = rs(x_mix)[-1][-1]
        rs.train()
        sr = F.interpolate(sr, x_mix.shape[2:4], mode='bilinear', align_corners=False)
        shc = sh.detach().cpu()
        print(f'[{name}] student logits rel err {rel(shc, sr.detach()):.2e}; |sig(s)-sig(t)| mean '
              f'{float((torch.sigmoid(sr) - torch.sigmoid(t_mix_r)).abs().mean()):.3e}')
        thr = 0.5
        cm_h = (torch.sigmoid(t_mix_h).max(1).values > thr)
        cm_r = (torch.sigmoid(t_mix_r).max(1).values > thr)
        band = (torch.sigmoid(t_mix_r).max(1).values - thr).abs()
        print(f'[{name}] cm flips {int((cm_h != cm_r).sum())}, min |maxsig-thr| {float(band.min()):.2e}')
        l_hh, _ = ops.consistency_loss(sh, t_mix_h.to(dev), thr)
        l_rr, _ = train_ref.consistency_loss(sr.detach(), t_mix_r, thr)
        l_hr, _ = train_ref.consistency_loss(shc, t_mix_r, thr)     # HIP student, ref teacher
        l_rh, _ = train_ref.consistency_loss(sr.detach(), t_mix_h, thr)   # ref student, HIP teacher
        l_hh_cpu, _ = train_ref.consistency_loss(shc, t_mix_h, thr)      # HIP operands, CPU loss arithmetic
        lr = float(l_rr)
        print(f'[{name}] loss ref {lr:.9g} hip {float(l_hh):.9g} rel {(float(l_hh) - lr) / lr:.2e} | '
              f'hip-s/ref-t {(float(l_hr) - lr) / lr:.2e} ref-s/hip-t {(float(l_rh) - lr) / lr:.2e} '
              f'hip-operands/cpu-loss {(float(l_hh_cpu) - lr) / lr:.2e}')
        # fp64 oracle of the same student pass for conditioning
        rs64 = models_ref.ListOutput(models_ref.SimpleUNet(2, 2, 4, 8)).double()
        rs64.load_state_dict(rs.state_dict())
        rs64.eval()
        s64 = F.interpolate(rs64(x_mix.double())[-1][-1], x_mix.shape[2:4], mode='bilinear', align_corners=False)
        l64, _ = train_ref.consistency_loss(s64.detach(), t_mix_r.double(), thr)
        print(f'[{name}] ref fp32 vs fp64 student: logits rel {rel(sr.detach(), s64.detach()):.2e}, '
              f'loss rel {(lr - float(l64)) / float(l64):.2e}')


if __name__ == '__main__' and len(sys.argv) == 1:
    main()


def steps():
    """G7's three steps through train.train_step vs the oracle in fp32 and fp64: per-step unsup loss, the
    gradient error before each optimizer step and the parameter error after it."""
    import cowmix
    import losses
    import train
    from models import simple_unet
    from models.adapters import ListOutput
    from ssseg import arena, optim
    from ssseg import nn as snn
    dev = torch.device('cuda:0')
    snn.set_compute_dtype(torch.float32)
    g = golden('trainsteps.npz')
    fn = lambda: ListOutput(simple_unet.UNet(2, num_blocks=2, first_channels=4, max_width=8))  # noqa: E731
    sd0 = {k[5:]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith('init.')}
    s, t = fn(), fn()
    s.load_state_dict(sd0)
    t.load_state_dict(sd0)
    s, t = s.to(dev), t.to(dev)
    for p in t.parameters():
        p.detach_()
    t.eval()
    arena.attach(s)
    arena.attach(t, with_grads=False)
    opt = optim.SGD(s.parameters(), lr=float(g['lr']), momentum=0.9, weight_decay=0.0005)
    cfg = {'train': dict(loss=losses.CalculateLoss([
        {'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'), 'weight': [0.5]}]),
        virtual_batch_size_multiplier=1, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
        sigma_range=(2, 4), confidence_threshold=0.5, consistency_loss_weight=10, ema_model_alpha=0.99,
        print_freq=1, gradient_clip_value=5.0)}
    imgs, masks, unl = (torch.from_numpy(g[k]) for k in ('imgs', 'masks', 'unl'))
    cowmix.NOISE_SOURCE = 'cpu'
    torch.manual_seed(int(g['rng_seed']))
    s.train()
    opt.zero_grad()
    hip = []
    orig_step = opt.step

    def rec_step(*a, **k):
        hip[-1]['grad'] = {n: p.grad.detach().double().cpu().clone() for n, p in s.named_parameters()}
        return orig_step(*a, **k)
    opt.step = rec_step
    for step in range(3):
        hip.append({})
        c, u, _ = train.train_step(s, t, opt, imgs[step].to(dev), masks[step].to(dev), unl[2 * step].to(dev),
                                   unl[2 * step + 1].to(dev), 30, step, cfg)
        hip[-1].update(u=float(u), s={k: v.double().cpu() for k, v in s.state_dict().items()},
                       t={k: v.double().cpu() for k, v in t.state_dict().items()})
    cowmix.NOISE_SOURCE = 'device'

    def oracle(dt):
        rs = models_ref.load_state(models_ref.ListOutput(models_ref.SimpleUNet(2, 2, 4, 8)), g, 'init.').to(dt)
        rt = models_ref.load_state(models_ref.ListOutput(models_ref.SimpleUNet(2, 2, 4, 8)), g, 'init.').to(dt)
        for p in rt.parameters():
            p.detach_()
        rt.eval()
        ro = torch.optim.SGD(rs.parameters(), lr=float(g['lr']), momentum=0.9, weight_decay=0.0005)
        recs = []
        orig = ro.step

        def rstep(*a, **k):
            recs[-1]['grad'] = {n: p.grad.detach().double().clone() for n, p in rs.named_parameters()}
            return orig(*a, **k)
        ro.step = rstep

        def on_step(k, rec):
            recs[-1].update(u=rec['unsup_loss'], s={a: b.double().clone() for a, b in rs.state_dict().items()},
                            t={a: b.double().clone() for a, b in rt.state_dict().items()})
            recs.append({})
        recs.append({})
        torch.manual_seed(int(g['rng_seed']))
        train_ref.train_epoch(rs, rt, ro, list(zip(imgs.to(dt), masks.to(dt))), iter(unl.to(dt)), 30,
                              train_ref.default_cfg(sigma_range=(2, 4), confidence_threshold=0.5), on_step=on_step)
        return recs[:3]
    r32, r64 = oracle(torch.float32), oracle(torch.float64)

    def err(a, b):   # worst per-tensor relative RMS error
        w = 0.0
        for k in b:
            if not b[k].dtype.is_floating_point:
                continue
            n = float(b[k].pow(2).mean().sqrt()) + 1e-30
            w = max(w, float((a[k].double() - b[k]).pow(2).mean().sqrt()) / n)
        return w
    for k in range(3):
        h, a, b = hip[k], r32[k], r64[k]
        line = (f'step {k}: unsup hip {h["u"]:.9g} ref32 {a["u"]:.9g} ref64 {b["u"]:.9g} golden {float(g["unsup_loss"][k]):.9g} | '
                f'rel hip-64 {(h["u"] - b["u"]) / b["u"]:.2e} ref32-64 {(a["u"] - b["u"]) / b["u"]:.2e}')
        if 'grad' in h and 'grad' in b:
            line += f' | grad err hip {err(h["grad"], b["grad"]):.2e} ref32 {err(a["grad"], b["grad"]):.2e}'
        line += (f' | student err hip {err(h["s"], b["s"]):.2e} ref32 {err(a["s"], b["s"]):.2e}'
                 f' | teacher err hip {err(h["t"], b["t"]):.2e} ref32 {err(a["t"], b["t"]):.2e}')
        d64 = {kk: b['s'][kk] - b['t'][kk] for kk in b['s'] if b['s'][kk].dtype.is_floating_point}
        dh = {kk: h['s'][kk] - h['t'][kk] for kk in d64}
        line += f' | (student-teacher) err hip {err(dh, d64):.2e}'
        print(line)


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'steps':
    steps()
