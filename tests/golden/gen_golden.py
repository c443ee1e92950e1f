"""Generate golden vectors from the reference (Luonic/semi-supervised_semantic_segmentation).

RUNS ONLY IN THE BUILD CONTAINER, where the reference is mounted read-only at /root/reference.
It imports the reference's own Python modules (with an empty `kornia` stub, which train.py imports
but never calls: reference/train.py:5, reversible_augmentations.py) and writes small .npz
fixtures next to this file. The fixtures are data (inputs + expected outputs); nothing from the
reference travels with them. Tests on the GPU box read only the .npz files.

Fixture index:
  G1  cowmix_*.npz      generate_cowmix_masks_like / generate_gaussian      (reference/cowmix.py:6-69)
  G2  mix.npz           mix_with_mask                                     (reference/cowmix.py:72-73)
  G3  consistency_*.npz train.train one step with stub models: BCE(+interp) loss, CowMix,
                        consistency loss value + gradients, EMA (reference/train.py:41-130)
  G4  lovasz.npz        binary_lovasz_loss_with_logits + lovasz_grad        (reference/losses.py:239-250, lovasz.py)
  G5  ema.npz           update_ema_variables                              (reference/mean_teacher.py:5-18)
  G6  model_*.npz       SimpleUNet / UNet(MobileNetV2) forwards            (reference/models/*.py)
  G7  trainsteps.npz    3 steps of train.train on a tiny SimpleUNet (DDP, gloo world 1)
  G9  metrics_*.npz     train.validate's Dice (argmax one-hot -> nearest resize -> metrics.dice_metric) and
                        lovasz.iou on the same predictions                 (reference/train.py:171-176,
                        metrics.py:1-7, lovasz.py:54-73)
  G10 inference.npz    models.inference_wrapper.InferenceWrapper on a stub model (reference/models/inference_wrapper.py)
  G6b model2_*.npz      HarDNet / Discriminator / MultiscaleFeatureDiscriminator / MultiscaleAttention(HRNet)
                        forwards (eval + train), input + selected parameter gradients, BN buffers; weights are
                        seeded (tests/seeded.py) and pinned by a state_dict SHA-256 instead of stored
  G11 msa_trainsteps.npz 2 steps of train.train on MultiscaleAttention(HigherHRNet-W32, 480, 2) at 128^2, bs 2 (config
                        C4's model family; DDP gloo world 1), fp32 and fp64; parameters / BN buffers after the steps
                        as seeded index samples                            (reference/train.py:41-130,
                        models/multiscale_attention.py:38-58)
  G12 rmi_*.npz         RMILoss forward + input gradient: the default-config RMI (radius 3, avg pool 4/4) and two
                        generic cases (3 classes / radius 2 / pool 3; radius 1 / no pooling)  (reference/losses.py:271-592)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [all | models2 | metrics | msa_trainsteps | rmi]
"""
import os
import sys
import types
import hashlib

import numpy as np

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))

sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.modules.setdefault('kornia', types.ModuleType('kornia'))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import cowmix  # noqa: E402  (reference)
import losses  # noqa: E402
import lovasz  # noqa: E402
import mean_teacher  # noqa: E402
import metrics  # noqa: E402
import train as ref_train  # noqa: E402
from models import simple_unet, unet  # noqa: E402
from models.encoders import mobilenetv2  # noqa: E402

torch.set_num_threads(8)
META = dict(torch_version=torch.__version__)


def sha(t):
    return hashlib.sha256(np.ascontiguousarray(t.detach().cpu().numpy()).tobytes()).hexdigest()


def save(name, **arrays):
    path = os.path.join(OUT, name)
    out = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        out[k] = np.asarray(v)
    out['torch_version'] = np.asarray(META['torch_version'])
    np.savez_compressed(path, **out)
    print(f'wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB')


def state_arrays(prefix, module):
    d = {}
    for k, v in module.state_dict().items():
        d[prefix + k] = v.detach().clone()
    return d


# ----------------------------------------------------------------------------------------------
# G1: CowMix masks
# ----------------------------------------------------------------------------------------------
def gen_cowmix():
    cases = [
        # (tag, seed, shape, mask_proportion_range, sigma_range, keep_field)
        ('a0', 0, (4, 3, 128, 128), (0.45, 0.55), (8, 32), True),
        ('a1', 1, (4, 3, 128, 128), (0.45, 0.55), (8, 32), False),
        ('a2', 2, (4, 3, 128, 128), (0.45, 0.55), (8, 32), False),
        ('b3', 3, (2, 3, 96, 80), (0.4, 0.6), (4, 16), True),
        ('c0', 0, (2, 3, 512, 512), (0.45, 0.55), (8, 32), False),
    ]
    for tag, seed, shape, pr, sr, keep_field in cases:
        example = torch.zeros(shape)
        torch.manual_seed(seed)
        mask = cowmix.generate_cowmix_masks_like(example, pr, sr)
        # Replay the reference RNG order (cowmix.py:44-55): rand(B) for p, rand(B) for sigma, normal.
        torch.manual_seed(seed)
        B = shape[0]
        p = torch.distributions.Uniform(torch.tensor(pr[0]), torch.tensor(pr[1])).rsample([B])
        import math
        sig = torch.exp(torch.distributions.Uniform(torch.tensor(math.log(float(sr[0]))),
                                                    torch.tensor(math.log(float(sr[1])))).rsample([B]))
        noise = torch.normal(mean=0, std=1, size=(B, 1) + tuple(shape[2:]), dtype=torch.float32)
        field = cowmix.dual_pass_gaussian_fileter2d(noise.transpose(0, 1), sig).transpose(1, 0)
        mean = field.mean(dim=(1, 2, 3))
        std = field.std(dim=(1, 2, 3))
        thr = torch.erfinv(2 * p - 1) * math.sqrt(2.0) * std + mean
        replay = (field > thr.view(B, 1, 1, 1)).float()
        assert torch.equal(replay, mask), 'RNG replay does not reproduce the reference mask'
        K = int(round(sig.max().item() * 3) * 2) + 1
        d = dict(seed=seed, shape=np.array(shape), prop_range=np.array(pr, dtype=np.float64),
                 sigma_range=np.array(sr, dtype=np.float64), p=p, sigma=sig, K=K,
                 noise_sha256=np.asarray(sha(noise)), mean=mean, std=std, thr=thr,
                 mask_bits=np.packbits(mask.numpy().astype(np.uint8).reshape(-1)),
                 # distance of every pixel to its threshold in units of std: the tie band
                 tie_band_count=int(((field - thr.view(B, 1, 1, 1)).abs()
                                     < 1e-5 * std.view(B, 1, 1, 1)).sum()))
        if keep_field:
            d['field'] = field
            d['noise'] = noise
        save(f'cowmix_{tag}.npz', **d)

    # generate_gaussian (cowmix.py:6-11): odd and even window sizes
    gs = {}
    for K, s in [(7, 1.3), (8, 2.0), (49, 8.0), (193, 31.7), (97, 16.2)]:
        gs[f'g_{K}'] = cowmix.generate_gaussian(K, torch.tensor(s))
        gs[f'sigma_{K}'] = np.float32(s)
    save('cowmix_gaussian.npz', **gs)


# ----------------------------------------------------------------------------------------------
# G2: mix_with_mask
# ----------------------------------------------------------------------------------------------
def gen_mix():
    g = torch.Generator().manual_seed(11)
    a = torch.randn(2, 3, 16, 24, generator=g)
    b = torch.randn(2, 3, 16, 24, generator=g)
    m = (torch.rand(2, 1, 16, 24, generator=g) > 0.5).float()
    save('mix.npz', a=a, b=b, mask=m, out=cowmix.mix_with_mask(a, b, m))


# ----------------------------------------------------------------------------------------------
# helpers for driving reference train.train
# ----------------------------------------------------------------------------------------------
class ScalarLog:
    def __init__(self):
        self.rows = []

    def add_scalar(self, name, value, step):
        self.rows.append((name, float(value), int(step)))


def ensure_pg():
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29533')
        dist.init_process_group('gloo', rank=0, world_size=1)


class StubLogits(nn.Module):
    """A 'model' whose logits are a learnable tensor (+0*x so autograd sees the input)."""

    def __init__(self, init):
        super().__init__()
        self.logits = nn.Parameter(init.clone())

    def forward(self, x):
        y = self.logits + 0.0 * x.sum()
        return [y], [y]


# ----------------------------------------------------------------------------------------------
# G3: one train.train step with stub models -> BCE/CalculateLoss, CowMix, consistency, EMA
# ----------------------------------------------------------------------------------------------
def gen_consistency():
    ensure_pg()
    cases = [
        # tag, seed, B, H, W, h, w, thr, epoch, logit_scale
        ('thr05', 5, 2, 64, 64, 32, 32, 0.5, 30, 3.0),
        ('thr097', 6, 3, 48, 40, 24, 20, 0.97, 30, 4.0),
        ('nan', 7, 2, 32, 32, 16, 16, 0.97, 30, 0.1),   # sigmoid < 0.97 everywhere -> 0/0 = NaN
        ('gated', 8, 2, 32, 32, 16, 16, 0.5, 10, 3.0),   # epoch <= 25 -> unsup loss * 0
    ]
    for tag, seed, B, H, W, h, w, thr, epoch, scale in cases:
        g = torch.Generator().manual_seed(seed)
        s_init = torch.randn(B, 2, h, w, generator=g) * scale
        t_init = torch.randn(B, 2, h, w, generator=g) * scale
        image = torch.rand(B, 3, H, W, generator=g)
        target_fg = (torch.rand(B, 1, H, W, generator=g) > 0.6).float()
        semantic_mask = torch.cat([1 - target_fg, target_fg], dim=1)
        ua = torch.rand(B, 3, H, W, generator=g)
        ub = torch.rand(B, 3, H, W, generator=g)
        student = StubLogits(s_init)
        teacher = StubLogits(t_init)
        mean_teacher.detach_model_parameters(teacher)
        teacher.eval()
        opt = torch.optim.SGD(student.parameters(), lr=0.0)
        cfg = {'train': dict(loss=losses.CalculateLoss([
            {'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'), 'weight': [0.5]}]),
            virtual_batch_size_multiplier=1, use_semi_supervised=True,
            mask_proportion_range=(0.45, 0.55), sigma_range=(4, 8), confidence_threshold=thr,
            consistency_loss_weight=10, ema_model_alpha=0.99, print_freq=1, gradient_clip_value=5.0)}
        log = ScalarLog()
        torch.manual_seed(1000 + seed)
        ref_train.train(student, teacher, opt, [{'image': image, 'semantic_mask': semantic_mask}],
                        iter([{'image': ua}, {'image': ub}]), epoch, 0, log, cfg, 'cpu')
        vals = {n: v for n, v, _ in log.rows}
        save(f'consistency_{tag}.npz', seed=seed, rng_seed=1000 + seed, thr=thr, epoch=epoch,
             s_logits=s_init, t_logits=t_init, image=image, semantic_mask=semantic_mask, ua=ua, ub=ub,
             sup_loss=np.float32(vals['train_classification_loss']),
             unsup_loss=np.float32(vals['train_unsupervised_loss']),
             grad=student.logits.grad, ema_after=teacher.logits.detach())


# ----------------------------------------------------------------------------------------------
# G4: Lovasz
# ----------------------------------------------------------------------------------------------
def gen_lovasz():
    g = torch.Generator().manual_seed(21)
    B, H, W = 3, 64, 64
    logits = (torch.randn(B, 2, H, W, generator=g) * 2.0).requires_grad_(True)
    fg = (torch.rand(B, 1, H, W, generator=g) > 0.55).float()
    fg[1] = 0.0  # an all-background image: valid = 0 path (losses.py:247)
    target = torch.cat([1 - fg, fg], dim=1)
    loss = losses.binary_lovasz_loss_with_logits(logits, target)
    loss.backward()
    gt = torch.tensor([1, 0, 1, 1, 0, 0, 1, 0], dtype=torch.float32)
    save('lovasz.npz', logits=logits.detach(), target=target, loss=loss.detach(), grad=logits.grad,
         gt_sorted=gt, lovasz_grad=lovasz.lovasz_grad(gt),
         lovasz_grad_1=lovasz.lovasz_grad(torch.tensor([1.0])))


# ----------------------------------------------------------------------------------------------
# G5: EMA
# ----------------------------------------------------------------------------------------------
def gen_ema():
    torch.manual_seed(31)
    student = simple_unet.UNet(2, num_blocks=2, first_channels=4, max_width=8)
    teacher = simple_unet.UNet(2, num_blocks=2, first_channels=4, max_width=8)
    for b in student.buffers():
        if torch.is_floating_point(b):
            b.uniform_(0.5, 1.5)
    before_t = state_arrays('t.', teacher)
    before_s = state_arrays('s.', student)
    mean_teacher.update_ema_variables(student, teacher, alpha=0.99)
    alias = all(eb.data_ptr() == sb.data_ptr() for eb, sb in zip(teacher.buffers(), student.buffers()))
    assert alias
    after = state_arrays('after.', teacher)
    save('ema.npz', alpha=0.99, buffers_aliased=alias, **before_t, **before_s, **after)


# ----------------------------------------------------------------------------------------------
# G6: model forwards
# ----------------------------------------------------------------------------------------------
def gen_models():
    specs = [
        ('simple_unet_t', lambda: simple_unet.UNet(2, num_blocks=3, first_channels=8, max_width=32,
                                                   train_upsampling=True), (2, 3, 32, 32)),
        ('simple_unet_b', lambda: simple_unet.UNet(2, num_blocks=3, first_channels=8, max_width=32,
                                                   train_upsampling=False), (2, 3, 36, 36)),
        ('unet_mbv2_t', lambda: unet.UNet(2, mobilenetv2.mobilenet_v2(width_mult=0.35), 32,
                                          train_upsampling=True), (2, 3, 64, 64)),
        ('unet_mbv2_b', lambda: unet.UNet(2, mobilenetv2.mobilenet_v2(width_mult=0.35), 32,
                                          train_upsampling=False), (2, 3, 64, 64)),
    ]
    for i, (tag, fn, shape) in enumerate(specs):
        torch.manual_seed(41 + i)
        m = fn()
        # non-trivial BN affine + running stats so eval mode is a real test
        with torch.no_grad():
            for mod in m.modules():
                if isinstance(mod, nn.BatchNorm2d):
                    mod.weight.uniform_(0.5, 1.5)
                    mod.bias.uniform_(-0.2, 0.2)
                    mod.running_mean.uniform_(-0.1, 0.1)
                    mod.running_var.uniform_(0.5, 2.0)
        init = state_arrays('init.', m)
        x = torch.rand(*shape)
        m.eval()
        with torch.no_grad():
            y_eval = m(x)
        m.train()
        y_train = m(x)
        # after the train-mode forward only the BN buffers change
        after = {k: v for k, v in state_arrays('after.', m).items() if 'running' in k or 'num_batches' in k}
        save(f'model_{tag}.npz', x=x, y_eval=y_eval, y_train=y_train.detach(), **init, **after)


# ----------------------------------------------------------------------------------------------
# G7: three reference train steps, tiny SimpleUNet, DDP on gloo world 1
# ----------------------------------------------------------------------------------------------
class ListOutput(nn.Module):
    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, x):
        y = self.model(x)
        return [y], [y]


def gen_trainsteps():
    ensure_pg()
    torch.manual_seed(51)
    fn = lambda: ListOutput(simple_unet.UNet(2, num_blocks=2, first_channels=4, max_width=8))  # noqa: E731
    student = fn()
    teacher = fn()
    teacher.load_state_dict(student.state_dict())
    init = state_arrays('init.', student)
    ddp = torch.nn.parallel.DistributedDataParallel(student)
    mean_teacher.detach_model_parameters(teacher)
    teacher.eval()
    opt = torch.optim.SGD(ddp.parameters(), lr=0.05, momentum=0.9, weight_decay=0.0005)
    g = torch.Generator().manual_seed(52)
    B, H, W, steps = 2, 32, 32, 3
    imgs = torch.rand(steps, B, 3, H, W, generator=g)
    fg = (torch.rand(steps, B, 1, H, W, generator=g) > 0.5).float()
    masks = torch.cat([1 - fg, fg], dim=2)
    unl = torch.rand(2 * steps, B, 3, H, W, generator=g)
    cfg = {'train': dict(loss=losses.CalculateLoss([
        {'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'), 'weight': [0.5]}]),
        virtual_batch_size_multiplier=1, use_semi_supervised=True,
        mask_proportion_range=(0.45, 0.55), sigma_range=(2, 4), confidence_threshold=0.5,
        consistency_loss_weight=10, ema_model_alpha=0.99, print_freq=1, gradient_clip_value=5.0)}
    log = ScalarLog()
    torch.manual_seed(53)
    ref_train.train(ddp, teacher, opt, [{'image': imgs[i], 'semantic_mask': masks[i]} for i in range(steps)],
                    iter([{'image': unl[i]} for i in range(2 * steps)]), 30, 0, log, cfg, 'cpu')
    sup = [v for n, v, _ in log.rows if n == 'train_classification_loss'][:steps]
    uns = [v for n, v, _ in log.rows if n == 'train_unsupervised_loss'][:steps]
    final_s = state_arrays('final_s.', student)
    final_t = state_arrays('final_t.', teacher)
    save('trainsteps.npz', imgs=imgs, masks=masks, unl=unl, rng_seed=53, lr=0.05,
         sup_loss=np.array(sup, np.float32), unsup_loss=np.array(uns, np.float32),
         **init, **final_s, **final_t)


# ----------------------------------------------------------------------------------------------
# G6b: the C3-C5 model families (seeded weights + SHA; inputs, outputs, gradients)
# ----------------------------------------------------------------------------------------------
def _yacs_shim():
    """higher_hrnet.py:23 imports yacs (absent here): a dict with attribute access is all it uses."""
    class CfgNode(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError:
                raise AttributeError(k)

        def __setattr__(self, k, v):
            self[k] = v
    yacs = types.ModuleType('yacs')
    cfgmod = types.ModuleType('yacs.config')
    cfgmod.CfgNode = CfgNode
    yacs.config = cfgmod
    sys.modules.setdefault('yacs', yacs)
    sys.modules.setdefault('yacs.config', cfgmod)


def sha_of(t):
    return hashlib.sha256(np.ascontiguousarray(t.detach().cpu().numpy()).tobytes()).hexdigest()


def gen_models2():
    sys.path.insert(0, os.path.dirname(OUT))      # tests/ (seeded.py)
    import seeded
    _yacs_shim()
    from functools import partial
    from models import discriminator, hardnet, higher_hrnet, multiscale_attention

    def msa():
        return multiscale_attention.MultiscaleAttention(
            partial(higher_hrnet.get_pose_net, cfg=higher_hrnet.POSE_HIGHER_RESOLUTION_NET), 480, 2)

    specs = [
        # tag, ctor, seed, input shapes, conv re-init, parameter grads to store
        ('hardnet', lambda: hardnet.HarDNet(n_classes=2), 61, [(2, 3, 256, 256)], None,
         ['base.0.conv.weight', 'base.4.layers.1.conv.weight', 'denseBlocksUp.4.layers.3.conv.weight',
          'finalConv.weight', 'finalConv.bias', 'base.0.norm.weight']),
        ('disc', lambda: discriminator.Discriminator(5, 2, 64, 512, 1), 62, [(2, 2, 64, 64)], None,
         ['net.0.0.weight', 'net.0.0.bias', 'net.1.0.weight', 'net.4.0.bias', 'net.5.0.weight']),
        ('msdisc', lambda: discriminator.MultiscaleFeatureDiscriminator([8, 16, 32, 64], [16, 32, 64, 128, 1]), 63,
         [(2, 8, 32, 32), (2, 16, 16, 16), (2, 32, 8, 8), (2, 64, 4, 4)], None, 'all'),
        ('msa_hrnet', msa, 64, [(2, 3, 128, 128)], 'he',
         ['model.stem.conv1.weight', 'model.stage3.mods.0.fuse_module.fuse_layers.2.0.0.conv.weight',
          'model.cls_head.2.weight', 'model.cls_head.2.bias', 'attention_head.0.bn.weight',
          'attention_head.2.weight', 'model.stage4.mods.2.branches.3.1.bn2.weight']),
    ]
    for tag, ctor, seed, shapes, conv_std, grad_names in specs:
        torch.manual_seed(seed)
        m = ctor()
        seeded.perturb(m, seed + 1000, conv_std)
        sha = seeded.state_sha(m)
        g = torch.Generator().manual_seed(seed + 2000)
        xs = [torch.rand(*s, generator=g) for s in shapes]
        arg = xs if len(xs) > 1 else xs[0]

        def logits(out):
            return out[1][-1] if isinstance(out, tuple) else out
        import copy
        m64 = copy.deepcopy(m).double()      # the same network in fp64: the yardstick for fp32 rounding
        d = dict(seed=seed, sha=np.asarray(sha), n_inputs=len(xs))
        gy = None
        for net, suf, dt in ((m, '', torch.float32), (m64, '64', torch.float64)):
            xin = [x.clone().to(dt) for x in xs]
            a = xin if len(xin) > 1 else xin[0]
            net.eval()
            with torch.no_grad():
                d['y_eval' + suf] = logits(net(a)).clone()
            net.train()
            for x in xin:
                x.requires_grad_(True)
            y_train = logits(net(a))
            if gy is None:
                gy = torch.randn(y_train.shape, generator=g)
            (y_train * gy.to(dt)).sum().backward()
            d['y_train' + suf] = y_train.detach()
            params = dict(net.named_parameters())
            names = list(params) if grad_names == 'all' else grad_names
            for i, x in enumerate(xin):     # large inputs are regenerated from the seed in the test (SHA-checked)
                d[f'shape{i}'] = np.array(xs[i].shape)
                if xs[i].numel() <= 200_000:
                    d[f'x{i}'] = xs[i]
                    d[f'xgrad{i}' + suf] = x.grad
                else:
                    d[f'x{i}_sha'] = np.asarray(sha_of(xs[i]))
            for n in names:
                d[f'grad{suf}.' + n] = params[n].grad
        if gy.numel() <= 200_000:
            d['gy'] = gy
        else:
            d['gy_sha'] = np.asarray(sha_of(gy))
        d = {k: (v.float() if isinstance(v, torch.Tensor) and v.dtype == torch.float64 else v) for k, v in d.items()}
        for k, v in m.state_dict().items():
            if 'running' in k or 'num_batches' in k:
                d['after.' + k] = v
        save(f'model2_{tag}.npz', **d)


# ----------------------------------------------------------------------------------------------
# G11: two reference train steps of config C4's model family (MultiscaleAttention over HigherHRNet-W32, 480 feature
# channels, 2 scales) at 128x128, bs 2, DDP on gloo world 1, fp32 and fp64
# ----------------------------------------------------------------------------------------------
def _sample_idx(n, i, k=256):
    g = torch.Generator().manual_seed(7000 + i)
    return torch.sort(torch.randperm(n, generator=g)[:k]).values


def gen_msa_trainsteps():
    """The student's parameters and BN buffers after 2 steps are stored as seeded index samples (256 elements per
    tensor, _sample_idx; the whole network is 29 M parameters); the fp64 run is the same reference code on a
    .double() copy with the CowMix draws taken in fp32 (the noise draw otherwise consumes the generator differently
    in fp64, giving a different mask) -- the fp32 rounding yardstick of tests/parity.py."""
    ensure_pg()
    sys.path.insert(0, os.path.dirname(OUT))      # tests/ (seeded.py)
    import copy
    import seeded
    _yacs_shim()
    from functools import partial
    from models import higher_hrnet, multiscale_attention
    seed = 64
    torch.manual_seed(seed)
    m = multiscale_attention.MultiscaleAttention(
        partial(higher_hrnet.get_pose_net, cfg=higher_hrnet.POSE_HIGHER_RESOLUTION_NET), 480, 2)
    seeded.perturb(m, seed + 1000, 'he')
    sha = seeded.state_sha(m)
    g = torch.Generator().manual_seed(seed + 3000)
    B, H, steps = 2, 128, 2
    imgs = torch.rand(steps, B, 3, H, H, generator=g)
    fg = (torch.rand(steps, B, 1, H, H, generator=g) > 0.5).float()
    masks = torch.cat([1 - fg, fg], dim=2)
    unl = torch.rand(2 * steps, B, 3, H, H, generator=g)
    cfg = {'train': dict(loss=losses.CalculateLoss([
        {'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'), 'weight': [0.5]}]),
        virtual_batch_size_multiplier=1, use_semi_supervised=True,
        mask_proportion_range=(0.45, 0.55), sigma_range=(4, 8), confidence_threshold=0.5,
        consistency_loss_weight=10, ema_model_alpha=0.99, print_freq=1, gradient_clip_value=5.0)}
    init = m.state_dict()
    d = dict(seed=seed, sha=np.asarray(sha), rng_seed=seed + 4000, lr=0.01, imgs_sha=np.asarray(sha_of(imgs)),
             masks_sha=np.asarray(sha_of(masks)), unl_sha=np.asarray(sha_of(unl)))
    orig_cm = cowmix.generate_cowmix_masks_like
    for dt, suf in ((torch.float32, ''), (torch.float64, '64')):
        student = copy.deepcopy(m).to(dt)
        teacher = copy.deepcopy(m).to(dt)
        ddp = torch.nn.parallel.DistributedDataParallel(student)
        mean_teacher.detach_model_parameters(teacher)
        teacher.eval()
        opt = torch.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9, weight_decay=0.0005)
        cowmix.generate_cowmix_masks_like = (lambda t, **kw: orig_cm(t.float(), **kw).to(t.dtype))
        log = ScalarLog()
        torch.manual_seed(seed + 4000)
        try:
            ref_train.train(ddp, teacher, opt, [{'image': imgs[i].to(dt), 'semantic_mask': masks[i].to(dt)}
                                                for i in range(steps)],
                            iter([{'image': unl[i].to(dt)} for i in range(2 * steps)]), 30, 0, log, cfg, 'cpu')
        finally:
            cowmix.generate_cowmix_masks_like = orig_cm
        d['sup_loss' + suf] = np.array([v for n, v, _ in log.rows if n == 'train_classification_loss'][:steps])
        d['unsup_loss' + suf] = np.array([v for n, v, _ in log.rows if n == 'train_unsupervised_loss'][:steps])
        for i, (k, v) in enumerate(student.state_dict().items()):
            if not torch.is_floating_point(v):
                d[f'final{suf}.{k}'] = v
                continue
            idx = _sample_idx(v.numel(), i)
            if not suf:
                d['idx.' + k] = idx
                d['init.' + k] = init[k].reshape(-1)[idx]
            d[f'final{suf}.{k}'] = v.detach().reshape(-1)[idx].double()
        print('msa trainsteps', suf or '32', d['sup_loss' + suf], d['unsup_loss' + suf])
    save('msa_trainsteps.npz', **d)


# ----------------------------------------------------------------------------------------------
# G9: validation metrics (Dice + IoU)
# ----------------------------------------------------------------------------------------------
def gen_metrics():
    cases = {'a': (3, (33, 47), (64, 80)), 'b': (2, (32, 32), (64, 64)), 'c': (2, (16, 16), (16, 16))}
    for tag, (B, (h, w), (H, W)) in cases.items():
        g = torch.Generator().manual_seed(41 + ord(tag))
        logits = torch.randn(B, 2, h, w, generator=g)
        logits[:, 1, :3, :] = logits[:, 0, :3, :]            # ties: argmax keeps class 0
        soft = torch.rand(B, 1, H, W, generator=g)
        soft[:, :, :2, :] = 0.5                               # mask ties: label 0, t1 = 0
        soft[0] = soft[0] * 0.4                               # an image with no foreground
        mask = torch.cat([1 - soft, soft], dim=1)
        # reference/train.py:171-176
        one_hot = torch.nn.functional.one_hot(torch.argmax(logits, dim=1), num_classes=2).permute(
            dims=(0, 3, 1, 2)).to(logits)
        pred_bin = torch.nn.functional.interpolate(one_hot, size=mask.size()[2:4], mode='nearest')
        mask_bin = (mask > 0.5).to(mask)
        dice = metrics.dice_metric(pred_bin[:, 1:], mask_bin[:, 1:])
        pred = torch.argmax(pred_bin, dim=1)
        label = torch.argmax(mask, dim=1)
        ious = lovasz.iou(pred, label, 2)
        save(f'metrics_{tag}.npz', logits=logits, mask=mask, dice=dice, dice_mean=dice.mean(),
             ious=np.asarray(ious, dtype=np.float64))


# ----------------------------------------------------------------------------------------------
# G10: InferenceWrapper
# ----------------------------------------------------------------------------------------------
def gen_inference():
    from models.inference_wrapper import InferenceWrapper

    g = torch.Generator().manual_seed(51)
    logits = torch.randn(1, 2, 37, 50, generator=g) * 3
    logits[0, 1, :2] = logits[0, 0, :2]                       # ties -> class 0

    class Stub(nn.Module):
        def forward(self, image):
            return [image], [logits, logits[:, :, ::2, ::2]]

    image = torch.rand(3, 75, 101, generator=g)
    mask, prob = InferenceWrapper(Stub())(image)
    save('inference.npz', logits=logits, image_hw=np.asarray([75, 101]), mask=mask, prob=prob)


# ----------------------------------------------------------------------------------------------
# G12: RMILoss
# ----------------------------------------------------------------------------------------------
RMI_CASES = {
    # name: (N, C, H, W, RMILoss kwargs, gout)
    'rmi_a': (2, 2, 91, 70, dict(num_classes=2, rmi_radius=3, rmi_pool='avg', rmi_pool_size=4, rmi_pool_stride=4), 1.0),
    'rmi_b': (2, 3, 50, 47, dict(num_classes=3, rmi_radius=2, rmi_pool='avg', rmi_pool_size=3, rmi_pool_stride=3), 0.5),
    'rmi_c': (3, 2, 12, 9, dict(num_classes=2, rmi_radius=1, rmi_pool='none', rmi_pool_size=4, rmi_pool_stride=4), 2.0),
}


def gen_rmi():
    """The reference's RMILoss on the CPU.  Its one device-specific line is `.type(torch.cuda.DoubleTensor)`
    (losses.py:549-550); torch.cuda.DoubleTensor is mapped to torch.DoubleTensor for the call (the arithmetic is
    the reference's own: fp32 pooling, fp64 covariances, torch.inverse, torch.cholesky).  Inputs: seeded logits with
    saturated patches (the clamp at losses.py:515) and one-hot blob targets (configs/default_config.py:147 shape)."""
    saved = torch.cuda.DoubleTensor
    torch.cuda.DoubleTensor = torch.DoubleTensor
    try:
        for i, (name, (N, C, H, W, kw, gout)) in enumerate(RMI_CASES.items()):
            g = torch.Generator().manual_seed(61 + i)
            logits = torch.randn(N, C, H, W, generator=g) * 3.0
            logits[0, 0, :5, :7] = 25.0                       # sigmoid == 1.0 in fp32 (clamp max, inclusive)
            logits[-1, -1, -4:, -6:] = -30.0                  # sigmoid < 1e-6 (clamped, zero gradient)
            blob = F.avg_pool2d(torch.rand(N, 1, H, W, generator=g), 5, 1, 2) > 0.5
            lab = torch.randint(0, C, (N, 1, H, W), generator=g)
            lab = torch.where(blob, lab, torch.zeros_like(lab))
            target = torch.zeros(N, C, H, W).scatter_(1, lab, 1.0)
            x = logits.clone().requires_grad_(True)
            loss = losses.RMILoss(**kw)(x, target)
            loss.backward(torch.tensor(gout))
            save(f'{name}.npz', logits=logits, target=target, loss=loss.detach(), grad=x.grad, gout=np.float32(gout),
                 **{k: np.asarray(v) for k, v in kw.items()})
    finally:
        torch.cuda.DoubleTensor = saved


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'rmi':
        gen_rmi()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'metrics':
        gen_metrics()
        gen_inference()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'models2':
        gen_models2()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'msa_trainsteps':
        gen_msa_trainsteps()
        sys.exit(0)
    gen_cowmix()
    gen_mix()
    gen_consistency()
    gen_lovasz()
    gen_ema()
    gen_models()
    gen_trainsteps()
    gen_models2()
    gen_metrics()
    gen_inference()
    gen_msa_trainsteps()
