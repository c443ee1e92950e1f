"""Pin the CPU oracle against golden vectors generated from the reference (tests/golden, G1-G7)."""
import hashlib

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import cowmix_ref, losses_ref, models_ref, rmi_ref, train_ref

COWMIX_CASES = ['a0', 'a1', 'a2', 'b3', 'c0']


@pytest.mark.parametrize('K', [7, 8, 49, 193, 97])
def test_gaussian_taps(K):
    g = golden('cowmix_gaussian.npz')
    ours = cowmix_ref.gaussian_taps(K, g[f'sigma_{K}'])
    np.testing.assert_allclose(ours, g[f'g_{K}'], rtol=2e-6, atol=1e-9)


@pytest.mark.parametrize('tag', COWMIX_CASES)
def test_cowmix_rng_replay_and_mask(tag):
    g = golden(f'cowmix_{tag}.npz')
    B, _, H, W = [int(v) for v in g['shape']]
    torch.manual_seed(int(g['seed']))
    p, sig, noise = cowmix_ref.draw_inputs(B, H, W, g['prop_range'], g['sigma_range'])
    assert np.array_equal(p, g['p']) and np.array_equal(sig, g['sigma'])
    assert hashlib.sha256(noise.reshape(B, 1, H, W).tobytes()).hexdigest() == str(g['noise_sha256'])
    assert cowmix_ref.window_size(sig) == int(g['K'])
    mask, field, thr, mean, std = cowmix_ref.cowmix_masks(noise, sig, p)
    ref = np.unpackbits(g['mask_bits'])[:B * H * W].reshape(B, H, W)
    if 'field' in g.files:
        np.testing.assert_allclose(field, g['field'].reshape(B, H, W), rtol=0, atol=2e-6)
    np.testing.assert_allclose(thr, g['thr'], rtol=1e-5, atol=1e-6)
    # bit-exact outside the tie band |f - thr| < 1e-5 * std
    band = np.abs(field - thr.reshape(B, 1, 1)) < 1e-5 * std.reshape(B, 1, 1)
    diff = (mask.astype(np.uint8) != ref)
    assert not (diff & ~band).any(), f'{int((diff & ~band).sum())} mask pixels differ outside the tie band'


def test_mix():
    g = golden('mix.npz')
    assert np.array_equal(cowmix_ref.mix(g['a'], g['b'], g['mask']), g['out'])


def test_lovasz_grad_vectors():
    g = golden('lovasz.npz')
    np.testing.assert_allclose(losses_ref.lovasz_grad(g['gt_sorted']), g['lovasz_grad'], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(losses_ref.lovasz_grad(np.ones(1, np.float32)), g['lovasz_grad_1'])


def test_binary_lovasz():
    g = golden('lovasz.npz')
    loss, grad = losses_ref.binary_lovasz(g['logits'], g['target'])
    np.testing.assert_allclose(loss, g['loss'], rtol=1e-5)
    np.testing.assert_allclose(grad, g['grad'], rtol=1e-4, atol=1e-7)
    assert np.all(grad[:, 0] == 0)


def rmi_kwargs(g):
    return dict(num_classes=int(g['num_classes']), radius=int(g['rmi_radius']), pool=str(g['rmi_pool']),
                pool_size=int(g['rmi_pool_size']), pool_stride=int(g['rmi_pool_stride']))


@pytest.mark.parametrize('case', ['rmi_a', 'rmi_b', 'rmi_c'])
def test_rmi(case):
    """G12: the RMILoss restatement reproduces the reference's loss and input gradient (bitwise on this torch)."""
    g = golden(f'{case}.npz')
    loss, grad = rmi_ref.rmi_loss_and_grad(g['logits'], g['target'], gout=float(g['gout']), **rmi_kwargs(g))
    np.testing.assert_allclose(loss, g['loss'], rtol=1e-6)
    np.testing.assert_allclose(grad, g['grad'], rtol=1e-5, atol=1e-9)
    assert (grad[g['logits'] < -20] == 0).all()          # sigmoid < 1e-6: clamped, no gradient


def test_ema():
    g = golden('ema.npz')
    keys = [k[2:] for k in g.files if k.startswith('t.') and 'running' not in k and 'num_batches' not in k]
    for k in keys:
        ours = losses_ref.ema_update(g['t.' + k], g['s.' + k], float(g['alpha']))
        assert np.array_equal(ours, g["after." + k])
    # buffers alias the student's (mean_teacher.py:16-18): teacher buffers after == student buffers
    for k in [k[2:] for k in g.files if k.startswith('s.') and 'running' in k]:
        assert np.array_equal(g['after.' + k], g['s.' + k])


@pytest.mark.parametrize('tag', ['thr05', 'thr097', 'nan', 'gated'])
def test_consistency_step(tag):
    """G3: one reference train step with stub logit models, restated with the numpy oracle."""
    g = golden(f'consistency_{tag}.npz')
    s, t, image, sm = g['s_logits'], g['t_logits'], g['image'], g['semantic_mask']
    B, _, H, W = image.shape
    up = lambda x: losses_ref.bilinear(x, (H, W))  # noqa: E731
    sup, g_sup = losses_ref.bce_logits_mean(up(s), sm)
    np.testing.assert_allclose(sup * 0.5, g['sup_loss'], rtol=1e-5)
    torch.manual_seed(int(g['rng_seed']))
    p, sig, noise = cowmix_ref.draw_inputs(B, H, W, (0.45, 0.55), (4, 8))
    m, *_ = cowmix_ref.cowmix_masks(noise, sig, p)
    m = m[:, None]
    t_mix = cowmix_ref.mix(up(t), up(t), m)  # stub teacher: same logits for both unlabeled images
    L, cm_mean, g_cons = losses_ref.consistency(up(s), t_mix, float(g['thr']))
    gate = 10.0 * float(int(g['epoch']) > 25)
    if tag == 'nan':
        assert np.isnan(g['unsup_loss']) and np.isnan(L)
        assert np.isnan(g['grad']).all()
        return
    np.testing.assert_allclose(L * gate, g['unsup_loss'], rtol=2e-5, atol=1e-7)
    grad = losses_ref.bilinear_backward(g_sup * 0.5 + g_cons * gate, (s.shape[2], s.shape[3]))
    np.testing.assert_allclose(grad, g['grad'], rtol=2e-4, atol=2e-8)
    np.testing.assert_allclose(losses_ref.ema_update(t, s, 0.99), g['ema_after'], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('tag,ctor', [
    ('simple_unet_t', lambda: models_ref.SimpleUNet(2, 3, 8, 32, train_upsampling=True)),
    ('simple_unet_b', lambda: models_ref.SimpleUNet(2, 3, 8, 32, train_upsampling=False)),
    ('unet_mbv2_t', lambda: models_ref.UNet(2, models_ref.mobilenet_v2(width_mult=0.35), 32, train_upsampling=True)),
    ('unet_mbv2_b', lambda: models_ref.UNet(2, models_ref.mobilenet_v2(width_mult=0.35), 32, train_upsampling=False)),
])
def test_model_forward(tag, ctor):
    g = golden(f'model_{tag}.npz')
    m = models_ref.load_state(ctor(), g, 'init.')
    x = torch.from_numpy(g['x'])
    m.eval()
    with torch.no_grad():
        np.testing.assert_allclose(m(x).numpy(), g['y_eval'], rtol=1e-4, atol=1e-5)
    m.train()
    with torch.no_grad():
        np.testing.assert_allclose(m(x).numpy(), g['y_train'], rtol=1e-4, atol=1e-5)
    sd = m.state_dict()
    for k in g.files:
        if k.startswith('after.'):
            np.testing.assert_allclose(sd[k[6:]].numpy(), g[k], rtol=1e-5, atol=1e-6)


def test_trainsteps():
    """G7: three reference train steps (SimpleUNet, SGD, clip, CowMix, EMA) vs the oracle step."""
    g = golden('trainsteps.npz')
    fn = lambda: models_ref.ListOutput(models_ref.SimpleUNet(2, 2, 4, 8))  # noqa: E731
    student = models_ref.load_state(fn(), g, 'init.')
    teacher = models_ref.load_state(fn(), g, 'init.')
    for p in teacher.parameters():
        p.detach_()
    teacher.eval()
    opt = torch.optim.SGD(student.parameters(), lr=float(g['lr']), momentum=0.9, weight_decay=0.0005)
    cfg = train_ref.default_cfg(sigma_range=(2, 4), confidence_threshold=0.5)
    imgs, masks, unl = (torch.from_numpy(g[k]) for k in ('imgs', 'masks', 'unl'))
    torch.manual_seed(int(g['rng_seed']))
    logs = train_ref.train_epoch(student, teacher, opt, list(zip(imgs, masks)), iter(unl), 30, cfg)
    np.testing.assert_allclose([r['sup_loss'] * 1.0 for r in logs], g['sup_loss'], rtol=1e-5)
    np.testing.assert_allclose([r['unsup_loss'] for r in logs], g['unsup_loss'], rtol=5e-3, atol=1e-8)
    sd_s, sd_t = student.state_dict(), teacher.state_dict()
    for k in sd_s:
        np.testing.assert_allclose(sd_s[k].numpy(), g['final_s.' + k], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(sd_t[k].numpy(), g['final_t.' + k], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('tag', ['a', 'b', 'c'])
def test_seg_metrics_vs_reference_golden(tag):
    """G9: validation Dice (reference train.py:171-176, metrics.py:1-7) and lovasz.iou, with ties in the
    logits and the mask, an all-background image, and non-integer / 2x / identity nearest resizes."""
    g = golden(f'metrics_{tag}.npz')
    dice, ious, _ = losses_ref.seg_metrics(g['logits'], g['mask'])
    np.testing.assert_array_equal(dice, g['dice'].reshape(-1))
    np.testing.assert_allclose(ious, g['ious'], rtol=1e-12)


def test_inference_head_vs_reference_golden():
    """G10: reference InferenceWrapper (bilinear to the image size, sigmoid, argmax one-hot) on stub logits;
    probabilities within 5e-6 (fp32 rounding of the resize)."""
    g = golden('inference.npz')
    mask, prob = losses_ref.inference_head(g['logits'], tuple(int(v) for v in g['image_hw']))
    np.testing.assert_array_equal(mask, g['mask'])
    np.testing.assert_allclose(prob, g["prob"], rtol=0, atol=5e-6)


def test_hardnet_restatement_vs_reference_golden():
    """oracle/hardnet_ref.py (the C5 network's CPU restatement) against the reference's own FC-HarDNet (golden G6b,
    model2_hardnet.npz): the same seed + perturbation gives the reference's weights (SHA-256 of the state_dict), and the
    eval / train forwards and the stored parameter gradients agree to fp32 rounding."""
    import seeded
    from oracle import hardnet_ref
    g = golden('model2_hardnet.npz')
    seed = int(g['seed'])
    torch.manual_seed(seed)
    m = hardnet_ref.HarDNet(n_classes=2)
    seeded.perturb(m, seed + 1000, None)
    assert seeded.state_sha(m) == str(g['sha'])
    gen = torch.Generator().manual_seed(seed + 2000)
    x = torch.rand(*[int(v) for v in g['shape0']], generator=gen)
    assert seeded.array_sha(x) == str(g['x0_sha'])
    m.eval()
    with torch.no_grad():
        ye = m(x)
    scale = float(np.abs(g['y_eval']).max())
    assert np.abs(ye.numpy() - g['y_eval']).max() <= 1e-5 * scale
    m.train()
    y = m(x)
    gy = torch.randn(y.shape, generator=gen)
    assert seeded.array_sha(gy) == str(g['gy_sha'])
    (y * gy).sum().backward()
    assert np.abs(y.detach().numpy() - g['y_train']).max() <= 1e-5 * float(np.abs(g['y_train']).max())
    params = dict(m.named_parameters())
    for k in g.keys():
        if k.startswith('grad.'):
            ref = g[k]
            assert np.abs(params[k[5:]].grad.numpy() - ref).max() <= 1e-4 * (np.abs(ref).max() + 1e-30), k
