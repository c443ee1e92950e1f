"""GPU parity of the CowMix / loss / interpolation / EMA / SGD kernels against the oracle and the
reference golden vectors.  Tolerances are stated per test."""
import hashlib

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import cowmix_ref, losses_ref, rmi_ref

pytestmark = pytest.mark.gpu


def ops():
    from ssseg import ops as o
    return o


@pytest.mark.parametrize('tag', ['a0', 'a1', 'a2', 'b3', 'c0'])
def test_cowmix_mask_bit_exact_outside_tie_band(hip_device, tag):
    g = golden(f'cowmix_{tag}.npz')
    B, _, H, W = [int(v) for v in g['shape']]
    torch.manual_seed(int(g['seed']))
    p, sig, noise = cowmix_ref.draw_inputs(B, H, W, g['prop_range'], g['sigma_range'])
    assert hashlib.sha256(noise.reshape(B, 1, H, W).tobytes()).hexdigest() == str(g['noise_sha256'])
    dev = hip_device
    mask, field, thr = ops().cowmix_mask(torch.from_numpy(noise).to(dev), torch.from_numpy(sig).to(dev),
                                         torch.from_numpy(p).to(dev), return_field=True)
    mask = mask.cpu().numpy().reshape(B, H, W)
    field = field.cpu().numpy().reshape(B, H, W)
    ref = np.unpackbits(g['mask_bits'])[:B * H * W].reshape(B, H, W)
    std = g['std'].reshape(B, 1, 1)
    np.testing.assert_allclose(thr.cpu().numpy(), g['thr'], rtol=1e-5, atol=1e-6)
    if 'field' in g.files:
        np.testing.assert_allclose(field, g['field'].reshape(B, H, W), rtol=0, atol=2e-6)
    band = np.abs(field - g['thr'].reshape(B, 1, 1)) < 1e-5 * std
    diff = mask.astype(np.uint8) != ref
    assert not (diff & ~band).any(), f'{int((diff & ~band).sum())} pixels differ outside the tie band'
    assert set(np.unique(mask)) <= {0.0, 1.0}


def test_cowmix_device_noise_statistics(hip_device):
    out = torch.empty(1 << 22, device=hip_device)
    ops().normal_(out, seed=1234, offset=0)
    x = out.double()
    assert abs(float(x.mean())) < 3e-3 and abs(float(x.std()) - 1) < 3e-3
    out2 = torch.empty_like(out)
    ops().normal_(out2, seed=1234, offset=0)
    assert torch.equal(out, out2)


def test_mix_bit_exact(hip_device):
    g = golden('mix.npz')
    a, b, m = (torch.from_numpy(g[k]).to(hip_device) for k in ('a', 'b', 'mask'))
    assert np.array_equal(ops().mix(a, b, m).cpu().numpy(), g['out'])


@pytest.mark.parametrize('shape,size,ac', [((2, 2, 32, 32), (64, 64), False), ((2, 3, 17, 23), (40, 31), False),
                                           ((1, 4, 8, 8), (16, 16), True), ((2, 2, 64, 48), (32, 24), False),
                                           ((1, 2, 9, 9), (9, 9), False)])
def test_bilinear_fwd_bwd(hip_device, shape, size, ac):
    rng = np.random.default_rng(0)
    x = rng.standard_normal(shape).astype(np.float32)
    gy = rng.standard_normal(shape[:2] + size).astype(np.float32)
    xt = torch.from_numpy(x).to(hip_device).requires_grad_(True)
    y = ops().interpolate_bilinear(xt, size, align_corners=ac)
    y.backward(torch.from_numpy(gy).to(hip_device))
    ref = torch.nn.functional.interpolate(torch.from_numpy(x), size=size, mode='bilinear', align_corners=ac)
    # the device kernels round every product (built without FMA contraction); PyTorch's CPU build may contract:
    # a few fp32 ulp apart
    np.testing.assert_allclose(y.detach().cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(y.detach().cpu().numpy(), losses_ref.bilinear(x, size, ac), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(xt.grad.cpu().numpy(), losses_ref.bilinear_backward(gy, shape[2:], ac),
                               rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('ac', [False, True])
@pytest.mark.parametrize('fmt,dt', [(torch.contiguous_format, torch.float32), (torch.channels_last, torch.bfloat16)])
def test_bilinear_identity_size_is_the_input(hip_device, ac, fmt, dt):
    """At the input's own size interpolate_bilinear returns the input (PyTorch's CPU kernels copy there): the kernel's
    (1, 0) weights reproduce the finite values bit for bit, and the gradient passes straight through."""
    o = ops()
    x = torch.randn(2, 3, 24, 40, device=hip_device).to(dt).contiguous(memory_format=fmt).requires_grad_(True)
    y = o.interpolate_bilinear(x, (24, 40), align_corners=ac)
    assert y is x
    yk = o._Bilinear.apply(x.detach(), (24, 40), ac)   # the kernel at identity size
    assert torch.equal(yk, x.detach())
    ref = torch.nn.functional.interpolate(x.detach().float().cpu(), size=(24, 40), mode='bilinear', align_corners=ac)
    assert torch.equal(ref, x.detach().float().cpu())


def test_bilinear_channels_last_bf16(hip_device):
    x = torch.randn(2, 8, 16, 16, device=hip_device).to(memory_format=torch.channels_last)
    y32 = ops().interpolate_bilinear(x, (32, 32), True)
    yb = ops().interpolate_bilinear(x.bfloat16(), (32, 32), True)
    assert yb.is_contiguous(memory_format=torch.channels_last)
    ref = torch.nn.functional.interpolate(x.cpu(), size=(32, 32), mode='bilinear', align_corners=True)
    np.testing.assert_allclose(y32.cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(yb.float().cpu().numpy(), ref.numpy(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('shape,size,ac', [((2, 32, 16, 16), (64, 64), False), ((3, 24, 13, 11), (26, 22), True),
                                           ((2, 16, 9, 7), (32, 29), False), ((1, 8, 40, 36), (20, 18), False)])
def test_bilinear_nhwc_vector_path_bitwise(hip_device, dt, shape, size, ac):
    """The 16-bit channels-last kernels (one thread per pixel and 8-channel chunk, HRNet / UNet feature maps) do the
    generic kernels' per-channel arithmetic: forward and backward are bit-identical to the generic path on the
    same values in NCHW layout (which the generic kernels handle)."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(shape, generator=g).to(dt).to(hip_device)
    gy = torch.randn(shape[:2] + size, generator=g).to(dt).to(hip_device)
    outs = []
    for fmt in (torch.channels_last, torch.contiguous_format):
        xt = x.contiguous(memory_format=fmt).clone().requires_grad_(True)
        y = ops().interpolate_bilinear(xt, size, align_corners=ac)
        y.backward(gy.contiguous(memory_format=fmt))
        outs.append((y.detach().contiguous(), xt.grad.contiguous()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    ref = torch.nn.functional.interpolate(x.float().cpu(), size=size, mode='bilinear', align_corners=ac)
    np.testing.assert_allclose(outs[0][0].float().cpu().numpy(), ref.numpy(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize('shape,size,ac', [((2, 32, 32, 32), (256, 256), False), ((2, 64, 17, 13), (34, 26), True),
                                           ((3, 16, 40, 36), (20, 18), False), ((1, 256, 8, 8), (64, 64), False)])
def test_bilinear_bwd_two_pass_bitwise(hip_device, shape, size, ac):
    """ssseg_bilinear_bwd_ws (separable rows / columns passes through an fp32 workspace, the activation resizes'
    backward) is bitwise the one-pass NHWC kernel (ssseg_bilinear_bwd), incl. 8x upsampling (HRNet fuse) and a
    downsampling resize."""
    from ssseg import native as N
    from ssseg import nn as snn
    n, c, h, w = shape
    oh, ow = size
    g = torch.Generator().manual_seed(7)
    gy = torch.randn(n, c, oh, ow, generator=g).to(torch.bfloat16).to(hip_device).contiguous(
        memory_format=torch.channels_last)
    outs = []
    for two in (False, True):
        gx = torch.empty(n, c, h, w, dtype=torch.bfloat16, device=hip_device).contiguous(
            memory_format=torch.channels_last)
        if two:
            snn._bilinear_bwd(gy, gx, n, c, h, w, oh, ow, N.strides4(gy), N.strides4(gx), ac)
        else:
            N.call('ssseg_bilinear_bwd', N.dev_ptr(gy), N.dev_ptr(gx), n, c, h, w, oh, ow, N.strides4(gy),
                   N.strides4(gx), int(ac), N.dt_code(gy), N.stream())
        torch.cuda.synchronize()
        outs.append(gx)
    assert torch.equal(outs[0], outs[1])


def test_bce_fwd_bwd(hip_device):
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((4, 2, 64, 64)) * 3).astype(np.float32)
    t = (rng.random((4, 2, 64, 64)) > 0.5).astype(np.float32)
    xt = torch.from_numpy(x).to(hip_device).requires_grad_(True)
    loss = ops().bce_with_logits_mean(xt, torch.from_numpy(t).to(hip_device))
    (loss * 0.5).backward()
    ref_l, ref_g = losses_ref.bce_logits_mean(x, t)
    np.testing.assert_allclose(float(loss.detach()), ref_l, rtol=1e-6)
    np.testing.assert_allclose(xt.grad.cpu().numpy(), ref_g * 0.5, rtol=1e-5, atol=1e-10)


@pytest.mark.parametrize('tag', ['thr05', 'thr097', 'nan', 'gated'])
def test_consistency_chain_vs_golden(hip_device, tag):
    """G3 through the HIP ops: interp -> BCE, CowMix (CPU-generator inputs) -> mix -> consistency."""
    o = ops()
    g = golden(f'consistency_{tag}.npz')
    dev = hip_device
    s = torch.from_numpy(g['s_logits']).to(dev).requires_grad_(True)
    t = torch.from_numpy(g['t_logits']).to(dev)
    B, _, H, W = g['image'].shape
    sm = torch.from_numpy(g['semantic_mask']).to(dev)
    sup = o.bce_with_logits_mean(o.interpolate_bilinear(s, (H, W)), sm) * 0.5
    torch.manual_seed(int(g['rng_seed']))
    p, sig, noise = cowmix_ref.draw_inputs(B, H, W, (0.45, 0.55), (4, 8))
    m = o.cowmix_mask(torch.from_numpy(noise).to(dev), torch.from_numpy(sig).to(dev), torch.from_numpy(p).to(dev))
    tu = o.interpolate_bilinear(t, (H, W))
    t_mix = o.mix(tu, tu, m)
    loss, cm = o.consistency_loss(o.interpolate_bilinear(s, (H, W)), t_mix, float(g['thr']))
    unsup = loss * (10.0 * float(int(g['epoch']) > 25))
    (sup + unsup).backward()
    np.testing.assert_allclose(float(sup), g['sup_loss'], rtol=1e-5)
    if tag == 'nan':
        assert np.isnan(float(unsup)) and torch.isnan(s.grad).all()
        return
    np.testing.assert_allclose(float(unsup), g['unsup_loss'], rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(s.grad.cpu().numpy(), g['grad'], rtol=2e-4, atol=2e-8)


def test_ema_bit_exact(hip_device):
    g = golden('ema.npz')
    keys = [k[2:] for k in g.files if k.startswith('t.') and 'running' not in k and 'num_batches' not in k]
    e = torch.cat([torch.from_numpy(g['t.' + k]).reshape(-1) for k in keys]).to(hip_device)
    p = torch.cat([torch.from_numpy(g['s.' + k]).reshape(-1) for k in keys]).to(hip_device)
    ref = np.concatenate([g['after.' + k].reshape(-1) for k in keys])
    ops().ema_update_(e, p, float(g['alpha']))
    assert np.array_equal(e.cpu().numpy(), ref)


def test_clip_sgd_matches_torch(hip_device):
    torch.manual_seed(3)
    params = [torch.randn(37, 5), torch.randn(1000), torch.randn(3, 3, 4)]
    grads = [torch.randn_like(q) * 3 for q in params]
    ref_p = [q.clone().requires_grad_(True) for q in params]
    for q, gr in zip(ref_p, grads):
        q.grad = gr.clone()
    opt = torch.optim.SGD(ref_p, lr=0.05, momentum=0.9, weight_decay=5e-4)
    flat_p = torch.cat([q.reshape(-1) for q in params]).to(hip_device)
    flat_g = torch.cat([q.reshape(-1) for q in grads]).to(hip_device)
    buf = torch.zeros_like(flat_p)
    shadow = torch.empty(flat_p.numel(), dtype=torch.bfloat16, device=hip_device)
    o = ops()
    for step in range(3):
        torch.nn.utils.clip_grad_norm_(ref_p, 5.0)
        opt.step()
        sq = torch.zeros(1, device=hip_device)
        o.sqnorm_(flat_g, sq)
        o.sgd_step_(flat_p, flat_g, buf, shadow, 0.05, 0.9, 5e-4, 5.0, sq, step == 0)
        for q, gr in zip(ref_p, grads):
            q.grad = gr.clone()
        flat_g = torch.cat([q.reshape(-1) for q in grads]).to(hip_device)
    ref = torch.cat([q.detach().reshape(-1) for q in ref_p]).numpy()
    np.testing.assert_allclose(flat_p.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(shadow.float().cpu().numpy(), ref, rtol=1e-2, atol=1e-2)


def _lovasz_hip(x, t, dev, gscale=1.0):
    import losses
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    loss = losses.binary_lovasz_loss_with_logits(xt, torch.from_numpy(t).to(dev))
    (loss * gscale).backward()
    return float(loss.detach()), xt.grad.cpu().numpy()


def test_lovasz_vs_reference_golden(hip_device):
    """G4 (reference losses.binary_lovasz_loss_with_logits on 3x2x64x64 incl. an all-background image):
    loss within 1e-5 relative (fp64 dot vs the reference's fp32 torch.dot), gradient within 1e-6."""
    g = golden('lovasz.npz')
    loss, grad = _lovasz_hip(g['logits'], g['target'], hip_device)
    np.testing.assert_allclose(loss, float(g['loss']), rtol=1e-5)
    np.testing.assert_allclose(grad, g['grad'], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('B,H,W,empty', [(4, 96, 80, 1), (1, 512, 512, None), (2, 45, 1, None), (3, 1, 1, 0),
                                         (2, 130, 129, 0)])
def test_lovasz_vs_oracle(hip_device, B, H, W, empty):
    """Radix-sorted device Lovász vs the oracle (stable argsort) on multi-tile segments (512^2 = 128 tiles),
    partial tiles, single-pixel images and an image with no foreground (valid = 0)."""
    rng = np.random.default_rng(B * 1000 + H)
    x = (rng.standard_normal((B, 2, H, W)) * 2).astype(np.float32)
    fg = rng.random((B, 1, H, W)) > 0.6
    if empty is not None:
        fg[empty] = False
    t = np.concatenate([~fg, fg], 1).astype(np.float32)
    loss, grad = _lovasz_hip(x, t, hip_device, gscale=0.7)
    ref_l, ref_g = losses_ref.binary_lovasz(x, t)
    np.testing.assert_allclose(loss, ref_l, rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(grad, ref_g * np.float32(0.7), rtol=1e-4, atol=2e-6)


def test_lovasz_bwd_from_fwd_bitwise(hip_device):
    """The autograd backward scatters the gradient the forward left in its workspace (ssseg_lovasz_bwd_from_fwd, no
    second sort): bit-identical to the stand-alone backward that sorts again (ssseg_lovasz_bwd), ties included."""
    from ssseg import native as N
    rng = np.random.default_rng(3)
    B, H, W = 3, 70, 66
    x = rng.choice(np.array([-1, 0, 0.5, 1, 2, 0.25], np.float32), size=(B, 2, H, W))
    fg = rng.random((B, 1, H, W)) > 0.5
    t = np.concatenate([~fg, fg], 1).astype(np.float32)
    _, grad = _lovasz_hip(x, t, hip_device, gscale=0.3)
    xt, tt = torch.from_numpy(x).to(hip_device), torch.from_numpy(t).to(hip_device)
    gx = torch.empty_like(xt)
    go = torch.full((), 0.3, device=hip_device)
    nb = N.lib().ssseg_lovasz_workspace_bytes(B, H * W)
    ws = N.workspace(nb, hip_device)
    N.call('ssseg_lovasz_bwd', N.dev_ptr(xt), N.dev_ptr(tt), B, 2, H * W, N.dev_ptr(go), N.dev_ptr(gx), N.dev_ptr(ws),
           nb, N.stream())
    torch.cuda.synchronize()
    assert np.array_equal(grad, gx.cpu().numpy())


def test_lovasz_ties_loss_invariant(hip_device):
    """Heavily tied errors (logits on a 5-value grid): the per-pixel gradient inside a tie depends on the
    sort's tie order (the reference's torch.sort is unstable), the loss and the per-image gradient sums
    over each tie group do not — compared against the oracle."""
    rng = np.random.default_rng(7)
    B, H, W = 3, 64, 48
    x = rng.choice(np.array([-1, 0, 0.5, 1, 2], np.float32), size=(B, 2, H, W))
    fg = rng.random((B, 1, H, W)) > 0.5
    t = np.concatenate([~fg, fg], 1).astype(np.float32)
    loss, grad = _lovasz_hip(x, t, hip_device)
    ref_l, ref_g = losses_ref.binary_lovasz(x, t)
    np.testing.assert_allclose(loss, ref_l, rtol=1e-5)
    d = fg[:, 0].astype(np.float32) - x[:, 1]
    err, sg = np.abs(d), np.sign(d)
    for b in range(B):
        for e in np.unique(err[b]):
            m = (err[b] == e) & (sg[b] != 0)   # Lovász weights g = -grad / sign; their sum per tie is order-free
            if m.any():
                np.testing.assert_allclose((-grad[b, 1][m] / sg[b][m]).sum(), (-ref_g[b, 1][m] / sg[b][m]).sum(),
                                           rtol=1e-4, atol=1e-5)
    assert np.all(grad[:, 0] == 0)


@pytest.mark.parametrize('tag', ['a', 'b', 'c'])
def test_seg_metrics_vs_reference_golden(hip_device, tag):
    """G9 on the device (ssseg_seg_metrics): per-image counts bit-exact with the oracle, Dice bit-exact
    with the reference's fp32 values, mean Dice within 1e-6 (fp64 vs fp32 mean), IoU within 1e-5; the
    logits are handed over as a strided 2-channel view of an 8-channel NHWC buffer (the heads' layout)."""
    g = golden(f'metrics_{tag}.npz')
    dev = hip_device
    B, _, h, w = g['logits'].shape
    phys = torch.zeros(B, h, w, 8, device=dev)
    phys[..., :2] = torch.from_numpy(g['logits']).to(dev).permute(0, 2, 3, 1)
    logits = phys.permute(0, 3, 1, 2)[:, :2]
    seg = ops().SegMetrics(dev)
    out = seg.update(logits, torch.from_numpy(g['mask']).to(dev)).cpu().numpy()
    _, _, counts = losses_ref.seg_metrics(g['logits'], g['mask'])
    np.testing.assert_array_equal(seg.counts.cpu().numpy(), counts)
    np.testing.assert_allclose(out[0], float(g['dice_mean']), rtol=1e-6)
    np.testing.assert_allclose(out[1:3], g['ious'], rtol=1e-5)
    np.testing.assert_allclose(out[3], g['ious'].mean(), rtol=1e-5)


def test_seg_metrics_running_totals_and_nan(hip_device):
    """Running dataset counts across batches (mIoU over the whole validation set), NaN logits follow
    torch.argmax (NaN is the maximum), 512x512 masks from 256x256 logits (the UNet /2 head)."""
    dev = hip_device
    g = torch.Generator().manual_seed(5)
    seg = ops().SegMetrics(dev)
    all_counts = []
    for i in range(3):
        logits = torch.randn(4, 2, 256, 256, generator=g)
        logits[0, 0, 0, :7] = float('nan')
        logits[1, 1, 3, :5] = float('nan')
        soft = torch.rand(4, 1, 512, 512, generator=g)
        mask = torch.cat([1 - soft, soft], 1)
        out = seg.update(logits.to(dev), mask.to(dev)).cpu().numpy()
        dice, _, counts = losses_ref.seg_metrics(logits.numpy(), mask.numpy())
        np.testing.assert_array_equal(seg.counts.cpu().numpy(), counts)
        np.testing.assert_allclose(out[0], dice.astype(np.float64).mean(), rtol=1e-6)
        all_counts.append(counts)
    tot = np.concatenate(all_counts).sum(0)
    np.testing.assert_array_equal(seg.total.cpu().numpy(), tot)
    np.testing.assert_allclose(out[1:3], [100 * tot[3] / tot[4], 100 * tot[5] / tot[6]], rtol=1e-5)


def test_inference_wrapper_vs_reference_golden(hip_device):
    """G10 through the drop-in models.inference_wrapper.InferenceWrapper (device bilinear + ssseg_prob_onehot):
    one-hot mask bit-exact with the reference except where the resized logits tie within 1e-5, sigmoid
    probabilities within 5e-6 (fp32 bilinear + sigmoid rounding on logits of magnitude ~10)."""
    from models.inference_wrapper import InferenceWrapper
    g = golden('inference.npz')
    dev = hip_device
    logits = torch.from_numpy(g['logits']).to(dev)

    class Stub(torch.nn.Module):
        def forward(self, image):
            return [image], [logits, logits[:, :, ::2, ::2]]

    H, W = (int(v) for v in g['image_hw'])
    mask, prob = InferenceWrapper(Stub())(torch.rand(3, H, W, device=dev))
    assert mask.shape == (2, H, W) and prob.shape == (2, H, W)
    prob = prob.cpu().numpy()
    np.testing.assert_allclose(prob, g["prob"], rtol=0, atol=5e-6)
    hi = losses_ref.bilinear(g['logits'], (H, W))[0]
    band = np.abs(hi[1] - hi[0]) < 1e-5
    diff = (mask.cpu().numpy() != g['mask']).any(0)
    assert not (diff & ~band).any()


@pytest.mark.parametrize('angle', [0.0, 17.5, -90.0, 33.0])
def test_reversible_rotate_vs_grid_sample(hip_device, angle):
    """reversible_augmentations.Rotate's kernel (kornia.rotate semantics: counter-clockwise about the centre,
    bilinear, zero padding; kornia absent so parity with it is unpinned) vs a torch grid_sample restatement of
    the same inverse map (align_corners=True pixel grid), forward and input gradient."""
    import math
    import torch.nn.functional as F
    from ssseg import ops
    g = torch.Generator().manual_seed(3)
    x = torch.rand(2, 3, 19, 24, generator=g, dtype=torch.float64)
    gy = torch.randn(2, 3, 19, 24, generator=g, dtype=torch.float64)
    N_, C, H, W = x.shape
    th = math.radians(angle)
    ys, xs = torch.meshgrid(torch.arange(H, dtype=torch.float64), torch.arange(W, dtype=torch.float64), indexing='ij')
    cx, cy = (W - 1) / 2, (H - 1) / 2
    sx = math.cos(th) * (xs - cx) - math.sin(th) * (ys - cy) + cx
    sy = math.sin(th) * (xs - cx) + math.cos(th) * (ys - cy) + cy
    grid = torch.stack([sx / (W - 1) * 2 - 1, sy / (H - 1) * 2 - 1], -1).expand(N_, H, W, 2)
    xr = x.clone().requires_grad_(True)
    yr = F.grid_sample(xr, grid, mode='bilinear', padding_mode='zeros', align_corners=True)
    yr.backward(gy)
    xd = x.float().to(hip_device).requires_grad_(True)
    y = ops.rotate(xd, angle)
    y.backward(gy.float().to(hip_device))
    assert float((y.detach().cpu().double() - yr.detach()).abs().max()) < 1e-5
    assert float((xd.grad.cpu().double() - xr.grad).abs().max()) < 1e-5
    if angle == 0.0:
        assert torch.equal(y.detach().cpu(), x.float())


def test_reversible_augmentations_roundtrip(hip_device):
    """apply() then reverse() on a smooth image: back to the input away from the rotated-out corners."""
    import reversible_augmentations as RA
    torch.manual_seed(0)
    yy, xx = torch.meshgrid(torch.linspace(-1, 1, 64), torch.linspace(-1, 1, 64), indexing='ij')
    img = torch.stack([torch.sin(2 * xx) * torch.cos(3 * yy)] * 2)[None].to(hip_device)
    rot = RA.Rotate(20)
    out = rot.reverse(rot.apply([img]))[0]
    c = (slice(None), slice(None), slice(20, 44), slice(20, 44))
    assert float((out[c] - img[c]).abs().max()) < 2e-2
    res = RA.Rescale(0.5, 0.75)
    small = res.apply([img])[0]
    assert small.shape[2] == int(64 * res.scale)
    back = res.reverse([small])[0]
    assert back.shape[2] in (63, 64)


def _rmi_hip(x, t, dev, gout=1.0, **kw):
    import losses as L
    mod = L.RMILoss(num_classes=kw['num_classes'], rmi_radius=kw['radius'], rmi_pool=kw['pool'],
                    rmi_pool_size=kw['pool_size'], rmi_pool_stride=kw['pool_stride'])
    xd = torch.from_numpy(np.ascontiguousarray(x)).to(dev).requires_grad_(True)
    loss = mod(xd, torch.from_numpy(np.ascontiguousarray(t)).to(dev))
    loss.backward(torch.tensor(gout, device=dev))
    return float(loss.detach().cpu()), xd.grad.cpu().numpy()


def _rmi_kw(g):
    return dict(num_classes=int(g['num_classes']), radius=int(g['rmi_radius']), pool=str(g['rmi_pool']),
                pool_size=int(g['rmi_pool_size']), pool_stride=int(g['rmi_pool_stride']))


@pytest.mark.parametrize('case', ['rmi_a', 'rmi_b', 'rmi_c'])
def test_rmi_vs_reference_golden(hip_device, case):
    """G12 (the reference's RMILoss: default config radius 3 / avg pool 4, 3 classes / radius 2 / pool 3, radius 1 /
    no pooling; saturated logits on both clamp bounds).  fp64 algebra in a different order (Cholesky-based inverse vs
    torch.inverse's LU): loss within 2e-6 relative, gradient within 1e-4 relative of the largest entry."""
    g = golden(f'{case}.npz')
    loss, grad = _rmi_hip(g['logits'], g['target'], hip_device, gout=float(g['gout']), **_rmi_kw(g))
    np.testing.assert_allclose(loss, float(g['loss']), rtol=2e-6)
    scale = float(np.abs(g['grad']).max())
    np.testing.assert_allclose(grad, g['grad'], rtol=1e-3, atol=1e-4 * scale)
    assert (grad[g['logits'] < -20] == 0).all()


def _rmi_inputs(N, C, H, W, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((N, C, H, W)) * 2.5).astype(np.float32)
    lab = rng.integers(0, C, size=(N, 1, H, W))
    lab = np.where(rng.random((N, 1, H, W)) > 0.3, lab, 0)
    t = (np.arange(C).reshape(1, C, 1, 1) == lab).astype(np.float32)
    return x, t


@pytest.mark.parametrize('N,C,H,W,kw', [
    (16, 2, 512, 512, dict(num_classes=2, radius=3, pool='avg', pool_size=4, pool_stride=4)),   # C2 shape, default RMI
    (2, 2, 91, 70, dict(num_classes=2, radius=3, pool='avg', pool_size=4, pool_stride=4)),      # uncovered last row
    (4, 2, 37, 29, dict(num_classes=2, radius=2, pool='none', pool_size=2, pool_stride=2)),
    (1, 4, 9, 9, dict(num_classes=2, radius=3, pool='avg', pool_size=2, pool_stride=2)),        # rows = N*C/ncls
])
def test_rmi_vs_oracle(hip_device, N, C, H, W, kw):
    """Device RMILoss vs the pinned oracle (rmi_ref) at the bench shape (bs 16, 512^2: 16129 positions per series,
    4 covariance chunks) and small / odd geometries; same tolerances as the golden test."""
    x, t = _rmi_inputs(N, C, H, W, N * 100 + H)
    loss, grad = _rmi_hip(x, t, hip_device, gout=0.75, **kw)
    ref_l, ref_g = rmi_ref.rmi_loss_and_grad(x, t, gout=0.75, **kw)
    np.testing.assert_allclose(loss, float(ref_l), rtol=2e-6)
    np.testing.assert_allclose(grad, ref_g, rtol=1e-3, atol=1e-4 * float(np.abs(ref_g).max()))


def test_rmi_deterministic_and_default_config_combo(hip_device):
    """Two runs are bitwise equal; the default config's CalculateLoss (BCE 0.5 + RMI 0.5, configs/default_config.py:
    141-148) on the device matches 0.5 * oracle BCE + 0.5 * oracle RMI."""
    import losses as L
    x, t = _rmi_inputs(4, 2, 128, 96, 5)
    a = _rmi_hip(x, t, hip_device, **dict(num_classes=2, radius=3, pool='avg', pool_size=4, pool_stride=4))
    b = _rmi_hip(x, t, hip_device, **dict(num_classes=2, radius=3, pool='avg', pool_size=4, pool_stride=4))
    assert a[0] == b[0] and np.array_equal(a[1], b[1])
    crit = L.CalculateLoss([
        {'loss_fn': L.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'), 'weight': [0.5]},
        {'loss_fn': L.RMILoss(num_classes=2, rmi_radius=3, rmi_pool='avg', rmi_pool_size=4, rmi_pool_stride=4),
         'weight': [0.5]}])
    xd = torch.from_numpy(x).to(hip_device)
    tot = float(crit([xd], torch.from_numpy(t).to(hip_device)).cpu())
    ref_bce = losses_ref.bce_logits_mean(x, t)
    ref_bce = ref_bce[0] if isinstance(ref_bce, tuple) else ref_bce
    ref_rmi, _ = rmi_ref.rmi_loss_and_grad(x, t)
    np.testing.assert_allclose(tot, 0.5 * float(ref_bce) + 0.5 * float(ref_rmi), rtol=1e-5)

