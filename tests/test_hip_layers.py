"""GPU parity of the layer engine (implicit-GEMM conv fwd/dgrad/wgrad, ConvTranspose2d, BatchNorm,
max-pool, concat/crop) against the plain PyTorch-CPU fp32 reference of the same op.

Tolerances: fp32 compute mode 1e-4 relative to the output's max magnitude (f32 MFMA is an exact
fp32 fma chain; the residual difference is summation order); bf16 mode 2e-2, fp16 mode 4e-3 relative RMS.
"""
import contextlib

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(params=['f32', 'bf16', 'f16'])
def mode(request):
    from ssseg import nn as snn
    dt = {'f32': torch.float32, 'bf16': torch.bfloat16, 'f16': torch.float16}[request.param]
    snn.set_compute_dtype(dt)
    yield request.param
    snn.set_compute_dtype(torch.bfloat16)


def _close(got, ref, mode, what):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = float(ref.abs().max()) + 1e-12
    if mode == 'f32':
        err = float((got - ref).abs().max()) / scale
        assert err < 1e-4, f'{what}: max rel err {err}'
    else:   # 16-bit storage: bf16 (8-bit mantissa) 2e-2, fp16 (11-bit) 4e-3 relative RMS
        err = float(((got - ref) ** 2).mean().sqrt() / (ref.pow(2).mean().sqrt() + 1e-12))
        assert err < (2e-2 if mode == 'bf16' else 4e-3), f'{what}: rel rms err {err}'


def _q(t, mode):
    """16-bit modes: the reference sees the same rounded inputs the kernels see (fp32 math after)."""
    if mode == 'bf16':
        return t.bfloat16().float()
    if mode == 'f16':
        return t.half().float()
    return t


def _act_in(x, dev):
    from ssseg import nn as snn
    return snn.to_act(x.to(dev))


def _act_out(y):
    """physical NHWC activation -> logical NCHW float tensor with real channels"""
    return y


CONV_CASES = [
    # cin, cout, k, stride, pad, dil, H, W, N
    (8, 16, 3, 1, 1, 1, 12, 10, 2),
    (16, 64, 1, 1, 0, 1, 9, 9, 2),
    (64, 32, 1, 2, 0, 1, 10, 11, 2),
    (16, 32, 3, 2, 1, 1, 13, 12, 2),
    (3, 64, 7, 2, 3, 1, 23, 22, 2),
    (32, 16, 3, 1, 2, 2, 11, 11, 1),
    (24, 40, 3, 1, 1, 1, 7, 9, 3),
    (128, 128, 3, 1, 1, 1, 8, 8, 2),
]


@pytest.mark.parametrize('cin,cout,k,s,p,d,H,W,n', CONV_CASES)
def test_conv2d_fwd_bwd(hip_device, mode, cin, cout, k, s, p, d, H, W, n):
    from ssseg import nn as snn
    torch.manual_seed(0)
    ref = torch.nn.Conv2d(cin, cout, k, s, p, d, bias=False)
    mod = snn.Conv2d(cin, cout, k, s, p, d, bias=False, head=True).to(hip_device)
    mod.load_state_dict(ref.state_dict())
    with torch.no_grad():
        ref.weight.copy_(_q(ref.weight, mode))
    x = _q(torch.randn(n, cin, H, W), mode)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    gy = _q(torch.randn_like(yr), mode)
    yr.backward(gy)
    xa = _act_in(x, hip_device).detach().requires_grad_(True)
    y = mod(xa)
    y.backward(gy.to(hip_device))
    _close(y, yr, mode, 'y')
    _close(mod.weight.grad, ref.weight.grad, mode, 'dW')
    _close(xa.grad[:, :cin], xr.grad, mode, 'dx')


@pytest.mark.parametrize('C,k,s,p,d,H,W,act', [(24, 3, 1, 1, 1, 9, 11, False), (32, 3, 2, 1, 1, 13, 12, 'relu6'),
                                                (16, 5, 1, 2, 1, 7, 8, False), (40, 3, 1, 2, 2, 10, 9, 'relu6'),
                                                (12, 3, 2, 1, 1, 9, 9, False)])
def test_depthwise_conv_fwd_bwd(hip_device, mode, C, k, s, p, d, H, W, act):
    """Depthwise conv (MobileNetV2, groups == C) fwd/dgrad/wgrad vs PyTorch fp32, with the fused ReLU6."""
    from ssseg import nn as snn
    torch.manual_seed(7)
    ref = torch.nn.Conv2d(C, C, k, s, p, d, groups=C, bias=False)
    mod = snn.Conv2d(C, C, k, s, p, d, groups=C, bias=False).to(hip_device)
    mod.load_state_dict(ref.state_dict())
    with torch.no_grad():
        ref.weight.copy_(_q(ref.weight, mode))
    x = _q(torch.randn(2, C, H, W), mode)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    relu6 = act == 'relu6' and mode == 'f32'   # mask flips at bf16 rounding of 0 / 6 (see the ConvT test)
    if relu6:
        yr = torch.clamp(yr, 0, 6)
    gy = _q(torch.randn_like(yr), mode)
    yr.backward(gy)
    xa = _act_in(x, hip_device).detach().requires_grad_(True)
    y = mod.forward_act(xa, snn.ACT_RELU6) if relu6 else mod(xa)
    y.backward(_act_in(gy, hip_device))
    _close(y[:, :C], yr, mode, 'y')
    _close(mod.weight.grad, ref.weight.grad, mode, 'dW')
    _close(xa.grad[:, :C], xr.grad, mode, 'dx')


@pytest.mark.parametrize('cin,cout,H,W', [(16, 8, 5, 6), (64, 32, 4, 4), (128, 64, 8, 7)])
def test_conv_transpose_relu(hip_device, mode, cin, cout, H, W):
    from ssseg import nn as snn
    torch.manual_seed(1)
    ref = torch.nn.ConvTranspose2d(cin, cout, 4, 2, 1)
    mod = snn.ConvTranspose2d(cin, cout, 4, 2, 1).to(hip_device)
    mod.load_state_dict(ref.state_dict())
    with torch.no_grad():
        ref.weight.copy_(_q(ref.weight, mode))
    x = _q(torch.randn(2, cin, H, W), mode)
    xr = x.clone().requires_grad_(True)
    # the fused ReLU is checked in fp32; in bf16 outputs within rounding of 0 flip the ReLU mask, which
    # swaps whole gradient terms, so the bf16 case checks the transposed conv itself
    relu = mode == 'f32'
    yr = F.relu(ref(xr)) if relu else ref(xr)
    gy = _q(torch.randn_like(yr), mode)
    yr.backward(gy)
    xa = _act_in(x, hip_device).detach().requires_grad_(True)
    y = mod.forward_relu(xa) if relu else mod(xa)
    gya = _act_in(gy, hip_device)
    y.backward(gya)
    _close(y.float().permute(0, 1, 2, 3)[:, :cout], yr, mode, 'y')
    _close(mod.weight.grad, ref.weight.grad, mode, 'dW')
    _close(mod.bias.grad, ref.bias.grad, mode, 'db')
    _close(xa.grad[:, :cin], xr.grad, mode, 'dx')


@pytest.mark.parametrize('C', [32, 12])
@pytest.mark.parametrize('train', [True, False])
@pytest.mark.parametrize('relu,residual', [(True, False), (False, False), (True, True)])
def test_batchnorm_act(hip_device, mode, train, relu, residual, C):
    """C=12: 8-byte chunks in f32 mode, a 16-byte chunk half in padding in bf16 mode (pad written 0)."""
    from ssseg import nn as snn
    torch.manual_seed(2)
    ref = torch.nn.BatchNorm2d(C)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.3, 0.3)
        ref.running_mean.uniform_(-0.2, 0.2)
        ref.running_var.uniform_(0.5, 2.0)
    mod = snn.BatchNorm2d(C).to(hip_device)
    mod.load_state_dict(ref.state_dict())
    ref.train(train)
    mod.train(train)
    x = _q(torch.randn(4, C, 9, 7) * 2 + 0.5, mode)
    r = _q(torch.randn(4, C, 9, 7), mode)
    xr = x.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True)
    yr = ref(xr)
    if residual:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    gy = _q(torch.randn_like(yr), mode)
    yr.backward(gy)
    xa = _act_in(x, hip_device).detach().requires_grad_(True)
    ra = _act_in(r, hip_device).detach().requires_grad_(True) if residual else None
    y = snn.bn_act(xa, mod, relu=relu, residual=ra)
    y.backward(_act_in(gy, hip_device))
    _close(y[:, :C], yr, mode, 'y')
    _close(xa.grad[:, :C], xr.grad, mode, 'dx')
    assert float(y.detach()[:, C:].abs().sum()) == 0 and float(xa.grad[:, C:].abs().sum()) == 0, 'padding channels'
    _close(mod.weight.grad, ref.weight.grad, mode, 'dgamma')
    _close(mod.bias.grad, ref.bias.grad, mode, 'dbeta')
    if residual:
        _close(ra.grad[:, :C], rr.grad, mode, 'dres')
    np.testing.assert_allclose(mod.running_mean.cpu().numpy(), ref.running_mean.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(mod.running_var.cpu().numpy(), ref.running_var.numpy(), rtol=1e-5, atol=1e-6)
    assert int(mod.num_batches_tracked) == int(ref.num_batches_tracked)


@pytest.mark.parametrize('kind,cin,cout,relu,residual', [
    ('conv', 24, 20, True, True), ('conv', 16, 64, False, False), ('conv', 64, 128, True, False),
    ('convT', 16, 12, True, False), ('convT', 32, 64, True, True)])
def test_conv_bn_act_fused_eval(hip_device, mode, monkeypatch, kind, cin, cout, relu, residual):
    """Eval BatchNorm (+ residual, ReLU) folded into the conv epilogue under no_grad (teacher forward)."""
    from ssseg import nn as snn
    torch.manual_seed(5)
    if kind == 'conv':
        rc, mc = torch.nn.Conv2d(cin, cout, 3, 1, 1, bias=True), snn.Conv2d(cin, cout, 3, 1, 1, bias=True)
        H, W = 11, 9
    else:
        rc, mc = torch.nn.ConvTranspose2d(cin, cout, 4, 2, 1), snn.ConvTranspose2d(cin, cout, 4, 2, 1)
        H, W = 5, 6
    rb, mb = torch.nn.BatchNorm2d(cout), snn.BatchNorm2d(cout)
    with torch.no_grad():
        rc.weight.copy_(_q(rc.weight, mode))
        rb.weight.uniform_(0.5, 1.5)
        rb.bias.uniform_(-0.3, 0.3)
        rb.running_mean.uniform_(-0.2, 0.2)
        rb.running_var.uniform_(0.5, 2.0)
    mc.load_state_dict(rc.state_dict())
    mb.load_state_dict(rb.state_dict())
    mc, mb = mc.to(hip_device), mb.to(hip_device)
    rb.eval()
    mb.eval()
    x = _q(torch.randn(2, cin, H, W), mode)
    with torch.no_grad():
        yr = rb(rc(x))
        r = _q(torch.randn_like(yr), mode)
        if residual:
            yr = yr + r
        if relu:
            yr = F.relu(yr)
        monkeypatch.setattr(snn, 'bn_act', lambda *a, **k: (_ for _ in ()).throw(AssertionError('not fused')))
        y = snn.conv_bn_act(mc, _act_in(x, hip_device), mb, relu=relu,
                            residual=_act_in(r, hip_device) if residual else None)
    _close(y[:, :cout], yr, mode, 'y')
    assert float(y[:, cout:].abs().sum()) == 0, 'padding channels'


@pytest.mark.parametrize('kind,cin,cout,relu,residual,bias', [
    ('conv', 24, 20, True, True, False), ('conv', 64, 128, True, False, True), ('conv', 16, 64, False, False, False),
    ('convT', 16, 12, True, False, True), ('convT', 32, 64, True, True, True)])
def test_conv_bn_act_fused_eval_grad(hip_device, mode, monkeypatch, kind, cin, cout, relu, residual, bias):
    """Differentiated conv -> eval BN (-> +residual) (-> ReLU) (the consistency pass): fused forward and the
    ssseg_bn_eval_bwd backward against PyTorch fp32 autograd (dx, dres, dW, dbias, dgamma, dbeta)."""
    from ssseg import nn as snn
    torch.manual_seed(6)
    if kind == 'conv':
        rc, mc = torch.nn.Conv2d(cin, cout, 3, 1, 1, bias=bias), snn.Conv2d(cin, cout, 3, 1, 1, bias=bias)
        H, W = 10, 9
    else:
        rc, mc = torch.nn.ConvTranspose2d(cin, cout, 4, 2, 1, bias=bias), snn.ConvTranspose2d(cin, cout, 4, 2, 1, bias=bias)
        H, W = 5, 6
    rb, mb = torch.nn.BatchNorm2d(cout), snn.BatchNorm2d(cout)
    with torch.no_grad():
        rc.weight.copy_(_q(rc.weight, mode))
        rb.weight.uniform_(0.5, 1.5)
        rb.bias.uniform_(-0.3, 0.3)
        rb.running_mean.uniform_(-0.2, 0.2)
        rb.running_var.uniform_(0.5, 2.0)
    mc.load_state_dict(rc.state_dict())
    mb.load_state_dict(rb.state_dict())
    mc, mb = mc.to(hip_device), mb.to(hip_device)
    rb.eval()
    mb.eval()
    x = _q(torch.randn(2, cin, H, W), mode)
    xr = x.clone().requires_grad_(True)
    yr = rb(rc(xr))
    r = _q(torch.randn_like(yr), mode)
    rr = r.clone().requires_grad_(True)
    if residual:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    gy = _q(torch.randn_like(yr), mode)
    yr.backward(gy)
    monkeypatch.setattr(snn, 'bn_act', lambda *a, **k: (_ for _ in ()).throw(AssertionError('not fused')))
    xa = _act_in(x, hip_device).detach().requires_grad_(True)
    ra = _act_in(r, hip_device).detach().requires_grad_(True) if residual else None
    y = snn.conv_bn_act(mc, xa, mb, relu=relu, residual=ra)
    y.backward(_act_in(gy, hip_device))
    _close(y[:, :cout], yr, mode, 'y')
    assert float(y.detach()[:, cout:].abs().sum()) == 0, 'padding channels'
    _close(xa.grad[:, :cin], xr.grad, mode, 'dx')
    if residual:
        _close(ra.grad[:, :cout], rr.grad, mode, 'dres')
    _close(mc.weight.grad, rc.weight.grad, mode, 'dW')
    if bias:
        _close(mc.bias.grad, rc.bias.grad, mode, 'dbias')
    _close(mb.weight.grad, rb.weight.grad, mode, 'dgamma')
    _close(mb.bias.grad, rb.bias.grad, mode, 'dbeta')


ALL_VARIANTS = [11] + list(range(1, 11)) + list(range(12, 29))


@pytest.mark.parametrize('kind,cin,cout,k,H', [('conv', 64, 128, 3, 19), ('conv', 128, 64, 1, 17), ('conv', 192, 256, 3, 9),
                                               ('conv', 64, 256, 1, 21), ('convT', 128, 64, 4, 7),
                                               ('conv', 256, 200, 1, 23), ('conv', 192, 1024, 1, 11),
                                               ('conv_s2', 128, 256, 1, 18), ('conv', 64, 64, 1, 64),
                                               # C % 64 != 0: the general-k LDS-DMA loader (64-wide n-tiles)
                                               ('conv', 32, 32, 3, 33), ('conv', 16, 64, 3, 20), ('conv', 8, 48, 3, 17),
                                               ('conv', 48, 50, 3, 15), ('conv', 96, 64, 3, 13), ('conv', 50, 28, 1, 19),
                                               ('conv_s2', 32, 64, 3, 26), ('convT', 32, 32, 4, 9),
                                               # W % 64 == 0, H % 4 == 0: the halo-tiled 3x3 kernel (variant 24)
                                               ('conv64', 64, 64, 3, 8), ('conv64', 128, 128, 3, 12),
                                               ('conv64', 192, 64, 3, 4), ('conv64', 64, 192, 3, 20),
                                               # 32 x 32 / 16 x 16 maps: the halo kernel's 32- and 16-wide tiles
                                               ('conv32', 64, 64, 3, 16), ('conv32', 128, 192, 3, 8),
                                               ('conv16', 64, 128, 3, 16), ('conv16', 192, 64, 3, 32),
                                               # 32 -> 32 channels: its halo form (variant 25)
                                               ('conv64', 32, 32, 3, 8), ('conv64', 32, 32, 3, 12),
                                               # vpad: 240 / 120 channels run the 64-aligned path over 256 / 128
                                               ('conv', 240, 120, 3, 11), ('conv64', 240, 120, 3, 4),
                                               # 1x1 over 64 / 128 channels: the pointwise kernel (variants 26, 27),
                                               # several tiles per wave, ragged last tile
                                               ('conv', 64, 256, 1, 150), ('conv', 128, 512, 1, 96)])
def test_conv_variants_bitwise(hip_device, kind, cin, cout, k, H):
    """Every bf16 engine variant (register-staged, LDS-DMA tile configs 1..10 and 12..23) accumulates the
    same MFMA k-sequence: forward and input-gradient outputs are bit-identical, so autotuning never changes
    results.  C % 64 != 0 layers run the general-k loader on the 64-wide configs (the others fall back to the
    register-staged kernel when forced), whose linear k order is the register-staged kernel's.  'conv64' maps
    (W = 64 or 128) run the halo-tiled 3x3 kernel (variant 24; variant 25 for 32 -> 32 channels) in the forward and the
    input gradient; 240 -> 120 runs every variant on the virtually padded contraction (ssseg.nn.vpad)."""
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    torch.manual_seed(11)
    Wd = H + 3
    if kind == 'conv64':
        kind, Wd = 'conv', 64 if cin != 64 or cout != 192 else 128
    elif kind in ('conv32', 'conv16'):
        kind, Wd = 'conv', int(kind[4:])
    if kind == 'conv':
        mod = snn.Conv2d(cin, cout, k, 1, k // 2, bias=False).to(hip_device)
    elif kind == 'conv_s2':
        mod = snn.Conv2d(cin, cout, k, 2, 0, bias=False).to(hip_device)
    else:
        mod = snn.ConvTranspose2d(cin, cout, k, 2, 1).to(hip_device)
    x = _act_in(torch.randn(2, cin, H, Wd), hip_device).detach().requires_grad_(True)
    outs = []
    try:
        for v in ALL_VARIANTS:
            N.call('ssseg_set_knob', 4, v)
            y = mod(x)
            gy = torch.ones_like(y)
            (gx,) = torch.autograd.grad(y, x, gy)
            torch.cuda.synchronize()
            outs.append((v, y.detach().clone(), gx.clone()))
    finally:
        N.call('ssseg_set_knob', 4, 0)
    for v, y, gx in outs[1:]:
        assert torch.equal(y, outs[0][1]), f'variant {v}: forward differs'
        assert torch.equal(gx, outs[0][2]), f'variant {v}: input gradient differs'


@pytest.mark.parametrize('n,H,W', [(4, 256, 256), (3, 20, 192)])
def test_hconv3s_persistent_bitwise(hip_device, n, H, W):
    """The 32 -> 32-channel halo kernel (variant 25) is persistent (<= 512 blocks looping over 4 x 64 tiles with the
    next halo in flight): more tiles than blocks (1024 at 4 x 256^2) and a ragged last round must give the gather
    kernel's outputs bit for bit, forward and input gradient, with and without the fused BN statistics."""
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    torch.manual_seed(3)
    conv = snn.Conv2d(32, 32, 3, 1, 1, bias=False).to(hip_device)
    bn = snn.BatchNorm2d(32).to(hip_device)
    x = _act_in(torch.randn(n, 32, H, W), hip_device).detach().requires_grad_(True)
    outs = []
    try:
        for v in (14, 25):
            N.call('ssseg_set_knob', 4, v)
            y = conv(x)
            (gx,) = torch.autograd.grad(y, x, torch.ones_like(y))
            bn.reset_running_stats()
            with torch.no_grad():
                z = snn.conv_bn_act(conv, x, bn, relu=True)
            torch.cuda.synchronize()
            outs.append((y.detach().clone(), gx.clone(), z.clone(), bn.running_mean.clone(), bn.running_var.clone()))
    finally:
        N.call('ssseg_set_knob', 4, 0)
    a, b = outs
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert torch.equal(a[2], b[2])
    torch.testing.assert_close(a[3], b[3], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(a[4], b[4], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('cin,cout,n,H,W', [(64, 256, 4, 64, 64), (128, 512, 3, 33, 40), (64, 64, 2, 9, 13),
                                            (128, 128, 2, 50, 31)])
def test_pointwise_kernel_bitwise(hip_device, cin, cout, n, H, W):
    """The register-direct pointwise kernel (variants 26 / 27, conv_pw.hip) vs the gather kernel (config 14): the
    folded eval-BN epilogue with ReLU, with and without a residual (+ the raw-accumulator copy: the differentiated
    consistency pass, output and every gradient), bit for bit, and a training BatchNorm fed by its fused statistics
    (per-wave rows instead of per-tile rows: fp32 summation order only) within 1e-6 of the gather kernel's.  (The
    64-pixel form, 26, takes no residual: forced there it falls back to the heuristic's kernel, so the residual pass
    is compared for 27 only.)"""
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    torch.manual_seed(8)
    conv = snn.Conv2d(cin, cout, 1, 1, 0, bias=False).to(hip_device)
    bn = snn.BatchNorm2d(cout).to(hip_device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    x = _act_in(torch.randn(n, cin, H, W) + 0.2, hip_device).detach().requires_grad_(True)
    res = _act_in(torch.randn(n, cout, H, W), hip_device).detach().requires_grad_(True)
    gy = _act_in(torch.randn(n, cout, H, W), hip_device)
    outs = {}
    try:
        for v in (14, 26, 27):
            N.call('ssseg_set_knob', 4, v)
            bn.train()
            bn.reset_running_stats()
            with torch.no_grad():
                z = snn.conv_bn_act(conv, x, bn, relu=True)
            o = {'train': (z.clone(), bn.running_mean.clone(), bn.running_var.clone())}
            bn.eval()
            for key, r in (('plain', None), ('res', res)):
                for t in (x, res, conv.weight):
                    t.grad = None
                y = snn.conv_bn_act(conv, x, bn, relu=True, residual=r)
                y.backward(gy)
                torch.cuda.synchronize()
                o[key] = [y.detach().clone(), x.grad.clone(), conv.weight.grad.clone()] + (
                    [res.grad.clone()] if r is not None else [])
            outs[v] = o
    finally:
        N.call('ssseg_set_knob', 4, 0)
    ref = outs[14]
    for v in (26, 27) if cin == 64 else (27,):   # 26: 64 channels only
        for key in ('plain', 'res') if v == 27 else ('plain',):
            for a, b, name in zip(outs[v][key], ref[key], ('y', 'dx', 'dW', 'dres')):
                assert torch.equal(a, b), (v, key, name)
        (z, rm, rv), (z0, rm0, rv0) = outs[v]['train'], ref['train']
        torch.testing.assert_close(rm, rm0, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(rv, rv0, rtol=1e-6, atol=1e-7)
        assert float((z.float() - z0.float()).abs().max()) <= 1e-2 * float(z0.float().abs().max())


WGRAD_CASES = [
    # cin, cout, k, stride, pad, dil, H, W, N   (the LDS-DMA weight-gradient kernel)
    (64, 64, 3, 1, 1, 1, 37, 29, 2),      # 64-channel kk-tiles, 64-channel co tile, several pixel splits
    (128, 192, 3, 1, 1, 1, 21, 19, 2),    # 128-channel kk-tiles, ragged co tile
    (256, 64, 1, 1, 0, 1, 45, 43, 3),     # 1x1, ragged last split
    (128, 128, 3, 2, 1, 1, 40, 37, 2),    # stride 2
    (64, 128, 3, 1, 2, 2, 23, 25, 2),     # dilation 2
    (512, 256, 1, 2, 0, 1, 18, 18, 2),    # strided 1x1 downsample
    (128, 64, 1, 1, 0, 1, 9, 11, 2),      # one split: dW written in its final layout directly
    # C % 64 != 0: the general-k tiles (a 64-wide kk-tile holds several taps; per-lane tap offsets)
    (32, 32, 3, 1, 1, 1, 37, 29, 2),      # HRNet-W32 branch
    (16, 64, 3, 1, 1, 1, 33, 31, 2),      # four taps per kk-tile
    (96, 64, 3, 2, 1, 1, 30, 28, 2),      # a tap boundary inside the second kk-tile, stride 2
    (40, 24, 1, 1, 0, 1, 25, 27, 2),      # 1x1, ragged kk-tile
    (32, 64, 3, 2, 1, 1, 34, 33, 2),      # HRNet-W32 transition (strided)
]


@pytest.mark.parametrize('cin,cout,k,s,p,d,H,W,n', WGRAD_CASES)
def test_wgrad_lds_dma(hip_device, cin, cout, k, s, p, d, H, W, n):
    """bf16 weight gradient on the LDS-DMA kernel (knob 8 = 0, the default) and on the register-staged
    kernel (knob 8 = -1) vs PyTorch fp32 on the same bf16-rounded operands.  The bf16 products are exact
    in fp32, so the kernels differ from the reference only by fp32 summation order: 1e-4 of max|dW|."""
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    torch.manual_seed(3)
    ref = torch.nn.Conv2d(cin, cout, k, s, p, d, bias=False)
    with torch.no_grad():
        ref.weight.copy_(ref.weight.bfloat16().float())
    mod = snn.Conv2d(cin, cout, k, s, p, d, bias=False).to(hip_device)
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(n, cin, H, W).bfloat16().float()
    yr = ref(x)
    gy = torch.randn_like(yr).bfloat16().float()
    yr.backward(gy)
    xa = snn.to_act(x.to(hip_device))
    gya = snn.to_act(gy.to(hip_device))
    grads = []
    try:
        for knob in (0, -1):
            N.call('ssseg_set_knob', 8, knob)
            mod.weight.grad = None
            mod(xa).backward(gya)
            torch.cuda.synchronize()
            grads.append(mod.weight.grad.detach().float().cpu())
    finally:
        N.call('ssseg_set_knob', 8, 0)
    gref = ref.weight.grad
    scale = float(gref.abs().max())
    for name, g in zip(('lds-dma', 'register-staged'), grads):
        err = float((g - gref).abs().max()) / scale
        assert err < 1e-4, f'{name}: max rel err {err}'


HALO_CASES = [
    # cin, cout, H, W, n, n2 (second pixel segment of a merged launch: 0 = none)
    (64, 64, 37, 64, 2, 0),       # one 64-channel block each way, column changes mid-split
    (128, 64, 20, 128, 2, 3),     # two channel blocks, two strips, merged launch with a different batch
    (384, 128, 9, 64, 3, 0),      # 6 x 2 channel blocks (the UNet decoder's 384 -> 128 shape)
    (64, 128, 64, 192, 1, 1),     # three strips, merged
    (64, 64, 1, 64, 1, 0),        # one row step: a single split writes dW directly
]


@pytest.mark.parametrize('cin,cout,H,W,n,n2', HALO_CASES)
def test_wgrad_halo3(hip_device, cin, cout, H, W, n, n2):
    """Halo-tiled 3x3 weight gradient (conv_wgrad_halo.hip, knob 11 = 0, the default for 3x3 / stride-1 / pad-1
    layers with W % 64 == 0) and the split-K LDS-DMA kernel (knob 11 = -1) vs PyTorch fp32 on the same bf16-rounded
    operands, single and merged (defer_wgrad: two backward passes, one launch over both pixel sets): fp32 summation
    order only, 1e-4 of max|dW|."""
    import contextlib
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    torch.manual_seed(5)
    ref = torch.nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
    with torch.no_grad():
        ref.weight.copy_(ref.weight.bfloat16().float())
    mod = snn.Conv2d(cin, cout, 3, 1, 1, bias=False).to(hip_device)
    mod.load_state_dict(ref.state_dict())
    passes = [n] + ([n2] if n2 else [])
    xs = [torch.randn(b, cin, H, W).bfloat16().float() for b in passes]
    gys = [torch.randn(b, cout, H, W).bfloat16().float() for b in passes]
    for x, gy in zip(xs, gys):
        ref(x).backward(gy)
    gref = ref.weight.grad
    grads = []
    try:
        for knob in (0, -1):
            N.call('ssseg_set_knob', 11, knob)
            mod.weight.grad = None
            for i, (x, gy) in enumerate(zip(xs, gys)):
                with (snn.defer_wgrad() if i == 0 and len(passes) > 1 else contextlib.nullcontext()):
                    mod(snn.to_act(x.to(hip_device))).backward(snn.to_act(gy.to(hip_device)))
            snn.flush_wgrad()
            torch.cuda.synchronize()
            grads.append(mod.weight.grad.detach().float().cpu())
    finally:
        N.call('ssseg_set_knob', 11, 0)
    scale = float(gref.abs().max())
    for name, g in zip(('halo', 'split-K'), grads):
        err = float((g - gref).abs().max()) / scale
        assert err < 1e-4, f'{name}: max rel err {err}'


@pytest.mark.parametrize('k,s,p,ceil', [(3, 2, 1, False), (2, 2, 0, True)])
def test_maxpool(hip_device, mode, k, s, p, ceil):
    from ssseg import nn as snn
    torch.manual_seed(3)
    x = _q(torch.randn(2, 16, 11, 9), mode)
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p, ceil_mode=ceil)
    gy = _q(torch.randn_like(yr), mode)
    yr.backward(gy)
    xa = _act_in(x, hip_device).detach().requires_grad_(True)
    y = snn.MaxPool2d(k, s, p, ceil_mode=ceil)(xa)
    y.backward(_act_in(gy, hip_device))
    _close(y, yr, mode, 'y')
    _close(xa.grad, xr.grad, mode, 'dx')


@pytest.mark.parametrize('H,W', [(12, 10), (13, 16)])
def test_maxpool_ties(hip_device, mode, H, W):
    """3x3 / stride-2 pool (the ResNet stem's: batched-load paths in misc.hip) on values with many ties: the
    forward keeps PyTorch's first-maximal-tap index, so the input gradient lands where PyTorch's does, exactly."""
    from ssseg import nn as snn
    torch.manual_seed(5)
    x = torch.randint(0, 3, (2, 16, H, W)).float()
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    gy = torch.randint(-4, 5, yr.shape).float()
    yr.backward(gy)
    xa = _act_in(x, hip_device).detach().requires_grad_(True)
    y = snn.MaxPool2d(3, 2, 1)(xa)
    y.backward(_act_in(gy, hip_device))
    assert torch.equal(y.detach().float().cpu(), yr.detach())
    assert torch.equal(xa.grad.float().cpu(), xr.grad)


def test_cat_crop(hip_device, mode):
    from ssseg import nn as snn
    torch.manual_seed(4)
    a = _q(torch.randn(2, 8, 10, 10), mode)
    b = _q(torch.randn(2, 16, 9, 9), mode)
    ar, br = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = torch.cat((ar[:, :, 0:9, 0:9], br), 1)
    gy = _q(torch.randn_like(yr), mode)
    yr.backward(gy)
    aa = _act_in(a, hip_device).detach().requires_grad_(True)
    ba = _act_in(b, hip_device).detach().requires_grad_(True)
    y = snn.cat_crop(aa, ba, 8, 16)
    y.backward(_act_in(gy, hip_device))
    _close(y, yr, mode, 'y')
    _close(aa.grad, ar.grad, mode, 'da')
    _close(ba.grad, br.grad, mode, 'db')


def test_no_cpu_fallback_for_layers():
    from ssseg import nn as snn
    mod = snn.Conv2d(8, 8, 3, padding=1)
    with pytest.raises(RuntimeError):
        mod(torch.randn(1, 8, 4, 4))


def _small_resnet_unet(dev):
    from models import unet
    from models.adapters import ListOutput
    from models.encoders import resnet
    torch.manual_seed(21)
    return ListOutput(unet.UNet(2, resnet.resnet50_encoder(), max_width=32, train_upsampling=True)).to(dev)


def test_batched_repack_after_weight_update(hip_device):
    """invalidate_packed() refreshes every cached fwd/dgrad/phase pack with one batched launch: a forward
    + backward after an in-place weight change equals a model that never packed the old weights."""
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    a = _small_resnet_unet(hip_device)
    b = _small_resnet_unet(hip_device)
    x = torch.rand(2, 3, 64, 64, device=hip_device)
    a.train()
    a(x)[-1][-1].float().sum().backward()          # packs fwd + dgrad layouts of every conv
    with torch.no_grad():
        for pa in a.parameters():
            pa.mul_(0.9)
    b.load_state_dict(a.state_dict())                 # same weights AND running statistics
    snn.invalidate_packed(a)
    a.eval()
    b.eval()
    with torch.no_grad():
        ya = a(x)[-1][-1]
        yb = b(x)[-1][-1]
    assert torch.equal(ya, yb)


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float32])
def test_batched_repack_matches_single_pack(hip_device, dt):
    """ssseg_weight_pack_batch (the LDS-tiled repack after an optimizer / EMA step) writes every packed layout --
    forward [K][R][S][C], flipped dgrad, ConvTranspose2d phases, strided-dgrad phases, 7x7 stem, channel padding --
    bit-identical to the one-pack-per-launch kernel ssseg_weight_pack."""
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(dt)
    torch.manual_seed(5)
    mods = [snn.Conv2d(3, 64, 7, 2, 3, bias=False), snn.Conv2d(64, 40, 3, 1, 1), snn.Conv2d(40, 256, 1),
            snn.Conv2d(256, 72, 3, 2, 1), snn.ConvTranspose2d(72, 24, 4, 2, 1), snn.Conv2d(24, 24, 5, 1, 2)]
    model = torch.nn.Sequential(*mods).to(hip_device)
    try:
        x = snn.to_act(torch.randn(2, 3, 32, 32, device=hip_device)).requires_grad_(True)
        y = x
        for m in mods:
            y = m(y)
        torch.autograd.backward(y, snn.to_act(torch.ones(y.shape, device=hip_device)))   # fwd + dgrad packs
        with torch.no_grad():
            for p in model.parameters():
                p.mul_(-0.7).add_(0.01)
        snn.invalidate_packed(model)                     # batched repack into the cached pack tensors
        torch.cuda.synchronize()
        npacks = 0
        for m in mods:
            w = m.weight.detach().contiguous()
            for key, t in m._ssseg_packs.items():
                Kd, Kr, Cd, Rs, Ss, Cp, layout, r0, rstep, Rn, s0, sstep, Sn = m._ssseg_specs[key]
                ref = torch.empty_like(t)
                N.call('ssseg_weight_pack', N.dev_ptr(w), N.dev_ptr(ref), Kd, Kr, Cd, Rs, Ss, Cp, layout, r0, rstep,
                       Rn, s0, sstep, Sn, N.dt_code(ref), N.stream())
                torch.cuda.synchronize()
                assert torch.equal(t, ref), (type(m).__name__, key)
                npacks += 1
        assert npacks >= 10
    finally:
        snn.set_compute_dtype(torch.bfloat16)


def test_folded_context_bitwise(hip_device):
    """snn.folded(model): one batched BN fold for the whole eval forward, bit-identical to per-layer folds,
    with and without autograd (teacher pass / consistency pass)."""
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    m = _small_resnet_unet(hip_device)
    x = torch.rand(2, 3, 64, 64, device=hip_device)
    m.train()
    m(x)                       # running stats move away from their init
    m.eval()
    with torch.no_grad():
        y0 = m(x)[-1][-1].clone()          # per-layer folds (records the conv/BN pairs)
        with snn.folded(m):
            y1 = m(x)[-1][-1].clone()
    assert torch.equal(y0, y1)
    xr = x.clone().requires_grad_(True)
    g0 = torch.autograd.grad(m(xr)[-1][-1].float().square().sum(), xr)[0]
    with snn.folded(m):
        out = m(xr)[-1][-1]
    g1 = torch.autograd.grad(out.float().square().sum(), xr)[0]
    assert torch.equal(g0, g1)


@pytest.mark.parametrize('C,P', [(64, 16 * 64 * 64), (200, 3 * 17 * 19), (1024, 16 * 16 * 16)])
def test_bn_fused_tails_match_unfused(hip_device, C, P):
    """ssseg_bn_stats_finalize == ssseg_bn_stats + ssseg_bn_finalize (the SyncBN path keeps the split form)
    and ssseg_bn_bwd_reduce_grad == ssseg_bn_bwd_reduce + ssseg_bn_param_grad, bit for bit (same reduction
    order; the tail only moves the per-channel math into the reduction kernel)."""
    from ssseg import native as N
    dev = hip_device
    g = torch.Generator().manual_seed(C)
    cp = (C + 7) // 8 * 8
    x = torch.zeros(P, cp, dtype=torch.bfloat16)
    x[:, :C] = (torch.randn(P, C, generator=g) * 2 + 0.5).bfloat16()
    dy = torch.zeros(P, cp, dtype=torch.bfloat16)
    dy[:, :C] = torch.randn(P, C, generator=g).bfloat16()
    x, dy = x.to(dev), dy.to(dev)
    nb = N.lib().ssseg_bn_workspace_bytes(C)
    ws = N.workspace(nb, dev)
    outs = []
    for fused in (False, True):
        sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
        mean = torch.empty(C, device=dev)
        inv = torch.empty(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        tail = (float(P), 1e-5, 0.1, N.dev_ptr(mean), N.dev_ptr(inv), N.dev_ptr(rm), N.dev_ptr(rv), N.dev_ptr(nbt))
        if fused:
            N.call('ssseg_bn_stats_finalize', N.dev_ptr(x), P, C, cp, N.BF16, N.dev_ptr(sums), N.dev_ptr(ws), nb,
                   *tail, N.stream())
        else:
            N.call('ssseg_bn_stats', N.dev_ptr(x), P, C, cp, N.BF16, N.dev_ptr(sums), N.dev_ptr(ws), nb, N.stream())
            N.call('ssseg_bn_finalize', N.dev_ptr(sums), C, *tail, N.stream())
        gamma = torch.linspace(0.5, 1.5, C, device=dev)
        beta = torch.linspace(-0.2, 0.2, C, device=dev)
        bsums = torch.empty(2 * C, dtype=torch.float64, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        args = (N.dev_ptr(dy), N.dev_ptr(x), None, P, C, cp, cp, cp, N.dev_ptr(mean), N.dev_ptr(inv),
                N.dev_ptr(gamma), N.dev_ptr(beta), 1, N.BF16, N.dev_ptr(bsums), N.dev_ptr(ws), nb)
        if fused:
            N.call('ssseg_bn_bwd_reduce_grad', *args, N.dev_ptr(dg), N.dev_ptr(db), N.stream())
        else:
            N.call('ssseg_bn_bwd_reduce', *args, N.stream())
            N.call('ssseg_bn_param_grad', N.dev_ptr(bsums), C, N.dev_ptr(dg), N.dev_ptr(db), N.stream())
        outs.append([t.cpu() for t in (sums, mean, inv, rm, rv, nbt, bsums, dg, db)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert int(outs[1][5]) == 1


@pytest.mark.parametrize('kind,cin,cout,k,s,H', [('conv', 64, 128, 3, 1, 19), ('conv', 128, 64, 1, 1, 17),
                                                 ('conv', 64, 256, 1, 2, 21), ('conv', 16, 40, 3, 1, 13),
                                                 ('convT', 128, 64, 4, 2, 7), ('conv', 8, 12, 3, 1, 11),
                                                 ('conv', 192, 320, 1, 1, 29)])
def test_fused_bn_stats_match_separate_pass(hip_device, mode, kind, cin, cout, k, s, H):
    """Training BatchNorm statistics from the producing conv's epilogue (ssseg_conv_epilogue.stats, fp64 tile
    partials of the stored output) == the separate statistics pass over that output (ssseg_bn_stats): same
    normalised output, same running statistics — for every bf16 engine variant (register-staged, each
    LDS-DMA tile config, with and without the LDS-staged epilogue) and the fp32 path."""
    from ssseg import native as N
    from ssseg import nn as snn
    torch.manual_seed(5)
    if kind == 'conv':
        conv = snn.Conv2d(cin, cout, k, s, k // 2, bias=False).to(hip_device)
    else:
        conv = snn.ConvTranspose2d(cin, cout, k, s, 1, bias=False).to(hip_device)
    bn = snn.BatchNorm2d(cout).to(hip_device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    x = _act_in(torch.randn(2, cin, H, H + 2) + 0.3, hip_device)
    variants = [(0, 0)] if mode == 'f32' else [(v, e) for v in ALL_VARIANTS for e in (0, -1)]
    try:
        for v, e in variants:
            N.call('ssseg_set_knob', 4, v)
            N.call('ssseg_set_knob', 7, e)
            outs = []
            for fused in (False, True):
                snn.set_fused_bn_stats(fused)
                bn.reset_running_stats()
                with torch.no_grad():
                    y = snn.conv_bn_act(conv, x, bn, relu=True)
                torch.cuda.synchronize()
                outs.append((y.float().cpu(), bn.running_mean.cpu().clone(), bn.running_var.cpu().clone()))
            (y0, m0, v0), (y1, m1, v1) = outs
            assert torch.allclose(m1, m0, rtol=1e-6, atol=1e-7), (v, e, 'running_mean')
            assert torch.allclose(v1, v0, rtol=1e-6, atol=1e-7), (v, e, 'running_var')
            tol = 1e-5 if mode == 'f32' else 1e-2
            assert float((y1 - y0).abs().max()) <= tol * (float(y0.abs().max()) + 1e-6), (v, e, 'output')
    finally:
        N.call('ssseg_set_knob', 4, 0)
        N.call('ssseg_set_knob', 7, 0)
        snn.set_fused_bn_stats(True)



@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("k,s,H,W", [(7, 2, 38, 256), (3, 2, 33, 512), (7, 1, 17, 128)])
def test_stem_conv_kernel(hip_device, dtype, k, s, H, W):
    """Image-input conv kernel (ssseg_conv_stem_epi: k = (s, c) of one filter row per MFMA step, operands
    straight from the image) vs the generic engine on the same layer: plain forward, training BatchNorm with
    fused statistics, eval BatchNorm folded with the raw accumulator kept (the differentiated consistency
    pass) and its gradients; both within fp32 rounding of each other (different k grouping), and the forward
    within the 16-bit tolerance of a PyTorch fp32 reference."""
    from ssseg import nn as snn
    snn.set_compute_dtype(dtype)
    tol = 1e-3
    try:
        torch.manual_seed(4)
        conv = snn.Conv2d(3, 64, k, s, k // 2, bias=False).to(hip_device)
        bn = snn.BatchNorm2d(64).to(hip_device)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
        x = torch.rand(2, 3, H, W)
        xa = _act_in(x, hip_device)
        outs = {}
        for stem in (False, True):
            snn.set_stem_kernel(stem)
            with torch.no_grad():
                y0 = conv(xa)
                bn.train()
                bn.reset_running_stats()
                y1 = snn.conv_bn_act(conv, xa, bn, relu=True)
                rm = bn.running_mean.clone()
                bn.eval()
            xg = xa.detach().clone().requires_grad_(False)
            conv.weight.grad = None
            y2 = snn.conv_bn_act(conv, xg, bn, relu=True)
            y2.backward(torch.ones_like(y2))
            torch.cuda.synchronize()
            outs[stem] = [t.detach().float().cpu().clone() for t in (y0, y1, rm, y2, conv.weight.grad)]
        for name, a, b in zip(('conv', 'train-bn', 'running_mean', 'eval-bn', 'dW'), outs[False], outs[True]):
            err = float((a - b).abs().max()) / (float(a.abs().max()) + 1e-6)
            # same 16-bit inputs and weights, fp32 accumulation in a different k order: outputs differ by at most
            # one 16-bit rounding step where a sum falls near a rounding boundary
            assert err <= (1e-2 if dtype == torch.bfloat16 else 2e-3), (name, err)
        ref = F.conv2d(_q(x, 'bf16' if dtype == torch.bfloat16 else 'f16'),
                       _q(conv.weight.detach().cpu(), 'bf16' if dtype == torch.bfloat16 else 'f16'), stride=s,
                       padding=k // 2)
        _close(outs[True][0][:, :64], ref, 'bf16' if dtype == torch.bfloat16 else 'f16', 'stem y')
    finally:
        snn.set_stem_kernel(True)
        snn.set_compute_dtype(torch.bfloat16)
    del tol


@pytest.mark.parametrize('cin,cout,H', [(256, 128, 8), (128, 64, 13), (64, 40, 6)])
def test_convT_phase_launch_bitwise(hip_device, cin, cout, H):
    """ConvTranspose2d(4,2,1) forward as ONE launch over its four output phases (ssseg_conv_igemm_phases) vs one
    launch per phase: bit-identical outputs (same MFMA k-sequence per output), for the plain + bias + ReLU
    epilogue, training BatchNorm with fused statistics (phase-major partial rows) and the eval fold with the raw
    copy; input gradients too."""
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    torch.manual_seed(8)
    conv = snn.ConvTranspose2d(cin, cout, 4, 2, 1).to(hip_device)
    bn = snn.BatchNorm2d(cout).to(hip_device)
    x = _act_in(torch.randn(2, cin, H, H + 1), hip_device)
    outs = {}
    try:
        for ph in (False, True):
            snn.set_phase_launch(ph)
            with torch.no_grad():
                y0 = conv.forward_relu(x)
                bn.train()
                bn.reset_running_stats()
                y1 = snn.conv_bn_act(conv, x, bn, relu=True)
                rv = bn.running_var.clone()
            bn.eval()
            xg = x.detach().clone().requires_grad_(True)
            y2 = snn.conv_bn_act(conv, xg, bn, relu=True)
            (gx,) = torch.autograd.grad(y2, xg, torch.ones_like(y2))
            torch.cuda.synchronize()
            outs[ph] = [t.detach().float().cpu().clone() for t in (y0, y1, rv, y2, gx)]
    finally:
        snn.set_phase_launch(True)
    for name, a, b in zip(('relu', 'train-bn', 'running_var', 'eval-bn', 'dx'), outs[False], outs[True]):
        if name == 'running_var':   # fp64 partial rows summed in another order across phases
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-8), name
        else:
            assert torch.equal(a, b), name


@pytest.mark.parametrize('relu', [True, False])
def test_eval_bn_backward_from_y_matches_aux(hip_device, mode, relu):
    """Differentiated eval pass without a residual: x_hat recovered from y (ssseg_bn_eval_bwd_grad_y, no raw
    accumulator copy) vs the raw-copy path: input, weight, gamma, beta gradients agree to the mode's rounding."""
    from ssseg import nn as snn
    torch.manual_seed(9)
    conv = snn.Conv2d(64, 96, 3, 1, 1, bias=True).to(hip_device)
    bn = snn.BatchNorm2d(96).to(hip_device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 1.5)
    bn.eval()
    x0 = _act_in(torch.randn(2, 64, 15, 17), hip_device)
    gy = _act_in(torch.randn(2, 96, 15, 17), hip_device)
    outs = {}
    try:
        for ymode in (False, True):
            snn.set_eval_bwd_from_y(ymode)
            for p in (conv.weight, conv.bias, bn.weight, bn.bias):
                p.grad = None
            x = x0.detach().clone().requires_grad_(True)
            y = snn.conv_bn_act(conv, x, bn, relu=relu)
            y.backward(gy)
            torch.cuda.synchronize()
            outs[ymode] = [t.detach().float().cpu().clone() for t in
                           (y, x.grad, conv.weight.grad, conv.bias.grad, bn.weight.grad, bn.bias.grad)]
    finally:
        snn.set_eval_bwd_from_y(True)
    tol = {'f32': 1e-5, 'bf16': 2e-2, 'f16': 4e-3}[mode]
    for name, a, b in zip(('y', 'dx', 'dW', 'db', 'dgamma', 'dbeta'), outs[False], outs[True]):
        err = float((a - b).abs().max()) / (float(a.abs().max()) + 1e-12)
        assert err <= tol, (name, err)


@pytest.mark.parametrize('kind,cin,cout,k,s,H,n1,n2', [('conv', 64, 128, 3, 1, 19, 2, 3), ('conv', 128, 64, 1, 1, 17, 3, 3),
                                                       ('conv', 128, 256, 3, 2, 18, 2, 1), ('conv', 3, 64, 7, 2, 21, 2, 2),
                                                       ('convT', 128, 64, 4, 2, 7, 2, 3), ('conv', 64, 64, 3, 1, 64, 4, 4)])
def test_wgrad_merged_two_passes(hip_device, mode, kind, cin, cout, k, s, H, n1, n2):
    """defer_wgrad + the next backward: ONE ssseg_conv_wgrad2 launch over both passes' pixels gives the summed
    weight gradient of the two backward passes (reference train.py:61,115 accumulate into one .grad):
    checked against fp32 PyTorch-CPU of both passes, and against the two separate launches (merge off)."""
    from ssseg import nn as snn
    torch.manual_seed(5)
    if kind == 'conv':
        mod = snn.Conv2d(cin, cout, k, s, k // 2, bias=True).to(hip_device)
        ref = torch.nn.Conv2d(cin, cout, k, s, k // 2, bias=True)
    else:
        mod = snn.ConvTranspose2d(cin, cout, k, s, 1, bias=True).to(hip_device)
        ref = torch.nn.ConvTranspose2d(cin, cout, k, s, 1, bias=True)
    ref.load_state_dict({kk: v.cpu() for kk, v in mod.state_dict().items()})
    xs = [torch.randn(n, cin, H, H) for n in (n1, n2)]
    gs = []
    for x in xs:
        y = ref(_q(x, mode))
        gs.append(torch.randn_like(y))
        (_q(gs[-1], mode) * y).sum().backward()
    ref_w = ref.weight.grad.clone()

    def run(merge):
        snn.set_wgrad_merge(merge)
        mod.weight.grad = None
        mod.bias.grad = None
        try:
            for i, (x, g) in enumerate(zip(xs, gs)):
                xa = snn.to_act(x.to(hip_device))
                y = mod(xa)
                with (snn.defer_wgrad() if i == 0 else contextlib.nullcontext()):
                    y.backward(snn.to_act(g.to(hip_device)))
                if i == 0 and merge:
                    assert snn.wgrad_pending() == 1
            snn.flush_wgrad()
            assert snn.wgrad_pending() == 0
            return mod.weight.grad.clone(), mod.bias.grad.clone()
        finally:
            snn.set_wgrad_merge(True)

    w_m, b_m = run(True)
    w_s, b_s = run(False)
    _close(w_m, ref_w, mode, 'merged dW')
    _close(b_m, ref.bias.grad, mode, 'merged db')
    _close(w_s, ref_w, mode, 'separate dW')
    scale = float(w_s.abs().max())
    assert float((w_m - w_s).abs().max()) <= 1e-5 * scale + 1e-7, 'merged vs separate launches'


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('cin,cout,H,n', [(176, 28, 16, 2), (133, 14, 32, 1), (78, 34, 8, 16), (512, 64, 4, 2)])
def test_conv_split_k_small_maps(hip_device, dtype, cin, cout, H, n):
    """deterministic split-K on tile-starved launches with a moderate contraction (HarDNet growth layers at 8^2-32^2,
    C % 64 != 0: the general-k loader starting at a slice's k-tile): forward, input and weight gradients vs PyTorch
    fp32 CPU, and run-to-run bitwise"""
    from ssseg import native as N
    from ssseg import nn as snn
    mode = 'bf16' if dtype == torch.bfloat16 else 'f16'
    snn.set_compute_dtype(dtype)
    try:
        cp = snn.rup(cin, snn.vec())
        d = snn._desc(N=n, H=H, W=H, C=cp, ldx=cp, OH=H, OW=H, K=snn.rup(cout, snn.vec()), R=3, S=3, sy=1, sx=1, dy=1,
                      dx=1, py=-1, px=-1, outH=H, outW=H, osy=1, osx=1, ooy=0, oox=0, ldy=snn.rup(cout, snn.vec()),
                      ldw=9 * cp)
        assert N.lib().ssseg_conv_igemm_workspace_bytes(snn.ctypes_ref(d), N.dt_code(torch.empty(0, dtype=dtype))) > 0
        torch.manual_seed(1)
        ref = torch.nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
        mod = snn.Conv2d(cin, cout, 3, 1, 1, bias=False).to(hip_device)
        mod.load_state_dict(ref.state_dict())
        with torch.no_grad():
            ref.weight.copy_(_q(ref.weight, mode))
        x = _q(torch.randn(n, cin, H, H), mode)
        xr = x.clone().requires_grad_(True)
        yr = ref(xr)
        gy = _q(torch.randn_like(yr), mode)
        yr.backward(gy)
        outs = []
        for _ in range(2):
            mod.zero_grad(set_to_none=True)
            xa = _act_in(x, hip_device).detach().requires_grad_(True)
            y = mod(xa)
            y.backward(snn.to_act(gy.to(hip_device)))
            outs.append((y[:, :cout].float().cpu(), xa.grad[:, :cin].float().cpu(), mod.weight.grad.cpu().clone()))
        _close(outs[0][0], yr, mode, 'y')
        _close(outs[0][1], xr.grad, mode, 'dx')
        _close(outs[0][2], ref.weight.grad, mode, 'dW')
        for a, b in zip(outs[0], outs[1]):
            assert torch.equal(a, b)
    finally:
        snn.set_compute_dtype(torch.bfloat16)


@pytest.mark.parametrize('act', [('leaky', 0.2), True])
def test_dgrad_applies_producer_activation_backward(hip_device, mode, act):
    """Conv4x4/s2 + LeakyReLU (or ReLU) feeding exactly one conv (the discriminator, discriminator.py:14-17): the
    consumer's input gradient applies the producer's activation backward in its epilogue
    (ssseg_conv_igemm_epi_actmask) -- same gradients as the separate activation-backward pass, within rounding."""
    from ssseg import nn as snn
    torch.manual_seed(4)
    c1 = snn.Conv2d(8, 32, 4, 2, 1).to(hip_device)
    c2 = snn.Conv2d(32, 48, 4, 2, 1).to(hip_device)
    x = _q(torch.randn(2, 8, 34, 30), mode)
    outs = []
    for on in (True, False):
        snn._CFG['act_mask'] = on
        try:
            c1.zero_grad(set_to_none=True)
            c2.zero_grad(set_to_none=True)
            xa = _act_in(x, hip_device).detach().requires_grad_(True)
            h = c1.forward_act(xa, act, single_use=True)
            assert h.__dict__.get('_ssseg_act_out') is not None
            y = c2(h)
            g = snn.to_act(_q(torch.randn(y.shape[0], 48, y.shape[2], y.shape[3],
                                          generator=torch.Generator().manual_seed(5)), mode).to(hip_device))
            y.backward(g)
            outs.append((xa.grad[:, :8].float().cpu(), c1.weight.grad.cpu().clone(), c1.bias.grad.cpu().clone()))
        finally:
            snn._CFG['act_mask'] = True
    for a, b, what in zip(outs[0], outs[1], ('dx', 'dW1', 'db1')):
        _close(a, b, mode, what)


@pytest.mark.parametrize('k2,s2,cout2,H,W', [(3, 1, 48, 19, 21), (1, 1, 128, 17, 18), (3, 2, 64, 20, 22),
                                             (3, 1, 64, 16, 64)])
def test_bn_backward_sums_from_consumer_dgrad(hip_device, mode, monkeypatch, k2, s2, cout2, H, W):
    """Training conv -> BN -> ReLU whose output feeds exactly one conv (Bottleneck bn1 / bn2, UNet conv3_0; reference
    resnet Bottleneck and unet.py:9-10): the consumer's input-gradient launch applies the ReLU backward and writes the
    BN backward's two channel sums in its epilogue (gradient statistics rows, ssseg_bn_gstat_finalize), and the BN
    backward skips its reduction pass over dy and x -- the same gradients as the separate pass within rounding (x_hat
    comes from y instead of x), for every engine variant (the (3, 1, 64, 16, 64) case reaches the halo kernels)."""
    from ssseg import native as N
    from ssseg import nn as snn
    torch.manual_seed(6)
    c1 = snn.Conv2d(16, 64, 3, 1, 1, bias=False).to(hip_device)
    bn = snn.BatchNorm2d(64).to(hip_device)
    c2 = snn.Conv2d(64, cout2, k2, s2, k2 // 2, bias=False).to(hip_device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    x = _q(torch.randn(2, 16, H, W), mode)
    calls = []
    real = N.call

    def spy(name, *a):
        calls.append(name)
        return real(name, *a)

    monkeypatch.setattr(N, 'call', spy)

    def run(on):
        snn.set_bn_grad_stats(on)
        for m in (c1, bn, c2):
            m.zero_grad(set_to_none=True)
        calls.clear()
        xa = _act_in(x, hip_device).detach().requires_grad_(True)
        h = snn.conv_bn_act(c1, xa, bn, relu=True, single_use=True)
        y = c2(h)
        g = snn.to_act(_q(torch.randn(y.shape[0], cout2, y.shape[2], y.shape[3],
                                      generator=torch.Generator().manual_seed(7)), mode).to(hip_device))
        y.backward(g)
        torch.cuda.synchronize()
        assert ('ssseg_bn_gstat_finalize_x' in calls) == on and ('ssseg_bn_bwd_reduce_grad' in calls) != on
        return (xa.grad[:, :16].float().cpu(), c1.weight.grad.cpu().clone(), bn.weight.grad.cpu().clone(),
                bn.bias.grad.cpu().clone(), c2.weight.grad.cpu().clone())

    variants = [0] if mode == 'f32' else ALL_VARIANTS
    try:
        ref = run(False)
        for v in variants:
            N.call('ssseg_set_knob', 4, v)
            got = run(True)
            for a, b, what in zip(got, ref, ('dx', 'dW1', 'dgamma', 'dbeta', 'dW2')):
                _close(a, b, mode, f'variant {v} {what}')
    finally:
        N.call('ssseg_set_knob', 4, 0)
        snn.set_bn_grad_stats(True)


@pytest.mark.parametrize('k2', [1, 3])
def test_bn_backward_sums_from_consumer_dgrad_ill_conditioned(hip_device, mode, k2):
    """The consumer-dgrad BN backward recovers x_hat = (y - beta) / gamma from the stored output y; where gamma is 0 or
    |beta| >> |gamma| (pretrained encoders have such channels) y's rounding swamps gamma * x_hat and dgamma would be
    a bias term or 0 (gamma == 0: such a channel could never move off zero).  Those channels take sum dy * x_hat from
    the masked gradient and x inside the finalize launch (ssseg_bn_gstat_finalize_x): dgamma / dbeta / dx equal the
    unfused reduction's within rounding on every channel -- gamma 0, 1e-3, 0.02 with beta +-2, and ordinary ones."""
    from ssseg import nn as snn
    torch.manual_seed(16)
    c1 = snn.Conv2d(16, 64, 3, 1, 1, bias=False).to(hip_device)
    bn = snn.BatchNorm2d(64).to(hip_device)
    c2 = snn.Conv2d(64, 32, k2, 1, k2 // 2, bias=False).to(hip_device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
        ill = torch.arange(0, 64, 3)
        bn.weight[ill] = torch.tensor([0.0, 1e-3, 0.02, -0.05] * 6, device=hip_device)[:len(ill)]
        bn.bias[ill] = torch.tensor([2.0, 1.5, -0.5, 1.0, 0.8, 2.5], device=hip_device).repeat(4)[:len(ill)]
    x = _q(torch.randn(2, 16, 20, 24), mode)

    def run(on):
        snn.set_bn_grad_stats(on)
        for m in (c1, bn, c2):
            m.zero_grad(set_to_none=True)
        xa = _act_in(x, hip_device).detach().requires_grad_(True)
        h = snn.conv_bn_act(c1, xa, bn, relu=True, single_use=True)
        y = c2(h)
        g = snn.to_act(_q(torch.randn(y.shape[0], 32, y.shape[2], y.shape[3],
                                      generator=torch.Generator().manual_seed(17)), mode).to(hip_device))
        y.backward(g)
        torch.cuda.synchronize()
        return (xa.grad[:, :16].float().cpu(), c1.weight.grad.cpu().clone(), bn.weight.grad.cpu().clone(),
                bn.bias.grad.cpu().clone())

    try:
        ref = run(False)
        got = run(True)
        assert float(ref[2][ill].abs().max()) > 0          # the true dgamma of the ill channels is not 0
        for a, b, what in zip(got, ref, ('dx', 'dW1', 'dgamma', 'dbeta')):
            _close(a, b, mode, what)
        # per channel on the ill ones: dgamma relative to that channel's own magnitude, not the tensor's max
        tol = {'f32': 1e-4, 'bf16': 2e-2, 'f16': 1e-2}[mode]
        for c in ill.tolist():
            r = float(ref[2][c])
            assert abs(float(got[2][c]) - r) <= tol * (abs(r) + 1e-3 * float(ref[2].abs().max())), (c, got[2][c], r)
    finally:
        snn.set_bn_grad_stats(True)


@pytest.mark.parametrize('deferred', [False, True])
@pytest.mark.parametrize('k2,s2,H,W', [(3, 1, 19, 21), (1, 1, 17, 18), (3, 2, 20, 22), (3, 1, 16, 64)])
def test_eval_bn_backward_in_consumer_dgrad(hip_device, mode, monkeypatch, deferred, k2, s2, H, W):
    """The differentiated eval pass (the consistency forward, reference train.py:90-92): conv -> eval BN -> ReLU whose
    output feeds exactly one conv (Bottleneck bn1 / bn2).  The consumer's input-gradient launch applies the ReLU
    backward AND the folded BN scale and writes the BN backward sums (gradient-statistics rows), so the producer's
    backward runs no BN pass at all (no ssseg_bn_eval_bwd_* for it): its parameter gradients come from
    ssseg_bn_gstat_finalize, or from the one deferred launch (ssseg_bn_param_grad_batch with the descriptor's x_hat
    transform).  Same gradients as the separate pass within rounding, for every engine variant."""
    from ssseg import native as N
    from ssseg import nn as snn
    torch.manual_seed(8)
    c1 = snn.Conv2d(16, 64, 3, 1, 1, bias=True).to(hip_device)
    bn1 = snn.BatchNorm2d(64).to(hip_device)
    c2 = snn.Conv2d(64, 64, k2, s2, k2 // 2, bias=False).to(hip_device)
    bn2 = snn.BatchNorm2d(64).to(hip_device)
    with torch.no_grad():
        for bn in (bn1, bn2):
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.3, 0.3)
            bn.running_mean.uniform_(-0.2, 0.2)
            bn.running_var.uniform_(0.5, 2.0)
    bn1.eval()
    bn2.eval()
    x = _q(torch.randn(2, 16, H, W), mode)
    calls = []
    real = N.call

    def spy(name, *a):
        calls.append(name)
        return real(name, *a)

    monkeypatch.setattr(N, 'call', spy)

    def run(on):
        snn.set_bn_grad_stats(on)
        for m in (c1, bn1, c2, bn2):
            m.zero_grad(set_to_none=True)
        calls.clear()
        xa = _act_in(x, hip_device).detach().requires_grad_(True)
        h = snn.conv_bn_act(c1, xa, bn1, relu=True, single_use=True)
        y = snn.conv_bn_act(c2, h, bn2, relu=True)
        g = snn.to_act(_q(torch.randn(y.shape[0], 64, y.shape[2], y.shape[3],
                                      generator=torch.Generator().manual_seed(9)), mode).to(hip_device))
        if deferred:
            with snn.defer_param_grads():
                y.backward(g)
        else:
            y.backward(g)
        torch.cuda.synchronize()
        n_bwd = sum(1 for c in calls if c.startswith('ssseg_bn_eval_bwd'))
        assert n_bwd == (1 if on else 2), (on, calls)
        if on and not deferred:
            assert 'ssseg_bn_gstat_finalize' in calls
        return (xa.grad[:, :16].float().cpu(), c1.weight.grad.cpu().clone(), c1.bias.grad.cpu().clone(),
                bn1.weight.grad.cpu().clone(), bn1.bias.grad.cpu().clone(), c2.weight.grad.cpu().clone(),
                bn2.weight.grad.cpu().clone())

    variants = [0] if mode == 'f32' else ALL_VARIANTS
    try:
        ref = run(False)
        for v in variants:
            N.call('ssseg_set_knob', 4, v)
            got = run(True)
            for a, b, what in zip(got, ref, ('dx', 'dW1', 'db1', 'dgamma1', 'dbeta1', 'dW2', 'dgamma2')):
                _close(a, b, mode, f'variant {v} {what}')
    finally:
        N.call('ssseg_set_knob', 4, 0)
        snn.set_bn_grad_stats(True)


@pytest.mark.parametrize('train', [True, False])
@pytest.mark.parametrize('head', [False, True])
def test_bn_backward_in_upsampler_or_head_dgrad(hip_device, mode, monkeypatch, train, head):
    """UNet decoder: UpBlock.conv3_1's BN+ReLU output feeds only the next block's ConvTranspose2d(4, 2, 1) upsampler
    (or the 1x1 head): that conv's input gradient carries the BN backward (gradient statistics; eval: also the folded
    scale) -- same gradients as the separate BN pass within rounding (reference unet.py:16-50, 63-102)."""
    from ssseg import native as N
    from ssseg import nn as snn
    torch.manual_seed(10)
    c1 = snn.Conv2d(16, 64, 3, 1, 1, bias=False).to(hip_device)
    bn = snn.BatchNorm2d(64).to(hip_device)
    c2 = (snn.Conv2d(64, 2, 1, bias=False, head=True) if head
          else snn.ConvTranspose2d(64, 32, 4, 2, 1)).to(hip_device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
    bn.train(train)
    x = _q(torch.randn(2, 16, 18, 20), mode)
    calls = []
    real = N.call

    def spy(name, *a):
        calls.append(name)
        return real(name, *a)

    monkeypatch.setattr(N, 'call', spy)

    def run(on):
        snn.set_bn_grad_stats(on)
        for m in (c1, bn, c2):
            m.zero_grad(set_to_none=True)
        calls.clear()
        xa = _act_in(x, hip_device).detach().requires_grad_(True)
        h = snn.conv_bn_act(c1, xa, bn, relu=True, single_use=True)
        y = c2(h) if head else c2.forward_relu(h)
        gen = torch.Generator().manual_seed(11)
        if head:
            g = _q(torch.randn(tuple(y.shape), generator=gen), mode).to(hip_device)
        else:
            g = snn.to_act(_q(torch.randn(y.shape[0], 32, y.shape[2], y.shape[3], generator=gen), mode).to(hip_device))
        y.backward(g)
        torch.cuda.synchronize()
        # (training BN: the _x form with the ill-conditioned-channel fallback; eval BN: the plain form)
        assert any(c.startswith('ssseg_bn_gstat_finalize') for c in calls) == on, (on, calls)
        return (xa.grad[:, :16].float().cpu(), c1.weight.grad.cpu().clone(), bn.weight.grad.cpu().clone(),
                bn.bias.grad.cpu().clone(), c2.weight.grad.cpu().clone())

    try:
        ref = run(False)
        got = run(True)
        for a, b, what in zip(got, ref, ('dx', 'dW1', 'dgamma', 'dbeta', 'dW2')):
            _close(a, b, mode, what)
    finally:
        snn.set_bn_grad_stats(True)


@pytest.mark.parametrize('nparts', [300, 511, 512, 700, 8200])
def test_pgrad_batch_long_tables(hip_device, nparts):
    """ssseg_bn_param_grad_batch over partial tables of every length the deferred eval-BN gradients produce (the
    consumer-dgrad gradient-statistics rows reach thousands: tables of >= 512 rows are folded in place first): the
    same sums as a float64 reference, with and without the descriptor's x_hat transform (scale, shift, mean_eff,
    invstd)."""
    import struct
    from ssseg import native as N
    g = torch.Generator().manual_seed(nparts)
    C = 72
    descs, outs, refs = [], [], []
    for gst in (False, True):
        part = torch.randn(2 * nparts, C, generator=g, dtype=torch.float64)
        scale = torch.rand(C, generator=g) + 0.5
        shift, mean, inv = torch.randn(C, generator=g), torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
        a = part[0::2].sum(0)
        b = part[1::2].sum(0)
        if gst:
            B = mean.double() * scale.double() + shift.double()
            b = (b - B * a) * (inv.double() / scale.double())
        dg, db, dbias = (torch.zeros(C, device=hip_device) for _ in range(3))
        dev = [t.to(hip_device) for t in (part, scale, shift, mean, inv)]
        outs.append((dg, db, dbias, dev))
        refs.append((b, a, scale.double() * a))
        gs = (dev[2].data_ptr(), dev[3].data_ptr(), dev[4].data_ptr()) if gst else (0, 0, 0)
        descs.append((dev[0].data_ptr(), nparts, C, dev[1].data_ptr(), dg.data_ptr(), db.data_ptr(), dbias.data_ptr())
                     + gs)
    blob = b''.join(struct.pack('<10q', *d) for d in descs)
    table = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(hip_device)
    N.call('ssseg_bn_param_grad_batch', N.dev_ptr(table), len(descs), C, N.stream())
    torch.cuda.synchronize()
    for (dg, db, dbias, _), (rg, rb, rbias) in zip(outs, refs):
        for got, ref in ((dg, rg), (db, rb), (dbias, rbias)):
            assert torch.allclose(got.cpu().double(), ref, rtol=1e-5, atol=1e-4 * (1 + float(ref.abs().max())))
