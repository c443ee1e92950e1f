"""GradJoin: the input gradients of an activation read by several native ops (a UNet skip, the input of a
ResNet block with a projection shortcut) are summed inside the consumers' own kernels (dgrad epilogue residual,
strided-dgrad phases, max-pool backward) instead of autograd's separate add.  Checked against the autograd sum
(set_grad_join(False)) on the same inputs: fp32 mode to fp32 rounding, bf16 mode to the layer tolerance."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(model, x, gy, join):
    from ssseg import nn as snn
    snn.set_grad_join(join)
    try:
        model.zero_grad(set_to_none=True)
        xa = x.clone().requires_grad_(True)
        y = model(xa)
        y.backward(gy)
        torch.cuda.synchronize()
        return ({n: p.grad.detach().float().cpu().clone() for n, p in model.named_parameters() if p.grad is not None},
                xa.grad.detach().float().cpu().clone(), y.detach().float().cpu())
    finally:
        snn.set_grad_join(True)


@pytest.mark.parametrize('dtype', ['f32', 'bf16'])
def test_unet_r50_grad_join_matches_autograd_sum(hip_device, dtype):
    from models import unet
    from models.encoders import resnet
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.float32 if dtype == 'f32' else torch.bfloat16)
    try:
        torch.manual_seed(0)
        model = unet.UNet(2, resnet.resnet50_encoder(), 64, train_upsampling=True).to(hip_device)
        x = torch.rand(2, 3, 64, 64, device=hip_device)
        gy = torch.randn(2, 2, 32, 32, device=hip_device)
        g0, dx0, y0 = _run(model, x, gy, False)
        g1, dx1, y1 = _run(model, x, gy, True)
    finally:
        snn.set_compute_dtype(torch.bfloat16)
    assert torch.equal(y0, y1)
    assert set(g0) == set(g1)
    rel = 1e-5 if dtype == 'f32' else 2e-2
    worst = []
    for n in g0:
        a, b = g0[n], g1[n]
        scale = float(a.abs().max()) + 1e-12
        err = float((a - b).abs().max()) / scale
        worst.append((err, n))
    worst.sort(reverse=True)
    print('worst parameter-gradient differences:', worst[:4])
    assert worst[0][0] <= rel, worst[:4]
    assert float((dx0 - dx1).abs().max()) <= rel * (float(dx0.abs().max()) + 1e-12)


def test_grad_join_any_consumer_order(hip_device):
    """Three consumers of one joined activation (a concat, a strided 1x1 conv, a max-pool), backward in whatever
    order autograd picks: the total input gradient equals the autograd sum."""
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.float32)
    try:
        torch.manual_seed(1)
        conv = snn.Conv2d(16, 32, 1, 2, 0, bias=False).to(hip_device)
        pool = snn.MaxPool2d(3, 2, 1)
        other = snn.to_act(torch.randn(2, 8, 12, 12, device=hip_device))
        x0 = snn.to_act(torch.randn(2, 16, 12, 12, device=hip_device))
        ga = snn.to_act(torch.randn(2, 32, 6, 6, device=hip_device))
        gb = snn.to_act(torch.randn(2, 16, 6, 6, device=hip_device))
        gc = snn.to_act(torch.randn(2, 24, 12, 12, device=hip_device))

        def run(join):
            snn.set_grad_join(join)
            x = x0.clone().requires_grad_(True)
            h = x * 1.0
            snn.mark_join(h)
            a = conv(h)
            b = pool(h)
            c = snn.cat_crop(other, h, 8, 16)
            torch.autograd.backward([a, b, c], [ga, gb, gc])
            torch.cuda.synchronize()
            return x.grad.detach().cpu().clone()
        g_sum, g_join = run(False), run(True)
    finally:
        snn.set_grad_join(True)
        snn.set_compute_dtype(torch.bfloat16)
    assert float((g_sum - g_join).abs().max()) <= 1e-5 * (float(g_sum.abs().max()) + 1e-12)


@pytest.mark.parametrize('dtype', ['f32', 'bf16'])
def test_batched_teacher_forward_bitwise(hip_device, dtype):
    """train_step runs the teacher's two eval passes (reference train.py:69-75) as ONE forward over both
    batches (snn.to_act_cat): the logits equal the two separate passes bit for bit."""
    from models import unet
    from models.encoders import resnet
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.float32 if dtype == 'f32' else torch.bfloat16)
    try:
        torch.manual_seed(2)
        model = unet.UNet(2, resnet.resnet50_encoder(), 64, train_upsampling=True).to(hip_device).eval()
        a = torch.rand(2, 3, 96, 96, device=hip_device)
        b = torch.rand(2, 3, 96, 96, device=hip_device)
        with torch.no_grad(), snn.folded(model):
            ya, yb = model(a).float().cpu(), model(b).float().cpu()
            yab = model(snn.to_act_cat([a, b])).float().cpu()
    finally:
        snn.set_compute_dtype(torch.bfloat16)
    assert torch.equal(yab[:2], ya) and torch.equal(yab[2:], yb)
