"""n-way channel concat (ssseg_nhwc_cat_n / ssseg_nhwc_split_n; reference hardnet.py:67,78 torch.cat(tin, 1)): the
concat packs each operand's real channels densely with the MFMA-vector padding written zero in the same launch, and
its backward writes every operand's gradient in one launch.  Both are pure data movement: bit-identical to
torch.cat / slicing of the real channels.  A layer output read by several concats (and a conv) sums the consumers'
gradients inside the split (snn.GradJoin): bitwise the autograd sum for concat-only consumers."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _act(dev, n, c, h, w, dtype, seed):
    from ssseg import nn as snn
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, c, h, w, generator=g).to(dtype)
    t = snn.new_act(n, snn.rup(c, snn.vec()), h, w, dtype, dev, zero=True)
    t[:, :c].copy_(x.to(dev))
    return t


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize('chans', [(10, 64), (10, 18, 64), (14, 24, 40, 96), (22, 38, 64, 320), (16, 16, 16, 16, 78),
                                   (2, 6, 4, 8)])
def test_cat_n_forward_backward_bitwise(hip_device, dtype, chans):
    from ssseg import nn as snn
    snn.set_compute_dtype(dtype)
    try:
        n, h, w = 2, 5, 7
        ts = [_act(hip_device, n, c, h, w, dtype, 10 + i).requires_grad_(True) for i, c in enumerate(chans)]
        y = snn.cat_n(ts, list(chans))
        total = sum(chans)
        ref = torch.cat([t[:, :c] for t, c in zip(ts, chans)], 1)
        assert y.shape[1] == snn.rup(total, snn.vec())
        assert torch.equal(y[:, :total], ref)
        assert not y[:, total:].any()
        gy = _act(hip_device, n, total, h, w, dtype, 99)
        y.backward(gy)
        c0 = 0
        for t, c in zip(ts, chans):
            assert t.grad.shape == t.shape
            assert torch.equal(t.grad[:, :c], gy[:, c0:c0 + c]), c
            assert not t.grad[:, c:].any()
            c0 += c
    finally:
        snn.set_compute_dtype(torch.bfloat16)


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_cat_n_join_sums_like_autograd(hip_device, dtype):
    """x feeds three concats (HarDNet layer 0 -> links of layers 2, 4 and 8): the joined gradient (summed inside the
    split launches, in backward order) equals autograd's separate adds bit for bit."""
    from ssseg import nn as snn
    snn.set_compute_dtype(dtype)
    grads = []
    try:
        for join in (True, False):
            snn.set_grad_join(join)
            base = _act(hip_device, 2, 64, 6, 6, dtype, 1)
            x = base.clone().requires_grad_(True)
            xs = snn.mark_join(x * 1)          # a non-leaf activation, like a layer output
            others = [_act(hip_device, 2, c, 6, 6, dtype, 20 + c).requires_grad_(True) for c in (10, 18, 30)]
            ys = [snn.cat_n([o, xs], [c, 64]) for o, c in zip(others, (10, 18, 30))]
            loss_parts = []
            for k, yk in enumerate(ys):
                gk = _act(hip_device, 2, yk.shape[1], 6, 6, dtype, 50 + k)
                loss_parts.append((yk, gk))
            torch.autograd.backward([p for p, _ in loss_parts], [g for _, g in loss_parts])
            grads.append(x.grad.clone())
    finally:
        snn.set_grad_join(True)
        snn.set_compute_dtype(torch.bfloat16)
    assert torch.equal(grads[0], grads[1])
