"""Virtual channel concat (ssseg_vcat; reference models/unet.py:44-45 torch.cat((x, skip), 1) feeding
UpBlock.conv3_0): the consuming conv's forward (LDS-DMA A-loader), weight gradient and merged two-pass weight
gradient read the two parts where they lie.  Every engine launch accumulates the same MFMA k-sequence from the
same bytes as on the materialised concat, so outputs, input gradients and weight gradients must be BIT-identical
to the copy path (snn.set_virtual_concat(False))."""
import contextlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _upblock(dev, cin, skip, cout, seed=3):
    from models.unet import UpBlock
    torch.manual_seed(seed)
    return UpBlock(cin, skip, cout, shrink=False, train_upsampling=True).to(dev)


def _run(block, x, skip, mode, vcat, gy=None):
    from ssseg import nn as snn
    snn.set_virtual_concat(vcat)
    try:
        block.zero_grad(set_to_none=True)
        xa = snn.to_act(x).detach().requires_grad_(mode != 'nograd')
        sa = snn.to_act(skip).detach().requires_grad_(mode != 'nograd')
        if mode == 'nograd':
            block.eval()
            with torch.no_grad():
                y = block(xa, sa)
            return [y.clone()]
        block.train(mode == 'train')
        if mode == 'merged':   # two backward passes, the first one's weight gradients deferred (train_step)
            outs = []
            for i in range(2):
                with (snn.defer_wgrad() if i == 0 else contextlib.nullcontext()):
                    y = block(xa, sa)
                    y.backward(gy)
                outs.append(y.detach().clone())
            snn.flush_wgrad()
        else:
            y = block(xa, sa)
            y.backward(gy)
            outs = [y.detach().clone()]
        return outs + [xa.grad.clone(), sa.grad.clone()] + [p.grad.clone() for p in block.parameters()]
    finally:
        snn.set_virtual_concat(True)
        block.train()


# (128, 64, 64, 32): conv3_0 at 64 x 64 runs the halo-tiled 3x3 weight gradient over the two parts
@pytest.mark.parametrize('cin,skip,cout,H', [(256, 256, 128, 16), (128, 64, 64, 33), (512, 1024, 128, 9),
                                            (128, 64, 64, 32)])
@pytest.mark.parametrize('mode', ['train', 'eval', 'nograd', 'merged'])
def test_upblock_virtual_concat_bitwise(hip_device, cin, skip, cout, H, mode):
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    block = _upblock(hip_device, cin, skip, cout)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, cin, H, H, generator=g).to(hip_device)
    s = torch.randn(2, skip, 2 * H, 2 * H, generator=g).to(hip_device)
    gy = snn.to_act(torch.randn(2, cout, 2 * H, 2 * H, generator=g).to(hip_device)) if mode != 'nograd' else None
    ref = _run(block, x, s, mode, False, gy)
    got = _run(block, x, s, mode, True, gy)
    assert len(ref) == len(got)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), f'{mode}: tensor {i} differs (max |d| {float((a.float() - b.float()).abs().max())})'


@pytest.mark.parametrize('cin,skip,cout', [(128, 192, 64), (128, 64, 192)])
@pytest.mark.parametrize('wcfg', [0, 2, 5, 10, 12])
def test_vcat_mixed_straddle_wgrad_configs(hip_device, cin, skip, cout, wcfg):
    """[64 | 192] and [192 | 64]: the seam sits inside one 128-wide kk-tile while the other lies wholly in one part,
    so the ST weight-gradient kernel runs straddling and non-straddling blocks in one launch (their per-stage LDS-DMA
    counts differ).  Forced 3- and 4-deep 128-wide configs (knob 9) must stay bitwise equal to the copy path."""
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    block = _upblock(hip_device, cin, skip, cout)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, cin, 24, 24, generator=g).to(hip_device)
    s = torch.randn(2, skip, 48, 48, generator=g).to(hip_device)
    gy = snn.to_act(torch.randn(2, cout, 48, 48, generator=g).to(hip_device))
    N.call('ssseg_set_knob', 9, wcfg)
    try:
        for mode in ('train', 'merged'):
            ref = _run(block, x, s, mode, False, gy)
            got = _run(block, x, s, mode, True, gy)
            for i, (a, b) in enumerate(zip(got, ref)):
                assert torch.equal(a, b), f'cfg {wcfg} {mode}: tensor {i} differs'
    finally:
        N.call('ssseg_set_knob', 9, 0)


def test_virtual_concat_is_not_copied(hip_device):
    """The lazy concat of an eligible UpBlock carries its parts and its memory is never written by the forward."""
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    a = snn.to_act(torch.randn(2, 128, 8, 8, device=hip_device))
    b = snn.to_act(torch.randn(2, 64, 8, 8, device=hip_device))
    y = snn.cat_crop(a, b, 128, 64, lazy=True)
    assert snn._vcat_of(y) is not None
    snn.materialize(y)
    assert snn._vcat_of(y) is None
    ref = snn.cat_crop(a, b, 128, 64)
    assert torch.equal(y, ref)
    # not eligible (fp32 mode / 64-unaligned part): an ordinary concat
    c = snn.to_act(torch.randn(2, 40, 8, 8, device=hip_device))
    assert snn._vcat_of(snn.cat_crop(a, c, 128, 40, lazy=True)) is None


@pytest.mark.parametrize('mode', ['train', 'eval'])
def test_virtual_concat_backward_writes_parts(hip_device, monkeypatch, mode):
    """conv3_0's input gradient goes straight into the two parts' gradients (ssseg_conv_igemm_epi_vsplit), the up
    part's with the upsampler's ReLU backward applied: no channel copy and no ssseg_act_bwd pass run in the forward
    or the backward of an eligible UpBlock (the gradients themselves are checked bitwise against the copy path by
    test_upblock_virtual_concat_bitwise)."""
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    block = _upblock(hip_device, 128, 64, 64)
    block.train(mode == 'train')
    x = snn.to_act(torch.randn(2, 128, 12, 12, device=hip_device)).requires_grad_(True)
    s = snn.to_act(torch.randn(2, 64, 24, 24, device=hip_device)).requires_grad_(True)
    calls = []
    real = N.call

    def spy(name, *args):
        calls.append(name)
        return real(name, *args)
    monkeypatch.setattr(N, 'call', spy)
    real_u = N.call_or_unsupported

    def spy_u(name, *args):
        calls.append(name)
        return real_u(name, *args)
    monkeypatch.setattr(N, 'call_or_unsupported', spy_u)
    y = block(x, s)
    y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    assert 'ssseg_conv_igemm_epi_vsplit' in calls
    assert 'ssseg_nhwc_copy' not in calls
    # the upsampler's ReLU backward runs inside the split launch (the up part's gradient arrives masked)
    assert 'ssseg_act_bwd' not in calls


def test_virtual_concat_second_consumer_raises(hip_device):
    """The split-output dgrad returns a never-written placeholder as the concat's input gradient: a second consumer of
    the lazy concat would have its gradient summed into that placeholder and lost, so the concat's backward raises."""
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    block = _upblock(hip_device, 128, 64, 64)
    x = snn.to_act(torch.randn(2, 128, 8, 8, device=hip_device)).requires_grad_(True)
    s = snn.to_act(torch.randn(2, 64, 16, 16, device=hip_device)).requires_grad_(True)
    up = block._upsample(x)
    cat = snn.cat_crop(up, s, 64, 64, lazy=True)
    assert snn._vcat_of(cat) is not None
    y = block.conv3_0(cat)
    other = cat.float().sum()   # a second consumer of the lazy concat
    with pytest.raises(RuntimeError, match='more than one consumer'):
        torch.autograd.backward([y, other], [torch.ones_like(y), torch.ones_like(other)])


def test_virtual_concat_part_modified_in_place_raises(hip_device):
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    block = _upblock(hip_device, 128, 64, 64)
    x = snn.to_act(torch.randn(2, 128, 8, 8, device=hip_device)).requires_grad_(True)
    s = snn.to_act(torch.randn(2, 64, 16, 16, device=hip_device))
    up = block._upsample(x)
    cat = snn.cat_crop(up, s, 64, 64, lazy=True)
    y = block.conv3_0(cat)
    s.mul_(2.0)
    with pytest.raises(RuntimeError, match='modified in place'):
        y.backward(torch.ones_like(y))
