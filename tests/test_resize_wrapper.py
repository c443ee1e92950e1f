"""ModelWrapper.ResizeWrapper (reference ModelWrapper.py:5-53): the size plan on the host (CPU) and the device
resize + pad against the torch-CPU restatement oracle/resize_ref.py (parity unpinned: the reference forward cannot
run, see ModelWrapper.py's docstring)."""
import pytest
import torch


@pytest.mark.parametrize('H,W,L', [(480, 640, 1024), (640, 480, 1024), (300, 1000, 1024), (1000, 300, 1024),
                                   (512, 512, 512), (100, 700, 512), (37, 53, 256), (1024, 1023, 1024)])
def test_resize_plan_matches_oracle_shapes(H, W, L):
    from ModelWrapper import resize_plan
    from oracle.resize_ref import resize_pad_ref
    th, tw, pl, pr, pt, pb = resize_plan(H, W, L)
    ref = resize_pad_ref(torch.zeros(1, 1, H, W), L)
    assert (th + pt + pb, tw + pl + pr) == tuple(ref.shape[2:])
    assert max(th, tw) == L
    short = tw + pl + pr if H > W else th + pt + pb
    assert short in (256, 512, 1024, 2048) and min(pl, pr, pt, pb) >= 0
    assert pr - pl in (0, 1) and pb - pt in (0, 1)


def test_resize_plan_no_size_class():
    from ModelWrapper import resize_plan
    with pytest.raises(ValueError):
        resize_plan(4000, 4000, 4096)


@pytest.mark.gpu
@pytest.mark.parametrize('H,W', [(480, 640), (640, 480), (300, 1000), (97, 53)])
def test_resize_wrapper_device_vs_oracle(hip_device, H, W):
    from ModelWrapper import ResizeWrapper
    from oracle.resize_ref import resize_pad_ref
    g = torch.Generator().manual_seed(5)
    x = torch.rand(2, 3, H, W, generator=g)
    seen = {}

    def model(inp):   # the wrapped model receives the resized, padded batch
        seen['x'] = inp
        return inp.sum()
    wrap = ResizeWrapper(model, larger_side_size=512)
    xd = x.to(hip_device).requires_grad_(True)
    out = wrap(xd)
    ref_in = resize_pad_ref(x.clone().requires_grad_(True), 512)
    got = seen['x'].cpu()
    assert got.shape == ref_in.shape
    assert torch.allclose(got, ref_in.detach(), atol=1e-5, rtol=1e-5), float((got - ref_in.detach()).abs().max())
    # gradient of sum(model input) w.r.t. the image: the bilinear backward from the interior view
    out.backward()
    xr = x.clone().requires_grad_(True)
    resize_pad_ref(xr, 512).sum().backward()
    assert torch.allclose(xd.grad.cpu(), xr.grad, atol=1e-4, rtol=1e-5)
