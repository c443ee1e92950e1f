"""Device train-time augmentations (data/device_augment.py, csrc/augment.hip): a batched restatement of the reference
config's albumentations pipelines (configs/default_config.py:179-212).  albumentations / cv2 are absent, so parity with
the reference pipeline is UNPINNED; the kernels are checked against the NumPy restatement of their own arithmetic
(oracle/augment_ref.py) and the host draws against the pipeline's parameter ranges and probabilities."""
import ctypes
import math

import numpy as np
import pytest
import torch

from oracle import augment_ref as R


def _aug():
    from data import device_augment as DA
    return DA


def test_param_structs_match_the_c_abi():
    DA = _aug()
    assert ctypes.sizeof(DA.WarpParams) == 80
    assert ctypes.sizeof(DA.ColorParams) == 60


def test_draws_follow_the_pipeline():
    """Host draws over many samples: ranges of every parameter and the OneOf / p frequencies of the config."""
    DA = _aug()
    aug = DA.DeviceAugment(64, seed=1)
    n = 4000
    _, color, gmaps, radius, _, nf = aug.draw(n, 80, 96, train=True)
    recs = aug.last_params
    angles = np.array([r['angle'] for r in recs])
    assert angles.min() >= -15 and angles.max() <= 15 and abs(angles.mean()) < 1.0
    crops = np.array([r['crop'] for r in recs])
    assert (crops[:, 0] <= 80).all() and (crops[:, 1] <= 96).all() and (crops[:, 2] + crops[:, 0] <= 80).all()
    area = crops[:, 0] * crops[:, 1] / (80 * 96)
    assert area.min() > 0.2 and area.max() <= 1.0
    freq = lambda key: sum(key in r for r in recs) / n   # noqa: E731
    assert abs(sum(r['hflip'] for r in recs) / n - 0.5) < 0.03
    assert freq('bc') == 1.0
    assert abs(freq('gray') - 0.1) < 0.02
    assert abs(freq('rgb_shift') + freq('hsv_shift') - 0.3) < 0.03
    assert abs(freq('blur_ksize') - 0.1) < 0.02
    assert abs(freq('iso') - 0.2) < 0.025
    dist = freq('elastic') + freq('grid') + freq('optical')
    assert abs(dist - 0.5) < 0.03 and abs(freq('optical') - 0.25) < 0.03
    assert nf == sum('elastic' in r for r in recs)
    al = np.array([r['bc'][0] for r in recs])
    assert al.min() >= 0.8 and al.max() <= 1.2
    assert set(r['blur_ksize'] for r in recs if 'blur_ksize' in r) == {3, 5, 7, 9}
    assert (radius[[('blur_ksize' in r) for r in recs]] > 0).all()


def test_affine_chain_identity():
    """No rotation, full crop, no flip: the composed map is the cv2.resize pixel-centre map."""
    DA = _aug()
    A = DA._compose([2.0, 0.0, 0.5, 0.0, 2.0, 0.5], [1.0, 0.0, 0.0, 0.0, 1.0, 0.0])
    assert A == [2.0, 0.0, 0.5, 0.0, 2.0, 0.5]
    M = DA.rotation_matrix(30.0, 10.0, 20.0)
    I = DA._compose(DA._affine_inv(M), M)
    np.testing.assert_allclose(I, [1, 0, 0, 0, 1, 0], atol=1e-12)


def _rand_warp(DA, rng, S, H, W, kind):
    p = DA.WarpParams()
    ang = rng.uniform(-15, 15)
    Rm = DA.rotation_matrix(ang, W / 2 - 0.5, H / 2 - 0.5)
    h, w, y0, x0 = 50, 60, 7, 11
    C = [w / S, 0.0, 0.5 * w / S - 0.5 + x0, 0.0, h / S, 0.5 * h / S - 0.5 + y0]
    A = DA._compose(DA._affine_inv(Rm), DA._compose(C, [-1.0, 0.0, S - 1.0, 0.0, 1.0, 0.0]))
    p.a[:] = A
    p.border = 1
    gmap = np.zeros(2 * S, np.float32)
    field = None
    if kind == 'elastic':
        p.distort = 1
        p.field = 0
        M = DA._affine_from_points(np.float32([[40, 40], [40, 24], [24, 24]]),
                                   np.float32([[41, 39.5], [40.2, 25], [23, 24.4]]))
        p.m[:] = DA._affine_inv(M)
        field = rng.uniform(-3, 3, size=(S, S, 2)).astype(np.float32)
    elif kind == 'grid':
        p.distort = 2
        gmap[:S] = DA.grid_axis(S, [1 + rng.uniform(-0.3, 0.3) for _ in range(6)], 5)
        gmap[S:] = DA.grid_axis(S, [1 + rng.uniform(-0.3, 0.3) for _ in range(6)], 5)
    elif kind == 'optical':
        p.distort, p.k, p.fx, p.fy, p.cx, p.cy = 3, rng.uniform(-1, 1), float(S), float(S), S * 0.5, S * 0.5 + 1
    return p, gmap, field


@pytest.mark.gpu
@pytest.mark.parametrize('kind', ['none', 'elastic', 'grid', 'optical'])
def test_warp_matches_oracle(hip_device, kind):
    from ssseg import native as N
    DA = _aug()
    rng = np.random.default_rng(3)
    n, H, W, S, Cm = 3, 70, 83, 48, 2
    img = rng.integers(0, 256, size=(n, H, W, 3), dtype=np.uint8)
    mask = (rng.random((n, H, W, Cm)) > 0.5).astype(np.uint8) * 255
    ps, gms, fls = zip(*[_rand_warp(DA, rng, S, H, W, kind) for _ in range(n)])
    arr = (DA.WarpParams * n)(*ps)
    for i in range(n):
        arr[i].field = i
    fields = np.stack([f if f is not None else np.zeros((S, S, 2), np.float32) for f in fls])
    d_p = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(hip_device)
    d_img, d_mask = torch.from_numpy(img).to(hip_device), torch.from_numpy(mask).to(hip_device)
    d_g, d_f = torch.from_numpy(np.stack(gms)).to(hip_device), torch.from_numpy(fields).to(hip_device)
    out = torch.empty((n, S, S, 3), device=hip_device)
    om = torch.empty((n, Cm, S, S), device=hip_device)
    N.call('ssseg_aug_warp', N.dev_ptr(d_img), N.dev_ptr(d_mask), Cm, n, H, W, N.dev_ptr(out), N.dev_ptr(om), S, S,
           N.dev_ptr(d_p), N.dev_ptr(d_g), N.dev_ptr(d_f), 0, N.stream())
    out01 = torch.empty((n, 3, S, S), device=hip_device)
    N.call('ssseg_aug_warp', N.dev_ptr(d_img), None, 0, n, H, W, N.dev_ptr(out01), None, S, S, N.dev_ptr(d_p),
           N.dev_ptr(d_g), N.dev_ptr(d_f), 1, N.stream())
    torch.cuda.synchronize()
    got, gm, g01 = out.cpu().numpy(), om.cpu().numpy(), out01.cpu().numpy()
    for i in range(n):
        pd = dict(a=list(arr[i].a), distort=arr[i].distort, m=list(arr[i].m), k=arr[i].k, cx=arr[i].cx, cy=arr[i].cy,
                  fx=arr[i].fx, fy=arr[i].fy, border=1)
        ref, rm = R.warp(img[i], mask[i], pd, S, gms[i], fields[i])
        d = np.abs(got[i] - ref)
        assert d.max() <= 1.0, d.max()            # float32 vs float64 coordinates: rounding ties only
        assert (d == 0).mean() > 0.99
        assert (gm[i] == rm).mean() > 0.995        # nearest: ties at half-pixel coordinates only
        np.testing.assert_allclose(g01[i], got[i].transpose(2, 0, 1) / 255.0, rtol=0, atol=1e-7)   # ToFloat


@pytest.mark.gpu
def test_color_matches_oracle(hip_device):
    from ssseg import native as N
    DA = _aug()
    rng = np.random.default_rng(5)
    n, H, W = 6, 17, 23
    img = rng.integers(0, 256, size=(n, H, W, 3)).astype(np.float32)
    cps = (DA.ColorParams * n)()
    specs = [dict(bc=1, alpha=1.13, beta=-0.07), dict(bc=1, alpha=0.85, beta=0.12, gray=1),
             dict(bc=1, alpha=1.0, beta=0.0, rgb=1, shift=[7.3, -9.1, 2.2]),
             dict(bc=1, alpha=0.93, beta=0.05, hsv=1, hsv_shift=[8.6, -7.2, 0.6]),
             dict(hsv=1, hsv_shift=[-9.5, 9.9, -0.8]), dict(gray=1)]
    for i, sp in enumerate(specs):
        for k, v in sp.items():
            if isinstance(v, list):
                getattr(cps[i], k)[:] = v
            else:
                setattr(cps[i], k, v)
    d_p = torch.frombuffer(bytearray(bytes(cps)), dtype=torch.uint8).to(hip_device)
    x = torch.from_numpy(img).to(hip_device)
    N.call('ssseg_aug_color', N.dev_ptr(x), n, H, W, N.dev_ptr(d_p), N.stream())
    got = x.cpu().numpy()
    for i, sp in enumerate(specs):
        ref = R.color(img[i], sp)
        d = np.abs(got[i] - ref)
        if set(sp) == {'gray'}:   # integer arithmetic (cv2's Q14 RGB2GRAY): bit-exact
            assert d.max() == 0, (i, d.max())
        assert d.max() <= 1.0, (i, d.max())
        assert (d == 0).mean() > 0.98, (i, (d == 0).mean())


def test_to_gray_known_answers():
    """The oracle's ToGray is OpenCV's 8-bit RGB2GRAY (albumentations to_gray): known answers of that conversion --
    pure red / green / blue -> 76 / 150 / 29, white -> 255 -- and its Q14 rounding (0.299 / 0.587 / 0.114 * 2^14 =
    4899 / 9617 / 1868, + 2^13, >> 14) where the float formula rounds the other way."""
    img = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [1, 0, 1]]], np.float64)
    y = R.color(img, dict(gray=1))[..., 0]
    assert y.tolist() == [[76, 150, 29, 255, 0, 0]]
    r, g, b = np.meshgrid(np.arange(0, 256, 3), np.arange(0, 256, 5), np.arange(0, 256, 7), indexing='ij')
    rgb = np.stack([r, g, b], -1).reshape(1, -1, 3).astype(np.float64)
    y = R.color(rgb, dict(gray=1))[0, :, 0]
    q14 = (r.ravel() * 4899 + g.ravel() * 9617 + b.ravel() * 1868 + 8192) >> 14
    assert (y == q14).all()
    flt = np.rint(0.299 * r + 0.587 * g + 0.114 * b).ravel()
    assert (flt != q14).any()   # the float formula is NOT the cv2 result everywhere


@pytest.mark.gpu
@pytest.mark.parametrize('sym,round8', [(0, 1), (1, 0)])
def test_blur_matches_oracle(hip_device, sym, round8):
    from ssseg import native as N
    DA = _aug()
    rng = np.random.default_rng(7)
    n, H, W, C = 4, 21, 30, 3 if round8 else 2
    x = (rng.integers(0, 256, size=(n, H, W, C)) if round8 else rng.uniform(-1, 1, size=(n, H, W, C))).astype(np.float32)
    radius = np.array([1, 0, 4, 2] if round8 else [24, 3, 0, 9], np.int32)
    weights = np.zeros((n, DA.WMAX), np.float32)
    for i, r in enumerate(radius):
        if r:
            t = DA.cv2_gaussian_taps(2 * r + 1) if round8 else DA.scipy_gaussian_taps(r / 4.0)
            t = t[:2 * r + 1]
            weights[i, :len(t)] = t
    xt = torch.from_numpy(x).to(hip_device)
    tmp = torch.empty_like(xt)
    d_r, d_w = torch.from_numpy(radius).to(hip_device), torch.from_numpy(weights).to(hip_device)   # alive past launch
    N.call('ssseg_aug_blur', N.dev_ptr(xt), N.dev_ptr(tmp), n, H, W, C, N.dev_ptr(d_r), N.dev_ptr(d_w), DA.WMAX, sym,
           round8, N.stream())
    got = xt.cpu().numpy()
    for i in range(n):
        ref = R.blur(x[i].astype(np.float64), int(radius[i]), weights[i].astype(np.float64), bool(sym), bool(round8))
        if round8:
            assert np.abs(got[i] - ref).max() <= 1.0 and (got[i] == ref).mean() > 0.98
        else:
            np.testing.assert_allclose(got[i], ref, atol=1e-5)


@pytest.mark.gpu
def test_iso_finish(hip_device):
    """ISONoise's HLS round trip + ToFloat (noise off: colour std 0, intensity 0) against the oracle, and the noise
    statistics: hue shift std and the luminance Poisson mean follow the sample's parameters."""
    from ssseg import native as N
    DA = _aug()
    rng = np.random.default_rng(9)
    n, H, W = 3, 64, 64
    img = rng.integers(0, 256, size=(n, H, W, 3)).astype(np.float32)
    cps = (DA.ColorParams * n)()
    cps[0].iso = 1                                            # the conversion chain alone
    cps[1].iso, cps[1].iso_color_std, cps[1].iso_intensity = 1, 0.0, 0.4   # luminance noise only
    d_p = torch.frombuffer(bytearray(bytes(cps)), dtype=torch.uint8).to(hip_device)
    x = torch.from_numpy(img).to(hip_device)
    out = torch.empty((n, 3, H, W), device=hip_device)
    st = torch.empty((n, 2), device=hip_device, dtype=torch.float64)
    N.call('ssseg_aug_iso_finish', N.dev_ptr(x), N.dev_ptr(out), n, H, W, N.dev_ptr(d_p), N.dev_ptr(st), 1234,
           N.stream())
    got = out.cpu().numpy()
    ref0 = R.iso_finish(img[0], dict(iso=1))
    # float32 (device) vs float64 (oracle) HLS round trips truncated to uint8 (astype): one level apart where the
    # round trip lands just below an integer
    d0 = np.abs(got[0] - ref0)
    assert d0.max() <= 1.0 / 255 + 1e-6 and (d0 < 1e-6).mean() > 0.5
    np.testing.assert_allclose(got[2], img[2].transpose(2, 0, 1) / 255.0, rtol=0, atol=1e-7)   # iso off: ToFloat
    # luminance-only noise: L' = L + k/255 (1 - L) with k ~ Poisson(std(L) * 0.4 * 255) -> L never decreases
    h0, l0, _ = R.rgb2hls(*(img[1][..., c] / 255.0 for c in range(3)))
    _, l1, _ = R.rgb2hls(*(got[1][c] for c in range(3)))
    lam = l0.std() * 0.4 * 255
    k = (l1 - l0) * 255 / np.maximum(1 - l0, 1e-3)
    sel = (1 - l0) > 0.2
    assert (l1 - l0 > -2.0 / 255).all()
    assert abs(k[sel].mean() - lam) < 0.15 * lam, (k[sel].mean(), lam)


@pytest.mark.gpu
def test_pipelines_end_to_end(hip_device):
    """DeviceAugment.train / .unsupervised on a batch: shapes, ranges, soft-mask values preserved (nearest), the
    mask's one-hot structure kept, reproducible with the same seed."""
    DA = _aug()
    rng = np.random.default_rng(11)
    n, H, W, S = 8, 96, 96, 64
    img = torch.from_numpy(rng.integers(0, 256, size=(n, H, W, 3), dtype=np.uint8)).to(hip_device)
    fg = (rng.random((n, H, W)) > 0.5).astype(np.uint8) * 255
    mask = torch.from_numpy(np.stack([255 - fg, fg], -1)).to(hip_device)
    outs = []
    for _ in range(2):
        aug = DA.DeviceAugment(S, seed=42, distort_p=1.0, blur_p=0.5, iso_p=0.5)
        x, m = aug.train(img, mask)
        u = aug.unsupervised(img)
        torch.cuda.synchronize()
        outs.append((x.cpu(), m.cpu(), u.cpu()))
    x, m, u = outs[0]
    assert x.shape == (n, 3, S, S) and m.shape == (n, 2, S, S) and u.shape == (n, 3, S, S)
    assert float(x.min()) >= 0 and float(x.max()) <= 1 and float(u.min()) >= 0 and float(u.max()) <= 1
    assert set(np.unique(m.numpy()).tolist()) <= {0.0, 1.0}
    np.testing.assert_array_equal(m[:, 0] + m[:, 1], np.ones((n, S, S)))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    assert math.isfinite(float(x.sum()))


@pytest.mark.gpu
def test_train_loop_applies_device_augment(hip_device):
    """train.train with train['device_augment'] (distributed_trainer builds it from train['device_augmentations']): the
    loaders deliver the host-only transforms' uint8 output (SyntheticSegDataset(uint8=True) stands in for
    SkinSegDataset with LongestMaxSize + PadIfNeeded, data/dataset.py:70-72), every labelled batch goes through
    DeviceAugment.train_batch and every unlabelled one through .unsupervised_batch before the step (the reference
    augments per sample on the host, dataset.py:73-74 / unsupervised_dataset.py:20-21): the step sees float NCHW
    crops, the same tensors a direct call with the same seed produces, and trains to finite losses."""
    import losses
    import train
    from data.synthetic import SyntheticSegDataset
    from models import simple_unet
    from models.adapters import ListOutput
    from ssseg import arena, optim
    DA = _aug()
    n, H, S = 2, 96, 64
    lab = SyntheticSegDataset(length=4, size=H, seed=1, uint8=True)
    unl = SyntheticSegDataset(length=8, size=H, seed=3, with_masks=False, uint8=True)
    dl = torch.utils.data.DataLoader(lab, batch_size=n)
    udl = torch.utils.data.DataLoader(unl, batch_size=n)
    torch.manual_seed(0)
    student = ListOutput(simple_unet.UNet(2, 3, 8, 32)).to(hip_device)
    teacher = ListOutput(simple_unet.UNet(2, 3, 8, 32)).to(hip_device)
    for p in teacher.parameters():
        p.detach_()
    teacher.eval()
    arena.attach(student)
    arena.attach(teacher, with_grads=False)
    opt = optim.SGD(student.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
    tc = dict(loss=losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits('mean'),
                                          'weight': [0.5]}]),
              virtual_batch_size_multiplier=1, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
              sigma_range=(2, 4), confidence_threshold=0.0, consistency_loss_weight=10, ema_model_alpha=0.99,
              print_freq=10 ** 9, gradient_clip_value=5.0, device_augment=DA.DeviceAugment(S, seed=7))
    seen = []
    real = train.run_step

    def spy(model, ema, o, image, mask, ua, ub, epoch, step, config):
        seen.append((image.clone(), mask.clone(), ua.clone(), ub.clone()))
        return real(model, ema, o, image, mask, ua, ub, epoch, step, config)

    train.run_step = spy
    try:
        train.train(student, teacher, opt, dl, iter(udl), 30, 0, None, {'train': tc}, hip_device)
    finally:
        train.run_step = real
    torch.cuda.synchronize()
    assert len(seen) == 2
    for image, mask, ua, ub in seen:
        assert image.shape == (n, 3, S, S) and image.dtype == torch.float32 and mask.shape == (n, 2, S, S)
        assert ua.shape == (n, 3, S, S) and ub.shape == (n, 3, S, S)
        assert float(image.max()) <= 1.0 and float(image.min()) >= 0.0
    # the same draws issued directly: labelled batch, then the two unlabelled batches, per step
    ref = DA.DeviceAugment(S, seed=7)
    uit = iter(udl)
    for (image, mask, ua, ub), batch in zip(seen, dl):
        b = ref.train_batch(batch)
        u0, u1 = ref.unsupervised_batch(next(uit)), ref.unsupervised_batch(next(uit))
        assert torch.equal(b['image'], image) and torch.equal(b['semantic_mask'], mask)
        assert torch.equal(u0['image'], ua) and torch.equal(u1['image'], ub)
    assert all(torch.isfinite(p).all() for p in student.parameters())
