"""Train-time augmentations on the device: the reference config's albumentations pipelines
(configs/default_config.py:179-205 train['augmentations'], :206-212 train['unsupervised_augmentations']), applied to a
whole batch in HBM after the host loader's LongestMaxSize + PadIfNeeded (data/transforms.py).

Per sample the parameters are drawn on the host with Python's `random`, transform by transform in the pipeline's
order and with albumentations' conventions (each transform's probability check, then its parameters; a OneOf picks
by its members' normalised probabilities); the batch is then augmented by four kernels (csrc/augment.hip):

* `ssseg_aug_warp` -- Rotate(limit=15) o RandomResizedCrop(scale=(0.25, 1), ratio=(0.75, 1.33)) o HorizontalFlip as
  ONE affine map, then one of ElasticTransform(120, 6, 3.6) / GridDistortion(5, 0.3) / OpticalDistortion(1, 0.5)
  (OneOf p=0.5) as a per-pixel coordinate map; image bilinear, mask nearest, reflect-101 borders (cv2 defaults of
  those transforms);
* `ssseg_aug_color` -- RandomBrightnessContrast(0.2, 0.2) (OneOf p=1), ToGray(p=0.1), RGBShift(10, 10, 10) /
  HueSaturationValue(10, 10, 1) (OneOf p=0.3), on the uint8 value grid;
* `ssseg_aug_blur` -- GaussianBlur(blur_limit=9) (OneOf p=0.1; cv2's kernels) and the elastic displacement fields;
* `ssseg_aug_iso_finish` -- ISONoise(color_shift=(0.01, 0.05), intensity=(0.1, 0.5)) (OneOf p=0.2) and ToFloat.

Deliberate differences (parity with albumentations / cv2 is unpinned: both are absent from this image): one
resampling for the whole geometric chain instead of one per transform (sharper, and no intermediate border
handling), the distortion resampled together with the affine chain -- i.e. before the colour ops instead of after
them (the colour ops are per pixel; only GaussianBlur's order relative to the distortion changes) -- and the
elastic / ISO noise drawn with Philox on the device instead of NumPy's MT19937.
"""
import ctypes
import math
import random

import numpy as np
import torch

from ssseg import native as N

WMAX = 64   # Gaussian taps per sample (radius <= 31)


class WarpParams(ctypes.Structure):
    _fields_ = [('a', ctypes.c_float * 6), ('distort', ctypes.c_int32), ('field', ctypes.c_int32),
                ('m', ctypes.c_float * 6), ('k', ctypes.c_float), ('cx', ctypes.c_float), ('cy', ctypes.c_float),
                ('fx', ctypes.c_float), ('fy', ctypes.c_float), ('border', ctypes.c_int32)]


class ColorParams(ctypes.Structure):
    _fields_ = [('bc', ctypes.c_int32), ('alpha', ctypes.c_float), ('beta', ctypes.c_float),
                ('gray', ctypes.c_int32),
                ('rgb', ctypes.c_int32), ('shift', ctypes.c_float * 3),
                ('hsv', ctypes.c_int32), ('hsv_shift', ctypes.c_float * 3),
                ('iso', ctypes.c_int32), ('iso_color_std', ctypes.c_float), ('iso_intensity', ctypes.c_float)]


def _affine_inv(m):
    """Inverse of a 2x3 affine map [[a, b, c], [d, e, f]]."""
    a, b, c, d, e, f = m
    det = a * e - b * d
    ia, ib, id_, ie = e / det, -b / det, -d / det, a / det
    return [ia, ib, -(ia * c + ib * f), id_, ie, -(id_ * c + ie * f)]


def _compose(p, q):
    """p o q for 2x3 affine maps (apply q first)."""
    return [p[0] * q[0] + p[1] * q[3], p[0] * q[1] + p[1] * q[4], p[0] * q[2] + p[1] * q[5] + p[2],
            p[3] * q[0] + p[4] * q[3], p[3] * q[1] + p[4] * q[4], p[3] * q[2] + p[4] * q[5] + p[5]]


def rotation_matrix(angle_deg, cx, cy):
    """cv2.getRotationMatrix2D(centre, angle, 1): dst = M src (positive angle = counter-clockwise on screen)."""
    a = math.cos(math.radians(angle_deg))
    b = math.sin(math.radians(angle_deg))
    return [a, b, (1 - a) * cx - b * cy, -b, a, b * cx + (1 - a) * cy]


def rrc_params(rng, H, W, scale, ratio):
    """albumentations RandomResizedCrop.get_params_dependent_on_targets: (crop_h, crop_w, y0, x0)."""
    area = H * W
    for _ in range(10):
        target = rng.uniform(*scale) * area
        ar = math.exp(rng.uniform(math.log(ratio[0]), math.log(ratio[1])))
        w = int(round(math.sqrt(target * ar)))
        h = int(round(math.sqrt(target / ar)))
        if 0 < w <= W and 0 < h <= H:
            i = rng.randint(0, H - h)
            j = rng.randint(0, W - w)
            return h, w, i, j
    in_ratio = W / H
    if in_ratio < min(ratio):
        w, h = W, int(round(W / min(ratio)))
    elif in_ratio > max(ratio):
        h, w = H, int(round(H * max(ratio)))
    else:
        w, h = W, H
    return h, w, (H - h) // 2, (W - w) // 2


def grid_axis(n, steps, num_steps):
    """GridDistortion's per-axis source coordinates (albumentations functional.grid_distortion)."""
    step = n // num_steps
    xx = np.zeros(n, np.float32)
    prev = 0.0
    for idx, x in enumerate(range(0, n, step)):
        end = min(x + step, n)
        cur = prev + step * steps[idx]
        xx[x:end] = np.linspace(prev, cur, end - x)
        prev = cur
    return xx


def cv2_gaussian_taps(ksize):
    """cv2.getGaussianKernel(ksize, 0): the fixed small tables for ksize <= 7, else sigma = 0.3((k-1)/2 - 1) + 0.8."""
    small = {1: [1.0], 3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
             7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}
    if ksize in small:
        return np.array(small[ksize], np.float64)
    sigma = 0.3 * ((ksize - 1) * 0.5 - 1) + 0.8
    x = np.arange(ksize) - (ksize - 1) / 2
    w = np.exp(-x * x / (2 * sigma * sigma))
    return w / w.sum()


def scipy_gaussian_taps(sigma, truncate=4.0):
    """scipy.ndimage.gaussian_filter's 1-D kernel (radius int(truncate * sigma + 0.5))."""
    r = int(truncate * sigma + 0.5)
    x = np.arange(-r, r + 1)
    w = np.exp(-0.5 * x * x / (sigma * sigma))
    return w / w.sum()


class DeviceAugment:
    """Batch augmenter.  `train(images, masks)` / `unsupervised(images)` take uint8 NHWC device tensors (the host
    loader's LongestMaxSize + PadIfNeeded output, equal sizes within a batch) and return float NCHW in [0, 1] (image)
    and [0, 1] soft masks, crop_size x crop_size.  The draws replay the pipeline: `last_params` keeps every sample's
    parameters (albumentations' ReplayCompose record)."""

    def __init__(self, crop_size, seed=0, rotate_limit=15, scale=(0.25, 1.0), ratio=(0.75, 1.33), hflip_p=0.5,
                 brightness=0.2, contrast=0.2, gray_p=0.1, color_p=0.3, rgb_shift=10, hsv=(10, 10, 1), blur_p=0.1,
                 blur_limit=(3, 9), iso_p=0.2, iso_color=(0.01, 0.05), iso_intensity=(0.1, 0.5), distort_p=0.5,
                 elastic=(120.0, 120 * 0.05, 120 * 0.03), grid=(5, 0.3), optical=(1.0, 0.5)):
        self.size = int(crop_size)
        self.rng = random.Random(seed)
        self.rotate_limit, self.scale, self.ratio, self.hflip_p = rotate_limit, scale, ratio, hflip_p
        self.brightness, self.contrast, self.gray_p, self.color_p = brightness, contrast, gray_p, color_p
        self.rgb_shift, self.hsv, self.blur_p, self.blur_limit = rgb_shift, hsv, blur_p, blur_limit
        self.iso_p, self.iso_color, self.iso_intensity = iso_p, iso_color, iso_intensity
        self.distort_p, self.elastic, self.grid, self.optical = distort_p, elastic, grid, optical
        self.last_params = None

    # ---- parameter draws (host, the pipeline's order) -----------------------------------------------------------
    def _geometry(self, H, W, train):
        rng, S = self.rng, self.size
        rec = {}
        A = [1.0, 0.0, 0.0, 0.0, 1.0, 0.0]   # crop grid -> input image
        if train:   # Rotate(limit=15, always_apply): p check, then the angle
            rng.random()
            rec['angle'] = rng.uniform(-self.rotate_limit, self.rotate_limit)
            R = rotation_matrix(rec['angle'], W / 2 - 0.5, H / 2 - 0.5)
        rng.random()   # RandomResizedCrop (always_apply)
        h, w, y0, x0 = rrc_params(rng, H, W, self.scale, self.ratio if train else (1.0, 1.0))
        rec['crop'] = (h, w, y0, x0)
        C = [w / S, 0.0, 0.5 * w / S - 0.5 + x0, 0.0, h / S, 0.5 * h / S - 0.5 + y0]   # cv2.resize INTER_LINEAR
        flip = rng.random() < self.hflip_p
        rec['hflip'] = flip
        F = [-1.0, 0.0, S - 1.0, 0.0, 1.0, 0.0] if flip else [1.0, 0.0, 0.0, 0.0, 1.0, 0.0]
        A = _compose(C, F)
        if train:
            A = _compose(_affine_inv(R), A)
        return A, rec

    def _color(self):
        rng = self.rng
        rec = {}
        cp = ColorParams()
        if rng.random() < 1.0:   # OneOf([RandomBrightnessContrast], p=1)
            rng.randint(0, 2 ** 32 - 1)   # OneOf's choice seed (one member)
            rng.random()
            cp.bc = 1
            cp.alpha = 1.0 + rng.uniform(-self.contrast, self.contrast)
            cp.beta = 0.0 + rng.uniform(-self.brightness, self.brightness)
            rec['bc'] = (cp.alpha, cp.beta)
        if rng.random() < self.gray_p:   # ToGray(p=0.1)
            cp.gray = 1
            rec['gray'] = True
        if rng.random() < self.color_p:   # OneOf([RGBShift, HueSaturationValue], p=0.3)
            pick = np.random.RandomState(rng.randint(0, 2 ** 32 - 1)).choice(2, p=[0.5, 0.5])
            rng.random()
            if pick == 0:
                cp.rgb = 1
                s = [rng.uniform(-self.rgb_shift, self.rgb_shift) for _ in range(3)]
                cp.shift[:] = s
                rec['rgb_shift'] = s
            else:
                cp.hsv = 1
                s = [rng.uniform(-self.hsv[0], self.hsv[0]), rng.uniform(-self.hsv[1], self.hsv[1]),
                     rng.uniform(-self.hsv[2], self.hsv[2])]
                cp.hsv_shift[:] = s
                rec['hsv_shift'] = s
        ksize = 0
        if rng.random() < self.blur_p:   # OneOf([GaussianBlur(blur_limit=9)], p=0.1)
            rng.randint(0, 2 ** 32 - 1)
            rng.random()
            ksize = int(rng.choice(list(range(self.blur_limit[0], self.blur_limit[1] + 1, 2))))
            rec['blur_ksize'] = ksize
        if rng.random() < self.iso_p:   # OneOf([ISONoise], p=0.2)
            rng.randint(0, 2 ** 32 - 1)
            rng.random()
            cs = rng.uniform(*self.iso_color)
            it = rng.uniform(*self.iso_intensity)
            cp.iso, cp.iso_color_std, cp.iso_intensity = 1, cs * 360.0 * it, it
            rec['iso'] = (cs, it)
        return cp, ksize, rec

    def _distortion(self, wp, S, gmap):
        rng = self.rng
        rec = {}
        if rng.random() < self.distort_p:   # OneOf([Elastic p=.5, Grid p=.5, Optical p=1], p=0.5)
            pick = int(np.random.RandomState(rng.randint(0, 2 ** 32 - 1)).choice(3, p=[0.25, 0.25, 0.5]))
            rng.random()
            if pick == 0:
                alpha, sigma, alpha_affine = self.elastic
                r = np.random.RandomState(rng.randint(0, 10000))
                c, sq = S // 2, min(S, S) // 3
                pts1 = np.float32([[c + sq, c + sq], [c + sq, c - sq], [c - sq, c - sq]])
                pts2 = pts1 + r.uniform(-alpha_affine, alpha_affine, size=pts1.shape).astype(np.float32)
                M = _affine_from_points(pts1, pts2)   # dst = M src (cv2.getAffineTransform)
                wp.distort = 1
                wp.m[:] = _affine_inv(M)
                rec['elastic'] = M
            elif pick == 1:
                num_steps, limit = self.grid
                sx = [1 + rng.uniform(-limit, limit) for _ in range(num_steps + 1)]
                sy = [1 + rng.uniform(-limit, limit) for _ in range(num_steps + 1)]
                gmap[:S] = grid_axis(S, sx, num_steps)
                gmap[S:] = grid_axis(S, sy, num_steps)
                wp.distort = 2
                rec['grid'] = (sx, sy)
            else:
                limit, shift = self.optical
                k = rng.uniform(-limit, limit)
                dx = round(rng.uniform(-shift, shift))
                dy = round(rng.uniform(-shift, shift))
                wp.distort, wp.k = 3, k
                wp.fx, wp.fy, wp.cx, wp.cy = float(S), float(S), S * 0.5 + dx, S * 0.5 + dy
                rec['optical'] = (k, dx, dy)
        return rec

    # ---- the batch ------------------------------------------------------------------------------------------------
    def _check(self, x, c):
        if not (x.is_cuda and x.dtype == torch.uint8 and x.dim() == 4 and x.is_contiguous()):
            raise ValueError('DeviceAugment: uint8 NHWC contiguous device tensors expected')
        if c is not None and x.shape[3] != c:
            raise ValueError(f'DeviceAugment: {c} channels expected, got {x.shape[3]}')

    def draw(self, n, H, W, train=True):
        """Host parameter draws of a batch of n samples (also what `last_params` records)."""
        S = self.size
        warp = (WarpParams * n)()
        color = (ColorParams * n)()
        gmaps = np.zeros((n, 2 * S), np.float32)
        radius = np.zeros(n, np.int32)
        weights = np.zeros((n, WMAX), np.float32)
        recs, nfield = [], 0
        for i in range(n):
            A, rec = self._geometry(H, W, train)
            warp[i].a[:] = A
            warp[i].border = 1
            if train:
                cp, ksize, crec = self._color()
                color[i] = cp
                rec.update(crec)
                if ksize:
                    taps = cv2_gaussian_taps(ksize)
                    radius[i] = ksize // 2
                    weights[i, :ksize] = taps
                rec.update(self._distortion(warp[i], S, gmaps[i]))
                if warp[i].distort == 1:
                    warp[i].field = nfield
                    nfield += 1
            recs.append(rec)
        self.last_params = recs
        return warp, color, gmaps, radius, weights, nfield

    def _upload(self, arr, dev):
        if isinstance(arr, np.ndarray):
            return torch.from_numpy(np.ascontiguousarray(arr)).to(dev, non_blocking=False)
        return torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)

    def train(self, images, masks):
        self._check(images, 3)
        self._check(masks, None)
        n, H, W, _ = images.shape
        S, dev = self.size, images.device
        stream = N.stream()
        warp, color, gmaps, radius, weights, nf = self.draw(n, H, W, True)
        d_warp, d_color = self._upload(warp, dev), self._upload(color, dev)
        d_gmaps = self._upload(gmaps, dev)
        fields = torch.empty((max(nf, 1), S, S, 2), device=dev, dtype=torch.float32)
        if nf:   # ElasticTransform displacement fields: uniform(-1, 1) -> scipy Gaussian(sigma) -> x alpha
            alpha, sigma, _ = self.elastic
            N.call('ssseg_aug_uniform_field', N.dev_ptr(fields), fields.numel(), self.rng.getrandbits(64), stream)
            taps = scipy_gaussian_taps(sigma)
            fr = np.full(nf, len(taps) // 2, np.int32)
            fw = np.zeros((nf, WMAX), np.float32)
            fw[:, :len(taps)] = taps * math.sqrt(alpha)   # both passes carry sqrt(alpha): the field is scaled by alpha
            self._blur(fields, torch.empty_like(fields), nf, S, S, 2, fr, fw, sym=1, round8=0, dev=dev, stream=stream)
        img = torch.empty((n, S, S, 3), device=dev, dtype=torch.float32)
        out_mask = torch.empty((n, masks.shape[3], S, S), device=dev, dtype=torch.float32)
        N.call('ssseg_aug_warp', N.dev_ptr(images), N.dev_ptr(masks), masks.shape[3], n, H, W, N.dev_ptr(img),
               N.dev_ptr(out_mask), S, S, N.dev_ptr(d_warp), N.dev_ptr(d_gmaps), N.dev_ptr(fields), 0, stream)
        N.call('ssseg_aug_color', N.dev_ptr(img), n, S, S, N.dev_ptr(d_color), stream)
        if radius.any():
            self._blur(img, torch.empty_like(img), n, S, S, 3, radius, weights, sym=0, round8=1, dev=dev, stream=stream)
        out = torch.empty((n, 3, S, S), device=dev, dtype=torch.float32)
        stats = torch.empty((n, 2), device=dev, dtype=torch.float64)
        N.call('ssseg_aug_iso_finish', N.dev_ptr(img), N.dev_ptr(out), n, S, S, N.dev_ptr(d_color), N.dev_ptr(stats),
               self.rng.getrandbits(64), stream)
        return out, out_mask

    def _blur(self, x, tmp, n, H, W, C, radius, weights, sym, round8, dev, stream):
        d_r, d_w = self._upload(radius, dev), self._upload(weights, dev)
        N.call('ssseg_aug_blur', N.dev_ptr(x), N.dev_ptr(tmp), n, H, W, C, N.dev_ptr(d_r), N.dev_ptr(d_w), WMAX, sym,
               round8, stream)

    def train_batch(self, batch):
        """A collated SkinSegDataset batch built with the host-only transforms (image uint8 [B, 3, H, W], semantic_mask
        float [B, C, H, W] in [0, 1], reference data/dataset.py:76-79 layout) -> the same dict, augmented on the
        device.  The NHWC uint8 views are layout plumbing (one copy each)."""
        img = batch['image'].cuda(non_blocking=True).permute(0, 2, 3, 1).contiguous()
        m = batch['semantic_mask'].cuda(non_blocking=True)
        m = (m * 255).round().to(torch.uint8).permute(0, 2, 3, 1).contiguous()
        x, mask = self.train(img, m)
        return dict(batch, image=x, semantic_mask=mask)

    def unsupervised_batch(self, batch):
        """A collated UnsupervisedImagesDataset batch (image uint8 [B, 3, H, W], host-only transforms) -> the same dict
        with the device-augmented float image (train['unsupervised_augmentations'], unsupervised_dataset.py:20-21)."""
        img = batch['image'].cuda(non_blocking=True).permute(0, 2, 3, 1).contiguous()
        return dict(batch, image=self.unsupervised(img))

    def unsupervised(self, images):
        """train['unsupervised_augmentations']: RandomResizedCrop(ratio=(1, 1)) + HorizontalFlip + ToFloat."""
        self._check(images, 3)
        n, H, W, _ = images.shape
        S, dev = self.size, images.device
        warp, _, gmaps, _, _, _ = self.draw(n, H, W, False)
        d_warp = self._upload(warp, dev)
        out = torch.empty((n, 3, S, S), device=dev, dtype=torch.float32)
        N.call('ssseg_aug_warp', N.dev_ptr(images), None, 0, n, H, W, N.dev_ptr(out), None, S, S, N.dev_ptr(d_warp),
               None, None, 1, N.stream())
        return out


def _affine_from_points(src, dst):
    """cv2.getAffineTransform: the 2x3 M with dst_i = M src_i for three point pairs."""
    A = np.zeros((6, 6))
    b = np.zeros(6)
    for i in range(3):
        x, y = src[i]
        A[2 * i] = [x, y, 1, 0, 0, 0]
        A[2 * i + 1] = [0, 0, 0, x, y, 1]
        b[2 * i], b[2 * i + 1] = dst[i]
    return [float(v) for v in np.linalg.solve(A, b)]
