"""TEST INFRASTRUCTURE ONLY (tests/ may import this; the product path never does).

NumPy restatement of the device augmentation kernels (csrc/augment.hip, data/device_augment.py), which restate the
reference config's albumentations pipelines (configs/default_config.py:179-212).  albumentations and cv2 are absent
from this image, so parity with the reference pipeline itself is UNPINNED: this oracle pins the kernels' own
arithmetic (OpenCV pixel-centre bilinear / nearest sampling, reflect-101 borders, the uint8-grid colour ops, cv2 /
scipy Gaussian taps, RGB <-> HLS / 8-bit HSV conversions), not albumentations' outputs.
"""
import numpy as np


def reflect101(i, n):
    i = np.asarray(i)
    if n == 1:
        return np.zeros_like(i)
    period = 2 * n - 2
    i = np.abs(i) % period
    return np.where(i >= n, period - i, i)


def reflect_sym(i, n):
    i = np.asarray(i)
    period = 2 * n
    i = np.where(i < 0, -i - 1, i) % period
    return np.where(i >= n, period - 1 - i, i)


def distort(p, S, gmap, field):
    """Crop-grid pixel coordinates after the sample's distortion (ssseg_aug_warp_params.distort)."""
    y, x = np.mgrid[0:S, 0:S].astype(np.float64)
    if p['distort'] == 1:   # ElasticTransform: Minv (x + dx, y + dy)
        ex, ey = x + field[..., 0], y + field[..., 1]
        m = p['m']
        return m[0] * ex + m[1] * ey + m[2], m[3] * ex + m[4] * ey + m[5]
    if p['distort'] == 2:   # GridDistortion: separable axis maps
        return np.broadcast_to(gmap[:S][None, :], (S, S)), np.broadcast_to(gmap[S:][:, None], (S, S))
    if p['distort'] == 3:   # OpticalDistortion (cv2.initUndistortRectifyMap, k1 = k2 = k)
        u, v = (x - p['cx']) / p['fx'], (y - p['cy']) / p['fy']
        r2 = u * u + v * v
        kr = 1 + p['k'] * r2 + p['k'] * r2 * r2
        return p['fx'] * u * kr + p['cx'], p['fy'] * v * kr + p['cy']
    return x, y


def warp(img, mask, p, S, gmap=None, field=None):
    """One sample: image HxWx3 uint8 -> SxSx3 float on the uint8 grid (bilinear), mask HxWxC uint8 -> CxSxS [0, 1]."""
    H, W = img.shape[:2]
    qx, qy = distort(p, S, gmap, field)
    a = p['a']
    sx, sy = a[0] * qx + a[1] * qy + a[2], a[3] * qx + a[4] * qy + a[5]
    x0, y0 = np.floor(sx), np.floor(sy)
    lx, ly = sx - x0, sy - y0
    x0, y0 = x0.astype(np.int64), y0.astype(np.int64)
    out = np.zeros((S, S, 3))
    for t in range(4):
        xx, yy = x0 + (t & 1), y0 + (t >> 1)
        wgt = (lx if t & 1 else 1 - lx) * (ly if t >> 1 else 1 - ly)
        if p['border'] == 1:
            xx, yy = reflect101(xx, W), reflect101(yy, H)
            ok = np.ones_like(wgt, bool)
        else:
            ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
            xx, yy = np.clip(xx, 0, W - 1), np.clip(yy, 0, H - 1)
        out += np.where(ok, wgt, 0)[..., None] * img[yy, xx].astype(np.float64)
    out = np.rint(np.clip(out, 0, 255))
    m = None
    if mask is not None:
        mx, my = np.rint(sx).astype(np.int64), np.rint(sy).astype(np.int64)
        if p['border'] == 1:
            mx, my = reflect101(mx, W), reflect101(my, H)
            m = mask[my, mx].astype(np.float64) / 255.0
        else:
            ok = (mx >= 0) & (mx < W) & (my >= 0) & (my < H)
            m = np.where(ok[..., None], mask[np.clip(my, 0, H - 1), np.clip(mx, 0, W - 1)], 0) / 255.0
        m = m.transpose(2, 0, 1)
    return out, m


def rgb2hsv8(r, g, b):
    mx, mn = np.maximum(r, np.maximum(g, b)), np.minimum(r, np.minimum(g, b))
    d = mx - mn
    v = mx
    s = np.where(mx > 0, 255 * d / np.where(mx > 0, mx, 1), 0)
    dd = np.where(d > 0, d, 1)
    hd = np.where(mx == r, 60 * (g - b) / dd, np.where(mx == g, 120 + 60 * (b - r) / dd, 240 + 60 * (r - g) / dd))
    hd = np.where(d > 0, np.where(hd < 0, hd + 360, hd), 0)
    h = np.rint(hd * 0.5)
    h = np.where(h >= 180, h - 180, h)
    return h, np.rint(s), np.rint(v)


def hsv82rgb(h, s, v):
    hd, sf = h * 2, s / 255
    c = v * sf
    hp = hd / 60
    x = c * (1 - np.abs(np.fmod(hp, 2) - 1))
    m = v - c
    sec = np.floor(hp).astype(np.int64) % 6
    z = np.zeros_like(c)
    r1 = np.select([sec == 0, sec == 1, sec == 2, sec == 3, sec == 4], [c, x, z, z, x], c)
    g1 = np.select([sec == 0, sec == 1, sec == 2, sec == 3, sec == 4], [x, c, c, x, z], z)
    b1 = np.select([sec == 0, sec == 1, sec == 2, sec == 3, sec == 4], [z, z, x, c, c], x)
    return tuple(np.rint(np.clip(t + m, 0, 255)) for t in (r1, g1, b1))


def color(img, p):
    """ssseg_aug_color on one HxWx3 [0, 255] image (float64)."""
    r, g, b = (img[..., i].astype(np.float64) for i in range(3))
    if p.get('bc'):
        al, be = p['alpha'], p['beta']
        r, g, b = (np.floor(np.clip(t * al + be * 255, 0, 255)) for t in (r, g, b))
    if p.get('gray'):   # albumentations to_gray = cv2 RGB2GRAY -> GRAY2RGB; OpenCV's 8-bit RGB2GRAY is the Q14 fixed
        # point CV_DESCALE(R*4899 + G*9617 + B*1868, 14) (coefficients 0.299 / 0.587 / 0.114 scaled by 2^14)
        ri, gi, bi = (t.astype(np.int64) for t in (r, g, b))
        y = ((ri * 4899 + gi * 9617 + bi * 1868 + 8192) >> 14).astype(np.float64)
        r = g = b = y
    if p.get('rgb'):
        r, g, b = (np.floor(np.clip(t + s, 0, 255)) for t, s in zip((r, g, b), p['shift']))
    if p.get('hsv'):
        h, s, v = rgb2hsv8(r, g, b)
        h = np.fmod(h + p['hsv_shift'][0], 180)
        h = np.floor(np.where(h < 0, h + 180, h))
        s = np.floor(np.clip(s + p['hsv_shift'][1], 0, 255))
        v = np.floor(np.clip(v + p['hsv_shift'][2], 0, 255))
        r, g, b = hsv82rgb(h, s, v)
    return np.stack([r, g, b], -1)


def blur(x, radius, weights, sym=False, round8=False):
    """Separable Gaussian of one HxWxC plane set (horizontal, then vertical)."""
    if radius == 0:
        return x.copy()
    H, W = x.shape[:2]
    refl = reflect_sym if sym else reflect101
    w = weights[:2 * radius + 1]
    tmp = np.zeros_like(x, dtype=np.float64)
    for k in range(-radius, radius + 1):
        tmp += w[k + radius] * x[:, refl(np.arange(W) + k, W)]
    out = np.zeros_like(tmp)
    for k in range(-radius, radius + 1):
        out += w[k + radius] * tmp[refl(np.arange(H) + k, H)]
    return np.rint(np.clip(out, 0, 255)) if round8 else out


def rgb2hls(r, g, b):
    mx, mn = np.maximum(r, np.maximum(g, b)), np.minimum(r, np.minimum(g, b))
    d = mx - mn
    l = 0.5 * (mx + mn)
    dd = np.where(d > 1e-12, d, 1)
    s = np.where(d > 1e-12, np.where(l < 0.5, d / np.where(mx + mn > 0, mx + mn, 1), d / np.where(2 - mx - mn > 0,
                                                                                               2 - mx - mn, 1)), 0)
    h = np.where(mx == r, 60 * (g - b) / dd, np.where(mx == g, 120 + 60 * (b - r) / dd, 240 + 60 * (r - g) / dd))
    h = np.where(d > 1e-12, np.where(h < 0, h + 360, h), 0)
    return h, l, s


def _hls_c(p, q, t):
    t = np.where(t < 0, t + 360, t)
    t = np.where(t >= 360, t - 360, t)
    return np.select([t < 60, t < 180, t < 240], [p + (q - p) * t / 60, q, p + (q - p) * (240 - t) / 60], p)


def hls2rgb(h, l, s):
    q = np.where(l < 0.5, l * (1 + s), l + s - l * s)
    p = 2 * l - q
    r, g, b = _hls_c(p, q, h + 120), _hls_c(p, q, h), _hls_c(p, q, h - 120)
    gray = s <= 0
    return np.where(gray, l, r), np.where(gray, l, g), np.where(gray, l, b)


def iso_finish(img, p, hue_noise=None, lum_noise=None):
    """ISONoise with the given per-pixel hue noise (already scaled) and Poisson luminance counts, then ToFloat
    (NCHW [0, 1]).  hue_noise / lum_noise None: no noise (the conversion chain alone)."""
    x = img.astype(np.float64)
    if p.get('iso'):
        h, l, s = rgb2hls(x[..., 0] / 255, x[..., 1] / 255, x[..., 2] / 255)
        if hue_noise is not None:
            h = h + hue_noise
            h = np.where(h < 0, h + 360, h)
            h = np.where(h > 360, h - 360, h)
        if lum_noise is not None:
            l = l + lum_noise / 255 * (1 - l)
        r, g, b = hls2rgb(h, l, s)
        x = np.stack([np.floor(np.clip(t * 255, 0, 255)) for t in (r, g, b)], -1)
    return (x / 255).transpose(2, 0, 1)
