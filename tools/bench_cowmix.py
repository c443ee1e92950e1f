"""CowMix mask generation at the C2 unlabeled batch (16 x 512^2; sigma in [8, 32] as bench.py, and two narrower ranges): device time of one
ssseg_cowmix_mask call (HIP events over 20 calls) and hashes of the smoothed field and the mask, for A/B of kernel
changes that must stay bit-identical (SSSEG_LIB_PATH selects another build).

    python tools/bench_cowmix.py
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import ops  # noqa: E402


def main():
    dev = torch.device('cuda')
    g = torch.Generator(device='cpu').manual_seed(3)
    for lo, hi in ((8.0, 32.0), (4.0, 16.0), (2.0, 5.0)):   # (8, 32): the bench config (bench.py)
        noise = torch.randn(16, 1, 512, 512, generator=g).to(dev)
        sigma = (lo + (hi - lo) * torch.rand(16, generator=g)).to(dev)
        p = (0.4 + 0.2 * torch.rand(16, generator=g)).to(dev)
        mask, field, thr = ops.cowmix_mask(noise, sigma, p, return_field=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.cowmix_mask(noise, sigma, p)
        e1.record()
        torch.cuda.synchronize()
        h = lambda t: hashlib.sha1(t.detach().cpu().numpy().tobytes()).hexdigest()[:16]  # noqa: E731
        print(f'sigma [{lo}, {hi}]: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per mask  field {h(field)}  '
              f'mask {h(mask)}  thr {h(thr)}')


if __name__ == '__main__':
    main()
