"""Batched weight repack (ssseg_weight_pack_batch, the refresh after every optimizer / EMA step) of the C2 student
(UNet-R50, forward + input-gradient layouts): device time per refresh (HIP events over 20) and a hash of every packed
tensor (A/B bit-identity; SSSEG_LIB_PATH selects another build).

    python tools/bench_pack.py
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from models import unet  # noqa: E402
from models.encoders import resnet  # noqa: E402
from ssseg import nn as snn  # noqa: E402


def main():
    snn.set_compute_dtype(torch.bfloat16)
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = unet.UNet(2, resnet.resnet50_encoder(), 128, train_upsampling=True).to(dev)
    x = torch.rand(2, 3, 256, 256, device=dev)
    model(x).float().sum().backward()   # creates every forward / input-gradient pack
    snn.invalidate_packed(model)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        snn.invalidate_packed(model)
    e1.record()
    torch.cuda.synchronize()
    h = hashlib.sha1()
    n = 0
    for m in model.modules():
        for key in sorted(getattr(m, '_ssseg_packs', {}) or {}, key=str):
            h.update(m._ssseg_packs[key].view(torch.uint8).cpu().numpy().tobytes())
            n += 1
    print(f'{n} packs: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per refresh  hash {h.hexdigest()[:16]}')


if __name__ == '__main__':
    main()
