"""HBM rates of the non-conv kernels the verdict asked for (CowMix mask generation + mixing, Lovász-softmax), at the
C2 / C3 step shapes: run the entry points a few times; under `rocprofv3 --kernel-trace --output-format csv` the trace
gives each kernel's duration, and --parse prices it against its algorithmic bytes (DESIGN.md §3 bytes per pixel).

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/aux -o a -- python tools/aux_kernels.py
    python tools/aux_kernels.py --parse gpurun_out/aux/a_kernel_trace.csv > profiles/r4_aux_kernels.txt
"""
import argparse
import collections
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

B, H, W = 16, 512, 512
PX = B * H * W
# algorithmic HBM bytes per launch (pixels of the batch x bytes per pixel; the sort keeps 32-bit keys and values)
BYTES = {
    'normal_kernel': 4 * PX,                       # noise write
    'cowmix_vblur_kernel': 8 * PX,                 # noise read + column-blurred field write
    'cowmix_hblur_kernel': 8 * PX,                 # field read + row-blurred field write (+ per-image sums)
    'cowmix_threshold_kernel': 8 * PX,             # field read + mask write
    'mix_kernel': (12 * 3 + 4) * PX,               # two 3-channel fp32 images + output + the mask
    'lovasz_prep_kernel': 20 * PX,                 # logit ch1 + 2-channel target read, key + value write
    'radix_hist_kernel': 4 * PX,                   # key read
    'radix_scatter_kernel': 16 * PX,               # key + value read and write
    'fg_count_kernel': 4 * PX,                     # value read
    'lovasz_grad_kernel': 12 * PX,                 # sorted key + value read, per-pixel gradient write
    'lovasz_bwd_kernel': 24 * PX,                  # logit + target + gradient read, 2-channel input gradient write
}


def run():
    import torch
    import cowmix
    import losses
    dev = torch.device('cuda')
    g = torch.Generator().manual_seed(3)
    ua = torch.rand(B, 3, H, W, generator=g).to(dev)
    ub = torch.rand(B, 3, H, W, generator=g).to(dev)
    logits = (torch.randn(B, 2, H, W, generator=g) * 2).to(dev).requires_grad_(True)
    fg = (torch.rand(B, 1, H, W, generator=g) > 0.5).float().to(dev)
    target = torch.cat([1 - fg, fg], 1).contiguous()
    for _ in range(5):
        m = cowmix.generate_cowmix_masks_like(ua, mask_proportion_range=(0.45, 0.55), sigma_range=(8, 32))
        cowmix.mix_with_mask(ua, ub, m)
        loss = losses.binary_lovasz_loss_with_logits(logits, target)
        loss.backward()
    torch.cuda.synchronize()
    print('ok', float(loss))


def parse(path):
    rows = [(r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in csv.DictReader(open(path))]
    agg = collections.defaultdict(list)
    for n, s, e in rows:
        n = n.replace('(anonymous namespace)::', '').replace('void ', '')
        key = n[:n.find('(')] if '(' in n else n
        key = key.split('<')[0]
        agg[key].append((e - s) / 1e3)
    print(f'# B={B} H={H} W={W}: per-launch median duration (last 5 launches of each) and algorithmic bytes')
    print(f'{"kernel":28s} {"launches":>8s} {"us":>9s} {"alg MB":>8s} {"TB/s":>6s}')
    for k, ts in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        t = sorted(ts[-5:])[len(ts[-5:]) // 2]
        b = BYTES.get(k)
        rate = f'{b / (t * 1e-6) / 1e12:6.2f}' if b else '     -'
        mb = f'{b / 1e6:8.1f}' if b else '       -'
        print(f'{k:28s} {len(ts):8d} {t:9.1f} {mb} {rate}')


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--parse')
    a = ap.parse_args()
    parse(a.parse) if a.parse else run()
