"""Bisect a world-2 DDP+SyncBN gradient mismatch: tiny ssseg models (conv-BN-ReLU chains with optional
max-pool / ConvTranspose2d) on two gloo ranks sharing the GPU vs the same steps on the concatenated batch on
CPU (torch.nn, fp64).  Prints the worst per-tensor gradient error per step for each model.

    python tools/diag_ddp.py
"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd')):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as tnn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

B, H, STEPS, WORLD = 2, 16, 3, 2


def build(kind, lib):
    """lib = ssseg.nn or torch.nn; same parameter names either way."""
    torch.manual_seed(0)
    mods = tnn.ModuleDict()
    mods['c1'] = lib.Conv2d(3, 8, 3, padding=1, bias=False)
    mods['b1'] = lib.BatchNorm2d(8)
    if 'pool' in kind:
        mods['p'] = lib.MaxPool2d(2, ceil_mode=True) if hasattr(lib, 'MaxPool2d') else tnn.MaxPool2d(2, ceil_mode=True)
    if 'convt' in kind:
        mods['t'] = lib.ConvTranspose2d(8, 8, 4, 2, 1)
        mods['bt'] = lib.BatchNorm2d(8)
    mods['c2'] = lib.Conv2d(8, 8, 3, padding=1, bias=False)
    mods['b2'] = lib.BatchNorm2d(8)
    mods['head'] = (lib.Conv2d(8, 2, 1, head=True) if lib is not tnn else tnn.Conv2d(8, 2, 1))
    return mods


def fwd(mods, x, native):
    if native:
        from ssseg import nn as snn
        x = snn.to_act(x)
        y = snn.conv_bn_act(mods['c1'], x, mods['b1'], relu=True)
        if 'p' in mods:
            y = mods['p'](y)
        if 't' in mods:
            y = snn.conv_bn_act(mods['t'], y, mods['bt'], relu=True)
        y = snn.conv_bn_act(mods['c2'], y, mods['b2'], relu=True)
        return mods['head'](y)
    y = F.relu(mods['b1'](mods['c1'](x)))
    if 'p' in mods:
        y = mods['p'](y)
    if 't' in mods:
        y = F.relu(mods['bt'](mods['t'](y)))
    y = F.relu(mods['b2'](mods['c2'](y)))
    return mods['head'](y)


def data(kind):
    g = torch.Generator().manual_seed(11)
    imgs = torch.rand(STEPS, WORLD, B, 3, H, H, generator=g)
    oh = (H // 2 if 'pool' in kind else H) * (2 if 'convt' in kind else 1)
    tg = (torch.rand(STEPS, WORLD, B, 2, oh, oh, generator=g) > 0.5).float()
    return imgs, tg


def worker(rank, port, kind, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=WORLD)
    try:
        from ssseg import nn as snn
        from ssseg import ops
        from ssseg.ddp import DistributedDataParallel
        snn.set_compute_dtype(torch.float32)
        dev = torch.device('cuda:0')
        mods = build(kind, snn).to(dev)
        ddp = DistributedDataParallel(mods, bucket_cap_mb=0.001)
        imgs, tg = data(kind)
        out = []
        for k in range(STEPS):
            for p in mods.parameters():
                p.grad.zero_()
            y = fwd(mods, imgs[k, rank].to(dev), True)
            t = tg[k, rank].to(dev)
            loss = ops.bce_with_logits_mean(y.contiguous() if False else y, t)
            ddp.arm()
            loss.backward()
            ddp.finish()
            torch.cuda.synchronize()
            out.append({n: p.grad.detach().cpu().numpy().copy() for n, p in mods.named_parameters()})
        q.put((rank, out))
    except Exception as exc:
        import traceback
        q.put((rank, repr(exc) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def oracle(kind):
    mods = build(kind, tnn).double()
    from ssseg import nn as snn
    ref = build(kind, snn)
    mods.load_state_dict({k: v.double() for k, v in ref.state_dict().items()})
    imgs, tg = data(kind)
    out = []
    for k in range(STEPS):
        mods.zero_grad()
        y = fwd(mods, torch.cat(list(imgs[k])).double(), False)
        loss = sum(F.binary_cross_entropy_with_logits(y[r * B:(r + 1) * B], tg[k, r].double())
                   for r in range(WORLD)) / WORLD
        loss.backward()
        out.append({n: p.grad.detach().numpy().copy() for n, p in mods.named_parameters()})
    return out


def main():
    import torch.multiprocessing as mp
    for kind in ('plain', 'pool', 'convt', 'pool+convt'):
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        s = socket.socket()
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
        s.close()
        procs = [ctx.Process(target=worker, args=(r, port, kind, q)) for r in range(WORLD)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=120) for _ in range(WORLD))
        for p in procs:
            p.join(30)
        if isinstance(res[0], str):
            print(kind, 'ERROR', res[0])
            continue
        ref = oracle(kind)
        for k in range(STEPS):
            gmax = max(float(np.abs(v).max()) for v in ref[k].values())
            worst = max((float(np.abs(res[0][k][n] - ref[k][n]).max() / max(np.abs(ref[k][n]).max(), 1e-4 * gmax)), n)
                        for n in ref[k])
            print(f'{kind:12s} step {k}: worst grad rel err {worst[0]:.2e} ({worst[1]})', flush=True)


if __name__ == '__main__':
    main()
