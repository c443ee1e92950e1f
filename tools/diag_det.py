"""Run-to-run determinism of one config's first train step: build, hook every module (forward outputs and
backward grad_outputs as bit checksums), run step 0; rebuild and repeat; print the first modules whose checksums
differ (forward order).

    python tools/diag_det.py [--config c3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tools'), ROOT, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd')]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def csum(t):
    if not isinstance(t, torch.Tensor) or not t.is_floating_point():
        return None
    t = t.detach().contiguous()
    v = t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)
    return int(v.to(torch.int64).sum()) * 1000003 + int((v.to(torch.int64) * torch.arange(
        v.numel(), device=v.device, dtype=torch.int64).view(v.shape).remainder(977)).sum())


def flat(o):
    if isinstance(o, torch.Tensor):
        return [o]
    if isinstance(o, (list, tuple)):
        return [t for x in o for t in flat(x)]
    return []


def run_once(name, path, dev):
    import full_size_steps as F
    import train
    model, ema, opt, cfg, tc, data, _, _ = F.build(name, path, dev)
    log = []
    hooks = []
    for tag, root in (('student', model), ('teacher', ema)):
        for mn, m in root.named_modules():
            if list(m.children()):
                continue
            hooks.append(m.register_forward_hook(
                lambda mod, i, o, k=f'{tag}.{mn}': log.append(('fwd', k, tuple(csum(t) for t in flat(o))))))
    out = train.train_step(model, ema, opt, *data, 30, 0, cfg)
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    params = [(n, csum(p)) for n, p in model.named_parameters()]
    return [float(t) for t in out], log, params


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c3')
    a = ap.parse_args()
    import full_size_steps as F
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:29541', rank=0, world_size=1)
    r1 = run_once(a.config, F.CFGS[a.config], dev)
    r2 = run_once(a.config, F.CFGS[a.config], dev)
    print('losses', r1[0], r2[0], 'equal', r1[0] == r2[0])
    n = 0
    for (k1, n1, c1), (k2, n2, c2) in zip(r1[1], r2[1]):
        if n1 != n2:
            print('order differs', n1, n2)
            break
        if c1 != c2:
            print('DIFF', k1, n1)
            n += 1
            if n >= 12:
                break
    print('forward records', len(r1[1]), len(r2[1]), 'differing shown', n)
    pd = [n for (n, c1), (_, c2) in zip(r1[2], r2[2]) if c1 != c2]
    print('params differing after the step:', len(pd), pd[:10])
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
