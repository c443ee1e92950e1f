"""Is the oracle's torch-CPU restatement a faithful CPU baseline?  

RUNS ONLY IN THE BUILD CONTAINER, where the reference is mounted read-only at /root/reference (same import
recipe as gen_golden.py: the reference's own modules with an empty `kornia` stub).  It times, on this
container's host cores and on identical synthetic data:

  reference  train.train (reference/train.py:25-147) over a DDP-wrapped (gloo, world 1) reference
             models/unet.py UNet with a ResNet-50 encoder (max_width=128, ConvTranspose2d up-sampling)
  oracle     oracle/train_ref.py train_epoch over oracle/models_ref.py's UNet-R50 (what bench.py's
             cpu_baseline leg times on the GPU box's host)

The reference has no ResNet-50 encoder: both runs use the oracle's resnet50_encoder module,
so the encoder arithmetic is identical and the comparison isolates the decoder + training-step restatement.
Protocol of BASELINE.md §4: torch.set_num_threads(len(os.sched_getaffinity(0))), fp32, 512x512, batch 2,
1 warm-up step + 3 timed steps, same seeds.  Writes profiles/<tag>_cpu_baseline_check.json.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/time_cpu_baseline.py [tag]
"""
import json
import os
import sys
import time
import types

REF = '/root/reference'
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.dont_write_bytecode = True

import torch  # noqa: E402

THREADS = len(os.sched_getaffinity(0))
torch.set_num_threads(THREADS)
SIZE, BATCH, TIMED = 512, 2, 3


def data():
    g = torch.Generator().manual_seed(7)
    n = TIMED + 1
    imgs = torch.rand(n, BATCH, 3, SIZE, SIZE, generator=g)
    fg = (torch.rand(n, BATCH, 1, SIZE, SIZE, generator=g) > 0.5).float()
    masks = torch.cat([1 - fg, fg], 2)
    unl = torch.rand(2 * n, BATCH, 3, SIZE, SIZE, generator=g)
    return imgs, masks, unl


def time_oracle():
    sys.path.insert(0, ROOT)
    from oracle import models_ref, train_ref
    torch.manual_seed(0)
    s = models_ref.ListOutput(models_ref.UNet(2, models_ref.resnet50_encoder(), 128, train_upsampling=True))
    t = models_ref.ListOutput(models_ref.UNet(2, models_ref.resnet50_encoder(), 128, train_upsampling=True))
    t.load_state_dict(s.state_dict())
    init = {k: v.clone() for k, v in s.state_dict().items()}
    for p in t.parameters():
        p.detach_()
    t.eval()
    opt = torch.optim.SGD(s.parameters(), lr=0.0001 * 9 / 4, momentum=0.9, weight_decay=0.0005)
    imgs, masks, unl = data()
    stamps = []
    torch.manual_seed(3)
    t0 = time.perf_counter()
    logs = train_ref.train_epoch(s, t, opt, list(zip(imgs, masks)), iter(unl), 30,
                                 train_ref.default_cfg(confidence_threshold=0.5),
                                 on_step=lambda step, rec: stamps.append(time.perf_counter()))
    steps = [stamps[0] - t0] + [b - a for a, b in zip(stamps, stamps[1:])]
    return steps, [r['sup_loss'] for r in logs], models_ref, init


def time_reference(models_ref, init):
    sys.path.insert(0, REF)
    sys.modules.setdefault('kornia', types.ModuleType('kornia'))
    import torch.distributed as dist
    import losses
    import mean_teacher
    import train as ref_train
    from models import unet
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29534')
        dist.init_process_group('gloo', rank=0, world_size=1)

    class ListOutput(torch.nn.Module):
        def __init__(self, model):
            super().__init__()
            self.model = model

        def forward(self, x):
            y = self.model(x)
            return [y], [y]

    class Log:
        def __init__(self):
            self.rows = []

        def add_scalar(self, name, value, step):
            self.rows.append((name, float(value), int(step)))

    torch.manual_seed(0)
    fn = lambda: ListOutput(unet.UNet(2, models_ref.resnet50_encoder(), max_width=128, train_upsampling=True))  # noqa: E731
    s, t = fn(), fn()
    s.load_state_dict(init)          # the oracle's initial weights (same parameter schema, strict)
    t.load_state_dict(s.state_dict())
    ddp = torch.nn.parallel.DistributedDataParallel(s)
    mean_teacher.detach_model_parameters(t)
    t.eval()
    opt = torch.optim.SGD(ddp.parameters(), lr=0.0001 * 9 / 4, momentum=0.9, weight_decay=0.0005)
    cfg = {'train': dict(loss=losses.CalculateLoss([
        {'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'), 'weight': [0.5]}]),
        virtual_batch_size_multiplier=1, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
        sigma_range=(8, 32), confidence_threshold=0.5, consistency_loss_weight=10, ema_model_alpha=0.99,
        print_freq=1, gradient_clip_value=5.0)}
    imgs, masks, unl = data()
    torch.manual_seed(3)
    steps = []
    log = Log()
    uit = iter([{'image': unl[i]} for i in range(2 * (TIMED + 1))])
    for k in range(TIMED + 1):      # one call per step: a step is timed whole, DataLoader-free
        t0 = time.perf_counter()
        ref_train.train(ddp, t, opt, [{'image': imgs[k], 'semantic_mask': masks[k]}], uit, 30, k, log, cfg, 'cpu')
        steps.append(time.perf_counter() - t0)
    sup = [v for n, v, _ in log.rows if n == 'train_classification_loss']
    return steps, sup


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'r3'
    o_steps, o_sup, models_ref, init = time_oracle()
    r_steps, r_sup = time_reference(models_ref, init)
    o = sum(o_steps[1:]) / TIMED
    r = sum(r_steps[1:]) / TIMED
    out = {
        'what': 'C2 semi-supervised train step on CPU (UNet-R50 mw128 ConvT up, 512x512, batch 2, fp32): the reference '
                'train.train vs the oracle restatement bench.py times as cpu_baseline',
        'threads': THREADS, 'timed_steps': TIMED, 'warmup_steps': 1,
        'reference_s_per_step': round(r, 3), 'oracle_s_per_step': round(o, 3),
        'reference_images_per_s': round(BATCH / r, 4), 'oracle_images_per_s': round(BATCH / o, 4),
        'oracle_over_reference_time': round(o / r, 3),
        'reference_steps_s': [round(v, 3) for v in r_steps], 'oracle_steps_s': [round(v, 3) for v in o_steps],
        'step0_sup_loss': {'reference': r_sup[0] if r_sup else None, 'oracle': o_sup[0]},
        'torch': torch.__version__,
        'note': 'step 0 of each run is the warm-up; both runs start from the same weights (the oracle init loaded '
                'strictly into the reference model) and data, so their step-0 supervised losses must agree',
    }
    path = os.path.join(ROOT, 'profiles', f'{tag}_cpu_baseline_check.json')
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
