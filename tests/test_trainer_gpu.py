"""The drop-in epoch loop (reference distributed_trainer.py:16-191 -> train.train :25-147 -> train.validate :150-195) on
the GPU at world size 1 over RCCL: loaders, the `cycle` over unlabelled batches, the train steps, validation, the
checkpoint dict and best.pth, the LR scheduler and the stop rule -- once with the captured-step replay of train.train
(ssseg.graph.StepGraph, the default) and once with every launch issued eagerly (SSSEG_TRAIN_GRAPH=0): the two runs
must end in bit-identical checkpoints."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd')

CFG = '''"""Tiny semi-supervised config for tests/test_trainer_gpu.py (bf16, SimpleUNet at 64x64, 5 steps per epoch)."""
from functools import partial

import torch

import losses
from data.synthetic import SyntheticSegDataset
from models.adapters import ListOutput
from models.simple_unet import UNet

common = dict(world_size=1, use_cpu=False, workers=1, output_dir={out!r}, num_classes=2, image_size=64,
              compute_dtype='bf16')
model = dict(model_fn=lambda: ListOutput(UNet(2, num_blocks=3, first_channels=16, max_width=64)))
train = dict(print_freq=2, batch_size_per_worker=2, virtual_batch_size_multiplier=1, num_dataloader_workers=0,
             crop_size=64, gradient_clip_value=5.0, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
             sigma_range=(4, 8), consistency_loss_weight=10, ema_model_alpha=0.99, confidence_threshold=0.5,
             pretrained_checkpoint_path='')
train['base_lr'] = 0.01
train['loss'] = losses.CalculateLoss([{{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'),
                                       'weight': [0.5]}}])
train['min_lr'] = train['base_lr'] * 2      # above the schedule's lr: the loop stops after one epoch
train['optimizer'] = partial(torch.optim.SGD, lr=train['base_lr'], momentum=0.9, weight_decay=0.0005)
train['lr_scheduler'] = partial(torch.optim.lr_scheduler.CosineAnnealingWarmRestarts, T_0=300, T_mult=2,
                                eta_min=train['base_lr'] * 0.01, last_epoch=-1)
train['dataset'] = partial(SyntheticSegDataset, length=10, size=64, seed=1, blob_sigma=4.0)
train['unsupervised_dataset'] = partial(SyntheticSegDataset, length=8, size=64, seed=3, with_masks=False)
val = dict(batch_size_per_worker=2, num_dataloader_workers=0,
           dataset=partial(SyntheticSegDataset, length=4, size=64, seed=2, blob_sigma=4.0))
'''

KEYS = {'epoch', 'best_metric', 'state_dict', 'ema_state_dict', 'optimizer'}   # distributed_trainer.py:173-179


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(cfg_path, port, graph, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['SSSEG_TRAIN_GRAPH'] = '1' if graph else '0'
    import sys
    sys.path[:0] = [ROOT, PKG]
    try:
        import torch.distributed as dist
        import distributed_trainer
        import train
        distributed_trainer.distributed_train(0, cfg_path)
        q.put({'captures': train._GRAPH['captures'], 'replays': train._GRAPH['replays'],
               'backend': dist.get_backend()})
        distributed_trainer.cleanup()
    except Exception as exc:
        import traceback
        q.put('ERROR ' + repr(exc) + '\n' + traceback.format_exc())


def _run(tmp, graph):
    import torch.multiprocessing as mp
    out = os.path.join(tmp, 'graph' if graph else 'eager')
    os.makedirs(out, exist_ok=True)
    cfg = os.path.join(tmp, f'cfg_{"graph" if graph else "eager"}.py')
    with open(cfg, 'w') as fh:
        fh.write(CFG.format(out=out))
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(cfg, _free_port(), graph, q))
    p.start()
    try:
        res = q.get(timeout=110)
    finally:
        p.join(30)
        if p.is_alive():
            p.kill()
    assert not isinstance(res, str), res
    return out, res


@pytest.mark.timeout(300)   # two spawned trainer processes, each up to 110 s
def test_distributed_train_one_epoch_graph_vs_eager(hip_device, tmp_path):
    tmp = str(tmp_path)
    out_g, res_g = _run(tmp, True)
    out_e, res_e = _run(tmp, False)
    assert res_g['backend'] == 'nccl'
    # 5 steps: 2 eager (autotune, BN fold table), the first optimizer step (step 1) eager too, then one capture and
    # replays of it for steps 2-4
    assert res_g['captures'] == 1 and res_g['replays'] == 3, res_g
    assert res_e['captures'] == 0 and res_e['replays'] == 0, res_e
    cks = []
    for out in (out_g, out_e):
        assert os.path.exists(os.path.join(out, 'best.pth'))
        ck = torch.load(os.path.join(out, 'checkpoint.pth'), map_location='cpu', weights_only=True)
        assert KEYS <= set(ck), set(ck)
        assert ck['epoch'] == 1
        cks.append(ck)
    g, e = cks
    for part in ('state_dict', 'ema_state_dict'):
        assert g[part].keys() == e[part].keys()
        for k in g[part]:
            assert torch.equal(g[part][k], e[part][k]), (part, k)
    mg = [v['momentum_buffer'] for v in g['optimizer']['state'].values()]
    me = [v['momentum_buffer'] for v in e['optimizer']['state'].values()]
    assert len(mg) == len(me) > 0
    for a, b in zip(mg, me):
        assert torch.equal(a, b)
    assert g['best_metric'] == e['best_metric']
    assert all(torch.isfinite(v).all() for v in g['state_dict'].values() if v.is_floating_point())
