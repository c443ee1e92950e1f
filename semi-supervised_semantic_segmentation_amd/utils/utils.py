"""Host utilities — drop-in for reference utils/utils.py."""
import os
import random

import numpy as np
import torch


def seed_everything(seed):
    random.seed(seed)
    os.environ['PYTHONHASHSEED'] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def calc_global_step(dataset_len, world_size, batch_size_per_worker, epoch):
    return int(dataset_len // (world_size * batch_size_per_worker) * epoch)


def get_trainable_params(model):
    return [p for p in model.parameters() if p.requires_grad]


def get_max_lr(optimizer):
    return max([float(g['lr']) for g in optimizer.param_groups] + [0.])


def freeze_bn(module):
    for layer in module.modules():
        if isinstance(layer, torch.nn.BatchNorm2d):
            layer.eval()


def reduce_tensor(inp):
    """utils.py:43-54: dist.reduce(SUM) to rank 0, in place (logging only)."""
    if not torch.distributed.is_initialized() or torch.distributed.get_world_size() < 2:
        return inp
    with torch.no_grad():
        torch.distributed.reduce(inp, dst=0)
    return inp


def memory_report():
    t = torch.cuda.get_device_properties(0).total_memory
    c = torch.cuda.memory_reserved(0)
    a = torch.cuda.memory_allocated(0)
    print('Mem:', t, c, a, c - a)


class AverageMeter:
    """Running average; accepts python numbers or device scalars (summed on device, no host sync
    until value()/average() is read)."""

    def __init__(self):
        self.initialized = False
        self.val = self.avg = self.sum = self.count = None

    def initialize(self, val, weight):
        self.val, self.sum, self.count = val, val * weight, weight
        self.initialized = True

    def update(self, val, weight=1):
        if isinstance(val, torch.Tensor):
            val = val.detach()
        if not self.initialized:
            self.initialize(val, weight)
        else:
            self.add(val, weight)

    def add(self, val, weight):
        self.val = val
        self.sum = self.sum + val * weight
        self.count += weight

    def value(self):
        return float(self.val)

    def average(self):
        return float(self.sum) / self.count if self.initialized else None
