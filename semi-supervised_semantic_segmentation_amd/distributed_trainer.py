"""Process launch + epoch loop — drop-in for reference distributed_trainer.py (distributed_train :16-191,
cleanup :194-195, main :198-208) on the MI355X stack: one process per GPU, RCCL ('nccl' backend),
native SyncBN (BatchNorm2d all-reduces its statistics across the group), ssseg DDP (bucketed RCCL
all-reduce over the flat gradient arena), fused SGD, checkpoint dict keys unchanged
(epoch, best_metric, state_dict, ema_state_dict, optimizer)."""
import os
import shutil
from itertools import cycle

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import config
import mean_teacher
import train
import utils.utils as utils
from ssseg import amp, arena
from ssseg import nn as snn
from ssseg import optim as soptim
from ssseg.ddp import DistributedDataParallel


def _writer(path, step):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(path, purge_step=step, flush_secs=30)
    except Exception:           # tensorboard is optional (absent in this image)
        return None


def attach_grad_scaler(optimizer, device):
    """fp16 mode: the device-side GradScaler.  Only ssseg's fused SGD unscales by 1/S and skips a non-finite
    step; any other optimizer would apply S-scaled gradients, so it is refused."""
    if not isinstance(optimizer, soptim.SGD):
        raise NotImplementedError(f'fp16 compute mode needs ssseg.optim.SGD (loss-scaled gradients are unscaled in '
                                  f'its fused step); got {type(optimizer).__name__}')
    optimizer.grad_scaler = amp.GradScaler(device)
    return optimizer.grad_scaler


def _scaler_state(opt):
    sc = getattr(opt, 'grad_scaler', None)
    return sc.state_dict() if sc is not None else None


def _load_scaler_state(opt, sd):
    sc = getattr(opt, 'grad_scaler', None)
    if sc is not None and sd is not None:
        sc.load_state_dict(sd)


def distributed_train(rank, cfg_path):
    utils.seed_everything(0)
    cfg = config.fromfile(cfg_path)
    world = cfg['common']['world_size']
    if cfg['common'].get('use_cpu'):
        raise RuntimeError('the MI355X trainer has no CPU path; the CPU execution of this step is oracle/train_ref.py')
    dist.init_process_group(backend='nccl', rank=rank, world_size=world)
    device = torch.device('cuda', rank % cfg['common']['workers'])
    torch.cuda.set_device(device)
    snn.set_compute_dtype({'fp32': torch.float32, 'fp16': torch.float16}.get(cfg['common'].get('compute_dtype'),
                                                                             torch.bfloat16))

    model = DistributedDataParallel(cfg['model']['model_fn']().to(device))
    ema_model = cfg['model']['model_fn']().to(device)
    mean_teacher.detach_model_parameters(ema_model)
    arena.attach(ema_model, with_grads=False)
    optimizer = soptim.from_config(cfg['train']['optimizer'], utils.get_trainable_params(model))
    fp16 = snn.compute_dtype() == torch.float16
    if fp16:   # dynamic loss scaling on the device (ssseg.amp): fp16's exponent range flushes small gradients
        attach_grad_scaler(optimizer, device)
    disc = None
    if cfg['model'].get('discriminator') is not None and cfg['train'].get('adversarial_loss_weight'):
        # config C5: the discriminator the reference config names (default_config.py:116-120) trained by the
        # build-defined adversarial branch (train.adversarial_terms / discriminator_step), its own DDP + SGD
        disc = DistributedDataParallel(cfg['model']['discriminator']().to(device))
        disc_opt = soptim.from_config(cfg['train']['discriminator_optimizer'], disc.parameters())
        if fp16:
            attach_grad_scaler(disc_opt, device)
        cfg['train']['adversarial'] = dict(discriminator=disc, optimizer=disc_opt,
                                           weight=float(cfg['train']['adversarial_loss_weight']))

    train_dir = cfg['common']['output_dir']
    pre = cfg['train'].get('pretrained_checkpoint_path') or ''
    if pre and os.path.exists(pre):
        ck = torch.load(pre, map_location='cpu', weights_only=True)
        model.module.load_state_dict(ck['state_dict'], strict=False)
        ema_model.load_state_dict(ck['state_dict'], strict=False)
        snn.invalidate_packed(model.module)
        snn.invalidate_packed(ema_model)
    ema_model.eval()
    last_epoch, best_metric = 0, None
    latest = os.path.join(train_dir, 'checkpoint.pth')
    if os.path.exists(latest):
        ck = torch.load(latest, map_location='cpu', weights_only=True)
        model.module.load_state_dict(ck['state_dict'], strict=False)
        ema_model.load_state_dict(ck['ema_state_dict'], strict=False)
        optimizer.load_state_dict(ck['optimizer'])
        _load_scaler_state(optimizer, ck.get('grad_scaler'))
        if disc is not None and 'discriminator_state_dict' in ck:
            disc.module.load_state_dict(ck['discriminator_state_dict'])
            cfg['train']['adversarial']['optimizer'].load_state_dict(ck['discriminator_optimizer'])
            _load_scaler_state(cfg['train']['adversarial']['optimizer'], ck.get('discriminator_grad_scaler'))
            snn.invalidate_packed(disc.module)
        best_metric, last_epoch = ck['best_metric'], ck['epoch']
        snn.invalidate_packed(model.module)
        snn.invalidate_packed(ema_model)
    lr_scheduler = cfg['train']['lr_scheduler'](optimizer)

    def loader(ds, bs, workers, drop_last=True):
        sampler = torch.utils.data.distributed.DistributedSampler(ds)
        return torch.utils.data.DataLoader(ds, batch_size=bs, sampler=sampler, pin_memory=True, drop_last=drop_last,
                                           num_workers=workers), sampler

    tc = cfg['train']
    if tc.get('device_augmentations') is not None:
        # train['device_augmentations'] = partial(DeviceAugment, crop_size, ...): the datasets deliver the host-only
        # transforms' uint8 output and train.train augments each batch on the device (a per-rank draw stream)
        tc['device_augment'] = tc['device_augmentations'](seed=1000 + rank)
    train_ds = tc['dataset']()
    train_dl, train_sampler = loader(train_ds, tc['batch_size_per_worker'], tc['num_dataloader_workers'])
    unsup_dl, _ = loader(tc['unsupervised_dataset'](), tc['batch_size_per_worker'], tc['num_dataloader_workers'])
    unsup_iter = cycle(iter(unsup_dl))
    val_dl, _ = loader(cfg['val']['dataset'](), cfg['val']['batch_size_per_worker'],
                       cfg['val']['num_dataloader_workers'], drop_last=False)
    gstep = lambda e: utils.calc_global_step(len(train_ds), world, tc['batch_size_per_worker'], e)  # noqa: E731
    writer = _writer(train_dir, gstep(last_epoch)) if rank == 0 else None

    for epoch in range(last_epoch, 300):
        if isinstance(lr_scheduler, torch.optim.lr_scheduler.CosineAnnealingWarmRestarts):
            lr_scheduler.step(epoch)
        train_sampler.set_epoch(epoch)
        if rank == 0 and writer is not None:
            writer.add_scalar('max_lr', utils.get_max_lr(optimizer), global_step=gstep(epoch))
        train.train(model, ema_model, optimizer, train_dl, unsup_iter, epoch, gstep(epoch), writer, cfg, device)
        dist.barrier()
        val_loss, _ = train.validate(model, val_dl, epoch, gstep(epoch + 1), writer, cfg, device)
        dist.barrier()
        if isinstance(lr_scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
            lr_scheduler.step(val_loss)
        if rank == 0:
            os.makedirs(train_dir, exist_ok=True)
            ck = {'epoch': epoch + 1, 'best_metric': val_loss, 'state_dict': model.module.state_dict(),
                  'ema_state_dict': ema_model.state_dict(), 'optimizer': optimizer.state_dict()}
            if fp16:   # extra keys only; the reference's five keys are unchanged
                ck['grad_scaler'] = _scaler_state(optimizer)
            if disc is not None:
                ck['discriminator_state_dict'] = disc.module.state_dict()
                ck['discriminator_optimizer'] = cfg['train']['adversarial']['optimizer'].state_dict()
                if fp16:
                    ck['discriminator_grad_scaler'] = _scaler_state(cfg['train']['adversarial']['optimizer'])
            torch.save(ck, latest)
            if best_metric is None or val_loss < best_metric:
                best_metric = val_loss
                shutil.copy2(latest, os.path.join(train_dir, 'best.pth'))
        dist.barrier()
        if utils.get_max_lr(optimizer) <= tc['min_lr']:
            break


def cleanup():
    dist.destroy_process_group()


def main(cfg_path='configs/c2_unet_r50.py'):
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '15001')
    cfg = config.fromfile(cfg_path)
    os.makedirs(cfg['common']['output_dir'], exist_ok=True)
    shutil.copy2(cfg_path, cfg['common']['output_dir'])
    mp.spawn(distributed_train, args=(cfg_path,), nprocs=cfg['common']['world_size'], join=True)


if __name__ == '__main__':
    import sys
    main(*sys.argv[1:2])
