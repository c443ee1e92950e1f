"""The train step's stream schedule (train.train_step): the teacher pass, the consistency forward and the consistency
backward on a side HIP stream, concurrent with the supervised backward, with every weight / bias gradient of both
backward passes held and replayed after the join (ssseg.nn.hold_wgrad / replay_held).  Reordering across streams
must not change a single bit: the same kernels run on the same operands, and every gradient tensor receives its
writes in the serial schedule's order.  Four steps (the first two always run serially: they autotune) of the C2
UNet-ResNet50 step at a small size, compared bitwise between the serial schedule and each overlap level."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dev, teacher, cons_fwd, cons_bwd, steps=4, size=128, batch=2):
    import cowmix
    import losses
    import train
    from models import unet
    from models.adapters import ListOutput
    from models.encoders import resnet
    from ssseg import arena, optim
    train._OVERLAP.update(teacher=teacher, consistency=cons_fwd, consistency_bwd=cons_bwd)
    train._OVERLAP['seen'].clear()
    cowmix._DEVICE_RNG['ctr'].clear()
    torch.manual_seed(0)
    student = ListOutput(unet.UNet(2, resnet.resnet50_encoder(), max_width=128, train_upsampling=True)).to(dev)
    teacher_m = ListOutput(unet.UNet(2, resnet.resnet50_encoder(), max_width=128, train_upsampling=True)).to(dev)
    teacher_m.load_state_dict(student.state_dict())
    for p in teacher_m.parameters():
        p.detach_()
    teacher_m.eval()
    arena.attach(student)
    arena.attach(teacher_m, with_grads=False)
    opt = optim.SGD(student.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
    cfg = {'train': dict(
        loss=losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits('mean'), 'weight': [0.5]}]),
        virtual_batch_size_multiplier=1, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
        sigma_range=(4, 8), consistency_loss_weight=10, ema_model_alpha=0.99, confidence_threshold=0.5,
        gradient_clip_value=5.0, print_freq=10 ** 9)}
    g = torch.Generator().manual_seed(5)
    recs = []
    student.train()
    opt.zero_grad()
    for step in range(steps):
        img = torch.rand(batch, 3, size, size, generator=g).to(dev)
        fg = (torch.rand(batch, 1, size, size, generator=g) > 0.5).float()
        mask = torch.cat([1 - fg, fg], 1).to(dev)
        ua = torch.rand(batch, 3, size, size, generator=g).to(dev)
        ub = torch.rand(batch, 3, size, size, generator=g).to(dev)
        out = train.train_step(student, teacher_m, opt, img, mask, ua, ub, 30, step, cfg)
        recs.append(torch.stack([t.float() for t in out]).cpu())
    torch.cuda.synchronize()
    return (recs, {k: v.detach().cpu().clone() for k, v in student.state_dict().items()},
            {k: v.detach().cpu().clone() for k, v in teacher_m.state_dict().items()})


def test_overlap_schedules_bitwise(hip_device):
    import train
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    saved = dict(train._OVERLAP)
    try:
        ref = _run(hip_device, False, False, False)
        for mode in ((True, False, False), (True, True, False), (True, True, True)):
            got = _run(hip_device, *mode)
            for k, (a, b) in enumerate(zip(ref[0], got[0])):
                assert torch.equal(a, b), (mode, k, a.tolist(), b.tolist())
            for part, (sa, sb) in (('student', (ref[1], got[1])), ('teacher', (ref[2], got[2]))):
                for key in sa:
                    assert torch.equal(sa[key], sb[key]), (mode, part, key)
    finally:
        train._OVERLAP.clear()
        train._OVERLAP.update(saved)
    assert all(bool(torch.isfinite(x).all()) for x in ref[0])
