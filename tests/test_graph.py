"""The captured training step (ssseg.graph.StepGraph, bench.py's default execution): replaying the HIP graph of one
C2 step (UNet-R50, mean teacher + CowMix, teacher pass on a side stream) gives BIT-identical losses, parameters, BN
running statistics and teacher weights to the same steps issued eagerly -- the graph holds the same kernels, and the
CowMix draws advance a device-side Philox counter (ssseg_cowmix_draw_dev) instead of a host offset."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graphed, device, steps=3, size=64, batch=2):
    import bench
    import cowmix
    import train
    from ssseg.graph import StepGraph
    model, teacher, opt, cfg = bench.build(batch, size, device)
    data = bench.synthetic_batches(steps + 2, batch, size, device, 0)
    for c in cowmix._DEVICE_RNG['ctr'].values():
        c.zero_()
    model.train()
    opt.zero_grad()
    # eager steps 0 and 1: step 0 tunes every conv geometry and registers the conv/BN pairs, step 1 builds the
    # teacher's BN fold table (host -> device, not capturable)
    losses = [train.train_step(model, teacher, opt, *data[k], 30, k, cfg) for k in range(2)]
    if graphed:
        g = StepGraph(lambda i, m, a, b: train.train_step(model, teacher, opt, i, m, a, b, 30, 2, cfg), *data[2])
        for k in range(2, steps + 2):
            losses.append(tuple(t.clone() for t in g(*data[k])))
    else:
        for k in range(2, steps + 2):
            losses.append(train.train_step(model, teacher, opt, *data[k], 30, k, cfg))
    torch.cuda.synchronize()
    state = {**{'s.' + k: v.detach().clone() for k, v in model.state_dict().items()},
             **{'t.' + k: v.detach().clone() for k, v in teacher.state_dict().items()}}
    return [tuple(float(t) for t in l) for l in losses], state


def test_graph_replay_matches_eager_bitwise(hip_device):
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    eager, s_e = _run(False, hip_device)
    graph, s_g = _run(True, hip_device)
    assert eager == graph, (eager, graph)
    assert all(torch.isfinite(torch.tensor(l)).all() for l in eager)
    for k in s_e:
        assert torch.equal(s_e[k], s_g[k]), k
