"""The live probe's fence-free timing events (csrc/probe.hip, ssseg.nn.ProbeEvent) used by bench.py's roofline leg:
they time a kernel like torch's default events do (same stream, same interval), and the probe rows they produce
cover every conv-engine launch of a layer."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_probe_event_times_like_torch_event(hip_device):
    from ssseg import nn as snn
    x = torch.randn(4096, 4096, device=hip_device)
    torch.cuda.synchronize()
    p0, p1 = snn.ProbeEvent(), snn.ProbeEvent()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    p0.record()
    torch.cuda._sleep(int(2e7))
    y = x @ x
    p1.record()
    t1.record()
    torch.cuda.synchronize()
    tp, tt = p0.elapsed_time(p1), t0.elapsed_time(t1)
    assert y.shape == x.shape
    assert 0.0 < tp <= tt * 1.05 + 0.05, (tp, tt)
    assert tp >= 0.5 * tt, (tp, tt)


def test_probe_rows_cover_conv_launches(hip_device):
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    conv = snn.Conv2d(64, 64, 3, padding=1, bias=False).to(hip_device)
    x = snn.to_act(torch.randn(2, 64, 32, 32, device=hip_device))
    rows = snn.probe(True)
    y = conv(x)
    snn.probe(False)
    torch.cuda.synchronize()
    assert tuple(y.shape) == (2, 64, 32, 32)
    assert len(rows) >= 1
    for e0, e1, flops, kind, _tag in rows:
        assert isinstance(e0, snn.ProbeEvent)
        assert e0.elapsed_time(e1) > 0.0 and flops > 0
