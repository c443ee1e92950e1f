"""Host logic of the fp16 loss scaler (CPU): the scaler attaches only to ssseg's fused SGD (the only optimizer
that unscales by 1/S and skips a non-finite step), and its state round-trips through a checkpoint dict."""
import pytest
import torch


def test_grad_scaler_refuses_torch_optimizer():
    import distributed_trainer
    m = torch.nn.Linear(4, 2)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    with pytest.raises(NotImplementedError):
        distributed_trainer.attach_grad_scaler(opt, torch.device('cpu'))
    assert getattr(opt, 'grad_scaler', None) is None


def test_grad_scaler_state_roundtrip():
    from ssseg import amp
    a = amp.GradScaler(torch.device('cpu'), init_scale=1024.0, growth_interval=7)
    a.state.copy_(torch.tensor([256.0, 5.0, 0.0, 1.0 / 256.0]))
    sd = a.state_dict()
    b = amp.GradScaler(torch.device('cpu'))
    b.load_state_dict(sd)
    assert torch.equal(a.state, b.state) and b.interval == 7 and b.get_scale() == 256.0
    sd['state'][0] = 1.0     # the saved copy is independent of the live state
    assert a.get_scale() == 256.0
