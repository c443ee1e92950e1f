"""Host-side checks of the loss modules (no GPU): constructor checks mirrored from the reference."""
import pytest


def test_rmi_rejects_unsupported():
    """RMILoss keeps the reference's assertions (losses.py:294-302) and refuses, at construction, the configurations
    the device kernels do not cover (radius > 3, max / interpolation pooling)."""
    import losses as L
    m = L.RMILoss(num_classes=2, rmi_radius=3, rmi_pool='avg', rmi_pool_size=4, rmi_pool_stride=4)
    assert m.pool_params() == (4, 4, 2) and m.half_d == 9
    assert L.RMILoss(num_classes=2, rmi_pool='none', rmi_pool_size=4, rmi_pool_stride=4).pool_params() == (1, 1, 0)
    assert L.RMILoss(num_classes=2, rmi_pool='max', rmi_pool_size=1, rmi_pool_stride=1).pool_params() == (1, 1, 0)
    with pytest.raises(NotImplementedError):
        L.RMILoss(num_classes=2, rmi_radius=4)
    with pytest.raises(NotImplementedError):
        L.RMILoss(num_classes=2, rmi_pool='max', rmi_pool_size=4, rmi_pool_stride=4)
    with pytest.raises(AssertionError):
        L.RMILoss(num_classes=2, rmi_pool_size=4, rmi_pool_stride=3)
    with pytest.raises(AssertionError):
        L.RMILoss(num_classes=2, rmi_radius=11)
