"""CPU-side checks of the C-ABI boundary: the library loads and exports every declared symbol."""
import ctypes

from ssseg import native


def test_library_exports_every_header_symbol():
    lib = native.lib()
    declared = native.header_symbols()
    assert len(declared) >= 10
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, f'declared in include/ssseg.h but not exported: {missing}'


def test_ctypes_table_matches_header():
    declared = set(native.header_symbols())
    bound = set(native.SIGS)
    assert declared == bound, f'header-only: {declared - bound}, binding-only: {bound - declared}'


def test_version_and_host_side_validation():
    lib = native.lib()
    assert lib.ssseg_version().decode().startswith('ssseg')
    assert lib.ssseg_cowmix_workspace_bytes(16, 512, 512) > 16 * 512 * 512 * 4
    # argument errors are detected on the host (no device touched): null pointers -> SSSEG_EINVAL
    assert lib.ssseg_mix(None, None, None, None, 1, 1, 1, 0, None) == -1
    assert lib.ssseg_cowmix_mask(None, None, None, 1, 8, 8, None, None, None, None, 0, None) == -1
    assert lib.ssseg_ema_update(None, None, 4, ctypes.c_double(0.99), None) == -1


def test_ops_refuse_cpu_tensors():
    import pytest
    import torch
    from ssseg import ops
    x = torch.zeros(1, 2, 4, 4)
    with pytest.raises(RuntimeError, match='HIP device tensor'):
        ops.bce_with_logits_mean(x, x)
