"""bench.py's parity leg (BASELINE.json 'mIoU parity'; north_star: logits within 1e-3 relative, argmax labels
bit-exact) at the bench geometry: the UNet-R50 student after a few bf16 training steps at 512^2, validated by the HIP
path in the fp32 parity mode and by the oracle (torch-CPU fp32 restatement of the network, numpy restatement of the
reference metrics, train.py:171-176, metrics.py:1-7, lovasz.py:54-73) on the same weights.  Every argmax flip must
lie inside the tie band |l1 - l0| < 1e-3 * max|l| of the oracle's logits; outside it the labels are bit-exact."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_parity_leg_flips_inside_tie_band(hip_device):
    import bench
    import train
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    model, teacher, opt, cfg = bench.build(2, 512, hip_device)
    data = bench.synthetic_batches(3, 2, 512, hip_device, 0)
    model.train()
    opt.zero_grad()
    for k in range(3):
        train.train_step(model, teacher, opt, *data[k], 30, k, cfg)
    torch.cuda.synchronize()
    out = bench.parity_leg(model, 512, hip_device, n_img=2)
    print(out)
    f32 = out['hip_fp32']
    assert f32['logits_max_err_rel'] <= 1e-3, f32
    assert out['argmax_mismatch_outside_band'] == 0, f32
    assert f32['argmax_mismatch_frac'] <= 1e-4, f32
    assert out['miou_abs_diff_fp32'] <= 1e-2 and out['dice_abs_diff_fp32'] <= 1e-4, out
