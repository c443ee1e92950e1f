"""CPU checks of the drop-in model surface: constructor signatures, parameter names and shapes match
the reference-restating oracle (so reference state_dicts load), and the UNet-R50 architecture has the
FLOP count the survey measured (95.94 GFLOP forward per 512x512 image)."""
import inspect

import pytest
import torch

from oracle import models_ref


def _sd_shapes(m):
    return {k: tuple(v.shape) for k, v in m.state_dict().items()}


def test_unet_r50_names_match_oracle():
    from models import unet
    from models.encoders import resnet
    prod = unet.UNet(2, resnet.resnet50_encoder(), 128, train_upsampling=True)
    ref = models_ref.UNet(2, models_ref.resnet50_encoder(), 128, train_upsampling=True)
    assert _sd_shapes(prod) == _sd_shapes(ref)
    n = sum(p.numel() for p in prod.parameters())
    assert n == 31_419_776          # 31,419,776 fp32 parameters


@pytest.mark.parametrize('up', [True, False])
def test_simple_unet_names_match_oracle(up):
    from models import simple_unet
    prod = simple_unet.UNet(2, 3, 8, 32, train_upsampling=up)
    ref = models_ref.SimpleUNet(2, 3, 8, 32, train_upsampling=up)
    assert _sd_shapes(prod) == _sd_shapes(ref)


def test_constructor_signatures_match_reference_surface():
    from models import simple_unet, unet
    assert list(inspect.signature(unet.UNet.__init__).parameters) == [
        'self', 'num_classes', 'encoder', 'max_width', 'norm_layer', 'train_upsampling']
    assert list(inspect.signature(unet.UpBlock.__init__).parameters) == [
        'self', 'in_channels', 'skip_in_channels', 'out_channels', 'shrink', 'norm_layer', 'train_upsampling']
    assert list(inspect.signature(simple_unet.UNet.__init__).parameters) == [
        'self', 'num_classes', 'num_blocks', 'first_channels', 'max_width', 'norm_layer', 'train_upsampling']


def test_unet_r50_flops_match_survey():
    from torch.utils.flop_counter import FlopCounterMode
    ref = models_ref.UNet(2, models_ref.resnet50_encoder(), 128, train_upsampling=True)
    with torch.device('meta'):
        x = torch.empty(1, 3, 512, 512)
    ref = ref.to('meta')
    with FlopCounterMode(display=False) as fc:
        ref(x)
    assert abs(fc.get_total_flops() / 1e9 - 95.94) < 0.05


def test_reference_state_dict_keys_load_into_product():
    """A checkpoint saved by the reference model tree (oracle restatement) loads strictly."""
    from models import simple_unet
    ref = models_ref.SimpleUNet(2, 3, 8, 32)
    prod = simple_unet.UNet(2, 3, 8, 32)
    prod.load_state_dict(ref.state_dict(), strict=True)


def test_mobilenetv2_encoder_tree_matches_reference_golden():
    """The drop-in MobileNetV2 encoder has the reference's module tree: the G6 state_dict (made by the
    reference mobilenetv2.py) loads strictly, endpoint depths match the reference's."""
    import numpy as np
    import torch
    from models import unet
    from models.encoders import mobilenetv2
    from conftest import golden
    g = golden("model_unet_mbv2_t.npz")
    m = unet.UNet(2, mobilenetv2.mobilenet_v2(width_mult=0.35), 32, train_upsampling=True)
    sd = {k[5:]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith('init.')}
    m.load_state_dict(sd, strict=True)
    assert m.encoder.endpoint_depths == [8, 8, 16, 32, 112]


@pytest.mark.parametrize('tag', ['hardnet', 'disc', 'msdisc', 'msa_hrnet'])
def test_c345_model_trees_reproduce_reference_weights(tag):
    """HarDNet / discriminators / MultiscaleAttention(HRNet): the same seed gives bit-identical weights to the
    reference's module tree (state_dict SHA-256 from golden G6b) — names, shapes, construction and init order."""
    import seeded
    from conftest import golden
    from test_hip_models_c345 import _ctor
    g = golden(f'model2_{tag}.npz')
    ctor, conv_std = _ctor(tag)
    torch.manual_seed(int(g['seed']))
    m = ctor()
    seeded.perturb(m, int(g['seed']) + 1000, conv_std)
    assert seeded.state_sha(m) == str(g['sha'])


def test_c345_parameter_counts_match_survey():
    from functools import partial
    from models import hardnet, higher_hrnet, multiscale_attention
    msa = multiscale_attention.MultiscaleAttention(
        partial(higher_hrnet.get_pose_net, cfg=higher_hrnet.POSE_HIGHER_RESOLUTION_NET), 480, 2)
    assert abs(sum(p.numel() for p in msa.parameters()) / 1e6 - 20.31) < 0.005      # 20.31 M
    assert abs(sum(p.numel() for p in hardnet.HarDNet(n_classes=2).parameters()) / 1e6 - 4.31) < 0.005


@pytest.mark.parametrize('fn', ['deeplabv3_resnet101', 'deeplabv3_resnet50', 'fcn_resnet50'])
def test_deeplab_names_match_oracle(fn):
    from models import deeplabv3
    prod, ref = getattr(deeplabv3, fn)(2), getattr(models_ref, fn)(2)
    assert _sd_shapes(prod) == _sd_shapes(ref)
    assert list(inspect.signature(getattr(deeplabv3, fn)).parameters)[0] == 'num_classes'


def test_deeplabv3_r101_params_and_flops_match_survey():
    from torch.utils.flop_counter import FlopCounterMode
    ref = models_ref.deeplabv3_resnet101(2)
    assert abs(sum(p.numel() for p in ref.parameters()) / 1e6 - 58.63) < 0.005      # 58.63 M
    ref = ref.to('meta').eval()          # eval: ASPP pooling's BN sees one value per channel at batch 1
    with torch.device('meta'):
        x = torch.empty(1, 3, 512, 512)
    with FlopCounterMode(display=False) as fc:
        ref(x)
    assert abs(fc.get_total_flops() / 1e9 - 482.3) < 0.1                           # 482.3 GFLOP
