"""ctypes binding of libssseg.so (the C ABI declared in include/ssseg.h).

The library is built in-tree (`make -C semi-supervised_semantic_segmentation_amd/csrc`, or
`__graft_entry__.build()`).  There is no fallback: if the library is missing, or a tensor handed to
an op is not on the HIP device, the call raises.
"""
import ctypes
import os
import re

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SSSEG_LIB_PATH') or os.path.join(_HERE, 'libssseg.so')   # override: A/B builds only
HEADER = os.path.join(_HERE, '..', '..', 'include', 'ssseg.h')

F32, BF16, F16, F64 = 0, 1, 2, 3
SSSEG_SUM, SSSEG_AVG = 0, 1
_ERRS = {-1: 'SSSEG_EINVAL', -2: 'SSSEG_EUNSUPPORTED', -3: 'SSSEG_EWORKSPACE', -4: 'SSSEG_ECOMM'}

vp, i64, i32, f32, f64, sz, u64 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                   ctypes.c_size_t, ctypes.c_uint64)
I64P = ctypes.POINTER(ctypes.c_int64)

class CatPart(ctypes.Structure):
    """ssseg_cat_part (include/ssseg.h): one operand of ssseg_nhwc_cat_n / ssseg_nhwc_split_n"""
    _fields_ = [('src', vp), ('dst', vp), ('add', vp), ('ld', i64), ('c', i64)]


def cat_parts(rows):
    """host table of (src, dst, add, ld, c) rows for the concat entry points (kept alive by the caller)"""
    return (CatPart * len(rows))(*[CatPart(*r) for r in rows])


# name -> (restype, argtypes); every entry must match include/ssseg.h
SIGS = {
    'ssseg_version': (ctypes.c_char_p, []),
    'ssseg_cowmix_workspace_bytes': (sz, [i64, i64, i64]),
    'ssseg_cowmix_mask': (i32, [vp, vp, vp, i64, i64, i64, vp, vp, vp, vp, sz, vp]),
    'ssseg_normal_f32': (i32, [vp, i64, u64, u64, vp]),
    'ssseg_mix': (i32, [vp, vp, vp, vp, i64, i64, i64, i32, vp]),
    'ssseg_cowmix_draw': (i32, [vp, vp, vp, i64, i64, f64, f64, f64, f64, u64, u64, vp]),
    'ssseg_cowmix_draw_dev': (i32, [vp, vp, vp, i64, i64, f64, f64, f64, f64, u64, vp, vp]),
    'ssseg_nchw_to_nhwc': (i32, [vp, vp, i64, i64, i64, i64, i64, i32, i32, vp]),
    'ssseg_nhwc_to_nchw': (i32, [vp, vp, i64, i64, i64, i64, i64, i32, i32, vp]),
    'ssseg_cast': (i32, [vp, vp, i64, i32, i32, vp]),
    'ssseg_bilinear_fwd': (i32, [vp, vp, i64, i64, i64, i64, i64, i64, I64P, I64P, i32, i32, vp]),
    'ssseg_bilinear_bwd': (i32, [vp, vp, i64, i64, i64, i64, i64, i64, I64P, I64P, i32, i32, vp]),
    'ssseg_bilinear_bwd_workspace_bytes': (sz, [i64, i64, i64, i64]),
    'ssseg_bilinear_bwd_ws': (i32, [vp, vp, i64, i64, i64, i64, i64, i64, I64P, I64P, i32, i32, vp, sz, vp]),
    'ssseg_aug_warp': (i32, [vp, vp, i64, i64, i64, i64, vp, vp, i64, i64, vp, vp, vp, i32, vp]),
    'ssseg_aug_color': (i32, [vp, i64, i64, i64, vp, vp]),
    'ssseg_aug_blur': (i32, [vp, vp, i64, i64, i64, i64, vp, vp, i64, i32, i32, vp]),
    'ssseg_aug_iso_finish': (i32, [vp, vp, i64, i64, i64, vp, vp, u64, vp]),
    'ssseg_aug_uniform_field': (i32, [vp, i64, u64, vp]),
    'ssseg_rotate_fwd': (i32, [vp, vp, i64, i64, i64, i64, f64, vp]),
    'ssseg_rotate_bwd': (i32, [vp, vp, i64, i64, i64, i64, f64, vp]),
    'ssseg_reduce_workspace_bytes': (sz, [i64]),
    'ssseg_bce_logits_fwd': (i32, [vp, vp, i64, vp, vp, sz, vp]),
    'ssseg_bce_logits_bwd': (i32, [vp, vp, i64, vp, vp, vp]),
    'ssseg_consistency_fwd': (i32, [vp, vp, i64, i64, i64, f32, vp, vp, sz, vp]),
    'ssseg_consistency_bwd': (i32, [vp, vp, i64, i64, i64, f32, vp, vp, vp, vp]),
    'ssseg_lovasz_workspace_bytes': (sz, [i64, i64]),
    'ssseg_lovasz_fwd': (i32, [vp, vp, i64, i64, i64, vp, vp, sz, vp]),
    'ssseg_lovasz_bwd': (i32, [vp, vp, i64, i64, i64, vp, vp, vp, sz, vp]),
    'ssseg_lovasz_bwd_from_fwd': (i32, [vp, vp, i64, i64, i64, vp, vp, vp, sz, vp]),
    'ssseg_rmi_workspace_bytes': (sz, [i64] * 9),
    'ssseg_rmi_fwd': (i32, [vp, vp] + [i64] * 9 + [i32, vp, vp, sz, vp]),
    'ssseg_rmi_bwd': (i32, [vp] + [i64] * 9 + [vp, vp, vp, sz, vp]),
    'ssseg_prob_onehot': (i32, [vp, i64, i64, vp, vp, vp]),
    'ssseg_seg_metrics': (i32, [vp, I64P, i64, i64, vp, I64P, i64, i64, i64, vp, vp, vp, vp]),
    'ssseg_ema_update': (i32, [vp, vp, i64, f64, vp]),
    'ssseg_scale_f32': (i32, [vp, i64, f32, vp]),
    'ssseg_axpby': (i32, [vp, f32, vp, f32, vp, i64, vp]),
    'ssseg_sigmoid_fwd': (i32, [vp, vp, i64, vp]),
    'ssseg_sigmoid_bwd': (i32, [vp, vp, vp, i64, vp]),
    'ssseg_sqnorm_accum': (i32, [vp, i64, vp, vp, sz, vp]),
    'ssseg_sgd_step': (i32, [vp, vp, vp, vp, i64, f32, f32, f32, f32, vp, i32, vp, vp]),
    'ssseg_amp_update': (i32, [vp, vp, f32, f32, i32, vp]),
    'ssseg_scale_by': (i32, [vp, vp, vp, i64, vp]),
    # convolution engine
    'ssseg_conv_igemm': (i32, [vp, vp, vp, vp, i32, i32, vp, i32, vp, sz, vp]),
    'ssseg_conv_igemm_phases': (i32, [vp, vp, vp, i32, i32, vp, i64, vp, vp, vp]),
    'ssseg_conv_igemm_phases_ws': (i32, [vp, vp, vp, i32, i32, vp, i64, vp, vp, vp, sz, vp]),
    'ssseg_conv_igemm_phases_workspace_bytes': (sz, [vp, i64, i32]),
    'ssseg_conv_stem_epi': (i32, [vp, vp, vp, vp, i32, vp, vp]),
    'ssseg_conv_igemm_epi': (i32, [vp, vp, vp, vp, i32, i32, vp, vp, sz, vp]),
    'ssseg_conv_igemm_epi_actmask': (i32, [vp, vp, vp, vp, i32, i32, vp, i32, f32, vp, sz, vp]),
    'ssseg_weight_pack_batch': (i32, [vp, i64, i32, vp]),
    'ssseg_dwconv_fwd': (i32, [vp, vp, vp, vp, i32, vp, vp]),
    'ssseg_dwconv_dgrad': (i32, [vp, vp, vp, vp, i32, vp]),
    'ssseg_dwconv_wgrad_workspace_bytes': (sz, [vp, i32]),
    'ssseg_dwconv_wgrad': (i32, [vp, vp, vp, vp, i32, i64, i32, vp, sz, vp]),
    'ssseg_conv_igemm_workspace_bytes': (sz, [vp, i32]),
    'ssseg_set_knob': (i32, [i32, i32]),
    'ssseg_tune_table_export': (i64, [vp, vp, i64]),
    'ssseg_tune_table_import': (i32, [vp, vp, i64, i32]),
    'ssseg_conv_wgrad_workspace_bytes': (sz, [vp, i32]),
    'ssseg_conv_wgrad': (i32, [vp, vp, vp, vp, i32, i64, i64, i32, i32, vp, sz, vp]),
    'ssseg_conv_wgrad2_workspace_bytes': (sz, [vp, i64, i32]),
    'ssseg_wgrad_defer_reduce': (i32, [i32]),
    'ssseg_wgrad_reduce_pending': (i64, []),
    'ssseg_wgrad_reduce_flush': (i32, [vp]),
    'ssseg_conv_wgrad2': (i32, [vp, vp, vp, vp, i64, vp, vp, i32, i64, i64, i32, i32, vp, sz, vp]),
    # virtual concat inputs (ssseg_vcat)
    'ssseg_conv_igemm_epi_vcat': (i32, [vp, vp, vp, vp, vp, i32, i32, vp, vp, sz, vp]),
    'ssseg_conv_igemm_epi_vsplit': (i32, [vp, vp, vp, vp, vp, i32, i32, vp, vp, sz, vp]),
    'ssseg_conv_wgrad_vcat': (i32, [vp, vp, vp, vp, vp, i32, i64, i64, i32, i32, vp, sz, vp]),
    'ssseg_conv_wgrad2_vcat': (i32, [vp, vp, vp, vp, vp, vp, i64, vp, vp, i32, i64, i64, i32, i32, vp, sz, vp]),
    'ssseg_weight_pack': (i32, [vp, vp, i64, i64, i64, i64, i64, i64, i32, i64, i64, i64, i64, i64, i64, i32, vp]),
    # batch norm
    'ssseg_bn_workspace_bytes': (sz, [i64]),
    'ssseg_bn_stats': (i32, [vp, i64, i64, i64, i32, vp, vp, sz, vp]),
    'ssseg_bn_partials_finalize': (i32, [vp, i64, i64, vp, f64, f32, f32, vp, vp, vp, vp, vp, vp]),
    'ssseg_bn_gstat_finalize': (i32, [vp, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    'ssseg_bn_gstat_finalize_x': (i32, [vp, i64, i64, vp, vp, vp, vp, vp, i64, i64, i32, vp, vp, vp, vp, vp]),
    'ssseg_channel_sum_grad': (i32, [vp, i64, i64, i64, i32, vp, vp, vp, sz, vp]),
    'ssseg_bn_finalize': (i32, [vp, i64, f64, f32, f32, vp, vp, vp, vp, vp, vp]),
    'ssseg_bn_eval_params': (i32, [vp, vp, f32, i64, vp, vp, vp]),
    'ssseg_bn_fold': (i32, [vp, vp, vp, vp, vp, f32, i64, i64, vp, vp, vp, vp, vp]),
    'ssseg_bn_fold_batch': (i32, [vp, i64, vp]),
    'ssseg_bn_eval_bwd': (i32, [vp, vp, vp, vp, vp, i64, i64, i64, vp, vp, vp, i32, i32, vp, vp, sz, vp]),
    'ssseg_bn_eval_bwd_grad_y': (i32, [vp, vp, vp, vp, i64, i64, i64, vp, vp, vp, vp, i32, i32, vp, vp, sz, vp, vp, vp,
                                      vp]),
    'ssseg_bn_eval_bwd_grad': (i32, [vp, vp, vp, vp, vp, i64, i64, i64, vp, vp, vp, i32, i32, vp, vp, sz, vp, vp,
                                      vp, vp]),
    'ssseg_bn_eval_param_grad': (i32, [vp, i64, vp, vp, vp, vp, vp]),
    'ssseg_bn_eval_bwd_part': (i32, [vp, vp, vp, vp, vp, i64, i64, i64, vp, vp, vp, vp, i32, i32, vp, sz, I64P, vp]),
    'ssseg_bn_param_grad_batch': (i32, [vp, i64, i64, vp]),
    'ssseg_bn_apply': (i32, [vp, vp, vp, i64, i64, i64, i64, i64, vp, vp, vp, vp, i32, i32, vp]),
    'ssseg_bn_bwd_reduce': (i32, [vp, vp, vp, i64, i64, i64, i64, i64, vp, vp, vp, vp, i32, i32, vp, vp, sz, vp]),
    'ssseg_bn_param_grad': (i32, [vp, i64, vp, vp, vp]),
    'ssseg_bn_bwd_reduce_grad': (i32, [vp, vp, vp, i64, i64, i64, i64, i64, vp, vp, vp, vp, i32, i32, vp, vp, sz, vp,
                                        vp, vp]),
    'ssseg_bn_stats_finalize': (i32, [vp, i64, i64, i64, i32, vp, vp, sz, f64, f32, f32, vp, vp, vp, vp, vp, vp]),
    'ssseg_bn_bwd_apply': (i32, [vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, vp, vp, vp, vp, i32, i32, vp, f64,
                                 i32, vp]),
    # pooling / copies
    'ssseg_maxpool_fwd': (i32, [vp, vp, vp, i64, i64, i64, i64, i64, i64, i64, i64, i64, i32, vp]),
    'ssseg_maxpool_bwd': (i32, [vp, vp, vp, i64, i64, i64, i64, i64, i64, i64, i64, i64, i32, vp]),
    'ssseg_maxpool_bwd_res': (i32, [vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, i64, i64, i64, i32, vp]),
    'ssseg_nhwc_copy': (i32, [vp, vp, i64, i64, i64, i64, i64, i64, i64, i64, i64, i64, i64, i64, i64, i64, i32, vp]),
    'ssseg_zero': (i32, [vp, sz, vp]),
    'ssseg_nhwc_cat_n': (i32, [vp, i64, vp, i64, i64, i32, vp]),
    'ssseg_nhwc_split_n': (i32, [vp, i64, vp, i64, i64, i32, vp]),
    'ssseg_act_bwd': (i32, [vp, vp, vp, i64, i32, f32, i32, vp]),
    'ssseg_relu_bwd': (i32, [vp, vp, vp, i64, i32, vp]),
    # pooling / elementwise primitives of the C3-C5 model families (csrc/pool.hip)
    'ssseg_avgpool_fwd': (i32, [vp, vp, i64, i64, i64, i64, i64, i64, i64, i64, i64, i32, vp]),
    'ssseg_avgpool_bwd': (i32, [vp, vp, i64, i64, i64, i64, i64, i64, i64, i64, i64, i32, vp]),
    'ssseg_global_avgpool_workspace_bytes': (sz, [i64, i64, i64]),
    'ssseg_global_avgpool_fwd': (i32, [vp, vp, i64, i64, i64, i64, i32, vp, sz, vp]),
    'ssseg_global_avgpool_bwd': (i32, [vp, vp, i64, i64, i64, i64, i32, vp]),
    'ssseg_add_n': (i32, [ctypes.POINTER(ctypes.c_void_p), i32, vp, i64, i32, f32, i32, vp]),
    'ssseg_dropout': (i32, [vp, vp, i64, f32, u64, u64, i32, vp]),
    'ssseg_dropout_dev': (i32, [vp, vp, i64, f32, u64, vp, i32, vp]),
    'ssseg_rng_take': (i32, [vp, vp, u64, vp]),
    'ssseg_att_blend_fwd': (i32, [vp, I64P, vp, I64P, vp, I64P, vp, i64, i64, i64, i64, vp]),
    'ssseg_att_blend_bwd': (i32, [vp, I64P, vp, I64P, vp, I64P, vp, I64P, vp, vp, vp, i64, i64, i64, i64, vp]),
    # collectives (csrc/comm.hip; ssseg/comm.py)
    'ssseg_comm_unique_id_bytes': (sz, []),
    'ssseg_comm_get_unique_id': (i32, [vp]),
    'ssseg_comm_init': (i32, [ctypes.POINTER(ctypes.c_void_p), vp, i32, i32, i32]),
    'ssseg_comm_destroy': (i32, [vp]),
    'ssseg_comm_async_error': (i32, [vp]),
    'ssseg_comm_last_error': (ctypes.c_char_p, []),
    'ssseg_allreduce_buckets': (i32, [vp, ctypes.POINTER(ctypes.c_void_p), I64P, i64, i32, i32, vp]),
    # probe timing events (csrc/probe.hip)
    'ssseg_probe_event_create': (i32, [ctypes.POINTER(ctypes.c_void_p)]),
    'ssseg_probe_event_record': (i32, [vp, vp]),
    'ssseg_probe_event_elapsed': (i32, [vp, vp, ctypes.POINTER(ctypes.c_float)]),
    'ssseg_probe_event_destroy': (i32, [vp]),
}


class ConvDesc(ctypes.Structure):
    """Mirror of ssseg_conv_desc (include/ssseg.h)."""
    _fields_ = [(n, ctypes.c_int64) for n in (
        'N', 'H', 'W', 'C', 'ldx', 'OH', 'OW', 'K', 'R', 'S', 'sy', 'sx', 'dy', 'dx', 'py', 'px',
        'outH', 'outW', 'osy', 'osx', 'ooy', 'oox', 'ldy', 'ldw')]


class ConvEpilogue(ctypes.Structure):
    """Mirror of ssseg_conv_epilogue (include/ssseg.h)."""
    _fields_ = [('scale', ctypes.c_void_p), ('shift', ctypes.c_void_p), ('residual', ctypes.c_void_p),
                ('ldr', ctypes.c_int64), ('aux', ctypes.c_void_p), ('relu', ctypes.c_int32), ('slope', ctypes.c_float),
                ('stats', ctypes.c_void_p), ('stats_ld', ctypes.c_int64), ('stats_rows', ctypes.c_void_p)]


class VCat(ctypes.Structure):
    """Mirror of ssseg_vcat (include/ssseg.h): second source of a virtual channel concat."""
    _fields_ = [('x2', ctypes.c_void_p), ('c1', ctypes.c_int64), ('ldx2', ctypes.c_int64)]


_lib = None


def header_symbols():
    """Function names declared in include/ssseg.h."""
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(ssseg_[a-z0-9_]+)\s*\(', text)))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'ssseg: native library not built ({LIB_PATH}); run __graft_entry__.build() '
                               'or make -C semi-supervised_semantic_segmentation_amd/csrc. There is no CPU fallback.')
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        # engine knobs for experiments, e.g. SSSEG_KNOBS="11=1,10=50" (ssseg_set_knob id=value pairs)
        for kv in filter(None, os.environ.get('SSSEG_KNOBS', '').split(',')):
            k, v = kv.split('=')
            if L.ssseg_set_knob(int(k), int(v)) != 0:
                raise ValueError(f'SSSEG_KNOBS: bad knob {kv!r}')
    return _lib


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f'ssseg: {name} failed with {_ERRS.get(rc, "hipError " + str(rc))}')


EUNSUPPORTED = -2


def call_or_unsupported(name, *args):
    """call(), except that SSSEG_EUNSUPPORTED is returned (False) instead of raised: the caller has another way."""
    rc = getattr(lib(), name)(*args)
    if rc == EUNSUPPORTED:
        return False
    if rc != 0:
        raise RuntimeError(f'ssseg: {name} failed with {_ERRS.get(rc, "hipError " + str(rc))}')
    return True


def stream():
    return torch.cuda.current_stream().cuda_stream


def dev_ptr(t, name='tensor'):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError(f'ssseg: {name} must be a HIP device tensor (no CPU fallback), got {t.device}')
    return t.data_ptr()


def dt_code(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float16:
        return F16
    raise RuntimeError(f'ssseg: unsupported dtype {t.dtype}')


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def strides4(t):
    arr = (ctypes.c_int64 * 4)(*t.stride())
    return arr
