"""ctypes binding of libcnf_hip.so (include/cnf.h).

This is the reference-side binding a Python caller uses: every entry point of the C ABI is
declared here with its argument types. The library is REQUIRED: there is no CPU fallback on
the product path; a missing or unloadable library raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
# CNF_LIB: load an alternative build of the same library (kernel-variant experiments)
LIB_PATH = Path(os.environ['CNF_LIB']) if os.environ.get('CNF_LIB') else _PKG / 'lib' / 'libcnf_hip.so'


class cnf_flow_desc(C.Structure):
    _fields_ = [('io_h', C.c_int), ('io_w', C.c_int), ('io_d', C.c_int), ('x_d', C.c_int),
                ('num_blocks', C.c_int),
                ('squeeze_factor_block_list', C.POINTER(C.c_int)),
                ('resnext_block_list', C.POINTER(C.c_int)),
                ('num_kernels_list', C.POINTER(C.c_int)),
                ('cardinality_list', C.POINTER(C.c_int)),
                ('lambda_y', C.c_float), ('ksize', C.c_int), ('layer_norm', C.c_int),
                ('dilations', C.c_int), ('group_mode', C.c_int), ('debug_options', C.c_char_p)]


class cnf_layer_info(C.Structure):
    _fields_ = [('kind', C.c_int), ('coupling_index', C.c_int), ('block', C.c_int),
                ('h', C.c_int), ('w', C.c_int), ('d', C.c_int), ('mask', C.c_int),
                ('hc', C.c_int), ('wc', C.c_int), ('dc1', C.c_int), ('dc2', C.c_int),
                ('num_kernels', C.c_int), ('cardinality', C.c_int), ('num_res_blocks', C.c_int),
                ('num_dilations', C.c_int), ('dilations', C.c_int * 8), ('num_prev_factors', C.c_int),
                ('fused_net', C.c_int)]


class cnf_toy_desc(C.Structure):
    _fields_ = [('io_shape', C.c_int), ('x_d', C.c_int), ('num_coupling_layers', C.c_int),
                ('intermediate_dims', C.c_int), ('num_layers', C.c_int), ('mask_indices', C.POINTER(C.c_int)),
                ('lambda_y', C.c_float)]


# per-layer completion callback of cnf_flow_backward_ex (void (*)(void* user, int coupling_index))
LAYER_DONE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int)

# (name, restype, argtypes)
_P = C.c_void_p
_F = C.c_void_p   # device float* as integer address
_SIGS = [
    ('cnf_plan_create', C.c_int, [C.POINTER(cnf_flow_desc), C.POINTER(_P)]),
    ('cnf_plan_destroy', None, [_P]),
    ('cnf_plan_num_layers', C.c_int, [_P]),
    ('cnf_plan_layer_info', C.c_int, [_P, C.c_int, C.POINTER(cnf_layer_info)]),
    ('cnf_plan_num_params', C.c_int64, [_P]),
    ('cnf_plan_num_param_tensors', C.c_int, [_P]),
    ('cnf_plan_param_tensor', C.c_int, [_P, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int64),
                                        C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ('cnf_plan_aux_floats', C.c_int64, [_P]),
    ('cnf_pack_params', C.c_int, [_P, _F, _F, _P]),
    ('cnf_plan_workspace_bytes', C.c_size_t, [_P, C.c_int]),
    ('cnf_flow_forward', C.c_int, [_P, _F, _F, _F, _F, _F, _P, C.c_int, _P]),
    ('cnf_flow_forward_noise', C.c_int, [_P, _F, _F, _F, C.c_float, C.c_float, C.c_uint64, C.c_uint64, _F, _F, _F, _P,
                                         C.c_int, _P]),
    ('cnf_flow_inverse', C.c_int, [_P, _F, _F, _F, _F, _P, C.c_int, _P]),
    ('cnf_coupling_forward', C.c_int, [_P, C.c_int, _F, _F, _F, _F, _F, _P, C.c_int, _P]),
    ('cnf_coupling_inverse', C.c_int, [_P, C.c_int, _F, _F, _F, _F, _P, C.c_int, _P]),
    ('cnf_squeeze', C.c_int, [_F, _F, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P]),
    ('cnf_channel_copy', C.c_int, [_F, C.c_int, C.c_int, _F, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, _P]),
    ('cnf_nll', C.c_int, [_P, _F, _F, _F, _F, _F, C.c_int, _P]),
    ('cnf_plan_train_workspace_bytes', C.c_size_t, [_P, C.c_int]),
    ('cnf_flow_forward_train', C.c_int, [_P, _F, _F, _F, _F, _F, _P, C.c_int, _P]),
    ('cnf_flow_backward', C.c_int, [_P, _F, _F, _F, _P, C.c_int, C.c_float, _F, _P]),
    ('cnf_flow_backward_ex', C.c_int, [_P, _F, _F, _F, _P, C.c_int, _F, _F, LAYER_DONE_FN, _P, _P]),
    ('cnf_coupling_backward', C.c_int, [_P, C.c_int, _F, _F, _F, _F, C.c_float, _P, C.c_int, _F, _P]),
    ('cnf_adam_step', C.c_int, [_F, _F, _F, _F, C.c_int64, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int,
                                _P]),
    ('cnf_toy_num_params', C.c_int64, [C.POINTER(cnf_toy_desc)]),
    ('cnf_toy_call', C.c_int, [C.POINTER(cnf_toy_desc), _F, _F, _F, _F, _F, C.c_int, C.c_int, _P]),
    ('cnf_toy_nll_sums', C.c_int, [_F, _F, C.c_int, _P]),
    ('cnf_logit', C.c_int, [_F, _F, C.c_int64, C.c_float, C.c_int, _P]),
    ('cnf_sr_preprocess', C.c_int, [_F, _F, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P]),
    ('cnf_down', C.c_int, [_F, _F, C.c_int, C.c_int, C.c_int, C.c_int, _P]),
    ('cnf_up', C.c_int, [_F, _F, C.c_int, C.c_int, C.c_int, C.c_int, _P]),
    ('cnf_instance_noise', C.c_int, [_F, _F, C.c_int64, C.c_float, C.c_uint64, C.c_uint64, _P]),
    ('cnf_plan_num_recorded_launches', C.c_int, [_P]),
    ('cnf_plan_recorded_launch_info', C.c_int, [_P, C.c_int, C.c_char_p, C.c_int,
                                                C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ('cnf_plan_relaunch', C.c_int, [_P, C.c_int, _P]),
    ('cnf_plan_set_launch_timing', C.c_int, [_P, C.c_int]),
    ('cnf_plan_launch_time_ms', C.c_int, [_P, C.c_int, C.POINTER(C.c_float)]),
    ('cnf_plan_weight_map', C.c_int64, [_P, C.c_int, C.POINTER(C.c_int64), C.c_int64]),
    ('cnf_comm_unique_id', C.c_int, [C.c_char_p]),
    ('cnf_comm_init', C.c_int, [C.c_int, C.c_int, C.c_char_p, C.POINTER(_P)]),
    ('cnf_comm_destroy', None, [_P]),
    ('cnf_allreduce_sum_f32', C.c_int, [_P, _F, C.c_size_t, _P]),
    ('cnf_nll_allreduce', C.c_int, [_P, _F, C.c_int, _F, _P]),
    ('cnf_last_error', C.c_char_p, []),
    ('cnf_version', C.c_char_p, []),
]

EXPORTED_SYMBOLS = [s[0] for s in _SIGS]

_lib = None


class CnfError(RuntimeError):
    pass


def load(path: os.PathLike | str | None = None):
    """Load libcnf_hip.so (raises if absent: the HIP path is mandatory)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise CnfError(f'{p} is missing: build it with `python -m arl_conditional_normalizing_flows_amd._build` '
                       f'(hipcc --offload-arch=gfx950). There is no CPU fallback.')
    lib = C.CDLL(str(p))
    for name, res, args in _SIGS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str = ''):
    if rc != 0:
        if rc == -1:
            raise AssertionError(f'{what}: {load().cnf_last_error().decode()}')
        raise CnfError(f'{what} failed ({rc}): {load().cnf_last_error().decode()}')


def ptr(t) -> int:
    """device pointer of a contiguous torch tensor (or None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()
