"""ctypes binding of libvadhip.so (the C ABI in include/vad.h).

There is no fallback: if the library is missing or no HIP device is present, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_LIB = None
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvadhip.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_U32 = ctypes.c_uint32
_F = ctypes.c_float
# int (*vad_bn_sync_fn)(void* user, int bn_layer, int phase, int64_t n, void* stream)
BN_SYNC_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                              ctypes.c_void_p)

_SIGS = {
    "vad_abi_version": (_I, []),
    "vad_last_error": (ctypes.c_char_p, []),
    "vad_rng_u24": (_I, [_U64, _U32, _U64, _I64, _I64, _I64, _P, _P]),
    "vad_synth_frames": (_I, [_U64, _U64, _I64, _I64, _I64, _I, _P, _P]),
    "vad_cad_num_slots": (_I, []),
    "vad_cad_slot_name": (ctypes.c_char_p, [_I]),
    "vad_cad_slot_numel": (_I64, [_I]),
    "vad_cad_slot_offset": (_I64, [_I]),
    "vad_cad_slot_group": (_I, [_I]),
    "vad_cad_param_floats": (_I64, []),
    "vad_cad_num_bufs": (_I, []),
    "vad_cad_buf_name": (ctypes.c_char_p, [_I]),
    "vad_cad_buf_numel": (_I64, [_I]),
    "vad_cad_buf_offset": (_I64, [_I]),
    "vad_cad_buf_floats": (_I64, []),
    "vad_cad_num_bn": (_I, []),
    "vad_cad_create": (_I, [_I, _I, _I, _I, ctypes.POINTER(_P)]),
    "vad_cad_destroy": (None, [_P]),
    "vad_cad_workspace_bytes": (_I64, [_P]),
    "vad_cad_bind": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vad_cad_forward": (_I, [_P, _P, _I, _U64, _U64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vad_cad_backward": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "vad_cad_backward_stage": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "vad_cad_wait_side": (_I, [_P, _P]),
    "vad_cad_wait_layer_grads": (_I, [_P, _I, _P]),
    "vad_cad_input_ready": (_I, [_P, _P]),
    "vad_cad_backward_ext": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vad_cad_optimizer_step": (_I, [_P, _F, _F, _F, _F, _F, _F, _F, _P, _P]),
    "vad_dense_forward": (_I, [_P, _I, _I, _P, _P, _I, _P, _I, _P, _I64, _P]),
    "vad_conv3x3_forward": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _P, _P, _P, _P]),
    "vad_conv3x3_dgrad": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _P, _P, _P, _P]),
    "vad_cad_debug_buffer": (_I, [_P, ctypes.c_char_p, _I, ctypes.POINTER(_P), ctypes.POINTER(_I64)]),
    "vad_cad_set_debug": (_I, [_P, ctypes.c_char_p, _I64]),
    "vad_cad_set_option": (_I, [_P, ctypes.c_char_p, _I64]),
    "vad_cad_conv_path": (_I, [_P, _I, _I]),
    "vad_cad_set_bn_sync": (_I, [_P, BN_SYNC_FN, _P, _I]),
    "vad_u8_to_clip": (_I, [_P, _I64, _I, _P, _P]),
    "vad_host_device_ptr": (_I, [_P, _P]),
    "vad_resize_u8": (_I, [_P, _I, _I, _P, _I, _I]),
    "vad_debug_d2h": (_I, [_P, _P, _I64]),
    "vad_cad_profile": (_I, [_P, _I, ctypes.c_char_p]),
    "vad_cad_profile_read": (_I, [_P, _P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I), _I]),
    "vad_cad_profile_marks": (_I, [_P, _P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), _I]),
    "vad_set_tuning": (_I, [ctypes.c_char_p, _I]),
    "vad_conv3x3_wgrad": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _I64, _P]),
    "vad_bn_bwd_apply": (_I, [_P, _P, _P, _I, _I, _P, _I, _P]),
    # minicausal (config 1)
    "vad_mc_create": (_I, [_I, _I, _I, _I, _I, ctypes.POINTER(_P)]),
    "vad_mc_destroy": (None, [_P]),
    "vad_mc_num_slots": (_I, [_P]),
    "vad_mc_slot_name": (ctypes.c_char_p, [_P, _I]),
    "vad_mc_slot_numel": (_I64, [_P, _I]),
    "vad_mc_slot_offset": (_I64, [_P, _I]),
    "vad_mc_param_floats": (_I64, [_P]),
    "vad_mc_num_bufs": (_I, [_P]),
    "vad_mc_buf_name": (ctypes.c_char_p, [_P, _I]),
    "vad_mc_buf_numel": (_I64, [_P, _I]),
    "vad_mc_buf_offset": (_I64, [_P, _I]),
    "vad_mc_buf_floats": (_I64, [_P]),
    "vad_mc_workspace_bytes": (_I64, [_P]),
    "vad_mc_bind": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vad_mc_forward": (_I, [_P, _P, _I, _U64, _U64, _I64, _P, _P, _P, _P, _P]),
    "vad_mc_backward": (_I, [_P, _P, _P]),
    "vad_mc_optimizer_step": (_I, [_P, _F, _F, _F, _F, _F, _F, _F, _P]),
    # a2 (avenue_training_script2.py)
    "vad_a2_num_slots": (_I, []),
    "vad_a2_slot_name": (ctypes.c_char_p, [_I]),
    "vad_a2_slot_numel": (_I64, [_I]),
    "vad_a2_slot_offset": (_I64, [_I]),
    "vad_a2_param_floats": (_I64, []),
    "vad_a2_create": (_I, [_I, _I, _I, _I, ctypes.POINTER(_P)]),
    "vad_a2_destroy": (None, [_P]),
    "vad_a2_workspace_bytes": (_I64, [_P]),
    "vad_a2_bind": (_I, [_P, _P, _P, _P, _P, _P, _P]),
    "vad_a2_forward": (_I, [_P, _P, _I, _U64, _U64, _I64, _I, _P, _P, _P, _P, _P]),
    "vad_a2_loss": (_I, [_P, _U64, _U64, _I64, _P, _P]),
    "vad_a2_loss_grads": (_I, [_P, _P, _P, _P]),
    "vad_a2_backward": (_I, [_P, _P, _P, _P, _P]),
    "vad_a2_optimizer_step": (_I, [_P, _F, _F, _F, _F, _F, _F, _P]),
    # bbox clip scorer (config 5)
    "vad_bbox_num_slots": (_I, []),
    "vad_bbox_slot_name": (ctypes.c_char_p, [_I]),
    "vad_bbox_slot_numel": (_I64, [_I]),
    "vad_bbox_slot_offset": (_I64, [_I]),
    "vad_bbox_param_floats": (_I64, []),
    "vad_bbox_create": (_I, [_I, _I, _I, _I, ctypes.POINTER(_P)]),
    "vad_bbox_destroy": (None, [_P]),
    "vad_bbox_workspace_bytes": (_I64, [_P]),
    "vad_bbox_bind": (_I, [_P, _P, _P]),
    "vad_bbox_forward": (_I, [_P, _P, _P, _P, _P, _P]),
    # cad1 memory autoencoder (causal_anomaly_detection1.py)
    "vad_ae_num_slots": (_I, []),
    "vad_ae_slot_name": (ctypes.c_char_p, [_I]),
    "vad_ae_slot_numel": (_I64, [_I]),
    "vad_ae_slot_offset": (_I64, [_I]),
    "vad_ae_param_floats": (_I64, []),
    "vad_ae_num_bufs": (_I, []),
    "vad_ae_buf_name": (ctypes.c_char_p, [_I]),
    "vad_ae_buf_numel": (_I64, [_I]),
    "vad_ae_buf_offset": (_I64, [_I]),
    "vad_ae_buf_floats": (_I64, []),
    "vad_ae_create": (_I, [_I, _I, ctypes.POINTER(_P)]),
    "vad_ae_destroy": (None, [_P]),
    "vad_ae_workspace_bytes": (_I64, [_P]),
    "vad_ae_bind": (_I, [_P] * 11),
    "vad_ae_forward": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "vad_ae_backward": (_I, [_P, _I, _P, _P, _P, _P]),
    "vad_ae_optimizer_step": (_I, [_P, _F, _F, _F, _F, _F, _F, _F, _P]),
    "vad_ae_update_memory": (_I, [_P, _P, _P, _I, _P]),
    "vad_ae_memory_score": (_I, [_P, _P, _P, _I, _P, _P]),
    "vad_a2_set_option": (_I, [_P, ctypes.c_char_p, _I64]),
    "vad_ae_debug_buffer": (_I, [_P, ctypes.c_char_p, _I, ctypes.POINTER(_P), ctypes.POINTER(_I64)]),
}


def lib():
    """Load libvadhip.so (after torch, so both share one HIP runtime)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first)
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libvadhip.so is not built ({LIB_PATH}); run __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(L, name)
        except AttributeError:  # (an older build, e.g. an A/B baseline: calling the entry point raises then)
            continue
        fn.restype = res
        fn.argtypes = args
    if L.vad_abi_version() != 1:
        raise RuntimeError("libvadhip ABI mismatch")
    _LIB = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError("libvadhip: " + lib().vad_last_error().decode())


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(device) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def require_hip(t) -> None:
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError("this build runs on MI355X (HIP) devices only; got a tensor on "
                           f"{getattr(t, 'device', type(t))}")


def host_device_ptr(t) -> int:
    """Device address of a pinned host tensor (kernels write it over PCIe; vad_host_device_ptr)."""
    if not t.is_pinned():
        raise ValueError("host_device_ptr: the tensor must be pinned")
    out = ctypes.c_void_p()
    check(lib().vad_host_device_ptr(t.data_ptr(), ctypes.addressof(out)))
    return out.value
