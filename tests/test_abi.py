"""C ABI checks that need no GPU: the library loads, exports every function include/vad.h declares, its slot
table matches the drop-in module's parameters, and errors come back as codes + text."""
import ctypes
import os
import re

import numpy as np
import torch

from oracle import rng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "vad.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vad_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from vad_amd import _native
    L = _native.lib()
    names = _declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert L.vad_abi_version() == 1


def test_slot_table_matches_module():
    from vad_amd import _native
    from vad_amd.cad import CausalAnomalyDetector
    L = _native.lib()
    torch.manual_seed(0)
    m = CausalAnomalyDetector()
    named = list(m.named_parameters())
    assert L.vad_cad_num_slots() == len(named)
    off_prev = -1
    for i, (k, p) in enumerate(named):
        assert L.vad_cad_slot_name(i).decode() == k
        assert L.vad_cad_slot_numel(i) == p.numel()
        off = L.vad_cad_slot_offset(i)
        assert off % 256 == 0 and off > off_prev
        off_prev = off
    assert L.vad_cad_param_floats() >= off_prev + named[-1][1].numel()
    bufs = [k for k in m.state_dict() if "running" in k]
    assert [L.vad_cad_buf_name(i).decode() for i in range(L.vad_cad_num_bufs())] == bufs
    groups = {L.vad_cad_slot_name(i).decode(): L.vad_cad_slot_group(i) for i in range(len(named))}
    assert groups["backbone.conv1.weight"] == 0 and groups["structure_learner.structure_params"] == 4
    assert groups["detector.detector_net.0.weight"] == 2 and groups["structure_learner.node_encoder.weight"] == 3


def test_ae_slot_table_matches_module():
    """cad1 VideoAutoEncoder: library slots = named_parameters(), buffers = the BN running stats in state_dict order."""
    from vad_amd import _native
    from vad_amd.ae import VideoAutoEncoder
    L = _native.lib()
    torch.manual_seed(0)
    m = VideoAutoEncoder()
    named = list(m.named_parameters())
    assert L.vad_ae_num_slots() == len(named)
    for i, (k, p) in enumerate(named):
        assert L.vad_ae_slot_name(i).decode() == k
        assert L.vad_ae_slot_numel(i) == p.numel()
        assert L.vad_ae_slot_offset(i) % 256 == 0
    assert [L.vad_ae_buf_name(i).decode() for i in range(L.vad_ae_num_bufs())] == \
        [k for k in m.state_dict() if "running" in k]
    h = ctypes.c_void_p()
    assert L.vad_ae_create(501, 8, ctypes.byref(h)) != 0  # update_memory writes B rows of the 500-row ring
    assert b"unsupported shape" in L.vad_last_error()


def test_error_codes_and_text():
    from vad_amd import _native
    L = _native.lib()
    h = ctypes.c_void_p()
    rc = L.vad_cad_create(0, 16, 227, 227, ctypes.byref(h))
    assert rc != 0
    assert b"unsupported shape" in L.vad_last_error()


def test_rng_contract_properties():
    keep = rng.dropout_keep(1, rng.S_DET_DROP1, 0, 0, 512, 512, 0.3)
    assert abs(keep.mean() - 0.7) < 0.01
    eps = rng.normal_eps(1, rng.S_EPS, 0, 0, 256, 256)
    assert abs(eps.mean()) < 0.02 and abs(eps.std() - 1) < 0.02
    a = rng.u24(5, 2, 3, np.arange(4), np.arange(7))
    b = rng.u24(5, 2, 3, np.arange(4), np.arange(7))
    assert (a == b).all() and a.max() < (1 << 24)
    assert not (rng.u24(5, 2, 4, np.arange(4), np.arange(7)) == a).all()  # the step changes the draws
    px = rng.pixels_u8(0, 0, 0, 2, 4096)
    assert px.dtype == np.uint8 and px.min() == 0 and px.max() == 255
