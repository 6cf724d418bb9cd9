import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libvadhip.so")
    config.addinivalue_line("markers", "slow: longer CPU parity cases")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        # VAD_TUNE="knob=v,knob=v": run the GPU suite with library tuning knobs set (A/B of kernel variants)
        for kv in filter(None, os.environ.get("VAD_TUNE", "").split(",")):
            from vad_amd import _native as nat
            k, v = kv.split("=")
            nat.check(nat.lib().vad_set_tuning(k.encode(), int(v)))
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
