"""Golden clip enumeration + labels of the reference datasets (build container only; the reference never travels).

Usage:  python tests/golden/make_dataset_golden.py [--ref /root/reference]

Builds the frame-folder tree of ``tests.golden.cases.DATASET_TREE`` (empty frame files: the reference's
constructors only list names) in a temp dir, runs the reference's own ``UCSDped2Dataset.__init__``
(causal_anomaly_detection.py:39-80) and ``UCSDped2SimpleDataset.__init__`` (minicausal_vad_complete3.py:104-190)
on it, and writes their (folder, frame names, start) sequences and labels to tests/golden/dataset_enum.json.
"""
import argparse
import io
import json
import os
import sys
import tempfile
from contextlib import redirect_stdout

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden.cases import DATASET_TREE, build_dataset_tree  # noqa: E402
from tests.golden.make_golden import _install_stubs, _load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    _install_stubs()
    cad = _load(a.ref, "causal_anomaly_detection.py", "ref_cad")
    mc = _load(a.ref, "minicausal_vad_complete3.py", "ref_mc")
    out = {"tree": DATASET_TREE, "cad": {}, "mc": {}}
    with tempfile.TemporaryDirectory() as root:
        build_dataset_tree(root, empty=True)
        for split in ("Train", "Test"):
            with redirect_stdout(io.StringIO()):
                d = cad.UCSDped2Dataset(root, split=split, transform=None, sequence_length=16)
            out["cad"][split] = {"sequences": [[os.path.basename(f), names, i] for f, names, i in d.sequences],
                                 "labels": [int(v) for v in d.labels]}
            with redirect_stdout(io.StringIO()):
                m = mc.UCSDped2SimpleDataset(root, subset=split, temporal_frames=8, spatial_size=64,
                                             max_clips_per_video=10, stride=4)
            out["mc"][split] = {"clips": [[os.path.relpath(p, root) for p in c] for c in m.video_clips],
                                "labels": [int(v) for v in m.labels]}
    with open(os.path.join(HERE, "dataset_enum.json"), "w") as f:
        json.dump(out, f)
    print("wrote dataset_enum.json:", {k: {s: len(v["labels"]) for s, v in out[k].items()} for k in ("cad", "mc")})


if __name__ == "__main__":
    main()
