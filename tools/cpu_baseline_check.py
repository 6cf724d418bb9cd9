"""Container-side check that bench.py's CPU baseline (the oracle's train step, oracle/cad_oracle.py) runs at the
reference's own speed: BASELINE.md requires the restatement to reproduce the imported reference's clips/s within
+-15 % before it counts as the baseline.  Imports the reference (build container only; it never travels to the GPU
box) exactly as tests/golden/make_golden.py does, runs its train_model over n config-2 batches (B=8, T=16,
1x227x227), times the oracle step on the same batches with the same threads, and writes the comparison to
profiles/<tag>_cpu_baseline_check.json.

Usage: python tools/cpu_baseline_check.py [--steps 4] [--tag r02]
"""
import argparse
import io
import json
import os
import sys
import time
from contextlib import redirect_stdout

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--tag", default="r02")
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--HW", type=int, default=227)
    args = ap.parse_args()
    import make_golden as mg
    from oracle import cad_oracle as co
    mg._install_stubs()
    cad = mg._load(args.ref, "causal_anomaly_detection.py", "ref_cad")
    B, T, S = args.B, args.T, args.HW
    batches = [(co.synth_clips(7, i, 0, B, T, S, S), co.synth_labels(0, B)) for i in range(args.steps + 1)]
    threads = torch.get_num_threads()

    # the reference: its own train_model (cad:609-790) over the batches, one epoch; the first batch is a warm-up
    torch.manual_seed(0)
    model = cad.CausalAnomalyDetector(num_factors=6, reid_dim=64)
    with redirect_stdout(io.StringIO()):
        cad.train_model(model, batches[:1], [], num_epochs=1, lr=3e-4)
        t0 = time.perf_counter()
        cad.train_model(model, batches[1:], [], num_epochs=1, lr=3e-4)
        ref_s = time.perf_counter() - t0

    # the oracle step on the same batches
    torch.manual_seed(0)
    sd = {k: v.clone() for k, v in cad.CausalAnomalyDetector(num_factors=6, reid_dim=64).state_dict().items()}
    params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v for k, v in sd.items() if "running" in k}
    state = {}
    co.cad_train_step(params, bufs, state, *batches[0], co.CadDraws.make(1, 0, 0, B, T))
    t0 = time.perf_counter()
    for i, (x, y) in enumerate(batches[1:]):
        co.cad_train_step(params, bufs, state, x, y, co.CadDraws.make(1, i + 1, 0, B, T))
    orc_s = time.perf_counter() - t0

    n = args.steps * B
    ref_v, orc_v = n / ref_s, n / orc_s
    out = {"workload": f"train step, B={B} clips x T={T} x 1x{S}x{S} (BASELINE config 2), {args.steps} steps after "
                       f"1 warm-up step",
           "threads": threads, "os_cpu_count": os.cpu_count(),
           "affinity": sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
           "reference_clips_per_s": round(ref_v, 3),
           "oracle_clips_per_s": round(orc_v, 3),
           "oracle_over_reference": round(orc_v / ref_v, 4),
           "within_15pct": abs(orc_v / ref_v - 1.0) <= 0.15,
           "reference_timed": "causal_anomaly_detection.py train_model (cad:609-790) imported with cv2/torchvision/"
                              "seaborn stubs (tests/golden/make_golden.py), per-epoch prints included",
           "oracle_timed": "oracle/cad_oracle.py cad_train_step (bench.py cpu_baseline leg)"}
    path = os.path.join(ROOT, "profiles", f"{args.tag}_cpu_baseline_check.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
