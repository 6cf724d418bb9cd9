"""Training-throughput benchmark of the MI355X hot path (BASELINE.json config 2 / 3).

One "step" = one fused train step of CausalAnomalyDetector (causal_anomaly_detection.py:669-690): forward
(backbone, detector, causal head, direct classifier), the multi-term loss, backward, clip_grad_norm_(1.0) and
AdamW — all in libvadhip kernels — on B=8 synthetic Avenue/UCSD-shaped clips of T=16 frames, 1x227x227, per GPU.
Data parallel for --gpus N > 1 (launched by torch.distributed.run): 8 clips per rank, gradients summed over
RCCL; value = all clips processed / max-over-ranks wall time (weak scaling).

Prints ONE JSON line (rank 0).  `roofline` covers the dominant kernel family of the step, timed live with HIP
events inside the timed region; `cpu_baseline` times the CPU oracle (oracle/cad_oracle.py, a port of the
reference step) on this host's cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "training clips/sec (B×T frames) at 1/2/4/8 MI355X; frame-AUC parity vs CPU ref"
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector == FP32 matrix peak
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
# fp32-equivalent peak of a kernel by products per bf16 K step (vad_cad_conv_path): split-bf16 runs six bf16 MFMA
# products per fp32 product, bf16-operand mode one, the f32 MFMA kernels run at the fp32 peak
PATH_PEAK = {6: PEAK_BF16_TFLOPS / 6, 2: PEAK_BF16_TFLOPS, 1: PEAK_BF16_TFLOPS, 0: PEAK_FP32_TFLOPS}
PEAK_HBM_GBPS = 8000.0     # MI355X_MICROARCH.md: HBM3E spec peak


def conv_shapes(B, T, H, W):
    """(NF, Ci, Co, OH, OW) of the eight 3x3 convs of ResNetBackbone (cad:121-139)."""
    NF = B * T
    h, w = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    out = []
    for ci, co, s in [(32, 32, 1), (32, 32, 1), (32, 64, 2), (64, 64, 1), (64, 128, 2), (128, 128, 1),
                      (128, 256, 2), (256, 256, 1)]:
        h, w = (h - 1) // s + 1, (w - 1) // s + 1
        out.append((NF, ci, co, h, w))
    return out


def algorithmic_work(label, B, T, H, W):
    """(bound, amount) per launch of a labelled kernel: FLOPs for MFMA convs, HBM bytes for elementwise."""
    fam, _, lay = label.partition("/L")
    cs = conv_shapes(B, T, H, W)
    if fam in ("conv_fwd", "conv_dgrad", "conv_wgrad"):
        NF, ci, co, oh, ow = cs[int(lay)]
        return "mfma", 2.0 * NF * oh * ow * co * ci * 9
    if fam in ("bn_bwd_reduce", "bn_bwd_apply"):
        NF, ci, co, oh, ow = cs[int(lay)]
        n = NF * oh * ow * co * 4.0
        return "hbm", (2 if fam == "bn_bwd_reduce" else 3) * n
    if fam == "conv1":
        NF = B * T
        oh, ow = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        return "mfma", 2.0 * NF * oh * ow * 32 * 49
    return None, None


CONV_FAMILIES = ("conv_fwd", "conv_dgrad", "conv_wgrad")


def conv_io(B, T, H, W):
    """(NF, Ci, Co, IH, IW, OH, OW) of the eight 3x3 convs (cad:121-139)."""
    out = []
    NF = B * T
    h, w = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    for ci, co, s in [(32, 32, 1), (32, 32, 1), (32, 64, 2), (64, 64, 1), (64, 128, 2), (128, 128, 1),
                      (128, 256, 2), (256, 256, 1)]:
        oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
        out.append((NF, ci, co, h, w, oh, ow))
        h, w = oh, ow
    return out


def conv_bytes(fam, layer, B, T, H, W, act_bytes):
    """Algorithmic HBM bytes of one conv launch: each activation operand read or written once (act_bytes per
    element: 4 fp32, 2 with bf16 activation storage) plus the fp32 weight (or weight-gradient) tensor once."""
    NF, ci, co, ih, iw, oh, ow = conv_io(B, T, H, W)[layer]
    x, y, w = NF * ih * iw * ci * act_bytes, NF * oh * ow * co * act_bytes, co * ci * 9 * 4
    return x + y + w  # fwd: x in, y out, W in; dgrad: dY in, dX out, W in; wgrad: dY, X in, dW out


def family_roofline(fam, live, pl, args, act_bytes):
    """Roofline of one conv family from the live HIP events of the timed region.  fp32 configs: MFMA-bound (SURVEY
    §8d), achieved = algorithmic FLOPs / time against the 157.3 TF fp32 peak (the kernels' own instruction peak --
    split-bf16 launches issue six bf16 products per fp32 product -- reported beside it).  bf16 config 4: HBM-bound,
    achieved = algorithmic bytes (conv_bytes) / time against 8 TB/s."""
    from vad_amd import _native as nat
    B, T, H, W = args.batch, args.T, args.H, args.W
    kind = {"conv_fwd": 0, "conv_dgrad": 1, "conv_wgrad": 2}[fam]
    flops = byts = ms_tot = ideal_s = 0.0
    launches = 0
    paths = {}
    per_layer = {}
    for lab, (ms, n) in live.items():
        f, _, lay = lab.partition("/L")
        if f != fam:
            continue
        l = int(lay)
        per_layer[lab] = round(1e3 * ms / max(n, 1), 2)
        work = algorithmic_work(lab, B, T, H, W)[1]
        flops += work * n
        byts += conv_bytes(fam, l, B, T, H, W, act_bytes) * n
        ms_tot += ms
        launches += n
        path = nat.lib().vad_cad_conv_path(pl.h, l, kind)
        paths[lab] = {6: "split-bf16", 2: "bf16-native", 1: "bf16-split1", 0: "f32"}.get(path, "?")
        ideal_s += work * n / (PATH_PEAK.get(path, PEAK_FP32_TFLOPS) * 1e12)
    sec = ms_tot * 1e-3
    tf, gbs = flops / sec / 1e12, byts / sec / 1e9
    if args.dtype == "bf16":
        r = {"bound": "hbm", "kernel": fam, "achieved": round(gbs, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
             "frac": round(gbs / PEAK_HBM_GBPS, 4), "traffic": None,
             "algorithmic_bytes_per_launch": round(byts / max(launches, 1)),
             "mfma_ceiling": {"achieved_tflops": round(tf, 2), "peak": PEAK_BF16_TFLOPS,
                              "frac": round(tf / PEAK_BF16_TFLOPS, 4)}}
    else:
        r = {"bound": "mfma", "kernel": fam, "achieved": round(tf, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
             "frac": round(tf / PEAK_FP32_TFLOPS, 4), "traffic": None,
             "algorithmic_bytes_per_launch": round(byts / max(launches, 1)),
             "instruction_peak": {"peak": round(flops / ideal_s / 1e12, 1),
                                  "frac": round(tf / (flops / ideal_s / 1e12), 4),
                                  "basis": "fp32-equivalent peak of each launch's kernel (f32 MFMA 157.3; "
                                           "split-bf16 2500/6), work-weighted harmonic mean over the family"}}
    r["launches_timed"] = launches
    r["avg_launch_us"] = round(1e3 * ms_tot / max(launches, 1), 2)
    r["kernel_paths"] = paths
    r["per_layer_us"] = dict(sorted(per_layer.items()))
    tag = f"cfg{args.config}"
    traffic, src = pmc_family("pmc_traffic", tag, fam, "hbm_bytes_per_launch")
    if traffic is not None:
        r["traffic"] = round(traffic)
        r["traffic_unit"] = "bytes/launch (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE)"
        r["traffic_source"] = src
        r["traffic_over_algorithmic"] = round(traffic / (byts / max(launches, 1)), 3)
    util, usrc = pmc_family("pmc_mfma", tag, fam, "mfma_util")
    if util is not None:
        r["mfma_util"] = round(util, 4)
        r["mfma_util_source"] = usrc
    return r


def pmc_family(kind, tag, family, key):
    """A conv family's PMC figure from the latest committed summary of THIS configuration
    (profiles/*_{tag}_{kind}.json, written by tools/pmc_traffic.py / pmc_mfma.py over rocprofv3 --pmc passes of
    `bench.py --config N`), or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{tag}_{kind}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        fam = json.load(f).get("families", {}).get(family)
    if not fam or fam.get(key) is None:
        return None, None
    return fam[key], os.path.relpath(files[-1], ROOT)


def cpu_quota():
    """CPUs this process may run on: the affinity mask, capped by the cgroup v2 CPU quota (the GPU box grants a
    16-CPU quota on a 256-CPU host; 256 threads under that quota run the CPU oracle 80x slower than 16)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return n


def host_cpu_info(threads):
    """Threads the CPU leg used, plus the host's logical CPU count and this process's affinity mask size."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"cores": threads, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cpu_quota": cpu_quota()}


def run_gpu(args, rank, world, local_rank):
    import torch
    import torch.distributed as dist
    from vad_amd import _native as nat
    from vad_amd.cad import CausalAnomalyDetector
    from vad_amd.train import CadTrainer, apply_memory_efficient_training

    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = CausalAnomalyDetector()
    with contextlib.redirect_stdout(io.StringIO()):
        apply_memory_efficient_training(model)
    model = model.to(dev)
    trainer = CadTrainer(model, lr=3e-4, seed=1234, prio_stream=args.prio_stream,
                         compute_dtype=torch.bfloat16 if args.dtype == "bf16" else torch.float32,
                         sync_bn=args.sync_bn)
    B, T, H, W = args.batch, args.T, args.H, args.W
    # synthetic clips resident in HBM before the timed region (device generator == oracle.rng.pixels_u8)
    pool = []
    for i in range(2):
        x = torch.empty(B, T, 1, H, W, device=dev)
        nat.check(nat.lib().vad_synth_frames(7, i, rank * B * T, B * T, H * W, 0, x.data_ptr(), nat.stream_of(dev)))
        pool.append(x)
    labels = torch.tensor([(rank * B + b) % 2 for b in range(B)], dtype=torch.int64, device=dev)
    torch.cuda.synchronize()  # (the clips are complete before every step: inputs_ready=True below)

    for i in range(args.warmup):
        trainer.step(pool[i % 2], labels, inputs_ready=True)
    torch.cuda.synchronize()

    # one instrumented step: per-label kernel times -> the dominant kernel family (largest summed time over the conv
    # families, the weight gradients included although they run on their own stream beside the input gradients)
    eng = trainer.eng
    eng.profile(True, "")
    trainer.step(pool[0], labels, inputs_ready=True)
    torch.cuda.synchronize()
    breakdown = eng.profile_read()
    fam_time = {}
    for lab, (ms, n) in breakdown.items():
        if lab.split("/L")[0] in CONV_FAMILIES:
            fam = lab.split("/L")[0]
            fam_time[fam] = fam_time.get(fam, 0.0) + ms
    dominant = max(fam_time, key=fam_time.get)
    # (the largest family on the critical stream: conv_wgrad is overlapped, DESIGN.md §3 Streams)
    critical = max((f for f in fam_time if f != "conv_wgrad"), key=fam_time.get)

    # timed region: K uninstrumented steps (the headline).  The per-family kernel times for the roofline come from a
    # separate instrumented phase right after it (every conv family's kernels dispatched with HIP start/stop events,
    # hipExtLaunchKernel, on the stream each runs on), so the headline carries no profiling overhead; that phase's own
    # step time is reported beside it (prof_ms_per_step)
    eng.profile(True, "conv_")  # clears the breakdown records
    eng.profile(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = t_loop0 = time.perf_counter()
    for i in range(args.steps):
        losses = trainer.step(pool[i % 2], labels, inputs_ready=True)
    t_enq = time.perf_counter()  # host enqueue time of the timed steps (== the step time when the host is the bound)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    n_prof = max(3, args.steps // max(1, args.prof_every))
    eng.profile(True, "conv_", reset=False)
    tp0 = time.perf_counter()
    for i in range(n_prof):
        trainer.step(pool[i % 2], labels, inputs_ready=True)
    torch.cuda.synchronize()
    prof_ms_per_step = 1e3 * (time.perf_counter() - tp0) / n_prof
    eng.profile(False, reset=False)
    live = eng.profile_read()
    # post-backbone chain (after the timed region, 3 more steps): end of the last forward conv to the start of the
    # first backbone-backward kernel (avgpool_bwd), kernel-dispatch events only on those two launches
    eng.profile(True, "conv_fwd/L7|avgpool_bwd")
    for i in range(3):
        trainer.step(pool[i % 2], labels, inputs_ready=True)
    torch.cuda.synchronize()
    marks = eng.profile_marks()
    eng.profile(False)
    chain = []
    for i, (lab, _, t1) in enumerate(marks):
        if lab == "conv_fwd/L7":
            nxt = [m for m in marks[i + 1:] if m[0] == "avgpool_bwd"]
            if nxt:
                chain.append(1e3 * (nxt[0][1] - t1))
    post_backbone_us = sorted(chain)[len(chain) // 2] if chain else None
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(losses[4].item())
    pl = eng.plans[(B, T, H, W)]
    act_bytes = 2 if args.dtype == "bf16" else 4
    families = {f: family_roofline(f, live, pl, args, act_bytes) for f in fam_time}
    roof = dict(families[dominant])
    roof["dominant_basis"] = ("largest summed kernel time over the conv families in an instrumented step "
                              "(weight gradients included: they overlap the input gradients on their own stream)")
    if critical != dominant:
        roof["critical_stream"] = families[critical]
    roof["families"] = {f: {k: r[k] for k in ("achieved", "frac", "avg_launch_us", "launches_timed", "per_layer_us")}
                        for f, r in families.items()}
    step_ms = 1e3 * elapsed / args.steps
    # parity probe (rank 0): one more forward on the first batch with the trained weights; the CPU leg re-runs it on
    # the oracle (cpu_baseline) and reports the score difference and the frame-AUC of both
    probe = None
    allreduce_bytes = 4 * trainer.allreduce_floats if trainer.dist else 0
    if rank == 0 and not args.no_cpu_baseline:  # (only the CPU leg reads it; PMC passes run without both)
        if trainer.sync_bn:  # (the probe runs on rank 0 alone: per-rank statistics, as the oracle leg computes them)
            eng.set_bn_sync(enable=False)
        o = eng.forward(pool[0], True, 777, 0, 0, labels)
        torch.cuda.synchronize()
        probe = dict(state={k: v.detach().cpu().clone() for k, v in model.state_dict().items()},
                     final=o["final"].cpu(), probs=o["probs"].cpu(), loss=float(o["losses"][4]))
        # held-out set for the frame-AUC parity: HELDOUT_BATCHES x B synthetic clips never trained on (seed 8), eval mode
        # (running statistics), labels i mod 2
        from oracle import cad_oracle as co
        held = []
        for k in range(HELDOUT_BATCHES):
            xh = co.synth_clips(8, k, 0, B, T, H, W).to(dev)
            held.append(eng.forward(xh, False, 0, 0, 0, None)["final"].cpu())
        torch.cuda.synchronize()
        probe["heldout"] = torch.cat(held)
    # input-inclusive leg (rank 0, N=1): the same step fed from pinned host u8 clips through ClipStager (batch k+1's
    # H2D copy and u8 -> fp32 conversion overlapping step k); never the headline value
    h2d = None
    if rank == 0 and world == 1 and args.h2d_steps > 0:
        from vad_amd.data import ClipStager
        stager = ClipStager(dev, mode=0)
        u8 = [torch.randint(0, 256, (B, T, 1, H, W), dtype=torch.uint8).pin_memory() for _ in range(2)]
        h = stager.issue(u8[0])

        def h2d_step(i):
            nonlocal h
            x, ready = stager.finish(h, wait=False), h.ready
            h = stager.issue(u8[(i + 1) % 2])
            trainer.step(x, labels, inputs_ready=ready)

        for i in range(2):  # warm-up
            h2d_step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.h2d_steps):
            h2d_step(i)
        h2d_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        stager.finish(h)
        torch.cuda.synchronize()
        h2d = {"value": round(B * args.h2d_steps / el, 3), "unit": "clips/s", "steps": args.h2d_steps,
               "ms_per_step": round(1e3 * el / args.h2d_steps, 4),
               "host_enqueue_ms_per_step": round(1e3 * h2d_enq / args.h2d_steps, 4),
               "bytes_h2d_per_step": B * T * H * W,
               "path": "pinned u8 host clips -> ClipStager.issue (H2D copy + u8->fp32 conversion on the stager stream, "
                    "batch k+1 during step k) -> step(inputs_ready=event): the early stem waits for it, the critical "
                    "stream does not"}
    # drop-in loop leg (rank 0, N=1): the package's own train_model inner loop (vad_amd.train.train_epoch) over a
    # loader of pinned host u8 clips -- prefetch + ClipStager, one fused step per batch, and the per-step host read of
    # the loss vector the reference does (loss.item(), cad:692) -- i.e. what a drop-in caller of train_model gets
    dropin = None
    if rank == 0 and world == 1 and args.h2d_steps > 0:
        from vad_amd.data import ClipStager
        from vad_amd.train import train_epoch
        stager = ClipStager(dev, mode=0)
        u8 = [torch.randint(0, 256, (B, T, 1, H, W), dtype=torch.uint8).pin_memory() for _ in range(2)]
        lab_cpu = labels.cpu()

        def loader(n):
            for i in range(n):
                yield u8[i % 2], lab_cpu

        train_epoch(trainer, loader(3), stager, log=None)  # warm-up
        torch.cuda.synchronize()
        n_loop = max(2 * args.h2d_steps, 10)
        t0 = time.perf_counter()
        tot, nb = train_epoch(trainer, loader(n_loop), stager, log=None)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        dropin = {"value": round(B * n_loop / el, 3), "unit": "clips/s", "steps": n_loop,
                  "ms_per_step": round(1e3 * el / n_loop, 4), "mean_total_loss": round(tot / max(nb, 1), 6),
                  "path": "vad_amd.train.train_epoch (train_model's inner loop): pinned u8 loader -> prefetch / "
                          "ClipStager (batch k+1 staged during step k) -> CadTrainer.step(inputs_ready=event, "
                          "host_losses=True) -> losses.tolist() every step (cad:692's loss.item())"}
    # whole-step algorithmic FLOP rate (all 3x3 convs fwd/dgrad/wgrad + conv1 fwd), for context
    conv_flops = sum(2.0 * NF * oh * ow * co * ci * 9 for NF, ci, co, oh, ow in conv_shapes(B, T, H, W))
    dgrad_flops = conv_flops - 2.0 * B * T * conv_shapes(B, T, H, W)[0][3] * conv_shapes(B, T, H, W)[0][4] * 32 * 32 * 9
    c1 = algorithmic_work("conv1", B, T, H, W)[1]
    step_flops = 2 * conv_flops + dgrad_flops + c1
    roof["instrumented_steps"] = n_prof
    roof["instrumented_ms_per_step"] = round(prof_ms_per_step, 4)
    return dict(elapsed=elapsed, step_ms=step_ms, host_enqueue_ms=1e3 * (t_enq - t_loop0) / args.steps, roof=roof,
                breakdown=breakdown, dominant=dominant,
                final_loss=final_loss, step_tflops=step_flops / (step_ms * 1e-3) / 1e12, probe=probe, h2d=h2d, dropin=dropin,
                allreduce_bytes=allreduce_bytes, post_backbone_us=post_backbone_us)


# SURVEY §8d fixed per-clip work of the train step: cfg 2 (T=16, 227^2, fp32) 20.25 GFLOP, MFMA-bound; cfg 4
# (T=32, 256^2, bf16 storage) 681 MB of HBM traffic (3 x 14.19 MB/frame x 32 frames / 2), HBM-bound
STEP_WORK = {(2, 16, 227, 227): ("mfma", 20.25e9), (4, 32, 256, 256): ("hbm", 681e6)}


def step_roofline(args, clips_per_s_per_gpu, step_tflops):
    """Whole-step fraction of the governing ceiling: clips/s per GPU x the fixed per-clip work."""
    key = (args.config, args.T, args.H, args.W)
    if key not in STEP_WORK:
        return {"bound": "mfma", "achieved": round(step_tflops, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(step_tflops / PEAK_FP32_TFLOPS, 4), "basis": "algorithmic conv FLOPs of the step"}
    bound, work = STEP_WORK[key]
    if bound == "mfma":
        a = clips_per_s_per_gpu * work / 1e12
        return {"bound": "mfma", "achieved": round(a, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(a / PEAK_FP32_TFLOPS, 4), "ceiling_clips_per_s": round(PEAK_FP32_TFLOPS * 1e12 / work),
                "basis": "SURVEY §8d F_clip = 20.25 GFLOP x clips/s per GPU"}
    a = clips_per_s_per_gpu * work / 1e9
    return {"bound": "hbm", "achieved": round(a, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": round(a / PEAK_HBM_GBPS, 4), "ceiling_clips_per_s": round(PEAK_HBM_GBPS * 1e9 / work),
            "basis": "SURVEY §8d B_clip = 681 MB x clips/s per GPU"}


HELDOUT_BATCHES = 8  # held-out clips for the frame-AUC parity: 8 x B (64 at the default B = 8)


def parity_check(args, probe):
    """CPU leg of the parity probe: the oracle forward (fp32, CPU) on the same clips, weights, BN state and draws
    as the GPU probe; max |score difference| (north star: 1e-4) and frame-AUC of both score sets (clip labels
    i mod 2 broadcast to the T frames of each clip)."""
    import torch
    from oracle import cad_oracle as co
    from vad_amd.evaluate import frame_auc
    B, T, H, W = args.batch, args.T, args.H, args.W
    sd = probe["state"]
    params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v.clone() for k, v in sd.items() if "running" in k}
    x = co.synth_clips(7, 0, 0, B, T, H, W)
    y = co.synth_labels(0, B)
    with torch.no_grad():
        ref = co.cad_forward(params, bufs, x, co.CadDraws.make(777, 0, 0, B, T), training=True)
        rl = co.cad_losses(ref, y)
    gpu_s, cpu_s = probe["final"].double(), ref["anomaly_scores"].double()
    # held-out frame-AUC: the same eval-mode scoring of the HELDOUT_BATCHES x B unseen clips on the oracle
    held_cpu = []
    with torch.no_grad():
        for k in range(HELDOUT_BATCHES):
            b2 = {kk: v.clone() for kk, v in sd.items() if "running" in kk}  # (the train-mode probe above moved bufs)
            r = co.cad_forward(params, b2, co.synth_clips(8, k, 0, B, T, H, W), co.CadDraws.make(0, 0, 0, B, T),
                               training=False)
            held_cpu.append(r["anomaly_scores"].double())
    hc, hg = torch.cat(held_cpu), probe["heldout"].double()
    yh = torch.arange(hc.numel()) % 2
    return {"max_abs_score_diff": float((gpu_s - cpu_s).abs().max()),
            "max_abs_prob_diff": float((probe["probs"].double() - ref["direct_predictions"].double()).abs().max()),
            "loss_rel_diff": abs(probe["loss"] - float(rl["total"])) / max(abs(float(rl["total"])), 1e-12),
            "frame_auc_gpu": frame_auc(hg.numpy(), yh.numpy(), T),
            "frame_auc_cpu": frame_auc(hc.numpy(), yh.numpy(), T),
            "heldout_max_abs_score_diff": float((hg - hc).abs().max()),
            "tolerance": 1e-4 if args.dtype == "fp32" else 2e-2,
            "sample": f"one train-mode forward of B={B} clips x T={T} x 1x{H}x{W} after the timed steps (scores, "
                      f"loss); frame-AUC and heldout_max_abs_score_diff: eval-mode scores of {hc.numel()} held-out "
                      f"synthetic clips (seed 8, never trained on), labels i mod 2 broadcast to the T frames"}


def cpu_baseline(args):
    """The CPU oracle (a port of the reference step) on this host: bounded sample of the same workload."""
    import torch
    from oracle import cad_oracle as co
    from vad_amd.cad import CausalAnomalyDetector
    threads = cpu_quota()  # every CPU this process may use (os.cpu_count() capped by affinity and cgroup quota)
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = CausalAnomalyDetector()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v for k, v in sd.items() if "running" in k}
    B, T, H, W = args.batch, args.T, args.H, args.W
    x = co.synth_clips(7, 0, 0, B, T, H, W)
    y = co.synth_labels(0, B)
    state = {}
    co.cad_train_step(params, bufs, state, x, y, co.CadDraws.make(1234, 0, 0, B, T))  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        co.cad_train_step(params, bufs, state, x, y, co.CadDraws.make(1234, n + 1, 0, B, T))
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or n >= 40:
            break
    return {"value": round(B * n / el, 3), "unit": "clips/s", **host_cpu_info(threads), "kind": "port",
            "sample": f"{n} train steps of B={B} clips x T={T} x 1x{H}x{W} (oracle/cad_oracle.py, torch CPU fp32, "
                      f"{threads} threads), after 1 warm-up step",
            "validated": "profiles/r02_cpu_baseline_check.json (oracle vs the imported reference, same host)"}


def run_bbox(args, rank, world, local_rank):
    """BASELINE config 5 (avenue_training_script_bbox.py scorer, bbox:339-368): 64 RGB 64x64 clips per rank with T
    drawn from {8, 16, 32}, scored in one packed batch per T (bbox.AnomalyVisualizer.predict_clips packing, the
    clips already resident in HBM).  A step scores every clip of the rank once."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from vad_amd import _native as nat
    from vad_amd.bbox import CausalAnomalyDetector as BboxDetector
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = BboxDetector().to(dev).eval()
    n = args.batch
    Ts = np.random.default_rng(5).choice([8, 16, 32], size=n * world)[rank * n:(rank + 1) * n]
    groups = {}
    for T in (8, 16, 32):
        k = int((Ts == T).sum())
        if k:
            x = torch.empty(k, 3, T, 64, 64, device=dev)
            nat.check(nat.lib().vad_synth_frames(11, 0, (rank * n) * 3 * 32, k * 3 * T, 64 * 64, 1, x.data_ptr(),
                                                 nat.stream_of(dev)))
            groups[T] = x

    def step():
        with torch.no_grad():
            return [model(x) for x in groups.values()]

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    frames = int(sum(x.shape[0] * x.shape[2] for x in groups.values()))
    probe = {T: (x[:2].cpu(), o[0].reshape(-1)[:2].cpu()) for (T, x), o in zip(groups.items(), out)}
    return dict(elapsed=elapsed, step_ms=1e3 * elapsed / args.steps, frames=frames, Ts=Ts.tolist(),
                state={k: v.detach().cpu().clone() for k, v in model.state_dict().items()}, probe=probe)


def bbox_cpu(args, r):
    """CPU leg of config 5: the oracle scorer (oracle/bbox_oracle.py) on a bounded sample, and parity of the GPU
    scores of the first two clips of every T bucket."""
    import torch
    from oracle import bbox_oracle as bo
    threads = cpu_quota()  # every CPU this process may use (os.cpu_count() capped by affinity and cgroup quota)
    torch.set_num_threads(threads)
    p = r["state"]
    diff = 0.0
    with torch.no_grad():
        for T, (x, s) in r["probe"].items():
            rs, _, _ = bo.bbox_forward(p, x)
            diff = max(diff, float((rs.reshape(-1) - s).abs().max()))
        x = bo.synth_clips(11, 0, 0, 4, 16, 64, 64)
        bo.bbox_forward(p, x)
        n, t0 = 0, time.perf_counter()
        while True:
            bo.bbox_forward(p, x)
            n += 1
            if time.perf_counter() - t0 >= min(args.cpu_seconds, 6.0) or n >= 200:
                break
        el = time.perf_counter() - t0
    return ({"value": round(4 * n / el, 3), "unit": "clips/s", **host_cpu_info(threads), "kind": "port",
             "sample": f"{n} forwards of 4 RGB clips x T=16 x 64x64 (oracle/bbox_oracle.py, torch CPU fp32, "
                       f"{threads} threads)"},
            {"max_abs_score_diff": diff, "tolerance": 1e-4, "sample": "first two clips of each T bucket"})


BBOX_FLOP_PER_FRAME = 2 * 4096 * 32 * 81 + 2 * 1024 * 64 * 864 // 2  # conv3d 3->32 @64^2 + 32->64 @32^2 (T/2)
BBOX_BYTES_PER_FRAME = 4 * (3 * 4096 + 2 * 32 * 4096 + 2 * 32 * 1024 // 2 + 2 * 64 * 1024 // 2)


def bbox_roofline(frames_per_s, frames_per_step):
    """Config 5 (inference) against both ceilings SURVEY §8d names: fp32 FLOPs (the two Conv3d layers) and HBM bytes
    (per-layer compulsory fp32 I/O: the clip, conv1's output written and read by the pool, the pool output written
    and read by conv2, conv2's output written and read by the adaptive pool), per frame of a clip."""
    tf = frames_per_s * BBOX_FLOP_PER_FRAME / 1e12
    gbs = frames_per_s * BBOX_BYTES_PER_FRAME / 1e9
    f_mfma, f_hbm = tf / PEAK_FP32_TFLOPS, gbs / PEAK_HBM_GBPS
    gov = "mfma" if f_mfma >= f_hbm else "hbm"
    r = {"bound": gov, "kernel": "whole step",
            "achieved": round(tf if gov == "mfma" else gbs, 3), "peak": PEAK_FP32_TFLOPS if gov == "mfma" else PEAK_HBM_GBPS,
            "unit": "TFLOP/s" if gov == "mfma" else "GB/s", "frac": round(max(f_mfma, f_hbm), 4),
            "traffic": None, "algorithmic_bytes_per_step": BBOX_BYTES_PER_FRAME * frames_per_step,
            "other_ceiling": {"unit": "GB/s" if gov == "mfma" else "TFLOP/s",
                              "achieved": round(gbs if gov == "mfma" else tf, 3),
                              "frac": round(f_hbm if gov == "mfma" else f_mfma, 4)},
            "basis": f"{BBOX_FLOP_PER_FRAME} FLOP and {BBOX_BYTES_PER_FRAME} B (per-layer compulsory fp32 I/O) per frame"
                     " x frames scored per second; governing = the ceiling with the larger fraction"}
    step, src = pmc_step("cfg5")
    if step is not None:
        r["traffic"] = round(step)
        r["traffic_unit"] = "HBM bytes per step (every kernel; PMC FETCH_SIZE x2 + WRITE_SIZE)"
        r["traffic_source"] = src
    return r


def pmc_step(tag):
    """Whole-step HBM bytes from the latest committed PMC summary of this configuration, or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{tag}_pmc_traffic.json")))
    if not files:
        return None, None
    st = json.load(open(files[-1])).get("step")
    return (st["hbm_bytes_per_step"], os.path.relpath(files[-1], ROOT)) if st else (None, None)


MC_TRAIN_FLOP_PER_CLIP = 566.3e6  # minicausal train step, T=16, 64x64


def run_mc(args, rank, world, local_rank):
    """BASELINE config 1 (minicausal_vad_complete3.py): StableTrainer.train_epoch over 32 clips (T=16, 1x64x64,
    x ~ U[0,1), labels alternating, batch 8: mc:503-599) on the HIP plan; one step = one epoch (4 iterations, with
    the reference's per-iteration host reads of loss / NaN status / accuracy)."""
    import torch
    from vad_amd import _native as nat
    from vad_amd.mc import SimpleVideoAnomalyDetector, StableTrainer
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = SimpleVideoAnomalyDetector(input_channels=1, temporal_frames=args.T, spatial_size=args.H)
    n, bs = args.batch, 8
    batches = []
    for k in range(n // bs):
        x = torch.empty(bs, 1, args.T, args.H, args.W, device=dev)
        nat.check(nat.lib().vad_synth_frames(0, 0, (rank * n + k * bs) * args.T, bs * args.T, args.H * args.W, 1,
                                             x.data_ptr(), nat.stream_of(dev)))
        y = torch.tensor([1.0 if (rank * n + k * bs + b) % 2 == 0 else 0.0 for b in range(bs)], device=dev)
        batches.append((x, y))
    tr = StableTrainer(model, batches, [], dev, lr=1e-3)
    for _ in range(args.warmup):
        tr.train_epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, acc = tr.train_epoch()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    model.eval()
    with torch.no_grad():
        probe = model(batches[0][0]).reshape(-1).cpu()
    state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    return dict(elapsed=elapsed, step_ms=1e3 * elapsed / args.steps, loss=loss, probe=probe, state=state,
                x0=batches[0][0].cpu())


def mc_cpu(args, r):
    """CPU leg of config 1: parity of the GPU eval scores (first batch, trained weights) against the oracle, and the
    oracle's StableTrainer iteration (oracle/mc_oracle.py) over the 4 batches of an epoch, timed."""
    import torch
    from oracle import mc_oracle as mo
    threads = cpu_quota()  # every CPU this process may use (os.cpu_count() capped by affinity and cgroup quota)
    torch.set_num_threads(threads)
    sd = r["state"]
    params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v.clone() for k, v in sd.items() if "running" in k}
    with torch.no_grad():
        ref = mo.mc_forward(params, bufs, r["x0"], None, False).reshape(-1)
    parity = {"max_abs_score_diff": float((ref - r["probe"]).abs().max()), "tolerance": 1e-4,
              "sample": "eval forward of the first batch (8 clips) after the timed epochs"}
    bs, T = 8, args.T
    batches = [(mo.synth_clips(0, 0, k * bs, bs, T, args.H, args.W), mo.synth_labels(k * bs, bs))
               for k in range(args.batch // bs)]
    state = {}
    p = {k: v.clone() for k, v in params.items()}
    mo.mc_train_step(p, bufs, state, *batches[0], mo.McDraws.make(1, 0, 0, bs))
    n, t0 = 0, time.perf_counter()
    while True:
        for k, (x, y) in enumerate(batches):
            mo.mc_train_step(p, bufs, state, x, y, mo.McDraws.make(1, n + 1, k * bs, bs))
        n += 1
        if time.perf_counter() - t0 >= args.cpu_seconds or n >= 50:
            break
    el = time.perf_counter() - t0
    return ({"value": round(args.batch * n / el, 3), "unit": "clips/s", **host_cpu_info(threads), "kind": "port",
             "sample": f"{n} epochs of {args.batch} clips (batch {bs}) x T={T} x 1x{args.H}x{args.W} "
                       f"(oracle/mc_oracle.py mc_train_step, torch CPU fp32, {threads} threads)"}, parity)


def ae_flops_per_clip(T):
    """Algorithmic FLOPs of one cad1 autoencoder train clip (SURVEY §8d counting: 2 per MAC, backward = 2x forward
    minus the first conv's input gradient).  Encoder per frame: convs 1.05 + 16.8 + 16.8 + 8.4 MFLOP + Linear 0.26;
    LSTM per frame 2 x 2 x 64 x 256; decoder once per clip (its T calls are identical): Linear 0.26 + transposed
    convs 8.4 + 16.8 + 16.8 + 1.05 MFLOP."""
    enc, lstm, dec, first = 43_253_760, 65_536, 43_253_760, 1_048_576
    return 3 * (T * (enc + lstm) + dec) - T * first


def run_ae(args, rank, world, local_rank):
    """cad1 (causal_anomaly_detection1.py) memory autoencoder, SURVEY §8f: one step = the fused train_model
    iteration (cad1:378-431: forward, MSE, memory-ring update, backward, NaN-grad check, clip_grad_norm_(0.1), Adam)
    on args.batch normal clips of T x 1x64x64 per rank, already resident in HBM."""
    import torch
    from vad_amd import _native as nat
    from vad_amd.ae import AeTrainer, VideoAutoEncoder
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = VideoAutoEncoder().to(dev)
    tr = AeTrainer(model, lr=1e-6)
    B, T = args.batch, args.T
    x = torch.empty(B, T, 1, 64, 64, device=dev)
    nat.check(nat.lib().vad_synth_frames(13, 0, rank * B * T, B * T, 64 * 64, 1, x.data_ptr(), nat.stream_of(dev)))
    x.clamp_(0.001, 0.999)  # the dataset's clamp (cad1:110-114)
    for _ in range(args.warmup):
        tr.step(x)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses = tr.step(x)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    lv = losses.cpu().tolist()
    ev = tr.eval_batch(x[:4])
    probe = {"x": x[:4].cpu(), "recon_error": ev["recon_error"].cpu(), "score": ev["anomaly_score"].cpu(),
             "state": {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}}
    return dict(elapsed=elapsed, step_ms=1e3 * elapsed / args.steps, loss=lv[0], status=lv[3], probe=probe)


def ae_cpu(args, r):
    """CPU leg of the cad1 line: parity of the GPU eval scores against the oracle (same weights / ring), and the
    oracle train step (oracle/ae_oracle.py) timed on a bounded sample."""
    import torch
    from oracle import ae_oracle as ae
    threads = cpu_quota()  # every CPU this process may use (os.cpu_count() capped by affinity and cgroup quota)
    torch.set_num_threads(threads)
    params, bufs, mem = ae.split_state(r["probe"]["state"])
    ev = ae.ae_eval_batch(params, bufs, mem, r["probe"]["x"])
    parity = {"max_abs_recon_error_diff": float((ev["recon_error"] - r["probe"]["recon_error"]).abs().max()),
              "max_abs_memory_score_diff": float((ev["outputs"]["anomaly_score"] - r["probe"]["score"]).abs().max()),
              "tolerance": 1e-4, "sample": "eval forward of 4 clips after the timed steps"}
    B, T = args.batch, args.T
    x = ae.synth_clips(13, 0, 0, B, T)
    y = torch.zeros(B, dtype=torch.int64)
    state = {}
    ae.ae_train_step(params, bufs, mem, state, x, y, lr=1e-6)
    n, t0 = 0, time.perf_counter()
    while True:
        ae.ae_train_step(params, bufs, mem, state, x, y, lr=1e-6)
        n += 1
        if time.perf_counter() - t0 >= args.cpu_seconds or n >= 100:
            break
    el = time.perf_counter() - t0
    return ({"value": round(B * n / el, 3), "unit": "clips/s", **host_cpu_info(threads), "kind": "port",
             "sample": f"{n} train steps of B={B} clips x T={T} x 1x64x64 (oracle/ae_oracle.py, torch CPU fp32, "
                       f"{threads} threads), after 1 warm-up step"}, parity)


def a2_flops_per_clip(T, H, W):
    """Algorithmic FLOPs of one a2 train clip (SURVEY §8d counting: 2 per MAC; backward = 2x forward minus the first
    conv's input gradient): the three k3 p1 Conv3d (strides (1,2,2), 2, 2; 3 -> 16 -> 32 -> 64 channels, a2:19-21) over
    their output voxels, fc 4096 -> 16 and the causal-discovery / graph-encoder / predictor Linears (a2:27-101)."""
    def out(n, s):
        return (n - 1) // s + 1
    d1, h1, w1 = T, out(H, 2), out(W, 2)
    d2, h2, w2 = out(d1, 2), out(h1, 2), out(w1, 2)
    d3, h3, w3 = out(d2, 2), out(h2, 2), out(w2, 2)
    c1 = d1 * h1 * w1 * 16 * 3 * 27
    c2 = d2 * h2 * w2 * 32 * 16 * 27
    c3 = d3 * h3 * w3 * 64 * 32 * 27
    lin = 4096 * 16 + 16 * 32 + 32 * 256 + 256 * 128 + 128 * 64 + 80 * 64 + 64 * 1
    fwd = c1 + c2 + c3 + lin
    return 2 * (3 * fwd - c1)


def run_a2(args, rank, world, local_rank):
    """a2 (avenue_training_script2.py) ImprovedMiniCausalVAD, SURVEY §8 row a15/a16: one step = the fused
    train_epoch_improved iteration (a2:218-245: forward, compute_improved_loss, the NaN check's host read of the loss,
    backward, clip_grad_norm_(0.5), AdamW) on args.batch RGB clips of T x 3x64x64 per rank, already resident in HBM."""
    import torch
    from vad_amd import _native as nat
    from vad_amd.a2 import ImprovedMiniCausalVAD
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    vad = ImprovedMiniCausalVAD(device=dev)
    B, T = args.batch, args.T
    # (B, 3, T, H, W): plane (clip, c, t) = keyed-hash u8 / 255 of global plane (clip * 3 + c) * T + t
    x = torch.empty(B, 3, T, args.H, args.W, device=dev)
    nat.check(nat.lib().vad_synth_frames(17, 0, rank * B * 3 * T, B * 3 * T, args.H * args.W, 1, x.data_ptr(),
                                         nat.stream_of(dev)))
    y = torch.zeros(B, device=dev)
    for _ in range(args.warmup):
        vad.train_step(x, y)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, comps, stepped = vad.train_step(x, y)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    xp = x[:4]
    preds, graphs, _ = vad.evaluate_improved([(xp, y[:4])])
    probe = {"x": xp.cpu(), "preds": preds, "graphs": graphs,
             "state": {k: v.detach().cpu().clone() for k, v in vad.model.state_dict().items()}}
    return dict(elapsed=elapsed, step_ms=1e3 * elapsed / args.steps, loss=loss, stepped=stepped, probe=probe)


def a2_cpu(args, r):
    """CPU leg of the a2 line: the GPU eval predictions / graphs after the timed steps against the oracle's forward on
    the same weights, and the oracle train step (oracle/a2_oracle.py) timed on a bounded sample."""
    import numpy as np
    import torch
    from oracle import a2_oracle as ao
    threads = cpu_quota()
    torch.set_num_threads(threads)
    params = {k: v.double() for k, v in r["probe"]["state"].items()}
    s, adj, _ = ao.a2_forward(params, r["probe"]["x"].double(), None, False)
    parity = {"max_abs_score_diff": float(np.abs(s.numpy().reshape(-1) - r["probe"]["preds"]).max()),
              "max_abs_adjacency_diff": float(np.abs(adj.numpy() - r["probe"]["graphs"]).max()),
              "tolerance": 1e-4, "sample": "eval forward of 4 clips after the timed steps (float64 oracle)"}
    B, T = args.batch, args.T
    params = {k: v.clone() for k, v in r["probe"]["state"].items()}
    x = ao.synth_clips(17, 0, 0, B, T, args.H, args.W)
    state = {}
    ao.a2_train_step(params, state, x, ao.A2Draws.make(17, 0, 0, B))
    n, t0 = 0, time.perf_counter()
    while True:
        ao.a2_train_step(params, state, x, ao.A2Draws.make(17, n + 1, 0, B))
        n += 1
        if time.perf_counter() - t0 >= args.cpu_seconds or n >= 200:
            break
    el = time.perf_counter() - t0
    return ({"value": round(B * n / el, 3), "unit": "clips/s", **host_cpu_info(threads), "kind": "port",
             "sample": f"{n} train steps of B={B} clips x 3x{T}x{args.H}x{args.W} (oracle/a2_oracle.py a2_train_step, "
                       f"torch CPU fp32, {threads} threads), after 1 warm-up step"}, parity)


def finish(world):
    """N > 1: every rank waits until rank 0 has run the CPU legs (after the timed region), then leaves the group."""
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


def launch_ranks(n, backend):
    """Run this command as n ranks (torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1) in a child
    process; returns its exit status.  Refuses (status 2) when fewer than n GPUs are visible for an RCCL run: the
    measurement would otherwise time a different configuration than the one named."""
    import socket
    import subprocess
    import torch
    visible = torch.cuda.device_count()  # (counting devices does not initialise the GPU on this image)
    if backend == "nccl" and visible < n:
        print(f"bench.py: --gpus {n} needs {n} GPUs, {visible} visible", file=sys.stderr, flush=True)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="2", choices=("1", "2", "4", "5", "cad1", "a2"),
                    help="BASELINE config: 1 = minicausal StableTrainer epoch over 32 clips T=16 64x64, "
                         "2 = T=16 227x227 fp32 (default), 4 = T=32 256x256 bf16 convs, "
                         "5 = bbox clip scorer, mixed T (inference); cad1 = the causal_anomaly_detection1.py "
                         "memory autoencoder train step (SURVEY §8f, not a BASELINE config); a2 = the "
                         "avenue_training_script2.py ImprovedMiniCausalVAD train step (SURVEY §8 a15/a16)")
    ap.add_argument("--batch", type=int, default=8, help="clips per GPU")
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--H", type=int, default=None)
    ap.add_argument("--W", type=int, default=None)
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default=None,
                    help="fp32: fp32 numerics; bf16: backbone 3x3 convs on bf16 operands (fp32 accumulate)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--prof-every", type=int, default=4,
                    help="after the timed region, steps // k instrumented steps (at least 3) give the roofline events")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--prio-stream", type=int, default=0, help="cad step on a high-priority stream (CadTrainer)")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="nccl (= RCCL over xGMI) for measurement; gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--breakdown-out", default=None, help="write the per-kernel breakdown JSON here")
    ap.add_argument("--sync-bn", action="store_true",
                    help="N>1: SyncBatchNorm mode (BN over the global batch = the reference's single-process step)")
    ap.add_argument("--h2d-steps", type=int, default=10,
                    help="steps of the input-inclusive leg (pinned u8 clips through ClipStager; 0 = skip)")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=V",
                    help="measurement only: set a libvadhip tuning knob (vad_set_tuning) before the run")
    args = ap.parse_args()
    # --gpus N: one process per GPU.  Launched without torch.distributed.run (no WORLD_SIZE), bench.py starts the N
    # ranks itself as a child torch.distributed.run before anything touches the GPU and exits with its status;
    # launched by torch.distributed.run, the world size must be N.
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, args.dist_backend))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} ranks were launched")
    if args.tune:
        from vad_amd import _native as nat
        for kv in args.tune:
            k, v = kv.split("=")
            nat.check(nat.lib().vad_set_tuning(k.encode(), int(v)))
    args.config = args.config if args.config in ("cad1", "a2") else int(args.config)
    preset = {1: (16, 64, 64, "fp32"), 2: (16, 227, 227, "fp32"), 4: (32, 256, 256, "bf16"), 5: (0, 64, 64, "fp32"),
              "cad1": (16, 64, 64, "fp32"), "a2": (8, 64, 64, "fp32")}[args.config]
    if args.config == 1 and args.batch == 8:
        args.batch = 32  # clips per epoch per rank (BASELINE config 1)
    if args.config == 5 and args.batch == 8:
        args.batch = 64  # clips per rank
    if args.config in ("cad1", "a2") and args.batch == 8:
        args.batch = 32
    args.T = args.T or preset[0]
    args.H = args.H or preset[1]
    args.W = args.W or preset[2]
    args.dtype = args.dtype or preset[3]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        if args.dist_backend == "gloo":
            # rehearsal of the multi-rank path on fewer GPUs than ranks (ranks share devices round-robin)
            local_rank %= torch.cuda.device_count()
        torch.cuda.set_device(local_rank)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    if args.config == 1:
        r = run_mc(args, rank, world, local_rank)
        if rank == 0:
            cpu, parity = (None, None) if args.no_cpu_baseline else mc_cpu(args, r)
            clips = world * args.batch * args.steps
            tflops = MC_TRAIN_FLOP_PER_CLIP * clips / r["elapsed"] / 1e12
            print(json.dumps({
                "metric": BASELINE_METRIC, "value": round(clips / r["elapsed"], 3), "unit": "clips/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["step_ms"], 4),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
                "data": "synthetic grayscale clips (keyed-hash u8 / 255), labels alternating; random-init weights "
                        "(torch.manual_seed(0))",
                "config": {"workload": "minicausal_vad_complete3.py StableTrainer epoch (mc:249-330), BASELINE "
                                       "config 1", "clips_per_gpu": args.batch, "batch": 8, "clip_len": args.T,
                           "frame": f"1x{args.H}x{args.W}", "parallelism": f"dp{world}",
                           "step": "one epoch (4 iterations)"},
                "roofline": {"bound": "mfma", "kernel": "whole step", "achieved": round(tflops, 3),
                             "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(tflops / PEAK_FP32_TFLOPS, 4),
                             "traffic": None, "basis": "566.3 MFLOP per train clip (SURVEY §8d) x clips / time"},
                "cpu_baseline": cpu, "parity": parity, "final_loss": r["loss"]}), flush=True)
        finish(world)
        return
    if args.config == "cad1":
        r = run_ae(args, rank, world, local_rank)
        if rank == 0:
            cpu, parity = (None, None) if args.no_cpu_baseline else ae_cpu(args, r)
            clips = world * args.batch * args.steps
            tflops = ae_flops_per_clip(args.T) * args.batch / (r["step_ms"] * 1e-3) / 1e12
            print(json.dumps({
                "metric": BASELINE_METRIC, "value": round(clips / r["elapsed"], 3), "unit": "clips/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["step_ms"], 4),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
                "data": "synthetic grayscale clips (keyed-hash u8 / 255, clamped to [0.001, 0.999]); random-init "
                        "weights (torch.manual_seed(0))",
                "config": {"workload": "causal_anomaly_detection1.py memory-autoencoder train_model step "
                                       "(cad1:378-431), SURVEY §8f", "clips_per_gpu": args.batch,
                           "global_batch": world * args.batch, "clip_len": args.T, "frame": "1x64x64",
                           "parallelism": f"dp{world}"},
                "roofline": {"bound": "mfma", "kernel": "whole step", "achieved": round(tflops, 3),
                             "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(tflops / PEAK_FP32_TFLOPS, 4),
                             "traffic": None,
                             "basis": f"{ae_flops_per_clip(args.T)} algorithmic FLOP per clip x clips / step time"},
                "cpu_baseline": cpu, "parity": parity, "final_loss": r["loss"], "final_status": r["status"]}),
                flush=True)
        finish(world)
        return
    if args.config == "a2":
        r = run_a2(args, rank, world, local_rank)
        if rank == 0:
            cpu, parity = (None, None) if args.no_cpu_baseline else a2_cpu(args, r)
            clips = world * args.batch * args.steps
            fpc = a2_flops_per_clip(args.T, args.H, args.W)
            tflops = fpc * args.batch / (r["step_ms"] * 1e-3) / 1e12
            a2_step_bytes, a2_src = pmc_step("cfga2") if (args.batch, args.T, args.H, args.W) == (32, 8, 64, 64) \
                else (None, None)
            print(json.dumps({
                "metric": BASELINE_METRIC, "value": round(clips / r["elapsed"], 3), "unit": "clips/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["step_ms"], 4),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
                "data": "synthetic RGB clips (keyed-hash u8 / 255); random-init weights (torch.manual_seed(0))",
                "config": {"workload": "avenue_training_script2.py ImprovedMiniCausalVAD train step (a2:218-245), "
                                       "SURVEY §8 a15/a16 (the reference loader's batch is 4: --batch 4)",
                           "clips_per_gpu": args.batch, "global_batch": world * args.batch, "clip_len": args.T,
                           "frame": f"3x{args.H}x{args.W}", "parallelism": f"dp{world}"},
                "roofline": {"bound": "mfma", "kernel": "whole step", "achieved": round(tflops, 3),
                             "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(tflops / PEAK_FP32_TFLOPS, 4),
                             "traffic": a2_step_bytes, "traffic_unit": "HBM bytes per step (every kernel; PMC "
                             "FETCH_SIZE x2 + WRITE_SIZE)", "traffic_source": a2_src,
                             "basis": f"{fpc} algorithmic FLOP per clip x clips / step time"},
                "cpu_baseline": cpu, "parity": parity, "final_loss": r["loss"], "stepped": r["stepped"]}),
                flush=True)
        finish(world)
        return
    if args.config == 5:
        r = run_bbox(args, rank, world, local_rank)
        if rank == 0:
            cpu, parity = (None, None) if args.no_cpu_baseline else bbox_cpu(args, r)
            clips = world * args.batch * args.steps
            print(json.dumps({
                "metric": BASELINE_METRIC, "value": round(clips / r["elapsed"], 3), "unit": "clips/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["step_ms"], 4),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
                "data": "synthetic RGB clips (keyed-hash u8 / 255), random-init weights (torch.manual_seed(0))",
                "config": {"workload": "avenue_training_script_bbox.py clip scorer (bbox:339-368), BASELINE config 5 "
                                       "(inference)", "clips_per_gpu": args.batch, "clip_len": "8/16/32 mixed",
                           "frame": "3x64x64", "packing": "one batch per T", "parallelism": f"dp{world}",
                           "frames_per_step_per_gpu": r["frames"]},
                "roofline": bbox_roofline(r["frames"] / (r["step_ms"] * 1e-3), r["frames"]),
                "cpu_baseline": cpu, "parity": parity}), flush=True)
        finish(world)
        return
    r = run_gpu(args, rank, world, local_rank)
    if rank == 0:
        cpu = None if args.no_cpu_baseline else cpu_baseline(args)
        parity = None if (args.no_cpu_baseline or r.get("probe") is None) else parity_check(args, r["probe"])
        clips = world * args.batch * args.steps
        out = {
            "metric": BASELINE_METRIC,
            "value": round(clips / r["elapsed"], 3),
            "unit": "clips/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["step_ms"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (keyed-hash u8 pixels, Normalize(0.5,0.5)); random-init weights (torch.manual_seed(0))",
            "config": {"workload": "causal_anomaly_detection.py train step (cad:669-690), BASELINE config "
                                   + (("2" if world == 1 else "3") if args.config == 2 else "4"),
                       "clips_per_gpu": args.batch, "global_batch": world * args.batch, "clip_len": args.T,
                       "frame": f"1x{args.H}x{args.W}", "parallelism": f"dp{world}"},
            "roofline": r["roof"],
            "cpu_baseline": cpu,
            "parity": parity,
            "h2d_inclusive": r.get("h2d"),
            "dropin_loop": r.get("dropin"),
            "bn_stats": "group (SyncBatchNorm)" if (args.sync_bn and world > 1) else "per rank",
            "step_roofline": step_roofline(args, clips / r["elapsed"] / world, r["step_tflops"]),
            "allreduce_bytes_per_step": r["allreduce_bytes"],
            "post_backbone_us": (round(r["post_backbone_us"], 1) if r.get("post_backbone_us") is not None else None),
            "host_enqueue_ms_per_step": round(r["host_enqueue_ms"], 4),
            "final_loss": r["final_loss"],
        }
        if args.breakdown_out:
            with open(args.breakdown_out, "w") as f:
                json.dump({"dominant": r["dominant"], "per_label_ms": r["breakdown"]}, f, indent=1)
        print(json.dumps(out), flush=True)
    finish(world)


if __name__ == "__main__":
    main()
