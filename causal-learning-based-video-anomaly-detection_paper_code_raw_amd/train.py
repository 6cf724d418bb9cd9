"""train_model / test_model / apply_memory_efficient_training of causal_anomaly_detection.py (cad:592-835),
driving the fused libvadhip step: forward + loss + backward + clip_grad_norm_(1.0) + AdamW in HIP kernels,
with an optional data-parallel gradient all-reduce (RCCL) between backward and the optimizer.
"""
from __future__ import annotations

import math
import re

import torch
import torch.distributed as dist

from .cad import CausalAnomalyDetector  # noqa: F401  (re-export for callers of this module)
from .data import ClipStager, prefetch


def apply_memory_efficient_training(model):
    """Freeze backbone.conv1 / backbone.bn1 (cad:592-607)."""
    for name, param in model.named_parameters():
        if "backbone.conv1" in name or "backbone.bn1" in name:
            param.requires_grad = False
    total = sum(p.numel() for p in model.parameters())
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    print(f"Total parameters: {total:,}")
    print(f"Trainable parameters: {trainable:,}")
    print(f"Frozen parameters: {total - trainable:,}")
    return model


class CadTrainer:
    """One fused train step per call; the building block of train_model and bench.py.

    Data parallel: one process per GPU; rank r processes global clips [r*B, (r+1)*B) of each step (RNG keyed by
    global clip index), grads (+ has-grad flags) are summed by bucketed all_reduces -- detector + causal head + direct
    classifier + flags during the backbone backward, the backbone in per-layer buckets as its layers finish
    (_backward_overlapped) -- and scaled by 1/world inside the optimizer kernel; BN running stats follow rank 0
    (broadcast right after each forward, DDP's broadcast_buffers).  No step blocks the host on the device.

    sync_bn=True (world > 1): SyncBatchNorm semantics -- every BN layer normalises over the whole group's batch
    (per-layer sums all-reduced in forward and backward), so the N-rank step equals the reference's single-process
    step on the global batch (BASELINE config 3: batch 64 over 8 GPUs); running stats then agree on every rank and
    are not broadcast.
    """

    def __init__(self, model, lr=3e-4, weight_decay=1e-5, eps=1e-8, betas=(0.9, 0.999), max_norm=1.0, seed=0,
                 process_group=None, engine=None, compute_dtype=None, sync_bn=False, force_dist=False,
                 prio_stream=False, skip_zero_detector=False):
        """force_dist: run the data-parallel protocol (broadcasts, bucketed all-reduces, SyncBN callback) even at
        world size 1 of an initialised process group -- exercises the collective path on one device (tests).
        skip_zero_detector (world > 1): all-reduce the ranks' detector has-grad flags after the forward and read the
        sum on the host; when it is zero (no box in range on any rank, cad:221-226) the detector's 13.3 MB of grads --
        zero on every rank -- are left out of the head bucket.  One small collective and a host wait per step instead
        of 13.3 MB on the wire: for interconnect-bound setups (the default sums it and never waits).
        prio_stream: run each step on a stream of the device's greatest priority (ordered after and before the
        caller's stream), so with the plan's low-priority weight-gradient stream (knob cad_stream_prio) the dispatcher
        prefers the critical path's workgroups."""
        self.model = model
        if compute_dtype is not None:
            model.set_compute_dtype(compute_dtype)
        self.eng = engine if engine is not None else model.engine()
        self.lr, self.wd, self.eps, self.betas, self.max_norm = lr, weight_decay, eps, betas, max_norm
        self.seed = seed
        self.step_idx = 0
        self.pg = process_group
        initialised = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if initialised else 1
        self.rank = dist.get_rank(process_group) if initialised else 0
        self.dist = initialised and (self.world > 1 or force_dist)
        self.eng.init_optimizer_state()
        self.sync_bn = bool(sync_bn) and self.dist
        self.skip_zero_detector = bool(skip_zero_detector) and self.dist
        self._det_flag = None
        # gradient buckets of the flat grad buffer (slot order: backbone | detector | causal head | direct classifier
        # | has-grad flags): everything from the detector on is one bucket, summed beside the backbone backward
        names = self.eng.slot_names
        i0 = next(i for i, n in enumerate(names) if n.startswith("detector."))
        i1 = next(i for i in range(i0, len(names)) if not names[i].startswith("detector."))
        self.det_range = (self.eng.slot_offset[i0], self.eng.slot_offset[i1])
        # backbone buckets [lo, hi) of the flat grad buffer, in the backward's order, each with the backbone layer
        # whose grads finish last in it: layer 7, layer 6, layers 5-4, layers 3-0 + the stem (the small layers are
        # merged: a collective costs ~10-30 us of latency at 8 ranks whatever its size)
        first = {}
        for i, n in enumerate(names):
            m = re.match(r"backbone\.layer(\d)\.(\d)\.", n)
            if m:
                l = 2 * (int(m.group(1)) - 1) + (0 if int(m.group(2)) < 3 else 1)
                first.setdefault(l, self.eng.slot_offset[i])
        first[8] = self.det_range[0]
        first[0] = 0
        self.bb_buckets = [(first[lo], first[hi], lo) for lo, hi in ((7, 8), (6, 7), (4, 6), (0, 4))]
        self.allreduce_floats = 0  # floats all-reduced by the last step (per rank, before the ring's 2(P-1)/P factor)
        self.prio_stream = None
        self._bufs_init, self._bufs_ev, self._arm_stream = False, None, None
        if prio_stream and self.eng.grads.is_cuda:
            self.prio_stream = torch.cuda.Stream(self.eng.device, priority=-1)
        if self.dist:
            dist.broadcast(self.eng.params, 0, group=process_group)
            dist.broadcast(self.eng.bufs, 0, group=process_group)
        if self.sync_bn:
            # the statistics travel on a communicator of their own, so on RCCL they are not queued behind the
            # head-grad all-reduce that overlaps the backbone backward (_backward_overlapped)
            ranks = dist.get_process_group_ranks(process_group) if process_group is not None else None
            self._bn_pg = dist.new_group(ranks=ranks)
            self.eng.set_bn_sync(self._bn_pg)

    def step(self, videos, labels, lr=None, want_outputs=False, inputs_ready=None, host_losses=False):
        """One training step; returns the (device) loss vector [cls, anomaly, causal, kl, total] (want_outputs: the
        forward's output dict, see CadEngine.forward).  host_losses=True: returns that vector as a CPU tensor instead
        -- the reference reads loss.item() every step (cad:692); here the forward's loss-tail kernel writes it into
        pinned host memory and the host waits only for the forward (an event), so the backward and optimizer it has
        already queued keep the device busy while the caller prepares the next step.  inputs_ready: None -- the clips are produced on the current
        stream, the step is ordered after it; True -- they are complete on the device already (staged and
        synchronised before); a torch.cuda.Stream -- its queued work completes them; a torch.cuda.Event -- its
        completion does (ClipStager.finish(h, wait=False) with h.ready).  Given, the frozen stem may start
        beside the previous step's queued tail (CadEngine.input_ready)."""
        if self.prio_stream is not None and self.eng.grads.is_cuda:
            # the step's critical path on a stream of the device's greatest priority (the plan's weight-gradient stream
            # runs at its least with knob cad_stream_prio), ordered after / before the caller's stream
            caller = torch.cuda.current_stream(self.eng.device)
            self.prio_stream.wait_stream(caller)
            with torch.cuda.stream(self.prio_stream):
                o = self._step(videos, labels, lr, want_outputs, inputs_ready, host_losses)
            caller.wait_stream(self.prio_stream)
            return o
        return self._step(videos, labels, lr, want_outputs, inputs_ready, host_losses)

    def _step(self, videos, labels, lr, want_outputs, inputs_ready=None, host_losses=False):
        eng = self.eng
        B = videos.shape[0]
        cur = torch.cuda.current_stream(eng.device) if eng.grads.is_cuda else None
        bcast = self.dist and not self.sync_bn
        if bcast and not self._bufs_init:
            # (the buffers of rank 0, before the first forward; later steps take them right after each forward)
            dist.broadcast(eng.bufs, 0, group=self.pg)
            self._bufs_init = True
            if cur is not None:
                self._bufs_ev = torch.cuda.Event()
                self._bufs_ev.record(cur)
        if (inputs_ready is not None and inputs_ready is not True and cur is not None
                and (videos.dtype != torch.float32 or not videos.is_contiguous())):
            # the forward converts these clips on the current stream: it must see them complete first (only fp32
            # contiguous clips, e.g. ClipStager's, are read in place by the early stem alone)
            if isinstance(inputs_ready, torch.cuda.Event):
                cur.wait_event(inputs_ready)
            else:
                cur.wait_stream(inputs_ready)
        if inputs_ready is not None and cur is not None:
            # the early stem waits for the inputs and for the last buffer broadcast (it updates bn1's running stats),
            # not for the previous step's tail on the current stream
            if self._arm_stream is None:
                self._arm_stream = torch.cuda.Stream(eng.device)
            if isinstance(inputs_ready, torch.cuda.Event):
                self._arm_stream.wait_event(inputs_ready)
            elif inputs_ready is not True:
                self._arm_stream.wait_stream(inputs_ready)
            if self._bufs_ev is not None:
                self._arm_stream.wait_event(self._bufs_ev)
            T, H, W = videos.shape[1], videos.shape[3], videos.shape[4]
            eng.input_ready(B, T, H, W, stream=self._arm_stream)
        lh = None
        if host_losses and not want_outputs and cur is not None:
            if getattr(self, "_loss_host", None) is None:
                # (one buffer: the host has read step k's losses before step k+1's forward is queued)
                self._loss_host = torch.zeros(5, dtype=torch.float32).pin_memory()
                self._loss_ev = torch.cuda.Event()
            lh = self._loss_host
        kw = {"loss_host": lh} if lh is not None else {}
        o = eng.forward(videos, True, self.seed, self.step_idx, self.rank * B, labels, want_outputs=want_outputs, **kw)
        # (the forward's per-rank "detector has a grad" flag; an engine without it: the grad buffer's flag after the
        # backward, see _head_bucket_start)
        self._det_flag = o["flags"][:1] if self.skip_zero_detector and "flags" in o else None
        if lh is not None:
            self._loss_ev.record(cur)
        if bcast:
            # the running statistics are final once the forward has run (the backward does not touch them): every
            # rank takes rank 0's here -- the values the reference's replicas start the next step from
            dist.broadcast(eng.bufs, 0, group=self.pg)
            if cur is not None:
                self._bufs_ev.record(cur)
        self.allreduce_floats = 0
        if self.dist and eng.grads.is_cuda:
            self._backward_overlapped()
        else:
            eng.backward(True)
            if self.dist:
                self._reduce(eng.grads[self._head_bucket_start():])  # detector + causal head + direct classifier + flags
                self._reduce(eng.grads[:self.det_range[0]])
        eng.optimizer_step(self.lr if lr is None else lr, self.betas, self.eps, self.wd, self.max_norm,
                           1.0 / self.world)
        self.step_idx += 1
        if lh is not None:
            self._loss_ev.synchronize()  # the forward (loss tail) is done; backward + optimizer may still run
            return lh.clone()
        if host_losses and not want_outputs:
            return o["losses"].cpu()
        return o if want_outputs else o["losses"]

    def _reduce(self, t):
        dist.all_reduce(t, group=self.pg)
        self.allreduce_floats += t.numel()

    def _backward_overlapped(self):
        """Backward in two stages with the gradient all-reduce in buckets (DDP's reduce-during-backward, with the
        splits chosen for this model's grad order):
          1. detector + causal head + direct classifier + the has-grad flags, summed on a side stream while the
             backbone backward runs on the compute stream (which waits only for the detector's input gradient).  The
             detector part (13.3 MB) is identically zero on every rank when no box is in range (every frame took the
             fallback box, cad:221-226) -- it is summed anyway: skipping it would need the flag on the host, i.e. a
             host wait on the device every step, while its all-reduce runs beside the ~1 ms backbone backward;
          2. the backbone in four buckets (self.bb_buckets), each issued behind the plan's event for the last of its
             layers to finish (vad_cad_wait_layer_grads), so layer 7's all-reduce runs beside layers 6-0's backward.
        The optimizer waits for all of them; the host never waits for the device.  Each element is summed over the
        same ranks as one all_reduce of the whole buffer, so results are identical to it."""
        eng = self.eng
        main = torch.cuda.current_stream(eng.device)
        if getattr(self, "_comm", None) is None:
            self._comm = torch.cuda.Stream(eng.device)
        side = self._comm
        d0 = self._head_bucket_start()
        # stage 2: the causal-head / detector backward keeps running on the plan's side stream while the backbone
        # (stage 1) starts; the all-reduce stream waits for both that side stream and the compute stream
        eng.backward(True, stage=2)
        eng.wait_side(side)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self._reduce(eng.grads[d0:])
        eng.backward(True, stage=1)
        for lo, hi, layer in self.bb_buckets:
            eng.wait_layer_grads(layer, side)
            with torch.cuda.stream(side):
                self._reduce(eng.grads[lo:hi])
        main.wait_stream(side)


    def _head_bucket_start(self):
        """Start of the head bucket in the flat grad buffer: the detector's first grad, or with skip_zero_detector
        and no rank's detector having a grad this step (the summed flag read on the host: the same decision on every
        rank), the slot after the detector's."""
        if not self.skip_zero_detector:
            return self.det_range[0]
        src = self._det_flag
        if src is None:  # (engines whose forward reports no flags: the grad buffer's, final after the backward)
            src = self.eng.grads[self.eng.param_floats:self.eng.param_floats + 1]
        f = src.detach().clone().float()
        self._reduce(f)
        self.det_flag_sum = float(f.item())
        return self.det_range[1] if self.det_flag_sum == 0.0 else self.det_range[0]


def _cosine_lr(base, epoch, t_max):
    return 0.5 * base * (1 + math.cos(math.pi * epoch / t_max))


def _eval_losses(model, videos, labels):
    eng = model.engine()
    o = eng.forward(videos, False, 0, 0, 0, labels)
    return o


def train_epoch(trainer, train_loader, stager, epoch=0, num_epochs=1, lr=None, log=print):
    """One epoch of train_model's inner loop (cad:637-700): per batch one fused step and the per-step loss read the
    reference does (loss.item(), cad:692), the running total and the batch print every 5 batches.  Returns
    (summed total loss, batches).  u8 clips (vad_amd.data datasets) are staged through pinned memory and normalised on
    the device one batch ahead, the step's early stem waiting for them (inputs_ready); the losses come back through
    pinned memory right after the forward (CadTrainer.step(host_losses=True)), so reading them does not drain the
    queued backward.  Float clips (the reference's own datasets) are copied as they are."""
    tot, nb = 0.0, 0
    for batch_idx, (videos, labels, ready) in enumerate(prefetch(train_loader, stager, with_ready=True)):
        try:
            l = trainer.step(videos, labels, lr=lr, inputs_ready=ready, host_losses=True).tolist()
            tot += l[4]
            nb += 1
            if batch_idx % 5 == 0 and log is not None:
                log(f"Epoch {epoch+1}/{num_epochs}, Batch {batch_idx+1}, Total: {l[4]:.6f}, Class: {l[0]:.6f}")
        except RuntimeError as e:
            if "out of memory" in str(e):
                print(f"CUDA out of memory at batch {batch_idx}. Skipping batch...")
                torch.cuda.empty_cache()
                continue
            raise
    return tot, nb


def train_model(model, train_loader, val_loader, num_epochs=20, lr=3e-4):
    """Training loop with the multi-objective loss (cad:609-790).  Returns (model, train_losses, val_losses)."""
    model = apply_memory_efficient_training(model)
    dev = torch.device("cuda", torch.cuda.current_device())
    model.to(dev)
    trainer = CadTrainer(model, lr=lr)
    stager = ClipStager(dev, mode=0)
    train_losses, val_losses = [], []
    print("Starting training with mixed precision: False")
    for epoch in range(num_epochs):
        model.train()
        cur_lr = _cosine_lr(lr, epoch, num_epochs)
        tot, nb = train_epoch(trainer, train_loader, stager, epoch, num_epochs, cur_lr)
        model.eval()
        vtot, vb, correct, total = 0.0, 0, 0, 0
        with torch.no_grad():
            for videos, labels in prefetch(val_loader, stager):
                o = _eval_losses(model, videos, labels)
                vtot += o["losses"][4].item()
                vb += 1
                correct += (o["probs"].argmax(1) == labels).sum().item()
                total += labels.numel()
        train_losses.append(tot / max(nb, 1))
        val_losses.append(vtot / max(vb, 1))
        print(f"Epoch {epoch+1}/{num_epochs}, Train Loss: {train_losses[-1]:.6f}, Val Loss: {val_losses[-1]:.6f}, "
              f"Val Accuracy: {correct / max(total, 1):.4f}")
    return model, train_losses, val_losses


def test_model(model, test_loader):
    """Scores every clip (cad:796-835); returns (scores, labels, outputs)."""
    model.eval()
    dev = next(model.parameters()).device
    scores, labels_all, outs = [], [], []
    with torch.no_grad():
        for videos, labels in prefetch(test_loader, ClipStager(dev, mode=0)):
            out = model(videos)
            scores.extend(out["anomaly_scores"].cpu().tolist())
            labels_all.extend(labels.cpu().tolist())
            outs.append(out)
    import numpy as np
    return np.array(scores), np.array(labels_all), outs
