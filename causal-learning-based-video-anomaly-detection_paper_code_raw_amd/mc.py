"""Drop-in SimpleVideoAnomalyDetector + StableTrainer of minicausal_vad_complete3.py (config 1), on the HIP plan.

Same class names, constructor signatures, submodule names (state_dict keys ``features.N.*``, ``classifier.N.*``),
initialisation order (mc:76-88: so a given torch seed draws the reference's weights) and forward return
``(B, 1)`` sigmoid scores (mc:90-102).  The compute goes through ``libvadhip.so`` (``vad_mc_*``): 3-D convs as
im2col + f32 MFMA GEMMs, train-mode BatchNorm3d, fused BN+ReLU+MaxPool3d, the classifier, BCE, and the
StableTrainer update (NaN/Inf skip, conditional clip, Adam with coupled L2) in device kernels.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn as nn

from . import _native as nat


class SimpleVideoAnomalyDetector(nn.Module):
    """mc:25-102.  ``forward(x)`` takes ``(B, C, T, H, W)`` and returns ``(B, 1)`` anomaly scores."""

    def __init__(self, input_channels=1, temporal_frames=8, spatial_size=64):
        super().__init__()
        self.temporal_frames = temporal_frames
        self.spatial_size = spatial_size
        self.features = nn.Sequential(
            nn.Conv3d(input_channels, 8, kernel_size=3, stride=1, padding=1), nn.BatchNorm3d(8), nn.ReLU(inplace=True),
            nn.MaxPool3d(kernel_size=(1, 2, 2), stride=(1, 2, 2)),
            nn.Conv3d(8, 16, kernel_size=3, stride=1, padding=1), nn.BatchNorm3d(16), nn.ReLU(inplace=True),
            nn.MaxPool3d(kernel_size=(2, 2, 2), stride=(2, 2, 2)),
            nn.Conv3d(16, 32, kernel_size=3, stride=1, padding=1), nn.BatchNorm3d(32), nn.ReLU(inplace=True),
            nn.MaxPool3d(kernel_size=(2, 2, 2), stride=(2, 2, 2)),
            nn.AdaptiveAvgPool3d((1, 1, 1)))
        self.classifier = nn.Sequential(
            nn.Dropout(0.5), nn.Linear(32, 16), nn.ReLU(inplace=True), nn.Dropout(0.3), nn.Linear(16, 8),
            nn.ReLU(inplace=True), nn.Linear(8, 1), nn.Sigmoid())
        self._initialize_weights()
        self.to(dtype=torch.float32)
        self._engine = None
        self._step = 0

    def _initialize_weights(self):
        for m in self.modules():
            if isinstance(m, nn.Conv3d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm3d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.constant_(m.bias, 0)

    # ------------------------------------------------------------------ HIP engine plumbing
    def engine(self, x: torch.Tensor) -> "McEngine":
        e = self._engine
        if e is None or e.device != x.device:
            e = McEngine(self, x.device)
            self._engine = e
        e.sync_from_module()
        e.use_shape(tuple(x.shape))
        return e

    def forward(self, x, *, seed=None, step=None, clip0=0):
        if x.dim() != 5:
            raise ValueError(f"Expected 5D tensor (B,C,T,H,W), got {x.shape}")
        nat.require_hip(x)
        if x.dtype != torch.float32:
            x = x.float()
        e = self.engine(x)
        if seed is None:
            seed = e.seed
        if step is None:
            step = self._step
            if self.training:
                self._step += 1
        params = [p for _, p in self.named_parameters()]  # slot order == named_parameters order
        return _McFunction.apply(x, e, self.training, seed, step, clip0, *params)


class _McFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, e, training, seed, step, clip0, *params):
        scores = e.forward(x.contiguous(), training, seed, step, clip0, labels=None)
        ctx.e = e
        return scores.view(-1, 1).clone()

    @staticmethod
    def backward(ctx, d_scores):
        e = ctx.e
        e.backward_from_scores(d_scores.reshape(-1).contiguous().float())
        grads = e.grad_views_for_autograd()
        return (None, None, None, None, None, None, *grads)


class _McPlan:
    """One C plan + workspace per input shape, bound to the engine's shared flat buffers."""

    def __init__(self, e: "McEngine", shape):
        lib = nat.lib()
        plan = ctypes.c_void_p()
        nat.check(lib.vad_mc_create(*shape, ctypes.byref(plan)))
        self.plan = plan
        self.ws = torch.empty(lib.vad_mc_workspace_bytes(plan) + 256, dtype=torch.uint8, device=e.device)
        base = (self.ws.data_ptr() + 255) // 256 * 256
        nat.check(lib.vad_mc_bind(plan, ctypes.c_void_p(base), nat.ptr(e.params), nat.ptr(e.grads), nat.ptr(e.bufs),
                                  nat.ptr(e.nbt), nat.ptr(e.exp_avg), nat.ptr(e.exp_avg_sq), nat.ptr(e.steps)))

    def __del__(self):
        try:
            if getattr(self, "plan", None):
                nat.lib().vad_mc_destroy(self.plan)
        except Exception:
            pass


class McEngine:
    """Flat device buffers (params / grads / BN buffers / Adam state, state_dict order) shared by per-shape plans."""

    def __init__(self, model: SimpleVideoAnomalyDetector, device):
        lib = nat.lib()
        self.device, self.model, self.seed = device, model, 1234
        C = model.features[0].in_channels
        probe = ctypes.c_void_p()
        nat.check(lib.vad_mc_create(1, C, 8, 8, 8, ctypes.byref(probe)))  # the slot table depends on C only
        try:
            self.slots = [(lib.vad_mc_slot_name(probe, i).decode(), lib.vad_mc_slot_offset(probe, i),
                           lib.vad_mc_slot_numel(probe, i)) for i in range(lib.vad_mc_num_slots(probe))]
            self.bufs_meta = [(lib.vad_mc_buf_name(probe, i).decode(), lib.vad_mc_buf_offset(probe, i),
                               lib.vad_mc_buf_numel(probe, i)) for i in range(lib.vad_mc_num_bufs(probe))]
            nparam, nbuf = lib.vad_mc_param_floats(probe), lib.vad_mc_buf_floats(probe)
        finally:
            lib.vad_mc_destroy(probe)
        f = dict(dtype=torch.float32, device=device)
        self.params = torch.zeros(nparam, **f)
        self.grads = torch.zeros(nparam + 256, **f)
        self.bufs = torch.zeros(nbuf, **f)
        self.nbt = torch.zeros(3, dtype=torch.int64, device=device)
        self.exp_avg = torch.zeros_like(self.params)
        self.exp_avg_sq = torch.zeros_like(self.params)
        self.steps = torch.zeros(len(self.slots), dtype=torch.int32, device=device)
        self.losses = torch.zeros(4, **f)  # bce, grad_norm, clipped, status
        self.flags = torch.zeros(4, dtype=torch.int32, device=device)
        sd = dict(model.named_parameters())
        self.param_views = [self.params[off:off + n].view_as(sd[name]) for name, off, n in self.slots]
        self._bound = False
        self.plans = {}
        self.cur = None
        self.scores = None

    def use_shape(self, shape):
        if shape not in self.plans:
            self.plans[shape] = _McPlan(self, shape)
        self.cur = self.plans[shape]
        if self.scores is None or self.scores.numel() != shape[0]:
            self.scores = torch.zeros(shape[0], dtype=torch.float32, device=self.device)

    def stream(self):
        return nat.stream_of(self.device)

    def sync_from_module(self):
        """Point the module's parameters / BN buffers at the flat device buffers (copied once)."""
        if self._bound:
            return
        m = self.model
        with torch.no_grad():
            sd = dict(m.named_parameters())
            for (name, off, n), view in zip(self.slots, self.param_views):
                view.copy_(sd[name].detach().to(self.device))
                mod_name, attr = name.rsplit(".", 1)
                setattr(m.get_submodule(mod_name), attr, nn.Parameter(view, requires_grad=sd[name].requires_grad))
            mods = dict(m.named_modules())
            for name, off, n in self.bufs_meta:
                mod_name, attr = name.rsplit(".", 1)
                mod = mods[mod_name]
                view = self.bufs[off:off + n].view_as(getattr(mod, attr))
                view.copy_(getattr(mod, attr).to(self.device))
                mod._buffers[attr] = view
            for i, b in enumerate(("features.1", "features.5", "features.9")):
                self.nbt[i] = int(mods[b].num_batches_tracked)
                mods[b]._buffers["num_batches_tracked"] = self.nbt[i:i + 1].view(())
        self._bound = True

    def forward(self, x, training, seed, step, clip0, labels=None):
        nat.check(nat.lib().vad_mc_forward(self.cur.plan, nat.ptr(x), int(training), ctypes.c_uint64(seed),
                                           ctypes.c_uint64(step), ctypes.c_int64(clip0),
                                           nat.ptr(labels) if labels is not None else None, nat.ptr(self.scores),
                                           nat.ptr(self.losses), nat.ptr(self.flags), self.stream()))
        return self.scores

    def backward(self):
        """Backward of the BCE loss of the last forward (StableTrainer path)."""
        nat.check(nat.lib().vad_mc_backward(self.cur.plan, None, self.stream()))

    def backward_from_scores(self, d_scores):
        nat.check(nat.lib().vad_mc_backward(self.cur.plan, nat.ptr(d_scores), self.stream()))

    def grad_views_for_autograd(self):
        return [self.grads[off:off + n].view_as(v).clone() for (name, off, n), v in zip(self.slots, self.param_views)]

    def optimizer_step(self, lr, wd=1e-5, b1=0.9, b2=0.999, eps=1e-8, clip_above=10.0, max_norm=1.0):
        nat.check(nat.lib().vad_mc_optimizer_step(self.cur.plan, ctypes.c_float(lr), ctypes.c_float(b1),
                                                  ctypes.c_float(b2), ctypes.c_float(eps), ctypes.c_float(wd),
                                                  ctypes.c_float(clip_above), ctypes.c_float(max_norm),
                                                  self.stream()))


class _AdamSurface:
    """The torch.optim.Adam surface StableTrainer exposes (mc:229-234): ``param_groups[0]['lr']`` is the live learning
    rate the device step uses (the reference's driver prints it every epoch, mc:414) and may be written; the Adam
    moments themselves live in the engine's flat device buffers.  ``zero_grad`` is a no-op (the fused step writes
    every grad)."""

    def __init__(self, lr, weight_decay=1e-5, eps=1e-8, betas=(0.9, 0.999)):
        self.param_groups = [{"lr": lr, "initial_lr": lr, "weight_decay": weight_decay, "eps": eps, "betas": betas}]
        self.defaults = dict(self.param_groups[0])

    def zero_grad(self, set_to_none=True):
        pass


class _StepLRSurface:
    """optim.lr_scheduler.StepLR(optimizer, step_size=15, gamma=0.7) (mc:237): ``step()`` once per epoch."""

    def __init__(self, optimizer, step_size=15, gamma=0.7):
        self.optimizer, self.step_size, self.gamma = optimizer, step_size, gamma
        self.base_lrs = [g["initial_lr"] for g in optimizer.param_groups]
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        for g, b in zip(self.optimizer.param_groups, self.base_lrs):
            g["lr"] = b * self.gamma ** (self.last_epoch // self.step_size)

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        return {"step_size": self.step_size, "gamma": self.gamma, "base_lrs": list(self.base_lrs),
                "last_epoch": self.last_epoch, "_last_lr": self.get_last_lr()}

    def load_state_dict(self, sd):
        self.step_size, self.gamma = sd["step_size"], sd["gamma"]
        self.base_lrs, self.last_epoch = list(sd["base_lrs"]), sd["last_epoch"]


class StableTrainer:
    """mc:218-420 with the train step on the HIP plan.  ``train_epoch`` / ``evaluate`` / ``train_model`` keep the
    reference's return values and history keys; ``optimizer`` / ``scheduler`` / ``criterion`` keep its attributes
    (Adam lr/wd 1e-5/eps 1e-8, StepLR(15, 0.7), BCELoss; mc:229-240)."""

    def __init__(self, model, train_loader, test_loader, device, lr=0.001):
        self.model = model.to(device)
        self.train_loader = train_loader
        self.test_loader = test_loader
        self.device = torch.device(device)
        self.optimizer = _AdamSurface(lr, weight_decay=1e-5, eps=1e-8)
        self.scheduler = _StepLRSurface(self.optimizer, step_size=15, gamma=0.7)
        self.criterion = nn.BCELoss()
        self.history = {"train_loss": [], "test_loss": [], "test_auc": [], "train_acc": [], "test_acc": []}
        self.best_auc = 0.0
        self.seed = 1234
        self.global_step = 0
        self.clip0 = 0

    @property
    def lr(self):
        return self.optimizer.param_groups[0]["lr"]

    @property
    def epoch(self):
        return self.scheduler.last_epoch

    def _lr(self):
        return self.optimizer.param_groups[0]["lr"]

    def _queue_step(self, data, targets):
        """Queue one mc:259-318 iteration on device and an asynchronous copy of its host-visible results (loss,
        status, correct count) into a pinned slot; returns the handle _finish reads."""
        data = data.to(device=self.device, dtype=torch.float32).contiguous()
        targets = targets.to(device=self.device, dtype=torch.float32).contiguous()
        self.model.train()
        e = self.model.engine(data)
        e.forward(data, True, self.seed, self.global_step, self.clip0, labels=targets)
        e.backward()
        g = self.optimizer.param_groups[0]
        e.optimizer_step(self._lr(), wd=g["weight_decay"], b1=g["betas"][0], b2=g["betas"][1], eps=g["eps"])
        self.global_step += 1
        self.clip0 += data.shape[0]
        if getattr(self, "_res_host", None) is None:
            self._res_host = torch.zeros(2, 3, dtype=torch.float32).pin_memory()
            self._res_ev = [torch.cuda.Event(), torch.cuda.Event()]
            self._slot = 0
        k = self._slot
        self._slot ^= 1
        corr = ((e.scores > 0.5).float() == targets).sum().reshape(1)
        dev = torch.cat([e.losses[0:1], e.losses[3:4], corr.float()])
        self._res_host[k].copy_(dev, non_blocking=True)
        self._res_ev[k].record()
        return k, targets.numel()

    def _finish(self, h):
        k, n = h
        self._res_ev[k].synchronize()
        loss, status, corr = self._res_host[k].tolist()
        # status 0: skipped before backward (not counted); 1: counted, no update (non-finite grads); 2: stepped
        counted = status > 0.5
        return loss, (int(corr) if counted else 0), n, counted

    def train_step(self, data, targets):
        """One mc:259-318 iteration on device; returns (loss, correct, n, counted) as host numbers."""
        return self._finish(self._queue_step(data, targets))

    def train_epoch(self):
        """mc:259-330 over the loader.  The host reads iteration k's loss / status / accuracy (the reference's
        per-iteration .item() reads) after it has queued iteration k+1, so the device never idles on the host round
        trip; the sums are the same numbers in the same order."""
        total_loss, correct, total = 0.0, 0, 0
        pending = None

        def take(h):
            nonlocal total_loss, correct, total
            loss, c, n, counted = self._finish(h)
            if counted:
                total_loss += loss
                correct += c
                total += n

        for data, targets in self.train_loader:
            h = self._queue_step(data, targets)
            if pending is not None:
                take(pending)
            pending = h
        if pending is not None:
            take(pending)
        n = len(self.train_loader)
        return (total_loss / n if n > 0 else 0), (correct / total if total > 0 else 0)

    def evaluate(self):
        import numpy as np
        from sklearn.metrics import roc_auc_score
        self.model.eval()
        total_loss, correct, total, outs, tars = 0.0, 0, 0, [], []
        with torch.no_grad():
            for data, targets in self.test_loader:
                data = data.to(device=self.device, dtype=torch.float32).contiguous()
                targets = targets.to(device=self.device, dtype=torch.float32)
                o = self.model(data).squeeze().float()
                if not torch.isfinite(o).all():
                    continue
                loss = torch.nn.functional.binary_cross_entropy(o, targets)
                if not torch.isfinite(loss):
                    continue
                total_loss += float(loss)
                outs.extend(o.cpu().numpy().reshape(-1).tolist())
                tars.extend(targets.cpu().numpy().reshape(-1).tolist())
                correct += int(((o > 0.5).float() == targets).sum())
                total += targets.numel()
        n = len(self.test_loader)
        avg = total_loss / n if n > 0 else float("inf")
        auc = 0.0
        if outs and len(set(tars)) > 1:
            pairs = [(o, t) for o, t in zip(outs, tars) if not (math.isnan(o) or math.isinf(o))]
            if pairs and len(set(t for _, t in pairs)) > 1:
                auc = float(roc_auc_score([t for _, t in pairs], [o for o, _ in pairs]))
        return avg, auc, (correct / total if total > 0 else 0)

    def train_model(self, epochs, save_path="simple_anomaly_model.pth"):
        for epoch in range(epochs):
            train_loss, train_acc = self.train_epoch()
            test_loss, test_auc, test_acc = self.evaluate()
            self.scheduler.step()
            for k, v in zip(("train_loss", "test_loss", "test_auc", "train_acc", "test_acc"),
                            (train_loss, test_loss, test_auc, train_acc, test_acc)):
                self.history[k].append(v)
            if test_auc > self.best_auc:
                self.best_auc = test_auc
                torch.save({"model_state_dict": self.model.state_dict(), "epoch": epoch, "best_auc": self.best_auc},
                           save_path)
            if epoch > 20 and test_auc < 0.55 and train_loss < 0.1:
                break
        return self.history
