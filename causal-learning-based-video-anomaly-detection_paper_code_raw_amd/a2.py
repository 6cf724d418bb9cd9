"""Drop-in for avenue_training_script2.py: the a2 CausalAnomalyDetector (a2:15-101) and ImprovedMiniCausalVAD
(a2:107-297) with forward / loss / backward / AdamW on the HIP plan (``vad_a2_*`` in libvadhip.so).

Same class names, constructor signatures, submodule names (state_dict keys ``feature_extractor.conv3d_1.weight``
... so the reference's ``best_improved_model.pth`` loads strictly), initialisation order and forward return
``(scores (B,1), causal_adj (B,16,16), features (B,16))``.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.nn as nn

from . import _native as nat


class CompactFeatureExtractor(nn.Module):
    """a2:15-35"""

    def __init__(self, input_channels=3, feature_dim=64):
        super().__init__()
        self.conv3d_1 = nn.Conv3d(input_channels, 16, (3, 3, 3), stride=(1, 2, 2), padding=1)
        self.conv3d_2 = nn.Conv3d(16, 32, (3, 3, 3), stride=(2, 2, 2), padding=1)
        self.conv3d_3 = nn.Conv3d(32, 64, (3, 3, 3), stride=(2, 2, 2), padding=1)
        self.adaptive_pool = nn.AdaptiveAvgPool3d((4, 4, 4))
        self.fc = nn.Linear(64 * 4 * 4 * 4, feature_dim)
        self.dropout = nn.Dropout(0.3)


class DifferentiableCausalDiscovery(nn.Module):
    """a2:37-66"""

    def __init__(self, num_variables=16, hidden_dim=32):
        super().__init__()
        self.num_variables = num_variables
        self.causal_net = nn.Sequential(nn.Linear(num_variables, hidden_dim), nn.ReLU(),
                                        nn.Linear(hidden_dim, num_variables * num_variables), nn.Sigmoid())

    def acyclicity_constraint(self, adj_matrix):
        """a2:62-66 (host-side helper, unchanged semantics)."""
        m = adj_matrix.mean(dim=0)
        return torch.trace(torch.matrix_power(m + 1e-8, 2))


class CausalAnomalyDetector(nn.Module):
    """a2:69-101.  forward(video_clips (B,3,T,H,W)) -> (anomaly_scores (B,1), causal_adj (B,16,16), features (B,16))."""

    def __init__(self, feature_dim=64, causal_dim=16, hidden_dim=128):
        super().__init__()
        self.feature_extractor = CompactFeatureExtractor(feature_dim=causal_dim)
        self.causal_discovery = DifferentiableCausalDiscovery(num_variables=causal_dim)
        self.graph_encoder = nn.Sequential(nn.Linear(causal_dim * causal_dim, hidden_dim), nn.ReLU(), nn.Dropout(0.3),
                                           nn.Linear(hidden_dim, 64))
        self.anomaly_predictor = nn.Sequential(nn.Linear(causal_dim + 64, 32), nn.ReLU(), nn.Linear(32, 1),
                                               nn.Sigmoid())
        self._engine = None
        self._step = 0

    def engine(self, x: torch.Tensor) -> "A2Engine":
        e = self._engine
        if e is None or e.device != x.device:
            e = A2Engine(self, x.device)
            self._engine = e
        e.sync_from_module()
        e.use_shape(tuple(x.shape))
        return e

    def forward(self, video_clips, *, seed=None, step=None, clip0=0):
        if video_clips.dim() != 5 or video_clips.shape[1] != 3:
            raise ValueError(f"Expected (B,3,T,H,W) clips, got {tuple(video_clips.shape)}")
        nat.require_hip(video_clips)
        x = video_clips.float().contiguous()
        e = self.engine(x)
        if seed is None:
            seed = e.seed
        if step is None:
            step = self._step
            if self.training:
                self._step += 1
        e.last_keys = (seed, step, clip0)
        params = [p for _, p in self.named_parameters()]
        return _A2Function.apply(x, e, self.training, seed, step, clip0, *params)


class _A2Function(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, e, training, seed, step, clip0, *params):
        s, adj, f = e.forward(x, training, seed, step, clip0, with_loss=False)
        ctx.e = e
        return s.view(-1, 1).clone(), adj.clone(), f.clone()

    @staticmethod
    def backward(ctx, d_s, d_adj, d_f):
        e = ctx.e
        e.backward(None if d_s is None else d_s.reshape(-1).contiguous().float(),
                   None if d_adj is None else d_adj.contiguous().float(),
                   None if d_f is None else d_f.contiguous().float())
        return (None, None, None, None, None, None, *e.grad_clones())


class _A2LossFunction(torch.autograd.Function):
    """compute_improved_loss on the engine's last forward; backward hands d total / d (scores, adj) upstream."""

    @staticmethod
    def forward(ctx, scores, adj, e, seed, step, clip0):
        e.loss(seed, step, clip0)
        ctx.e = e
        return e.losses[0].clone()

    @staticmethod
    def backward(ctx, g):
        ds, dadj = ctx.e.loss_grads()
        return (ds.view(-1, 1) * g, dadj * g, None, None, None, None)


class _A2Plan:
    def __init__(self, e, shape):
        lib = nat.lib()
        B, C, T, H, W = shape
        plan = ctypes.c_void_p()
        nat.check(lib.vad_a2_create(B, T, H, W, ctypes.byref(plan)))
        self.plan = plan
        self.B = B
        self.ws = torch.empty(lib.vad_a2_workspace_bytes(plan) + 256, dtype=torch.uint8, device=e.device)
        base = (self.ws.data_ptr() + 255) // 256 * 256
        nat.check(lib.vad_a2_bind(plan, ctypes.c_void_p(base), nat.ptr(e.params), nat.ptr(e.grads),
                                  nat.ptr(e.exp_avg), nat.ptr(e.exp_avg_sq), nat.ptr(e.steps)))
        f = dict(dtype=torch.float32, device=e.device)
        self.scores, self.adj, self.feats = torch.zeros(B, **f), torch.zeros(B, 16, 16, **f), torch.zeros(B, 16, **f)
        self.d_s, self.d_adj = torch.zeros(B, **f), torch.zeros(B, 16, 16, **f)
        self.borrow = False

    def __del__(self):
        try:
            if getattr(self, "plan", None):
                nat.lib().vad_a2_destroy(self.plan)
        except Exception:
            pass


class A2Engine:
    """Flat device buffers (params / grads / AdamW state, named_parameters order) shared by per-shape plans."""

    def __init__(self, model, device):
        lib = nat.lib()
        self.device, self.model, self.seed = device, model, 1234
        self.slots = [(lib.vad_a2_slot_name(i).decode(), lib.vad_a2_slot_offset(i), lib.vad_a2_slot_numel(i))
                      for i in range(lib.vad_a2_num_slots())]
        names = [n for n, _ in model.named_parameters()]
        if names != [s[0] for s in self.slots]:
            raise NotImplementedError("the HIP a2 plan supports the reference dims (feature_dim=64, causal_dim=16, "
                                      "hidden_dim=128) only")
        n = lib.vad_a2_param_floats()
        f = dict(dtype=torch.float32, device=device)
        self.params, self.grads = torch.zeros(n, **f), torch.zeros(n, **f)
        self.exp_avg, self.exp_avg_sq = torch.zeros(n, **f), torch.zeros(n, **f)
        self.steps = torch.zeros(len(self.slots), dtype=torch.int32, device=device)
        self.losses = torch.zeros(10, **f)
        sd = dict(model.named_parameters())
        self.param_views = [self.params[o:o + k].view_as(sd[nm]) for nm, o, k in self.slots]
        self._bound = False
        self.plans, self.cur, self.last_keys = {}, None, (0, 0, 0)

    def use_shape(self, shape):
        if shape not in self.plans:
            self.plans[shape] = _A2Plan(self, shape)
        self.cur = self.plans[shape]

    def sync_from_module(self):
        if self._bound:
            return
        m = self.model
        with torch.no_grad():
            sd = dict(m.named_parameters())
            for (name, o, k), view in zip(self.slots, self.param_views):
                view.copy_(sd[name].detach().to(self.device))
                mod_name, attr = name.rsplit(".", 1)
                setattr(m.get_submodule(mod_name), attr, nn.Parameter(view, requires_grad=sd[name].requires_grad))
        self._bound = True

    def stream(self):
        return nat.stream_of(self.device)

    def forward(self, x, training, seed, step, clip0, with_loss, borrow_input=False):
        """borrow_input: x stays unchanged until the backward (the fused train step): conv3d_1 reads it in place."""
        p = self.cur
        if p.borrow != bool(borrow_input):
            nat.check(nat.lib().vad_a2_set_option(p.plan, b"borrow_input", int(bool(borrow_input))))
            p.borrow = bool(borrow_input)
        nat.check(nat.lib().vad_a2_forward(p.plan, nat.ptr(x), int(training), ctypes.c_uint64(seed),
                                           ctypes.c_uint64(step), ctypes.c_int64(clip0), int(with_loss),
                                           nat.ptr(p.scores), nat.ptr(p.adj), nat.ptr(p.feats),
                                           nat.ptr(self.losses) if with_loss else None, self.stream()))
        return p.scores, p.adj, p.feats

    def set_host_losses(self, buf):
        """Let the current plan's forward also write its 10 loss words into `buf` (a pinned CPU tensor; None: stop)."""
        p = self.cur
        ptr = buf.data_ptr() if buf is not None else 0
        if getattr(p, "host_ptr", 0) != ptr:
            nat.check(nat.lib().vad_a2_set_option(p.plan, b"host_losses", ctypes.c_int64(ptr)))
            p.host_ptr = ptr

    def loss(self, seed, step, clip0):
        nat.check(nat.lib().vad_a2_loss(self.cur.plan, ctypes.c_uint64(seed), ctypes.c_uint64(step),
                                        ctypes.c_int64(clip0), nat.ptr(self.losses), self.stream()))

    def loss_grads(self):
        p = self.cur
        nat.check(nat.lib().vad_a2_loss_grads(p.plan, nat.ptr(p.d_s), nat.ptr(p.d_adj), self.stream()))
        return p.d_s.clone(), p.d_adj.clone()

    def backward(self, d_s=None, d_adj=None, d_f=None):
        nat.check(nat.lib().vad_a2_backward(self.cur.plan, nat.ptr(d_s) if d_s is not None else None,
                                            nat.ptr(d_adj) if d_adj is not None else None,
                                            nat.ptr(d_f) if d_f is not None else None, self.stream()))

    def grad_clones(self):
        return [self.grads[o:o + k].view_as(v).clone() for (_, o, k), v in zip(self.slots, self.param_views)]

    def optimizer_step(self, lr, weight_decay, max_norm, betas=(0.9, 0.999), eps=1e-8):
        nat.check(nat.lib().vad_a2_optimizer_step(self.cur.plan, ctypes.c_float(lr), ctypes.c_float(betas[0]),
                                                  ctypes.c_float(betas[1]), ctypes.c_float(eps),
                                                  ctypes.c_float(weight_decay), ctypes.c_float(max_norm),
                                                  self.stream()))


class _ParamGroups:
    """The slice of the torch optimizer surface the reference's driver reads (param_groups[0]['lr']) and writes into
    its checkpoints (a2:438-455: ``optimizer.state_dict()``).  The AdamW moments live in the engine's flat device
    buffers; ``state_dict`` exports them in torch.optim.AdamW's layout (one entry per parameter, named_parameters
    order) so a checkpoint written here loads into the reference's optimizer and vice versa."""

    def __init__(self, lr, weight_decay, model_ref=None):
        self.param_groups = [{"lr": lr, "weight_decay": weight_decay, "betas": (0.9, 0.999), "eps": 1e-8}]
        self._model_ref = model_ref

    def _engine(self):
        m = self._model_ref() if self._model_ref is not None else None
        return getattr(m, "_engine", None)

    def state_dict(self):
        g = dict(self.param_groups[0])
        e = self._engine()
        n = len(list(self._model_ref().parameters())) if self._model_ref is not None else 0
        state = {}
        if e is not None:
            steps = e.steps.cpu().tolist()
            for i, (_, o, k) in enumerate(e.slots):
                if steps[i] > 0:
                    shape = e.param_views[i].shape
                    state[i] = {"step": torch.tensor(float(steps[i])),
                                "exp_avg": e.exp_avg[o:o + k].view(shape).detach().cpu().clone(),
                                "exp_avg_sq": e.exp_avg_sq[o:o + k].view(shape).detach().cpu().clone()}
        g.update(amsgrad=False, maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
                 params=list(range(n)))
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, sd):
        g = sd["param_groups"][0]
        for k in ("lr", "weight_decay", "betas", "eps"):
            if k in g:
                self.param_groups[0][k] = tuple(g[k]) if k == "betas" else float(g[k])
        self._pending = sd.get("state", {})
        e = self._engine()
        if e is not None:
            self.push_state(e)

    def push_state(self, e):
        """Copy loaded moments into the engine's device buffers (called once the engine exists)."""
        st = getattr(self, "_pending", None)
        if not st:
            return
        steps = [0] * len(e.slots)
        with torch.no_grad():
            for i, (_, o, k) in enumerate(e.slots):
                s = st.get(i, st.get(str(i)))
                if s is None:
                    continue
                e.exp_avg[o:o + k].copy_(s["exp_avg"].reshape(-1).to(e.exp_avg))
                e.exp_avg_sq[o:o + k].copy_(s["exp_avg_sq"].reshape(-1).to(e.exp_avg_sq))
                steps[i] = int(float(s["step"]))
            e.steps.copy_(torch.tensor(steps, dtype=torch.int32))
        self._pending = None


class _Plateau:
    """ReduceLROnPlateau(mode='min', factor=0.5, patience=5) semantics (torch defaults: rel threshold 1e-4)."""

    def __init__(self, opt, factor=0.5, patience=5, threshold=1e-4, min_lr=0.0, eps=1e-8):
        self.opt, self.factor, self.patience, self.threshold, self.min_lr, self.eps = (
            opt, factor, patience, threshold, min_lr, eps)
        self.best, self.bad = float("inf"), 0

    def state_dict(self):
        return {"factor": self.factor, "patience": self.patience, "threshold": self.threshold,
                "min_lrs": [self.min_lr], "eps": self.eps, "best": self.best, "num_bad_epochs": self.bad,
                "mode": "min", "threshold_mode": "rel", "cooldown": 0, "cooldown_counter": 0}

    def load_state_dict(self, sd):
        self.factor, self.patience = float(sd["factor"]), int(sd["patience"])
        self.threshold, self.eps = float(sd["threshold"]), float(sd["eps"])
        self.min_lr = float(sd.get("min_lrs", [0.0])[0])
        self.best, self.bad = float(sd["best"]), int(sd["num_bad_epochs"])

    def step(self, metric):
        if metric < self.best * (1 - self.threshold):
            self.best, self.bad = metric, 0
        else:
            self.bad += 1
        if self.bad > self.patience:
            for g in self.opt.param_groups:
                new = max(g["lr"] * self.factor, self.min_lr)
                if g["lr"] - new > self.eps:
                    g["lr"] = new
            self.bad = 0


LOSS_KEYS = ("anomaly_loss", "acyclicity_loss", "sparsity_loss", "consistency_loss", "structure_loss", "edge_count",
             "sparsity_ratio")


def _check_batch(B):
    """A single-clip batch fails in the reference: ``anomaly_scores.squeeze()`` is 0-d while the pseudo-targets are
    (1,), and ``F.binary_cross_entropy`` raises (a2:139-147; reproduced by running the reference on B=1)."""
    if B == 1:
        raise ValueError("Using a target size (torch.Size([1])) that is different to the input size "
                         "(torch.Size([])) is deprecated. Please ensure they have the same size.")


class ImprovedMiniCausalVAD:
    """a2:107-297 on the HIP plan: model / optimizer / scheduler attributes, compute_improved_loss,
    train_epoch_improved, evaluate_improved."""

    def __init__(self, device="cuda"):
        self.device = device
        self.model = CausalAnomalyDetector().to(device)
        self.optimizer = _ParamGroups(lr=0.0005, weight_decay=0.001, model_ref=lambda: self.model)
        self.anomaly_weight, self.causal_weight, self.sparsity_weight, self.consistency_weight = 1.0, 0.01, 0.001, 0.01
        self.scheduler = _Plateau(self.optimizer, factor=0.5, patience=5)
        self.seed = 1234
        self.global_step = 0
        self.clip0 = 0

    def compute_improved_loss(self, anomaly_scores, causal_adj, targets, features):
        """Loss of the model's last forward (the labels are ignored: pseudo-labels, a2:139-141).  Returns
        (total loss tensor with autograd into the model's backward, components dict)."""
        _check_batch(anomaly_scores.shape[0])
        e = self.model._engine
        seed, step, clip0 = e.last_keys
        total = _A2LossFunction.apply(anomaly_scores, causal_adj, e, seed, step, clip0)
        vals = e.losses.cpu().tolist()
        return total, dict(zip(LOSS_KEYS, vals[1:8]))

    def train_step(self, videos, labels):
        """One a2:218-245 iteration fused on device (forward + loss + backward + clip + AdamW)."""
        _check_batch(videos.shape[0])
        videos = videos.to(self.device, dtype=torch.float32).contiguous()
        self.model.train()
        e = self.model.engine(videos)
        self.optimizer.push_state(e)
        g = self.optimizer.param_groups[0]
        # The reference reads the loss after the forward and skips the backward and the step on NaN (a2:230-232).
        # Here the forward's copy kernel also writes the losses into pinned host memory (plan option host_losses),
        # the backward and the optimizer step are queued at once -- the optimizer kernels skip the update on device
        # when the loss is NaN (status word losses[9]) and the backward's grads are overwritten by the next one --
        # and the host waits for the forward only, so the device never idles on the host round trip.
        if getattr(self, "_loss_host", None) is None:
            self._loss_host = torch.zeros(10, dtype=torch.float32).pin_memory()
            self._loss_ev = torch.cuda.Event()
        e.set_host_losses(self._loss_host)
        e.forward(videos, True, self.seed, self.global_step, self.clip0, with_loss=True, borrow_input=True)
        self._loss_ev.record()
        e.backward()
        e.optimizer_step(g["lr"], g["weight_decay"], max_norm=0.5)
        self._loss_ev.synchronize()
        vals = self._loss_host.tolist()
        comps = dict(zip(LOSS_KEYS, vals[1:8]))
        stepped = not np.isnan(vals[0])
        self.global_step += 1
        self.clip0 += videos.shape[0]
        return vals[0], comps, stepped

    def train_epoch_improved(self, dataloader):
        total_loss = 0.0
        comps_sum = {k: 0.0 for k in LOSS_KEYS}
        for batch_idx, (videos, labels) in enumerate(dataloader):
            loss, comps, stepped = self.train_step(videos, labels)
            if not stepped:
                print(f"NaN loss detected at batch {batch_idx}, skipping...")
                continue
            total_loss += loss
            for k, v in comps.items():
                comps_sum[k] += v
        n = len(dataloader)
        avg = total_loss / n
        self.scheduler.step(avg)
        return avg, {k: v / n for k, v in comps_sum.items()}

    def evaluate_improved(self, dataloader):
        self.model.eval()
        preds, graphs = [], []
        with torch.no_grad():
            for videos, _ in dataloader:
                videos = videos.to(self.device, dtype=torch.float32).contiguous()
                s, adj, f = self.model(videos)
                preds.extend(s.squeeze().cpu().numpy().reshape(-1).tolist())
                graphs.append(adj.cpu().numpy())
        preds = np.array(preds, dtype=np.float32)
        graphs = np.vstack(graphs)
        e = np.sum(graphs > 0.1, axis=(1, 2))
        metrics = {"mean_score": float(np.mean(preds)), "std_score": float(np.std(preds)),
                   "min_score": float(np.min(preds)), "max_score": float(np.max(preds)),
                   "score_range": float(np.max(preds) - np.min(preds)), "avg_edges": float(np.mean(e)),
                   "avg_sparsity": float(np.mean(e / 256)),
                   "unique_graphs": len(np.unique(graphs.reshape(len(graphs), -1), axis=0))}
        return preds, graphs, metrics

    def save_checkpoint(self, path, **extra):
        """The a2:438-455 checkpoint dict: model / optimizer (/ scheduler) state plus caller extras (epoch, ...)."""
        ck = {"model_state_dict": self.model.state_dict(), "optimizer_state_dict": self.optimizer.state_dict(),
              "scheduler_state_dict": self.scheduler.state_dict()}
        ck.update(extra)
        torch.save(ck, str(path))

    def load_checkpoint(self, path):
        """Load an a2-format checkpoint (incl. the shipped best_improved_model.pth) or a bare state_dict.  Only
        tensors and plain containers are read (weights_only=True)."""
        ck = torch.load(str(path), map_location="cpu", weights_only=True)
        sd = ck.get("model_state_dict", ck) if isinstance(ck, dict) else ck
        self.model.load_state_dict(sd)
        if isinstance(ck, dict) and "optimizer_state_dict" in ck:
            self.optimizer.load_state_dict(ck["optimizer_state_dict"])
        if isinstance(ck, dict) and "scheduler_state_dict" in ck:
            self.scheduler.load_state_dict(ck["scheduler_state_dict"])
        return ck


class MiniCausalVAD(ImprovedMiniCausalVAD):
    """The ``MiniCausalVAD`` surface avenue_training_script1.py drives (a1:19,104,141,160,180-181,187,210): ``.model``
    (whose forward returns the (scores, adj, features) 3-tuple, a1:51), ``.device``, ``.optimizer.param_groups``
    (a1:107-108), ``train_epoch(loader) -> (loss, components)`` with the anomaly/acyclicity/sparsity/consistency
    keys (a1:141-154), ``evaluate(loader) -> (predictions, labels, causal_graphs)`` (a1:160,187) and
    ``save_model/load_model(path)`` (a1:180-181,205,210).  The module a1 imports it from (``minicausal_vad``,
    a1:20) is not in the reference repo, so this restates it on the a2 model and loss it shares its 16x16 causal
    graph and loss keys with; the default lr 1e-3 is the one a1:107 treats as the constructor's.  Semantics beyond
    a1's call sites are parity unpinned."""

    def __init__(self, device="cuda", learning_rate=0.001):
        super().__init__(device)
        self.optimizer.param_groups[0]["lr"] = learning_rate

    def train_epoch(self, dataloader):
        return self.train_epoch_improved(dataloader)

    def evaluate(self, dataloader):
        self.model.eval()
        preds, labels, graphs = [], [], []
        with torch.no_grad():
            for videos, y in dataloader:
                videos = videos.to(self.device, dtype=torch.float32).contiguous()
                s, adj, _ = self.model(videos)
                preds.append(s.reshape(-1).cpu().numpy())
                labels.append(np.asarray(torch.as_tensor(y).reshape(-1).cpu().numpy(), dtype=np.float32))
                graphs.append(adj.cpu().numpy())
        return np.concatenate(preds), np.concatenate(labels), np.concatenate(graphs)

    def save_model(self, path):
        self.save_checkpoint(path, global_step=self.global_step)

    def load_model(self, path):
        ck = self.load_checkpoint(path)
        if isinstance(ck, dict) and "global_step" in ck:
            self.global_step = int(ck["global_step"])
