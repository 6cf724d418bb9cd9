"""Drop-in VideoAutoEncoder + train_model / calculate_anomaly_scores of causal_anomaly_detection1.py (cad1), on the
HIP plan (``vad_ae_*`` in libvadhip.so).

The module keeps the reference's class name, constructor signature, submodule names (state_dict keys
``encoder.N.*``, ``decoder.N.*``, ``temporal_encoder.*`` and the buffers ``normal_memory`` / ``memory_ptr`` /
``temperature``), module creation order and init_weights (cad1:29-41, 124-199), so ``torch.manual_seed(s)`` draws
the reference's weights and its checkpoints load; ``forward()`` returns the reference dict (cad1:316-321) and torch
autograd runs through it.  Every op runs in device kernels: the per-frame encoder convs (im2col + f32 MFMA GEMMs)
with per-frame-index train-mode BatchNorm, the LSTM recurrence and its BPTT, the decoder once per clip, the
reconstruction MSE, the memory-ring score / update, and the train_model update (non-finite-grad skip,
clip_grad_norm_(0.1), Adam with coupled L2).  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from . import _native as nat
from .a2 import _ParamGroups, _Plateau
from .engine import _set_buffer

LATENT, HW = 64, 64


def init_weights(m):
    """cad1:29-41."""
    if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
        nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="leaky_relu")
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)
    elif isinstance(m, nn.Linear):
        nn.init.xavier_normal_(m.weight, gain=0.5)
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)
    elif isinstance(m, nn.BatchNorm2d):
        nn.init.constant_(m.weight, 1)
        nn.init.constant_(m.bias, 0)


def safe_normalize(tensor, dim=-1, eps=1e-8):
    """cad1:43-47."""
    return tensor / torch.clamp(torch.norm(tensor, dim=dim, keepdim=True), min=eps)


def check_and_fix_nan(tensor, name="tensor"):
    """cad1:49-54 (NaN -> 0)."""
    return torch.where(torch.isnan(tensor), torch.zeros_like(tensor), tensor)


def safe_mse_loss(pred, target, eps=1e-8):
    """cad1:323-338: MSE, the L1 mean when that is not finite, a constant 0 when neither is."""
    diff = check_and_fix_nan(pred) - check_and_fix_nan(target)
    loss = torch.mean(diff * diff)
    if not bool(torch.isfinite(loss)):
        loss = torch.mean(torch.abs(diff))
        if not bool(torch.isfinite(loss)):
            return torch.tensor(0.0, device=pred.device, requires_grad=True)
    return loss


def reconstruction_loss(original, reconstructed):
    """cad1:340-344."""
    return safe_mse_loss(reconstructed, original)


def _clip_input(frames):
    nat.require_hip(frames)
    if frames.dim() != 5:
        raise ValueError(f"Expected 5D tensor (B,T,C,H,W), got {tuple(frames.shape)}")
    if tuple(frames.shape[2:]) != (1, HW, HW):
        raise ValueError("VideoAutoEncoder takes (B, T, 1, 64, 64) clips (its Linear(128*4*4) fixes 64x64 frames, "
                         f"cad1:151), got {tuple(frames.shape)}")
    return frames.to(torch.float32).contiguous()


class VideoAutoEncoder(nn.Module):
    """cad1:124-321.  forward(frames (B, T, 1, 64, 64)) -> {'reconstructed', 'sequence_feature', 'frame_features',
    'anomaly_score'}."""

    def __init__(self, input_channels=1, latent_dim=64):
        super().__init__()

        def act():
            return nn.LeakyReLU(0.1, inplace=True)

        enc = []
        for ci, co in ((input_channels, 32), (32, 64), (64, 128), (128, 128)):
            enc += [nn.Conv2d(ci, co, 4, stride=2, padding=1), nn.BatchNorm2d(co), act()]
        self.encoder = nn.Sequential(*enc, nn.Flatten(), nn.Linear(128 * 4 * 4, latent_dim), nn.Tanh())
        dec = [nn.Linear(latent_dim, 128 * 4 * 4), act(), nn.Unflatten(1, (128, 4, 4))]
        for ci, co in ((128, 128), (128, 64), (64, 32)):
            dec += [nn.ConvTranspose2d(ci, co, 4, stride=2, padding=1), nn.BatchNorm2d(co), act()]
        self.decoder = nn.Sequential(*dec, nn.ConvTranspose2d(32, input_channels, 4, stride=2, padding=1),
                                     nn.Sigmoid())
        self.temporal_encoder = nn.LSTM(input_size=latent_dim, hidden_size=latent_dim, num_layers=1,
                                        batch_first=True, dropout=0.0)
        self.register_buffer("normal_memory", torch.zeros(500, latent_dim))
        self.register_buffer("memory_ptr", torch.zeros(1, dtype=torch.long))
        self.memory_size = 500
        self.apply(init_weights)
        self.register_buffer("temperature", torch.tensor(1.0))

    # ------------------------------------------------------------------ HIP engine plumbing
    def engine(self) -> "AeEngine":
        e = self.__dict__.get("_vad_engine")
        if e is None or not e.is_bound():
            e = AeEngine(self)
            self.__dict__["_vad_engine"] = e
        return e

    def update_memory(self, features):
        """cad1:201-219 on the device-resident ring."""
        self.engine().update_memory(features)

    def encode_sequence(self, frames):
        """cad1:221-246 -> (sequence_feature (B, 64), frame_features (B, T, 64)); not differentiable (use forward)."""
        o = self.engine().forward(_clip_input(frames), stages=1, training=self.training)
        return o["sequence_feature"], o["frame_features"]

    def decode_sequence(self, sequence_feature, sequence_length):
        """cad1:248-260 -> (B, T, 1, 64, 64); not differentiable (use forward)."""
        nat.require_hip(sequence_feature)
        seq = sequence_feature.detach().to(torch.float32).contiguous()
        return self.engine().forward(None, stages=2, training=self.training, seq_in=seq,
                                     T=int(sequence_length))["reconstructed"]

    def compute_anomaly_score(self, sequence_feature):
        """cad1:262-301."""
        return self.engine().memory_score(sequence_feature)

    def forward(self, frames):
        x = _clip_input(frames)
        e = self.engine()
        params = [p for _, p in self.named_parameters()]
        recon, seq, ff, score = _AeFunction.apply(x, e, self.training, *params)
        return {"reconstructed": recon, "sequence_feature": seq, "frame_features": ff, "anomaly_score": score}


class _AeFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, e, training, *params):
        o = e.forward(x, stages=3, training=training)
        ctx.e = e
        ctx.mark_non_differentiable(o["anomaly_score"])
        return o["reconstructed"], o["sequence_feature"], o["frame_features"], o["anomaly_score"]

    @staticmethod
    def backward(ctx, d_recon, d_seq, d_ff, d_score):
        ctx.e.backward(False, d_recon, d_seq, d_ff)
        return (None, None, None, *ctx.e.grad_views())


class _AePlan:
    """One C plan + workspace per (B, T), bound to the engine's shared flat buffers."""

    def __init__(self, e, B, T):
        L = nat.lib()
        h = ctypes.c_void_p()
        nat.check(L.vad_ae_create(B, T, ctypes.byref(h)))
        self.h = h
        self.ws = torch.empty(L.vad_ae_workspace_bytes(h) + 256, dtype=torch.uint8, device=e.device)
        self.bind(e)

    def bind(self, e):
        base = (self.ws.data_ptr() + 255) // 256 * 256
        nat.check(nat.lib().vad_ae_bind(self.h, base, e.params.data_ptr(), e.grads.data_ptr(), e.bufs.data_ptr(),
                                        e.nbt.data_ptr(), e.memory.data_ptr(), e.mptr.data_ptr(), nat.ptr(e.exp_avg),
                                        nat.ptr(e.exp_avg_sq), nat.ptr(e.steps)))

    def __del__(self):
        try:
            if getattr(self, "h", None):
                nat.lib().vad_ae_destroy(self.h)
        except Exception:
            pass


class AeEngine:
    """Flat device buffers of one VideoAutoEncoder -- params / grads / BN running stats / counters / memory ring /
    Adam state; the module's parameters and buffers are views into them -- shared by per-(B, T) plans."""

    def __init__(self, model):
        L = nat.lib()
        p0 = next(model.parameters())
        nat.require_hip(p0)
        if model.encoder[0].in_channels != 1 or model.temporal_encoder.hidden_size != LATENT:
            raise NotImplementedError("the HIP plan implements VideoAutoEncoder(input_channels=1, latent_dim=64), "
                                      "the reference's configuration (cad1:687)")
        self.model, self.device = model, p0.device
        self.slots = [(L.vad_ae_slot_name(i).decode(), L.vad_ae_slot_offset(i), L.vad_ae_slot_numel(i))
                      for i in range(L.vad_ae_num_slots())]
        named = list(model.named_parameters())
        if [k for k, _ in named] != [s[0] for s in self.slots]:
            raise RuntimeError("model parameters do not match the libvadhip slot table")
        f = dict(dtype=torch.float32, device=self.device)
        self.params = torch.zeros(L.vad_ae_param_floats(), **f)
        self.grads = torch.zeros_like(self.params)
        self.bufs = torch.zeros(L.vad_ae_buf_floats(), **f)
        named_bufs = dict(model.named_buffers())
        nbt_names = [k for k in named_bufs if k.endswith("num_batches_tracked")]
        self.nbt = torch.zeros(len(nbt_names), dtype=torch.int64, device=self.device)
        with torch.no_grad():
            for (k, p), (_, off, nel) in zip(named, self.slots):
                if p.numel() != nel:
                    raise RuntimeError(f"parameter {k}: {p.numel()} elements, library expects {nel}")
                view = self.params[off:off + nel].view_as(p)
                view.copy_(p.data)
                p.data = view
            for i in range(L.vad_ae_num_bufs()):
                k, off, nel = L.vad_ae_buf_name(i).decode(), L.vad_ae_buf_offset(i), L.vad_ae_buf_numel(i)
                view = self.bufs[off:off + nel].view_as(named_bufs[k])
                view.copy_(named_bufs[k])
                _set_buffer(model, k, view)
            for i, k in enumerate(nbt_names):
                self.nbt[i].copy_(named_bufs[k].reshape(()))
                _set_buffer(model, k, self.nbt[i])
            self.memory = named_bufs["normal_memory"].detach().to(**f).clone().contiguous()
            self.mptr = named_bufs["memory_ptr"].detach().to(device=self.device, dtype=torch.int64).clone()
            _set_buffer(model, "normal_memory", self.memory)
            _set_buffer(model, "memory_ptr", self.mptr)
        self.exp_avg = self.exp_avg_sq = self.steps = None
        self.losses = torch.zeros(4, **f)  # mse, grad norm, clipped, status
        self.plans = {}
        self.cur = None

    def is_bound(self) -> bool:
        m = self.model
        return (next(m.parameters()).data_ptr() == self.params.data_ptr()
                and m.normal_memory.data_ptr() == self.memory.data_ptr())

    def plan(self, B, T) -> _AePlan:
        if (B, T) not in self.plans:
            self.plans[(B, T)] = _AePlan(self, B, T)
        return self.plans[(B, T)]

    def init_optimizer_state(self):
        if self.exp_avg is None:
            self.exp_avg = torch.zeros_like(self.params)
            self.exp_avg_sq = torch.zeros_like(self.params)
            self.steps = torch.zeros(len(self.slots), dtype=torch.int32, device=self.device)
            for p in self.plans.values():
                p.bind(self)

    def stream(self):
        return nat.stream_of(self.device)

    def forward(self, x, stages=3, training=True, loss_mode=0, seq_in=None, T=None, outputs=True):
        """One plan forward (stages 1 encode / 2 decode / 3 both; loss_mode 0 none / 1 eval MSE / 2 train_model
        iteration).  Returns fresh output tensors and the device loss vector."""
        if stages & 1:
            B, T = int(x.shape[0]), int(x.shape[1])
        else:
            B = int(seq_in.shape[0])
        pl = self.plan(B, T)
        dev = self.device
        o = {}
        if outputs:
            o["sequence_feature"] = torch.empty(B, LATENT, device=dev)
            if stages & 1:
                o["frame_features"] = torch.empty(B, T, LATENT, device=dev)
            if stages & 2:
                o["reconstructed"] = torch.empty(B, T, 1, HW, HW, device=dev)
            if stages == 3:
                o["anomaly_score"] = torch.empty(B, device=dev)
            if loss_mode:
                o["recon_error"] = torch.empty(B, device=dev)
        nat.check(nat.lib().vad_ae_forward(
            pl.h, nat.ptr(x), nat.ptr(seq_in), stages, 1 if training else 0, loss_mode,
            nat.ptr(o.get("reconstructed")), nat.ptr(o.get("sequence_feature")), nat.ptr(o.get("frame_features")),
            nat.ptr(o.get("anomaly_score")), nat.ptr(o.get("recon_error")), self.losses.data_ptr(), self.stream()))
        o["losses"] = self.losses
        self.cur = pl
        return o

    def backward(self, use_loss, d_recon=None, d_seq=None, d_ff=None):
        c = [None if t is None else t.to(torch.float32).contiguous() for t in (d_recon, d_seq, d_ff)]
        nat.check(nat.lib().vad_ae_backward(self.cur.h, 1 if use_loss else 0, *[nat.ptr(t) for t in c],
                                            self.stream()))

    def optimizer_step(self, lr, weight_decay=1e-6, max_norm=0.1, betas=(0.9, 0.999), eps=1e-8, grad_scale=1.0):
        self.init_optimizer_state()
        nat.check(nat.lib().vad_ae_optimizer_step(self.cur.h, lr, betas[0], betas[1], eps, weight_decay, max_norm,
                                                  grad_scale, self.stream()))

    def grad_views(self):
        return [self.grads[off:off + n].view_as(p).clone()
                for (_, off, n), (_, p) in zip(self.slots, self.model.named_parameters())]

    def update_memory(self, features):
        f = features.detach().to(device=self.device, dtype=torch.float32).reshape(-1, LATENT).contiguous()
        nat.check(nat.lib().vad_ae_update_memory(self.memory.data_ptr(), self.mptr.data_ptr(), f.data_ptr(),
                                                 int(f.shape[0]), self.stream()))

    def memory_score(self, sequence_feature):
        s = sequence_feature.detach().to(device=self.device, dtype=torch.float32).reshape(-1, LATENT).contiguous()
        out = torch.empty(s.shape[0], device=self.device)
        nat.check(nat.lib().vad_ae_memory_score(self.memory.data_ptr(), self.mptr.data_ptr(), s.data_ptr(),
                                                int(s.shape[0]), out.data_ptr(), self.stream()))
        return out


class AeTrainer:
    """The fused train_model iteration (cad1:378-431) on already selected normal clips: forward + MSE + memory-ring
    update + backward + non-finite-grad skip + clip_grad_norm_(max_norm) + Adam in device kernels, no host
    synchronisation.  ``step`` returns the device vector [mse, grad_norm, clipped, status] (status 0: skipped
    before backward -- a non-finite input; 1: non-finite grads, no step; 2: stepped).

    Data parallel (an initialised process group): each rank trains on its own clips, the flat gradient buffer is
    summed with one all_reduce and scaled by 1/world inside the optimizer, BN running stats follow rank 0 (DDP's
    broadcast_buffers); BN batch statistics and the memory ring stay per rank."""

    def __init__(self, model, lr=5e-7, weight_decay=1e-6, max_norm=0.1, betas=(0.9, 0.999), eps=1e-8,
                 optimizer=None, process_group=None):
        import torch.distributed as dist
        self.model = model
        self.optimizer = optimizer if optimizer is not None else _ParamGroups(lr=lr, weight_decay=weight_decay)
        self.max_norm, self.betas, self.eps = max_norm, betas, eps
        self.eng = model.engine()
        self.eng.init_optimizer_state()
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        if self.world > 1:
            dist.broadcast(self.eng.params, 0, group=process_group)
            dist.broadcast(self.eng.bufs, 0, group=process_group)

    def step(self, videos):
        e = self.eng
        self.model.train()
        x = _clip_input(videos)
        if self.world > 1:
            import torch.distributed as dist
            dist.broadcast(e.bufs, 0, group=self.pg)
        e.forward(x, stages=3, training=True, loss_mode=2, outputs=False)
        e.backward(True)
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(e.grads, group=self.pg)
        g = self.optimizer.param_groups[0]
        e.optimizer_step(g["lr"], g["weight_decay"], self.max_norm, self.betas, self.eps, 1.0 / self.world)
        return e.losses

    def eval_batch(self, videos):
        """Eval-mode forward with the batch MSE and per-clip errors (cad1:460-464, 542-552)."""
        self.model.eval()
        return self.eng.forward(_clip_input(videos), stages=3, training=False, loss_mode=1)


def train_model(model, train_loader, val_loader, num_epochs=30, lr=5e-7, save_path="best_robust_autoencoder.pth"):
    """cad1:346-524 driving the fused HIP iteration.  Returns (model, train_losses, val_losses)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    model.to(dev)
    optimizer = _ParamGroups(lr=lr, weight_decay=1e-6)
    scheduler = _Plateau(optimizer, factor=0.8, patience=3, min_lr=1e-7)
    trainer = AeTrainer(model, optimizer=optimizer)
    best_loss, patience, patience_counter = float("inf"), 10, 0
    train_losses, val_losses = [], []
    print("Training memory-based autoencoder...")
    for epoch in range(num_epochs):
        model.train()
        train_loss, num_batches, valid_batches = 0.0, 0, 0
        for batch_idx, (videos, labels) in enumerate(train_loader):
            normal_mask = torch.as_tensor(labels) == 0  # only normal clips train (cad1:373-378)
            if not bool(normal_mask.any()):
                continue
            videos = videos[normal_mask.to(videos.device)]
            if videos.shape[0] == 0:
                continue
            loss, _, _, status = trainer.step(videos.to(dev)).tolist()
            if status < 0.5:  # non-finite input: skipped before the forward (cad1:385-387)
                continue
            if status > 1.5:
                train_loss += loss
                valid_batches += 1
            num_batches += 1
            if batch_idx % 20 == 0:
                print(f"Epoch {epoch + 1}/{num_epochs}, Batch {batch_idx + 1}, Loss: {loss:.4f}, "
                      f"Memory: {int(model.memory_ptr[0])}/{model.memory_size}")
        if valid_batches == 0:
            print("No valid batches in this epoch!")
            break
        model.eval()
        val_loss, val_scores, val_labels, valid_val = 0.0, [], [], 0
        with torch.no_grad():
            for videos, labels in val_loader:
                videos = videos.to(dev)
                if bool(torch.isnan(videos).any()):
                    continue
                o = trainer.eval_batch(videos)
                vl = float(o["losses"][0])
                # safe_mse_loss: with an Inf pixel both the MSE and the L1 fallback are Inf -> 0 (cad1:331-336)
                val_loss += vl if math.isfinite(vl) else 0.0
                val_scores.extend(o["anomaly_score"].cpu().numpy().tolist())
                val_labels.extend(np.asarray(torch.as_tensor(labels).cpu()).reshape(-1).tolist())
                valid_val += 1
        if valid_val == 0:
            print("No valid validation batches!")
            continue
        avg_train, avg_val = train_loss / max(valid_batches, 1), val_loss / max(valid_val, 1)
        train_losses.append(avg_train)
        val_losses.append(avg_val)
        scheduler.step(avg_val)
        normal = [s for s, y in zip(val_scores, val_labels) if y == 0]
        abnormal = [s for s, y in zip(val_scores, val_labels) if y == 1]
        separation = float(np.mean(abnormal) - np.mean(normal)) if normal and abnormal else 0.0
        print(f"Epoch {epoch + 1}/{num_epochs}: Train Loss {avg_train:.4f}, Val Loss {avg_val:.4f}, "
              f"valid batches {valid_batches}/{num_batches}, memory {int(model.memory_ptr[0])}/{model.memory_size}, "
              f"separation {separation:.4f}, LR {optimizer.param_groups[0]['lr']:.6f}")
        if not np.isnan(avg_val) and avg_val < best_loss:
            best_loss, patience_counter = avg_val, 0
            torch.save(model.state_dict(), save_path)
        else:
            patience_counter += 1
            if patience_counter >= patience:
                print(f"Early stopping after {patience} epochs without improvement")
                break
    try:
        model.load_state_dict(torch.load(save_path, map_location=dev, weights_only=True))
    except Exception:
        print("Using final model")
    return model, train_losses, val_losses


def calculate_anomaly_scores(model, test_loader):
    """cad1:526-564: (0.7 * per-clip reconstruction MSE + 0.3 * memory score, labels, MSEs, memory scores)."""
    model.eval()
    e = model.engine()
    scores, labels_all, recon, memory = [], [], [], []
    with torch.no_grad():
        for videos, labels in test_loader:
            videos = videos.to(e.device)
            if bool(torch.isnan(videos).any()):
                continue
            o = e.forward(_clip_input(videos), stages=3, training=False, loss_mode=1)
            err, ms = o["recon_error"], o["anomaly_score"]
            scores.extend((0.7 * err + 0.3 * ms).cpu().numpy().tolist())
            labels_all.extend(np.asarray(torch.as_tensor(labels).cpu()).reshape(-1).tolist())
            recon.extend(err.cpu().numpy().tolist())
            memory.extend(ms.cpu().numpy().tolist())
    return np.array(scores), np.array(labels_all), np.array(recon), np.array(memory)
