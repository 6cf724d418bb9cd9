"""Data-parallel test helpers: an oracle-backed stand-in for CadEngine (CPU, test infrastructure) and the
single-process emulation of one DP step that both the CPU and the GPU tests compare against."""
import numpy as np
import torch

from oracle import cad_oracle as co


class OracleEngine:
    """CPU engine with CadEngine's interface (flat params/grads/bufs, forward/backward/optimizer_step),
    computing with oracle/cad_oracle.py.  Grad/flag/optimizer semantics mirror libvadhip's."""

    def __init__(self, model):
        from vad_amd import _native as nat
        L = nat.lib()  # slot layout only: no device call
        n = L.vad_cad_num_slots()
        self.slot_names = [L.vad_cad_slot_name(i).decode() for i in range(n)]
        self.slot_offset = [L.vad_cad_slot_offset(i) for i in range(n)]
        self.slot_numel = [L.vad_cad_slot_numel(i) for i in range(n)]
        self.slot_group = [L.vad_cad_slot_group(i) for i in range(n)]
        self.param_floats = L.vad_cad_param_floats()
        self.shapes = {k: p.shape for k, p in model.named_parameters()}
        self.params = torch.zeros(self.param_floats)
        self.grads = torch.zeros(self.param_floats + 256)
        sd = model.state_dict()
        for k, off, nel in zip(self.slot_names, self.slot_offset, self.slot_numel):
            self.params[off:off + nel] = sd[k].reshape(-1)
        self.buf_names = [k for k in sd if "running" in k]
        self.bufs = torch.cat([sd[k].reshape(-1).clone() for k in self.buf_names])
        self.exp_avg = self.exp_avg_sq = self.steps = None
        self._last = None
        self.bn_sync = None

    def set_bn_sync(self, process_group=None, enable=True):
        import torch.distributed as dist
        self.bn_sync = (process_group if process_group is not None else dist.group.WORLD) if enable else None

    def _pdict(self):
        return {k: self.params[o:o + n].view(self.shapes[k]) for k, o, n in
                zip(self.slot_names, self.slot_offset, self.slot_numel)}

    def _bdict(self):
        out = {}
        o = 0
        for k in self.buf_names:
            c = {"bn1": 32, "layer1": 32, "layer2": 64, "layer3": 128, "layer4": 256}[k.split(".")[1]]
            out[k] = self.bufs[o:o + c]
            o += c
        return out

    def init_optimizer_state(self):
        if self.exp_avg is None:
            self.exp_avg = torch.zeros_like(self.params)
            self.exp_avg_sq = torch.zeros_like(self.params)
            self.steps = torch.zeros(len(self.slot_names), dtype=torch.int32)

    def forward(self, x, training, seed, step, clip0, labels=None, want_outputs=True):
        B, T = x.shape[:2]
        p = {k: v.detach().clone().requires_grad_(not k.startswith(co.FROZEN_PREFIXES)) for k, v in self._pdict().items()}
        bufs = self._bdict()
        draws = co.CadDraws.make(seed, step, clip0, B, T)
        out = co.cad_forward(p, bufs, x, draws, training=training, sync_group=self.bn_sync)
        losses = co.cad_losses(out, labels)
        self._last = (p, losses, out)
        lv = torch.stack([losses[k].detach() for k in ("classification", "anomaly", "causal", "kl", "total")])
        return {"losses": lv}

    def backward(self, use_loss=True):
        p, losses, out = self._last
        names = [n for n in self.slot_names if not n.startswith(co.FROZEN_PREFIXES)]
        gs = torch.autograd.grad(losses["total"], [p[n] for n in names], allow_unused=True)
        self.grads.zero_()
        flags = [0.0, 0.0]
        for n, g in zip(names, gs):
            if g is None:
                continue
            i = self.slot_names.index(n)
            self.grads[self.slot_offset[i]:self.slot_offset[i] + self.slot_numel[i]] = g.reshape(-1)
            if self.slot_group[i] == 2:
                flags[0] = 1.0
            if self.slot_group[i] == 3:
                flags[1] = 1.0
        self.grads[self.param_floats:self.param_floats + 2] = torch.tensor(flags)

    def optimizer_step(self, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5, max_norm=1.0, grad_scale=1.0,
                       total_norm=None):
        self.init_optimizer_state()
        g = self.grads[:self.param_floats] * grad_scale
        norm = float(torch.sqrt((g.double() ** 2).sum()))
        coef = min(1.0, max_norm / (norm + 1e-6))
        fl = self.grads[self.param_floats:self.param_floats + 2]
        for i, grp in enumerate(self.slot_group):
            if not (grp == 1 or (grp == 2 and fl[0] > 0) or (grp == 3 and fl[1] > 0)):
                continue
            self.steps[i] += 1
            st = int(self.steps[i])
            o, n = self.slot_offset[i], self.slot_numel[i]
            newp, m, v = co.adamw_update(self.params[o:o + n], g[o:o + n] * coef, self.exp_avg[o:o + n],
                                         self.exp_avg_sq[o:o + n], st, lr, betas[0], betas[1], eps, weight_decay)
            self.params[o:o + n], self.exp_avg[o:o + n], self.exp_avg_sq[o:o + n] = newp, m, v


def emulate_dp_steps(eng, batches, world, nsteps, lr=3e-4, seed=0):
    """Single-process reference of CadTrainer under DDP semantics: per-rank forward/backward on each rank's clips,
    grads (and flags) summed, 1/world scaling in the optimizer, BN buffers following rank 0."""
    eng.init_optimizer_state()
    for step in range(nsteps):
        acc = torch.zeros_like(eng.grads)
        bufs0 = eng.bufs.clone()
        keep = None
        for r in range(world):
            x, y = batches[r]
            eng.bufs.copy_(bufs0)
            eng.forward(x, True, seed, step, r * x.shape[0], y, want_outputs=False)
            eng.backward(True)
            acc += eng.grads
            if r == 0:
                keep = eng.bufs.clone()
        eng.bufs.copy_(keep)
        eng.grads.copy_(acc)
        eng.optimizer_step(lr, grad_scale=1.0 / world)


def make_batches(world, B, T, H, W, seed=3):
    return [(co.synth_clips(seed, 0, r * B, B, T, H, W), co.synth_labels(r * B, B)) for r in range(world)]
