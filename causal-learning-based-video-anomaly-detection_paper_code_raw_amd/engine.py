"""CadEngine: owns the flat device buffers of one CausalAnomalyDetector and drives libvadhip.

Layout (all on the model's HIP device):
  * params : one fp32 buffer, every nn.Parameter of the model is a view into it (slot order = state_dict order,
             offsets from the library, 256-float aligned) -> state_dict / load_state_dict keep working;
  * grads  : same layout + a 256-float tail whose first two floats are the "has grad" flags of the detector and
             the structure learner (summed by the data-parallel all-reduce together with the grads);
  * bufs   : BatchNorm running_mean / running_var, also viewed by the module buffers;
  * nbt    : the nine num_batches_tracked counters (int64);
  * exp_avg / exp_avg_sq / steps : AdamW state, created on the first optimizer step.
One plan (+ workspace) per input shape (B, T, H, W).
"""
from __future__ import annotations

import ctypes

import torch

from . import _native as nat

GROUP_FROZEN, GROUP_ALWAYS, GROUP_DET, GROUP_STRUCT, GROUP_NEVER = range(5)


class _Plan:
    def __init__(self, engine, B, T, H, W):
        L = nat.lib()
        h = ctypes.c_void_p()
        nat.check(L.vad_cad_create(B, T, H, W, ctypes.byref(h)))
        self.h = h
        nat.check(L.vad_cad_set_option(h, b"conv_bf16", 1 if engine.compute_dtype == torch.bfloat16 else 0))
        # (the workspace is carved for the options set before the size query: the training stem's buffers only when
        # the stem trains -- CadEngine.plan builds a new plan when that changes)
        self.stem_grad = engine.stem_trains()
        self.ws_stem = self.stem_grad
        nat.check(L.vad_cad_set_option(h, b"stem_grad", 1 if self.stem_grad else 0))
        self.shape = (B, T, H, W)
        nbytes = L.vad_cad_workspace_bytes(h)
        self.ws = torch.empty(int(nbytes) + 256, dtype=torch.uint8, device=engine.device)
        base = (self.ws.data_ptr() + 255) // 256 * 256
        e = engine
        nat.check(L.vad_cad_bind(h, base, e.params.data_ptr(), e.grads.data_ptr(), e.bufs.data_ptr(),
                                 e.nbt.data_ptr(), nat.ptr(e.exp_avg), nat.ptr(e.exp_avg_sq), nat.ptr(e.steps)))
        self._sync_cb = None
        self.apply_bn_sync(engine)

    def apply_bn_sync(self, engine):
        """Install (or clear) the SyncBatchNorm callback: an all-reduce of the plan's [2C] double sums buffer over
        the engine's process group, on the current stream."""
        L = nat.lib()
        if engine.bn_sync is None:
            self._sync_cb = None
            nat.check(L.vad_cad_set_bn_sync(self.h, nat.BN_SYNC_FN(), None, 1))
            return
        import torch.distributed as dist
        group, world = engine.bn_sync
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        nat.check(L.vad_cad_debug_buffer(self.h, b"bn_sync", 0, ctypes.byref(p), ctypes.byref(n)))
        off = p.value - self.ws.data_ptr()
        sums = self.ws[off:off + 4 * n.value].view(torch.float64)

        def _cb(user, bn_layer, phase, count, stream):
            try:
                dist.all_reduce(sums[:count], group=group)
                return 0
            except Exception as exc:  # reported through the library's error path
                print(f"vad bn sync (layer {bn_layer}, phase {phase}) failed: {exc!r}")
                return 1

        self._sync_cb = nat.BN_SYNC_FN(_cb)  # kept alive as long as the plan
        nat.check(L.vad_cad_set_bn_sync(self.h, self._sync_cb, None, world))

    def rebind(self, engine):
        e = engine
        base = (self.ws.data_ptr() + 255) // 256 * 256
        nat.check(nat.lib().vad_cad_bind(self.h, base, e.params.data_ptr(), e.grads.data_ptr(), e.bufs.data_ptr(),
                                         e.nbt.data_ptr(), nat.ptr(e.exp_avg), nat.ptr(e.exp_avg_sq),
                                         nat.ptr(e.steps)))

    def __del__(self):
        try:
            if self.h:
                nat.lib().vad_cad_destroy(self.h)
        except Exception:
            pass


class CadEngine:
    def __init__(self, model: torch.nn.Module):
        L = nat.lib()
        self.model = model
        p0 = next(model.parameters())
        nat.require_hip(p0)
        self.device = p0.device
        n = L.vad_cad_num_slots()
        self.slot_names = [L.vad_cad_slot_name(i).decode() for i in range(n)]
        self.slot_numel = [L.vad_cad_slot_numel(i) for i in range(n)]
        self.slot_offset = [L.vad_cad_slot_offset(i) for i in range(n)]
        self.slot_group = [L.vad_cad_slot_group(i) for i in range(n)]
        self.param_floats = L.vad_cad_param_floats()
        named = list(model.named_parameters())
        if [k for k, _ in named] != self.slot_names:
            raise RuntimeError("model parameters do not match the libvadhip slot table")
        for (k, p), nel in zip(named, self.slot_numel):
            if p.numel() != nel:
                raise RuntimeError(f"parameter {k}: {p.numel()} elements, library expects {nel}")
        dev = self.device
        self.params = torch.zeros(self.param_floats, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(self.param_floats + 256, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for (k, p), off in zip(named, self.slot_offset):
                view = self.params[off:off + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
        nb = L.vad_cad_num_bufs()
        self.buf_names = [L.vad_cad_buf_name(i).decode() for i in range(nb)]
        self.buf_offset = [L.vad_cad_buf_offset(i) for i in range(nb)]
        self.bufs = torch.zeros(L.vad_cad_buf_floats(), dtype=torch.float32, device=dev)
        named_bufs = dict(model.named_buffers())
        with torch.no_grad():
            for k, off in zip(self.buf_names, self.buf_offset):
                b = named_bufs[k]
                view = self.bufs[off:off + b.numel()].view_as(b)
                view.copy_(b)
                _set_buffer(model, k, view)
        nbt_names = [k for k in named_bufs if k.endswith("num_batches_tracked")]
        if len(nbt_names) != L.vad_cad_num_bn():
            raise RuntimeError("unexpected number of BatchNorm layers")
        self.nbt = torch.zeros(len(nbt_names), dtype=torch.int64, device=dev)
        with torch.no_grad():
            for i, k in enumerate(nbt_names):
                self.nbt[i].copy_(named_bufs[k].reshape(()))
                _set_buffer(model, k, self.nbt[i])
        # (the stem's Parameter objects, for the per-call requires_grad check: building the named-parameter dict
        # costs ~0.3 ms of host time, twice per step, on the step's critical path where the GPU runs short kernels)
        self._stem_params = [p for k, p in named if k in self.STEM]
        self.exp_avg = self.exp_avg_sq = self.steps = None
        self.bn_sync = None  # (process_group, world) in SyncBatchNorm mode
        self._compute_dtype = torch.float32
        self.plans = {}
        self.generation = 0
        self._last = None
        self._loss_buf = None

    # ------------------------------------------------------------------ bookkeeping
    @property
    def compute_dtype(self):
        """torch.float32 (default: fp32 numerics) or torch.bfloat16 (backbone 3x3 convs on bf16 operands with fp32
        accumulation, BASELINE config 4; everything else stays fp32)."""
        return self._compute_dtype

    @compute_dtype.setter
    def compute_dtype(self, dt):
        if dt not in (torch.float32, torch.bfloat16):
            raise ValueError(f"compute_dtype must be torch.float32 or torch.bfloat16, got {dt}")
        self._compute_dtype = dt
        for p in self.plans.values():
            nat.check(nat.lib().vad_cad_set_option(p.h, b"conv_bf16", 1 if dt == torch.bfloat16 else 0))

    def set_bn_sync(self, process_group=None, enable: bool = True):
        """SyncBatchNorm mode: in training forwards every BatchNorm layer normalises with the statistics of the whole
        process group's batch (and its backward uses the group's mean terms), so an N-rank step of B clips per rank
        equals the reference's single-process step on the N*B-clip batch (cad:116,131,136 normalise over all B*T
        frames).  enable=False restores per-rank statistics (DDP's default)."""
        import torch.distributed as dist
        if enable:
            world = dist.get_world_size(process_group)
            self.bn_sync = (process_group, world)
        else:
            self.bn_sync = None
        for p in self.plans.values():
            p.apply_bn_sync(self)

    def is_bound(self) -> bool:
        p = next(self.model.parameters())
        return p.data_ptr() == self.params.data_ptr() and p.device == self.device

    def init_optimizer_state(self):
        if self.exp_avg is None:
            self.exp_avg = torch.zeros_like(self.params)
            self.exp_avg_sq = torch.zeros_like(self.params)
            self.steps = torch.zeros(len(self.slot_names), dtype=torch.int32, device=self.device)
            for p in self.plans.values():
                p.rebind(self)

    def plan(self, B, T, H, W) -> _Plan:
        key = (B, T, H, W)
        pl = self.plans.get(key)
        if pl is None or (self.stem_trains() and not pl.ws_stem):
            # (a plan carved for the frozen stem has no room for conv1's activation: a training stem needs a new one)
            pl = self.plans[key] = _Plan(self, B, T, H, W)
        return pl

    def grad_view(self, i):
        off = self.slot_offset[i]
        return self.grads[off:off + self.slot_numel[i]]

    # ------------------------------------------------------------------ compute
    def forward(self, x: torch.Tensor, training: bool, seed: int, step: int, clip0: int, labels=None,
                want_outputs: bool = True, loss_host=None):
        """Runs the fused forward.  want_outputs=False returns only the loss vector (no output copies); with
        loss_host (a pinned 5-float CPU tensor) the loss-tail kernel writes the vector straight into it over PCIe,
        so a host read needs only an event recorded after this call, not the queued backward and optimizer."""
        nat.require_hip(x)
        if x.dim() != 5:
            raise ValueError(f"Expected 5D tensor (B,T,C,H,W), got {tuple(x.shape)}")
        B, T, C, H, W = x.shape
        if C != 1:
            raise ValueError("ResNetBackbone here takes single-channel frames (input_channels=1, cad:515)")
        x0 = x
        x = x.contiguous().float()
        pl = self.plan(B, T, H, W)
        # (before the forward: a training stem needs conv1's activation stored, a frozen one is recomputed in place)
        self._set_stem_grad(pl)
        armed, self._armed = getattr(self, "_armed", None), None
        if armed is not None and armed is not pl:  # (armed for another plan: that arm must not outlive this call)
            nat.check(nat.lib().vad_cad_set_option(armed.h, b"input_armed", 0))
        elif armed is pl and x.data_ptr() != x0.data_ptr():  # the input was converted here, on the current stream
            nat.check(nat.lib().vad_cad_input_ready(pl.h, ctypes.c_void_p(
                torch.cuda.current_stream(self.device).cuda_stream)))
        dev = self.device
        if not want_outputs:
            if loss_host is not None:
                if loss_host.numel() != 5 or loss_host.dtype != torch.float32 or not loss_host.is_contiguous():
                    raise ValueError("loss_host: a contiguous 5-float pinned CPU tensor")
                loss_ptr, loss_t = nat.host_device_ptr(loss_host), loss_host
            else:
                if self._loss_buf is None:
                    self._loss_buf = torch.empty(5, device=dev)
                loss_ptr, loss_t = self._loss_buf.data_ptr(), self._loss_buf
            lab = None if labels is None else labels.to(device=dev, dtype=torch.int64).contiguous()
            nat.check(nat.lib().vad_cad_forward(
                pl.h, x.data_ptr(), 1 if training else 0, seed & ((1 << 64) - 1), step, clip0, nat.ptr(lab),
                None, None, None, None, None, None, None, None, None, loss_ptr, None, nat.stream_of(dev)))
            self.generation += 1
            self._last = (pl, lab, x)
            return {"losses": loss_t}
        o = dict(
            final=torch.empty(B, device=dev), probs=torch.empty(B, 2, device=dev),
            causal=torch.empty(B, device=dev), kl=torch.empty(B, device=dev),
            z=torch.empty(B, 5, 6, device=dev), adj=torch.empty(B, 6, 6, device=dev),
            nmax=torch.empty(B, dtype=torch.int32, device=dev), boxes=torch.empty(B, T, 5, 4, device=dev),
            counts=torch.empty(B, T, dtype=torch.int32, device=dev), losses=torch.empty(5, device=dev),
            flags=torch.empty(2, dtype=torch.int32, device=dev))
        lab = None
        if labels is not None:
            lab = labels.to(device=dev, dtype=torch.int64).contiguous()
        nat.check(nat.lib().vad_cad_forward(
            pl.h, x.data_ptr(), 1 if training else 0, seed & ((1 << 64) - 1), step, clip0, nat.ptr(lab),
            o["final"].data_ptr(), o["probs"].data_ptr(), o["causal"].data_ptr(), o["kl"].data_ptr(),
            o["z"].data_ptr(), o["adj"].data_ptr(), o["nmax"].data_ptr(), o["boxes"].data_ptr(),
            o["counts"].data_ptr(), o["losses"].data_ptr(), o["flags"].data_ptr(), nat.stream_of(dev)))
        self.generation += 1
        self._last = (pl, lab, x)
        return o

    def backward(self, use_loss: bool, d_final=None, d_probs=None, d_causal=None, d_kl=None, d_z=None, d_adj=None,
                 stage: int = -1, d_boxes=None):
        """stage -1: whole backward; 0: everything but the backbone (grads outside [0, backbone_floats) final);
        1: the backbone (after stage 0 or 2); 2: stage 0 whose causal-head / detector grads finish on the plan's side
        stream (order a consumer after them with wait_side).  d_boxes: grad of the (B, T, 5, 4) detections output."""
        pl, lab, _ = self._last
        self._set_stem_grad(pl)
        c = [t.contiguous() if t is not None else None for t in (d_final, d_probs, d_causal, d_kl, d_z, d_adj)]
        if d_boxes is not None:
            nat.check(nat.lib().vad_cad_backward_ext(pl.h, stage, 1 if use_loss else 0, *[nat.ptr(t) for t in c],
                                                     nat.ptr(d_boxes.contiguous().float()),
                                                     nat.stream_of(self.device)))
            return
        if stage == -1:
            nat.check(nat.lib().vad_cad_backward(pl.h, 1 if use_loss else 0, *[nat.ptr(t) for t in c],
                                                 nat.stream_of(self.device)))
        else:
            nat.check(nat.lib().vad_cad_backward_stage(pl.h, stage, 1 if use_loss else 0, *[nat.ptr(t) for t in c],
                                                       nat.stream_of(self.device)))

    def wait_layer_grads(self, layer: int, stream):
        """Make `stream` wait until every grad of backbone layer `layer` (0..7; layer 0 with the stem's) of the last
        queued backbone backward is final (per-layer data-parallel buckets)."""
        pl = self._last[0]
        nat.check(nat.lib().vad_cad_wait_layer_grads(pl.h, layer, ctypes.c_void_p(stream.cuda_stream)))

    def input_ready(self, B: int, T: int, H: int, W: int, stream=None):
        """Arm the next forward of the (B, T, H, W) plan: its input clips are complete once the work queued on `stream`
        (a torch.cuda.Stream; default: the current stream) at this call is, so its frozen stem may run beside what
        the current stream still has queued (the previous step's tail).  One-shot (vad_cad_input_ready)."""
        pl = self.plan(B, T, H, W)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        nat.check(nat.lib().vad_cad_input_ready(pl.h, ctypes.c_void_p(s.cuda_stream)))
        self._armed = pl

    def wait_side(self, stream):
        """Make `stream` (a torch.cuda.Stream) wait for everything queued so far on the last plan's side stream (the
        stage-2 backward's head / detector grads)."""
        pl = self._last[0]
        nat.check(nat.lib().vad_cad_wait_side(pl.h, ctypes.c_void_p(stream.cuda_stream)))

    STEM = ("backbone.conv1.weight", "backbone.conv1.bias", "backbone.bn1.weight", "backbone.bn1.bias")

    def stem_trains(self) -> bool:
        """backbone.conv1 / bn1 take grads unless frozen (apply_memory_efficient_training, cad:592-598)."""
        return any(p.requires_grad for p in self._stem_params)

    def _set_stem_grad(self, pl):
        on = self.stem_trains()
        if getattr(pl, "stem_grad", None) != on:
            nat.check(nat.lib().vad_cad_set_option(pl.h, b"stem_grad", 1 if on else 0))
            pl.stem_grad = on
        self.stem_grad_on = on

    @property
    def backbone_floats(self) -> int:
        """Length of the backbone's leading run of slots in the flat buffers (named_parameters order)."""
        return next(o for n, o in zip(self.slot_names, self.slot_offset) if not n.startswith("backbone."))

    def profile(self, enable: bool, only_prefix: str = "", reset: bool = True):
        """HIP-event timing of the plan's labelled launches (all plans of this engine).  enable=False pauses (the
        records are kept); enable=True clears them first unless reset=False."""
        code = (1 if reset else 2) if enable else 0
        for pl in self.plans.values():
            nat.check(nat.lib().vad_cad_profile(pl.h, code, only_prefix.encode()))

    def profile_read(self, shape=None) -> dict:
        """{label: (total_ms, launches)} recorded since profile(True) (synchronises the stream)."""
        pl = self.plans[shape] if shape is not None else self._last[0]
        cap = 256
        labels = ctypes.create_string_buffer(64 * cap)
        tot = (ctypes.c_double * cap)()
        cnt = (ctypes.c_int * cap)()
        n = nat.lib().vad_cad_profile_read(pl.h, labels, tot, cnt, cap)
        if n < 0:
            nat.check(1)
        out = {}
        for i in range(min(n, cap)):
            lab = labels.raw[64 * i:64 * (i + 1)].split(b"\0", 1)[0].decode()
            out[lab] = (tot[i], cnt[i])
        return out

    def profile_marks(self, shape=None) -> list:
        """[(label, start_ms, end_ms)] of every recorded launch in record order, relative to the first record's start
        (synchronises the stream)."""
        pl = self.plans[shape] if shape is not None else self._last[0]
        cap = 4096
        labels = ctypes.create_string_buffer(64 * cap)
        t0 = (ctypes.c_double * cap)()
        t1 = (ctypes.c_double * cap)()
        n = nat.lib().vad_cad_profile_marks(pl.h, labels, t0, t1, cap)
        if n < 0:
            nat.check(1)
        return [(labels.raw[64 * i:64 * (i + 1)].split(b"\0", 1)[0].decode(), t0[i], t1[i]) for i in range(min(n, cap))]

    def optimizer_step(self, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5, max_norm=1.0, grad_scale=1.0,
                       total_norm=None):
        self.init_optimizer_state()
        pl = self._last[0]
        nat.check(nat.lib().vad_cad_optimizer_step(pl.h, lr, betas[0], betas[1], eps, weight_decay, max_norm,
                                                   grad_scale, nat.ptr(total_norm), nat.stream_of(self.device)))


def _set_buffer(model, dotted, tensor):
    mod = model
    parts = dotted.split(".")
    for p in parts[:-1]:
        mod = getattr(mod, p)
    mod._buffers[parts[-1]] = tensor


def engine_for(model) -> CadEngine:
    eng = model.__dict__.get("_vad_engine")
    if eng is None or not eng.is_bound():
        eng = CadEngine(model)
        model.__dict__["_vad_engine"] = eng
    return eng
