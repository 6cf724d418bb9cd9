"""Drop-in for avenue_training_script_bbox.py's clip scorer (config 5) on the HIP plan (``vad_bbox_*``).

``CausalAnomalyDetector`` (bbox:51-101) keeps the class name, constructor, submodule names (state_dict keys
``encoder.0.weight`` ...) and forward return ``(anomaly_score.squeeze(), causal_adj (B,16,16), features (B,1024))``;
it runs in eval mode (the reference only ever scores clips with it: AnomalyVisualizer, bbox:339-368).
``AnomalyVisualizer.predict_anomaly_for_clip`` mirrors bbox:339-368; ``predict_clips`` scores a list of clips of
mixed lengths T by packing them into one batch per T (no layer couples clips, so this is exact).  The reference's
person detectors and drawing code (cv2 / yolov5) are out of scope.
"""
from __future__ import annotations

import ctypes
from collections import defaultdict
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

from . import _native as nat


class CausalAnomalyDetector(nn.Module):
    """bbox:51-101"""

    def __init__(self, input_channels=3, hidden_dim=64, num_frames=8):
        super().__init__()
        self.num_frames = num_frames
        self.encoder = nn.Sequential(
            nn.Conv3d(input_channels, 32, kernel_size=3, stride=1, padding=1), nn.ReLU(), nn.MaxPool3d(2),
            nn.Conv3d(32, 64, kernel_size=3, stride=1, padding=1), nn.ReLU(), nn.AdaptiveAvgPool3d((1, 4, 4)))
        self.feature_dim = 64 * 16
        self.causal_net = nn.Sequential(nn.Linear(self.feature_dim, 256), nn.ReLU(), nn.Linear(256, 16 * 16))
        self.classifier = nn.Sequential(nn.Linear(self.feature_dim, 128), nn.ReLU(), nn.Dropout(0.3),
                                        nn.Linear(128, 1), nn.Sigmoid())
        self._engine = None

    def forward(self, x):
        if self.training:
            raise NotImplementedError("the HIP bbox scorer runs in eval mode (call .eval(); the reference never "
                                      "trains this model)")
        if x.dim() != 5 or x.shape[1] != 3:
            raise ValueError(f"Expected (B,3,T,H,W) clips, got {tuple(x.shape)}")
        nat.require_hip(x)
        e = self._engine
        if e is None or e.device != x.device:
            e = self._engine = BboxEngine(self, x.device)
        e.sync_from_module()
        s, adj, f = e.forward(x.float().contiguous())
        return s.squeeze(), adj, f


class _BboxPlan:
    def __init__(self, e, shape):
        lib = nat.lib()
        B, C, T, H, W = shape
        plan = ctypes.c_void_p()
        nat.check(lib.vad_bbox_create(B, T, H, W, ctypes.byref(plan)))
        self.plan = plan
        self.ws = torch.empty(lib.vad_bbox_workspace_bytes(plan) + 256, dtype=torch.uint8, device=e.device)
        base = (self.ws.data_ptr() + 255) // 256 * 256
        nat.check(lib.vad_bbox_bind(plan, ctypes.c_void_p(base), nat.ptr(e.params)))

    def __del__(self):
        try:
            if getattr(self, "plan", None):
                nat.lib().vad_bbox_destroy(self.plan)
        except Exception:
            pass


class BboxEngine:
    def __init__(self, model, device):
        lib = nat.lib()
        self.device, self.model = device, model
        self.slots = [(lib.vad_bbox_slot_name(i).decode(), lib.vad_bbox_slot_offset(i), lib.vad_bbox_slot_numel(i))
                      for i in range(lib.vad_bbox_num_slots())]
        if [n for n, _ in model.named_parameters()] != [s[0] for s in self.slots]:
            raise NotImplementedError("the HIP bbox plan supports the reference layout (input_channels=3) only")
        self.params = torch.zeros(lib.vad_bbox_param_floats(), dtype=torch.float32, device=device)
        self._bound = False
        self.plans = {}

    def sync_from_module(self):
        if self._bound:
            return
        m = self.model
        with torch.no_grad():
            sd = dict(m.named_parameters())
            for name, off, n in self.slots:
                view = self.params[off:off + n].view_as(sd[name])
                view.copy_(sd[name].detach().to(self.device))
                mod_name, attr = name.rsplit(".", 1)
                setattr(m.get_submodule(mod_name), attr, nn.Parameter(view, requires_grad=sd[name].requires_grad))
        self._bound = True

    def forward(self, x):
        shape = tuple(x.shape)
        if shape not in self.plans:
            self.plans[shape] = _BboxPlan(self, shape)
        p = self.plans[shape]
        B = shape[0]
        f = dict(dtype=torch.float32, device=self.device)
        s, adj, feats = torch.empty(B, **f), torch.empty(B, 16, 16, **f), torch.empty(B, 1024, **f)
        nat.check(nat.lib().vad_bbox_forward(p.plan, nat.ptr(x), nat.ptr(s), nat.ptr(adj), nat.ptr(feats),
                                             nat.stream_of(self.device)))
        return s.view(B, 1), adj, feats


class AnomalyVisualizer:
    """The model-facing part of bbox:103-368: checkpoint loading and clip scoring."""

    def __init__(self, model_path: str | None = None, device="cuda"):
        self.device = device
        self.model = self.load_trained_model(model_path)

    def load_trained_model(self, model_path):
        model = CausalAnomalyDetector().to(self.device)
        if model_path and Path(model_path).exists():
            ck = torch.load(model_path, map_location="cpu", weights_only=True)
            sd = ck.get("model_state_dict", ck.get("state_dict", ck)) if isinstance(ck, dict) else ck
            model.load_state_dict(sd)
        model.eval()
        return model

    def predict_anomaly_for_clip(self, video_clip):
        """bbox:339-368: one (3,T,H,W) clip (numpy or tensor) -> (score, causal graph (16,16), features (1024,))."""
        t = torch.from_numpy(video_clip).float() if isinstance(video_clip, np.ndarray) else video_clip.float()
        if t.dim() == 4:
            t = t.unsqueeze(0)
        with torch.no_grad():
            s, adj, f = self.model(t.to(self.device))
        return float(s.squeeze().cpu().numpy()), adj.squeeze().cpu().numpy(), f.squeeze().cpu().numpy()

    def predict_clips(self, clips, process_group=None):
        """Score clips of mixed lengths: one packed batch per T; results in input order.

        Data parallel (BASELINE config 5): with an initialised process group of world size P every rank passes the
        same clip list, scores the clips of each length group at positions r, r+P, ... (an even share of every T
        bucket), and the (score, graph, features) triples are exchanged with one all_gather_object at the end;
        no layer couples clips, so the result equals the single-process one."""
        import torch.distributed as dist
        world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        rank = dist.get_rank(process_group) if world > 1 else 0
        groups = defaultdict(list)
        for i, c in enumerate(clips):
            t = torch.from_numpy(c).float() if isinstance(c, np.ndarray) else c.float()
            groups[tuple(t.shape)].append((i, t))
        mine = {}
        with torch.no_grad():
            for shape, items in groups.items():
                items = items[rank::world]
                if not items:
                    continue
                x = torch.stack([t for _, t in items]).to(self.device)
                s, adj, f = self.model(x)
                s = s.reshape(-1).cpu().numpy()
                adj, f = adj.cpu().numpy(), f.cpu().numpy()
                for k, (i, _) in enumerate(items):
                    mine[i] = (float(s[k]), adj[k], f[k])
        if world > 1:
            parts = [None] * world
            dist.all_gather_object(parts, mine, group=process_group)
            for p in parts:
                mine.update(p)
        return [mine[i] for i in range(len(clips))]
