"""Drop-in CausalAnomalyDetector (causal_anomaly_detection.py:508-586) running on libvadhip.

The nn.Module tree mirrors the reference exactly — class names, constructor signatures, attribute names,
Sequential indices and the order in which submodules are created — so that
  * ``torch.manual_seed(s); CausalAnomalyDetector()`` draws bit-identical initial weights,
  * state_dict keys match and reference checkpoints load,
  * ``model(videos)`` returns the reference's dict (cad:578-586).
The torch submodules are parameter containers only: every forward/backward runs in HIP kernels through the
C ABI (include/vad.h).  Randomness (dropout masks, VAE noise) comes from the keyed counter RNG of the
library; in the module API the key is drawn from torch's default generator, so torch.manual_seed still makes
runs reproducible.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import engine as _eng


# ---------------------------------------------------------------------------------------------- helpers
def _conv_stage(cin: int, cout: int, stride: int) -> nn.Sequential:
    """[Conv3x3(stride) BN ReLU, Conv3x3 BN ReLU] (ResNetBackbone._make_layer, cad:128-139)."""
    mods = []
    for i in range(2):
        mods += [nn.Conv2d(cin if i == 0 else cout, cout, 3, stride=stride if i == 0 else 1, padding=1),
                 nn.BatchNorm2d(cout), nn.ReLU(inplace=True)]
    return nn.Sequential(*mods)


def _mlp(widths, dropout_after=(), final_act=None) -> nn.Sequential:
    """Linear/ReLU stack; Dropout(p) follows the ReLU of hidden layer i when i is in dropout_after."""
    mods = []
    drops = dict(dropout_after)
    for i in range(len(widths) - 1):
        mods.append(nn.Linear(widths[i], widths[i + 1]))
        if i < len(widths) - 2:
            mods.append(nn.ReLU())
            if i in drops:
                mods.append(nn.Dropout(drops[i]))
    if final_act is not None:
        mods.append(final_act)
    return nn.Sequential(*mods)


# ---------------------------------------------------------------------------------------------- stages
class ResNetBackbone(nn.Module):
    """Per-frame CNN (cad:110-158): conv7x7/s2 + BN + ReLU + maxpool, four 2-conv stages, AdaptiveAvgPool(4,6)."""

    def __init__(self, input_channels=1, output_dim=256):
        super().__init__()
        self.conv1 = nn.Conv2d(input_channels, 32, 7, stride=2, padding=3)
        self.bn1 = nn.BatchNorm2d(32)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        for i, (cin, cout, s) in enumerate([(32, 32, 1), (32, 64, 2), (64, 128, 2), (128, output_dim, 2)], 1):
            setattr(self, f"layer{i}", _conv_stage(cin, cout, s))
        self.avgpool = nn.AdaptiveAvgPool2d((4, 6))


class SimplePedestrianDetector(nn.Module):
    """Box regressor MLP 6144->512->256->128->64->20 with the reference's pedestrian-position bias (cad:160-230)."""

    PRIOR_BOXES = [180, 120, 25, 50, 150, 100, 20, 45, 210, 140, 30, 55, 120, 80, 22, 48, 240, 160, 28, 52]

    def __init__(self, feature_dim):
        super().__init__()
        self.feature_dim = feature_dim
        self.detector_net = _mlp([feature_dim, 512, 256, 128, 64, 20], dropout_after=((0, 0.3), (1, 0.2)))
        self.init_weights()

    def init_weights(self):
        with torch.no_grad():
            self.detector_net[-1].bias.data = torch.tensor(self.PRIOR_BOXES, dtype=torch.float32)


class TrajectoryTracker(nn.Module):
    """ReID MLP 4->32->64->64 on boxes; trajectories = [box, reid] zero-padded per clip (cad:232-274)."""

    def __init__(self, max_tracks=20, reid_dim=64):
        super().__init__()
        self.max_tracks = max_tracks
        self.reid_dim = reid_dim
        self.reid_net = _mlp([4, 32, reid_dim, reid_dim])


class TrajectoryEncoder(nn.Module):
    """GRU over each trajectory, last hidden -> Linear(64, 32) (cad:276-309)."""

    def __init__(self, input_dim, latent_dim=32, hidden_dim=64):
        super().__init__()
        self.input_dim = input_dim
        self.latent_dim = latent_dim
        self.gru = nn.GRU(input_dim, hidden_dim, batch_first=True, bidirectional=False)
        self.encoder = nn.Linear(hidden_dim, latent_dim)


class CausalFactorExtractor(nn.Module):
    """VAE head: 32->32->32, mu / logvar (num_factors), reparameterised z and per-clip KL (cad:311-352)."""

    def __init__(self, input_dim, num_factors=6, hidden_dim=32):
        super().__init__()
        self.num_factors = num_factors
        self.encoder = nn.Sequential(nn.Linear(input_dim, hidden_dim), nn.ReLU(),
                                     nn.Linear(hidden_dim, hidden_dim), nn.ReLU())
        self.mu_head = nn.Linear(hidden_dim, num_factors)
        self.logvar_head = nn.Linear(hidden_dim, num_factors)


class CausalStructureLearner(nn.Module):
    """Node encoder + pairwise edge MLP -> num_factors^2 adjacency (cad:354-398)."""

    def __init__(self, num_factors, hidden_dim=32):
        super().__init__()
        self.num_factors = num_factors
        self.node_encoder = nn.Linear(num_factors, hidden_dim)
        self.edge_predictor = nn.Sequential(nn.Linear(hidden_dim * 2, hidden_dim), nn.ReLU(),
                                            nn.Linear(hidden_dim, 1), nn.Sigmoid())
        self.structure_params = nn.Parameter(torch.randn(num_factors, num_factors))


class DynamicsPredictor(nn.Module):
    """(A z^T)^T then MLP 6->32->32->6 (cad:400-426)."""

    def __init__(self, num_factors, hidden_dim=32):
        super().__init__()
        self.num_factors = num_factors
        self.dynamics_net = _mlp([num_factors, hidden_dim, hidden_dim, num_factors])


class EnhancedAnomalyScorer(nn.Module):
    """0.5 causal + 0.3 motion + 0.2 temporal sigmoid scorers (cad:428-502)."""

    def __init__(self, num_factors):
        super().__init__()
        self.num_factors = num_factors
        self.causal_scorer = _mlp([num_factors * 3, 64, 32, 1], dropout_after=((0, 0.2),), final_act=nn.Sigmoid())
        self.motion_scorer = _mlp([num_factors * 2, 32, 16, 1], final_act=nn.Sigmoid())
        self.temporal_scorer = _mlp([num_factors, 32, 16, 1], final_act=nn.Sigmoid())


# ---------------------------------------------------------------------------------------------- autograd bridge
class _CadFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, x, training, seed, step, clip0, *params):
        o = engine.forward(x, training, seed, step, clip0)
        ctx.engine = engine
        ctx.generation = engine.generation
        ctx.mark_non_differentiable(o["nmax"], o["counts"])
        return o["final"], o["probs"], o["causal"], o["kl"], o["z"], o["adj"], o["nmax"], o["boxes"], o["counts"]

    @staticmethod
    def backward(ctx, d_final, d_probs, d_causal, d_kl, d_z, d_adj, d_nmax, d_boxes, d_counts):
        eng = ctx.engine
        if eng.generation != ctx.generation:
            raise RuntimeError("libvadhip keeps the activations of the most recent forward only: call backward "
                               "before running the model again")
        eng.backward(False, d_final, d_probs, d_causal, d_kl, d_z, d_adj, d_boxes=d_boxes)
        flags = eng.grads[eng.param_floats:eng.param_floats + 2].tolist()
        grads = []
        for i, g in enumerate(eng.slot_group):
            live = (g == _eng.GROUP_ALWAYS or (g == _eng.GROUP_DET and flags[0] > 0)
                    or (g == _eng.GROUP_STRUCT and flags[1] > 0) or (g == _eng.GROUP_FROZEN and eng.stem_grad_on))
            grads.append(eng.grad_view(i).view(eng.model_param_shapes[i]).clone() if live else None)
        return (None, None, None, None, None, None, *grads)


# ---------------------------------------------------------------------------------------------- the model
class CausalAnomalyDetector(nn.Module):
    """Complete causal anomaly detection model (cad:508-586), HIP-backed."""

    def __init__(self, num_factors=6, reid_dim=64):
        super().__init__()
        if num_factors != 6 or reid_dim != 64:
            raise ValueError("libvadhip implements the reference configuration num_factors=6, reid_dim=64")
        self.backbone = ResNetBackbone(input_channels=1, output_dim=256)
        self.detector = SimplePedestrianDetector(256 * 4 * 6)
        self.tracker = TrajectoryTracker(reid_dim=reid_dim)
        self.traj_encoder = TrajectoryEncoder(4 + reid_dim, latent_dim=32)
        self.causal_extractor = CausalFactorExtractor(32, num_factors=num_factors)
        self.structure_learner = CausalStructureLearner(num_factors)
        self.dynamics_predictor = DynamicsPredictor(num_factors)
        self.anomaly_scorer = EnhancedAnomalyScorer(num_factors)
        self.direct_classifier = _mlp([256 * 4 * 6, 512, 256, 128, 64, 2], dropout_after=((0, 0.3), (1, 0.2)),
                                      final_act=nn.Softmax(dim=-1))

    def engine(self) -> _eng.CadEngine:
        eng = _eng.engine_for(self)
        eng.model_param_shapes = [p.shape for p in self.parameters()]
        dt = getattr(self, "_compute_dtype", torch.float32)
        if eng.compute_dtype != dt:
            eng.compute_dtype = dt
        return eng

    def set_compute_dtype(self, dtype):
        """torch.float32 (default, fp32 numerics) or torch.bfloat16: the backbone's 3x3 convs take bf16 operands
        with fp32 accumulation (BASELINE config 4); BN, heads, losses and AdamW stay fp32.  An extension of the
        reference surface (which runs fp32 on CPU and fp16 autocast on CUDA, cad:644-668)."""
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"compute dtype must be torch.float32 or torch.bfloat16, got {dtype}")
        self._compute_dtype = dtype
        return self

    def forward(self, video_frames, *, seed=None, step=0, clip0=0):
        """video_frames: (B, T, 1, H, W) on a HIP device.  Returns the reference's output dict."""
        eng = self.engine()
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if self.training else 0
        params = list(self.parameters())
        final, probs, causal, kl, z, adj, nmax, boxes, counts = _CadFunction.apply(
            eng, video_frames, self.training, seed, step, clip0, *params)
        B, T = video_frames.shape[:2]
        nm = nmax.tolist()
        cnt = counts.tolist()
        return {
            "anomaly_scores": final,
            "causal_factors": [z[b, :nm[b]] for b in range(B)],
            "adjacency_matrices": [adj[b] for b in range(B)],
            "kl_losses": [kl[b] for b in range(B)],
            "detections": [[boxes[b, t, :cnt[b][t]] for t in range(T)] for b in range(B)],
            "direct_predictions": probs,
            "causal_anomaly_scores": causal,
        }
