"""MI355X-native hot path of pvvkishore/Causal-Learning-Based-Video-Anomaly-Detection_Paper_Code_Raw.

Drop-in modules (reference names and state_dict keys) whose forward/backward/optimizer run in hand-written
HIP kernels for gfx950 (libvadhip.so, C ABI in include/vad.h).  Import through the ``vad_amd`` alias.
"""
from .cad import (CausalAnomalyDetector, CausalFactorExtractor, CausalStructureLearner, DynamicsPredictor,  # noqa
                  EnhancedAnomalyScorer, ResNetBackbone, SimplePedestrianDetector, TrajectoryEncoder,
                  TrajectoryTracker)
from .train import CadTrainer, apply_memory_efficient_training, test_model, train_model  # noqa: F401
