"""Import target for avenue_training_script1.py's ``from minicausal_vad import MiniCausalVAD`` (a1:20): the class
lives in :mod:`.a2` next to the a2 model and loss it runs on."""
from .a2 import MiniCausalVAD  # noqa: F401
