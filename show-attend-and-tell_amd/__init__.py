"""sat_amd — MI355X-native Show-Attend-and-Tell training path.

Drop-in for the reference's encoder.py / attention.py / decoder.py and the inner
loop of train.py (yvokeller/Show-Attend-and-Tell): same module API, state_dict
keys and CLI flags; compute runs in hand-written gfx950 HIP kernels behind the
C ABI in include/sat_hip.h (libsat_hip.so, loaded with ctypes).
"""
from . import _lib
from ._lib import SatPolicy as Policy
from .attention import Attention
from .data import PackedImages, collate_packed
from .decoder import Decoder
from .encoder import Encoder
from .loss import caption_loss, special_ids, StepMetrics, RunningMeters
from .optim import Adam

__all__ = ["Attention", "Decoder", "Encoder", "caption_loss", "special_ids", "StepMetrics", "RunningMeters", "Adam",
           "PackedImages", "collate_packed"]
