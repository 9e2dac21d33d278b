"""funasr_amd — MI355X-native (gfx950) Paraformer / SenseVoiceSmall inference behind FunASR's
AutoModel contract.

Importing the package does not touch the GPU. Compute lives in libpfm_hip.so (C ABI,
include/pfm.h); `funasr_amd.runtime` binds it. Build with `python -m funasr_amd.build`.
"""
from .config import (ParaformerConfig, SenseVoiceConfig, paraformer_large, paraformer_tiny,  # noqa: F401
                     sense_voice_small, sense_voice_tiny)
from .register import tables  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: AutoModel / Paraformer import torch
    if name == "AutoModel":
        from .auto_model import AutoModel
        return AutoModel
    if name == "Paraformer":
        from .model import Paraformer
        return Paraformer
    if name == "SenseVoiceSmall":
        from .sense_voice import SenseVoiceSmall
        return SenseVoiceSmall
    raise AttributeError(name)
