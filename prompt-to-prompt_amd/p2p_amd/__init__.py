"""p2p_amd -- MI355X-native Prompt-to-Prompt attention-control hot path.

Host side (Python / PyTorch-ROCm) of the library; the kernels live in ``libp2p_hip.so``
(C ABI: ``include/p2p_hip.h``).  Module map, mirroring the reference files:

* ``ptp_utils``    -- register_attention_control, sampling loop, word/time tables
* ``seq_aligner``  -- token alignment and mapper tables
* ``controllers``  -- main.py's AttentionControl / Store / Edit / Replace / Refine / Reweight /
                      LocalBlend / get_equalizer / aggregate_attention
* ``null_text``    -- null_text.py's flavour of the same
* ``programs``     -- device edit programs (cross-attention edits as data)
* ``unet`` / ``ddim`` / ``pipeline`` -- the SD-v1.4-shaped caller around the hot path
"""
from . import config  # noqa: F401
from .tokenizer import StandInTokenizer, default_tokenizer  # noqa: F401

__all__ = ["config", "StandInTokenizer", "default_tokenizer"]
