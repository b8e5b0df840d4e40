"""Process-wide switches of the attention path.

COMPUTE selects the MFMA precision of the fused kernels:
  "bf16" -- production path (bf16 operands, f32 accumulate / softmax / edits / stores);
  "f32"  -- check mode (exact-f32 v_mfma_f32_32x32x2_f32), parity within 1e-5.
"""
from __future__ import annotations

import contextlib
import os

COMPUTE = os.environ.get("P2P_COMPUTE", "bf16")

# main.py:18 / null_text.py:22: run the CFG halves as two U-Net calls; the controllers then
# skip the first num_att_layers calls of every step (main.py:77-79).
LOW_RESOURCE = False


def set_compute(mode: str):
    global COMPUTE
    if mode not in ("bf16", "f32"):
        raise ValueError(f"compute mode {mode!r} (bf16 | f32)")
    COMPUTE = mode


def get_compute() -> str:
    return COMPUTE


@contextlib.contextmanager
def compute_mode(mode: str):
    old = COMPUTE
    set_compute(mode)
    try:
        yield
    finally:
        set_compute(old)
