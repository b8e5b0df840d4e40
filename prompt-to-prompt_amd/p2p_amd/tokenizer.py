"""Deterministic stand-in for the CLIP BPE tokenizer.

The reference builds every edit table through exactly two tokenizer calls:
``tokenizer.encode(text) -> [BOS, ids..., EOS]`` (``seq_aligner.py:108-109``,
``ptp_utils.py:253``) and ``tokenizer.decode([id]) -> piece`` (``ptp_utils.py:253``),
plus ``tokenizer(prompts, padding="max_length", max_length=77, ...)`` in the sampling
loop (``ptp_utils.py:144-156``).  The real CLIP vocabulary is not available offline, so
this class reproduces that interface deterministically:

* words are lower-cased and split on single spaces;
* a word longer than ``long_word`` characters is split into ``piece_len``-character
  pieces (``"lasagna" -> "lasa", "gna"``), which exercises the multi-token branches of
  the mapper builders (``seq_aligner.py:164-172``);
* a piece's id is a CRC32 hash of the piece text, so ids never depend on call order.

The golden fixtures under ``tests/golden`` store the id lists they were built from.
"""
from __future__ import annotations

import zlib
from typing import Dict, List, Sequence

import torch

BOS_ID = 49406
EOS_ID = 49407


class _Batch:
    def __init__(self, input_ids: torch.Tensor):
        self.input_ids = input_ids

    def __getitem__(self, key):
        return getattr(self, key)


class StandInTokenizer:
    bos_token_id = BOS_ID
    eos_token_id = EOS_ID
    pad_token_id = EOS_ID
    model_max_length = 77

    def __init__(self, piece_len: int = 4, long_word: int = 6):
        self.piece_len = piece_len
        self.long_word = long_word
        self._pieces: Dict[int, str] = {BOS_ID: "<|startoftext|>", EOS_ID: "<|endoftext|>"}

    # -- word -> pieces -> ids -------------------------------------------------
    def pieces(self, word: str) -> List[str]:
        if len(word) <= self.long_word:
            return [word]
        return [word[i:i + self.piece_len] for i in range(0, len(word), self.piece_len)]

    def piece_id(self, piece: str) -> int:
        pid = 1000 + zlib.crc32(piece.encode("utf-8")) % 48000
        self._pieces.setdefault(pid, piece)
        return pid

    def encode(self, text: str) -> List[int]:
        ids = [BOS_ID]
        for word in text.lower().split(" "):
            if not word:
                continue
            ids.extend(self.piece_id(p) for p in self.pieces(word))
        ids.append(EOS_ID)
        return ids

    def decode(self, ids: Sequence[int]) -> str:
        return "".join(self._pieces.get(int(i), "") for i in ids)

    # -- batch call used by the sampling loop ----------------------------------
    def __call__(self, prompts, padding="max_length", max_length=None, truncation=True,
                 return_tensors="pt"):
        if isinstance(prompts, str):
            prompts = [prompts]
        max_length = max_length or self.model_max_length
        rows = []
        for p in prompts:
            ids = self.encode(p)
            if truncation and len(ids) > max_length:
                ids = ids[:max_length - 1] + [EOS_ID]
            ids = ids + [self.pad_token_id] * (max_length - len(ids))
            rows.append(ids)
        return _Batch(torch.tensor(rows, dtype=torch.int64))


_DEFAULT = None


def default_tokenizer() -> StandInTokenizer:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = StandInTokenizer()
    return _DEFAULT
