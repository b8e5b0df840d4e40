"""Word-index and time/word schedule tables (host side).

``get_word_inds`` follows ``ptp_utils.py:245-263`` (identical copy at ``seq_aligner.py:131-149``);
the alpha schedule follows ``ptp_utils.py:266-297``, including its truncation
``int(bound * (num_steps + 1))`` and its in-place completion of a caller's dict with
``"default_": (0., 1.)``.  Pinned bit-exact by ``tests/golden/tables.npz``.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple, Union

import numpy as np
import torch


def get_word_inds(text: str, word_place, tokenizer):
    """Token positions (1-based, BOS = 0) of the word(s) selected by string or word index."""
    words = text.split(" ")
    if type(word_place) is str:
        targets = [i for i, w in enumerate(words) if w == word_place]
    elif type(word_place) is int:
        targets = [word_place]
    else:
        targets = word_place
    found = []
    if len(targets) > 0:
        pieces = [tokenizer.decode([tok]).strip("#") for tok in tokenizer.encode(text)][1:-1]
        consumed, word = 0, 0
        for pos, piece in enumerate(pieces):
            consumed += len(piece)
            if word in targets:
                found.append(pos + 1)
            if consumed >= len(words[word]):
                word += 1
                consumed = 0
    return np.array(found)


def update_alpha_time_word(alpha: torch.Tensor, bounds: Union[float, Tuple[float, float]], prompt_ind: int,
                           word_inds: Optional[torch.Tensor] = None):
    if type(bounds) is float:
        bounds = 0, bounds
    rows = alpha.shape[0]
    start, end = int(bounds[0] * rows), int(bounds[1] * rows)
    cols = torch.arange(alpha.shape[2]) if word_inds is None else word_inds
    alpha[:start, prompt_ind, cols] = 0
    alpha[start:end, prompt_ind, cols] = 1
    alpha[end:, prompt_ind, cols] = 0
    return alpha


def get_time_words_attention_alpha(prompts, num_steps,
                                   cross_replace_steps: Union[float, Dict[str, Tuple[float, float]]],
                                   tokenizer, max_num_words: int = 77):
    """[num_steps + 1, B - 1, 1, 1, max_num_words] 0/1 schedule of the cross-attention edit."""
    if type(cross_replace_steps) is not dict:
        cross_replace_steps = {"default_": cross_replace_steps}
    if "default_" not in cross_replace_steps:
        cross_replace_steps["default_"] = (0., 1.)
    n_edits = len(prompts) - 1
    alpha = torch.zeros(num_steps + 1, n_edits, max_num_words)
    for e in range(n_edits):
        alpha = update_alpha_time_word(alpha, cross_replace_steps["default_"], e)
    for word, bounds in cross_replace_steps.items():
        if word == "default_":
            continue
        per_edit = [get_word_inds(prompts[e + 1], word, tokenizer) for e in range(n_edits)]
        for e, inds in enumerate(per_edit):
            if len(inds) > 0:
                alpha = update_alpha_time_word(alpha, bounds, e, inds)
    return alpha.reshape(num_steps + 1, n_edits, 1, 1, max_num_words)
