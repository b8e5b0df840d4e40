"""Token alignment and word-mapper tables (host side, built once per controller).

Same public names and results as the reference ``seq_aligner.py``; the tables feed the
device edit programs (``programs.py``).  Behaviour kept bit-exact on purpose, quirks
included (pinned by ``tests/golden/tables.npz``):

* Needleman-Wunsch with gap 0 / match 1 / mismatch -1 and tie order left > up > diag
  (``seq_aligner.py:61-76``);
* the refinement tail ``mapper[L:] = len(y) + arange`` (``:117``) and ``-1`` for inserted
  target tokens (``:93``);
* the replacement walk that, after the last replaced word, writes ``mapper[j, j]`` rather
  than ``mapper[i, j]`` (``:180-183``) and spreads ``1/len(target)`` over multi-token
  targets (``:170-172``).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from .ptp_words import get_word_inds  # noqa: F401  (re-exported, as seq_aligner.py:131 does)

GAP, MATCH, MISMATCH = 0, 1, -1
# trace-back codes of seq_aligner.py:50-55
_LEFT, _UP, _DIAG, _STOP = 1, 2, 3, 4


class ScoreParams:
    """seq_aligner.py:18-29."""

    def __init__(self, gap, match, mismatch):
        self.gap = gap
        self.match = match
        self.mismatch = mismatch

    def mis_match_char(self, x, y):
        return self.match if x == y else self.mismatch


def get_matrix(size_x: int, size_y: int, gap: int) -> np.ndarray:
    """Score matrix with the gap-penalised first row/column (seq_aligner.py:46-50)."""
    m = np.zeros((size_x + 1, size_y + 1), dtype=np.int32)
    m[0, :] = np.arange(size_y + 1, dtype=np.int32) * gap
    m[:, 0] = np.arange(size_x + 1, dtype=np.int32) * gap
    return m


def get_traceback_matrix(size_x: int, size_y: int) -> np.ndarray:
    t = np.zeros((size_x + 1, size_y + 1), dtype=np.int32)
    t[0, :] = _LEFT
    t[:, 0] = _UP
    t[0, 0] = _STOP
    return t


def global_align(x: Sequence[int], y: Sequence[int], score: ScoreParams):
    nx, ny = len(x), len(y)
    score_m = get_matrix(nx, ny, score.gap)
    trace = get_traceback_matrix(nx, ny)
    for i in range(1, nx + 1):
        xi = x[i - 1]
        row_prev, row = score_m[i - 1], score_m[i]
        for j in range(1, ny + 1):
            cand_left = int(row[j - 1]) + score.gap
            cand_up = int(row_prev[j]) + score.gap
            cand_diag = int(row_prev[j - 1]) + score.mis_match_char(xi, y[j - 1])
            best = max(cand_left, cand_up, cand_diag)
            row[j] = best
            # ties resolve left, then up, then diagonal
            trace[i, j] = _LEFT if best == cand_left else (_UP if best == cand_up else _DIAG)
    return score_m, trace


def get_aligned_sequences(x, y, trace_back):
    """Walk the trace back; return aligned sequences and the y->x token map [(j, i|-1)]."""
    xs: List = []
    ys: List = []
    pairs: List[Tuple[int, int]] = []
    i, j = len(x), len(y)
    while i > 0 or j > 0:
        code = int(trace_back[i, j])
        if code == _DIAG:
            i, j = i - 1, j - 1
            xs.append(x[i])
            ys.append(y[j])
            pairs.append((j, i))
        elif code == _LEFT:
            j -= 1
            xs.append("-")
            ys.append(y[j])
            pairs.append((j, -1))
        elif code == _UP:
            i -= 1
            xs.append(x[i])
            ys.append("-")
        else:  # _STOP
            break
    pairs.reverse()
    return xs, ys, torch.tensor(pairs, dtype=torch.int64)


def get_mapper(x: str, y: str, tokenizer, max_len: int = 77):
    """Refinement map of target tokens onto source tokens (seq_aligner.py:107-118)."""
    x_ids = tokenizer.encode(x)
    y_ids = tokenizer.encode(y)
    _, trace = global_align(x_ids, y_ids, ScoreParams(GAP, MATCH, MISMATCH))
    base = get_aligned_sequences(x_ids, y_ids, trace)[-1]
    n = base.shape[0]
    alphas = torch.ones(max_len)
    alphas[:n] = (base[:, 1] != -1).float()
    mapper = torch.zeros(max_len, dtype=torch.int64)
    mapper[:n] = base[:, 1]
    mapper[n:] = len(y_ids) + torch.arange(max_len - len(y_ids))
    return mapper, alphas


def get_refinement_mapper(prompts, tokenizer, max_len: int = 77):
    maps, alphas = zip(*[get_mapper(prompts[0], p, tokenizer, max_len) for p in prompts[1:]])
    return torch.stack(maps), torch.stack(alphas)


def get_replacement_mapper_(x: str, y: str, tokenizer, max_len: int = 77):
    """Word-replacement mapper of one edit (seq_aligner.py:152-185)."""
    wx, wy = x.split(" "), y.split(" ")
    if len(wx) != len(wy):
        raise ValueError(f"attention replacement edit can only be applied on prompts with the same length"
                         f" but prompt A has {len(wx)} words and prompt B has {len(wy)} words.")
    changed = [k for k in range(len(wy)) if wy[k] != wx[k]]
    src_inds = [get_word_inds(x, k, tokenizer) for k in changed]
    tgt_inds = [get_word_inds(y, k, tokenizer) for k in changed]
    m = np.zeros((max_len, max_len))
    i = j = 0
    nxt = 0
    while i < max_len and j < max_len:
        if nxt < len(src_inds) and src_inds[nxt][0] == i:
            s, t = src_inds[nxt], tgt_inds[nxt]
            if len(s) == len(t):
                m[s, t] = 1
            else:
                share = 1 / len(t)
                for tt in t:
                    m[s, tt] = share
            nxt += 1
            i += len(s)
            j += len(t)
        else:
            # before the last replaced word the walk is diagonal in (i, j); after it the
            # reference writes the (j, j) diagonal
            if nxt < len(src_inds):
                m[i, j] = 1
            else:
                m[j, j] = 1
            i += 1
            j += 1
    return torch.from_numpy(m).float()


def get_replacement_mapper(prompts, tokenizer, max_len: int = 77):
    return torch.stack([get_replacement_mapper_(prompts[0], p, tokenizer, max_len) for p in prompts[1:]])
