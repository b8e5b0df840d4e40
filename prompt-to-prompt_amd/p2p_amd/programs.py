"""Device edit programs for the fused cross-attention kernel.

Every cross-attention edit of the reference is, per edit ``e`` and output word ``w``,

    R[w]   = post[w] * ( c_rep[w] * P_e[w] + sum_t val[t] * P_0[row[t]] )     t in column w
    P_e'   = alpha[w] * R[w] + (1 - alpha[w]) * P_e[w]

with the rows/values stored as a compressed column list:

* AttentionReplace  (main.py:217-218)  c_rep 0, column w of the mapper (``einsum('hpw,bwn')``);
* AttentionRefine   (main.py:235-239)  c_rep 1 - a[w], one term (mapper[w] mod n, a[w]);
  a ``-1`` mapper entry gathers column n-1 as torch's negative indexing does;
* AttentionReweight (main.py:258-264)  c_rep 0, one term (w, eq[w]); chained on a Replace or
  Refine controller it keeps the inner terms and sets post = eq.

Zeros of the dense mapper are skipped, so the column sums are the reference's with the
zero terms removed (exact for single-entry columns, which is every column the mapper
builders produce except multi-token source words).

Blob layout (include/p2p_hip.h; COLS = 128 column stride, TMAX = 8 term planes):
    header  int32[8] = n_edits, n_cols, tmax, COLS, dense, dense_offset, 0, 0
    per edit e, at byte 32 + e * REC_BYTES:
        c_rep f32[COLS] | post f32[COLS] | term {i32 row, f32 val}[TMAX][COLS]
    dense (when every term value is exact in f16), at byte dense_offset:
        f16 [n_edits][96 source words][96 target words] -- the mapper as an MFMA operand
Plane t of column w holds the t-th term of that column, (0, 0.0) past its last one; the kernel
walks the first ``tmax`` planes for every column (a wave-uniform loop of independent loads), and
the padding adds +0.0 after the real terms, so the sums keep the sparse order exactly.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

PROGRAM_COLS = 128
PROGRAM_TMAX = 8
REC_BYTES = 2 * 4 * PROGRAM_COLS + 8 * PROGRAM_TMAX * PROGRAM_COLS
HEADER_BYTES = 32
DENSE = 96
F_DENSE = 1


@dataclass
class EditProgram:
    n_edits: int
    n_cols: int
    c_rep: np.ndarray               # [E, n_cols] f32
    post: np.ndarray                # [E, n_cols] f32
    terms: List[List[List[tuple]]] = field(default_factory=list)  # [E][w] -> [(row, val)]

    @property
    def tmax(self) -> int:
        return max([len(col) for cols in self.terms for col in cols] + [0])

    def blob(self) -> np.ndarray:
        E, n = self.n_edits, self.n_cols
        if n > PROGRAM_COLS:
            raise ValueError(f"{n} words exceed the program column stride {PROGRAM_COLS}")
        tmax = self.tmax
        if tmax > PROGRAM_TMAX:
            raise ValueError(f"a target word gathers {tmax} source words (> {PROGRAM_TMAX})")
        rec = np.zeros((E, REC_BYTES // 4), np.uint32)
        for e in range(E):
            rec[e, :n] = np.asarray(self.c_rep[e], np.float32).view(np.uint32)
            rec[e, PROGRAM_COLS:PROGRAM_COLS + n] = np.asarray(self.post[e], np.float32).view(np.uint32)
            planes = rec[e, 2 * PROGRAM_COLS:].reshape(PROGRAM_TMAX, PROGRAM_COLS, 2)
            for w in range(n):
                for t, (r, v) in enumerate(self.terms[e][w]):
                    planes[t, w, 0] = np.uint32(np.int32(r).view(np.uint32))
                    planes[t, w, 1] = np.float32(v).view(np.uint32)
        dense = self.dense_f16()
        dense_off = HEADER_BYTES + E * REC_BYTES if dense is not None else 0
        header = np.array([E, n, tmax, PROGRAM_COLS, int(dense is not None), dense_off, 0, 0], np.int32)
        parts = [header.view(np.uint8), rec.view(np.uint8).ravel()]
        if dense is not None:
            parts.append(dense.view(np.uint8).ravel())
        return np.concatenate(parts)

    def dense_f16(self) -> Optional[np.ndarray]:
        """The mappers as f16 [E, 96, 96] (row = source word, col = target word), or None when a
        term value is not exactly representable in f16 (the kernel then gathers in f32)."""
        E, n = self.n_edits, self.n_cols
        if n > DENSE:
            return None
        m = torch.zeros(E, DENSE, DENSE, dtype=torch.float32)
        for e in range(E):
            for w in range(n):
                for (r, v) in self.terms[e][w]:
                    m[e, r, w] = float(np.float32(v))
        mb = m.to(torch.float16)
        if not torch.equal(mb.float(), m):
            return None
        return mb.view(torch.int16).numpy().view(np.uint16)

    def to_device(self, device) -> torch.Tensor:
        blob = self.blob()
        t = torch.from_numpy(blob.copy()).to(device)
        t.p2p_flags = F_DENSE if int(blob[16:20].view(np.int32)[0]) else 0   # p2p_group.flags
        t.p2p_n_edits = self.n_edits                                          # p2p_group.n_edits
        return t


def replace_program(mapper: torch.Tensor) -> EditProgram:
    """mapper: [E, n, n] float (seq_aligner.get_replacement_mapper)."""
    m = mapper.detach().to("cpu", torch.float32).numpy()
    E, n, _ = m.shape
    terms = []
    for e in range(E):
        cols = []
        for w in range(n):
            nz = np.nonzero(m[e, :, w])[0]
            cols.append([(int(r), float(m[e, r, w])) for r in nz])
        terms.append(cols)
    return EditProgram(E, n, np.zeros((E, n), np.float32), np.ones((E, n), np.float32), terms)


def refine_program(mapper: torch.Tensor, alphas: torch.Tensor) -> EditProgram:
    """mapper: [E, n] int64 (may hold -1); alphas: [E, n] or [E, 1, 1, n] float."""
    mp = mapper.detach().cpu().numpy().astype(np.int64)
    a = alphas.detach().to("cpu", torch.float32).reshape(mp.shape).numpy()
    E, n = mp.shape
    c_rep = (np.float32(1.0) - a).astype(np.float32)   # torch: 1 - alphas in f32
    terms = [[[(int(mp[e, w] % n), float(a[e, w]))] for w in range(n)] for e in range(E)]
    return EditProgram(E, n, c_rep, np.ones((E, n), np.float32), terms)


def reweight_program(equalizer: torch.Tensor, n_edits: int, inner: Optional[EditProgram]) -> EditProgram:
    """equalizer: [E_eq, n] with E_eq in {1, n_edits} (broadcast of main.py:262-263)."""
    eq = equalizer.detach().to("cpu", torch.float32).numpy()
    if eq.ndim != 2 or eq.shape[0] not in (1, n_edits):
        raise ValueError(f"equalizer of shape {tuple(eq.shape)} does not broadcast over {n_edits} edits")
    n = eq.shape[1]
    rows = [eq[e if eq.shape[0] > 1 else 0] for e in range(n_edits)]
    if inner is None:
        terms = [[[(w, float(rows[e][w]))] for w in range(n)] for e in range(n_edits)]
        return EditProgram(n_edits, n, np.zeros((n_edits, n), np.float32), np.ones((n_edits, n), np.float32),
                           terms)
    if inner.n_edits != n_edits or inner.n_cols != n:
        raise ValueError("chained controller has a different number of edits / words")
    if not np.all(inner.post == 1.0):
        raise ValueError("reweight chained on a reweight is not a fused program")
    post = np.stack(rows).astype(np.float32)
    return EditProgram(n_edits, n, inner.c_rep.copy(), post, inner.terms)
