"""Oracle restatement of the host edit tables (pure Python; TEST INFRASTRUCTURE ONLY)."""
from __future__ import annotations

import torch


def word_positions(text, selector, tok):
    """ptp_utils.py:245-263 -- token indices (1-based) of the selected word(s)."""
    words = text.split(" ")
    if isinstance(selector, str):
        wanted = {i for i in range(len(words)) if words[i] == selector}
    elif isinstance(selector, int):
        wanted = {selector}
    else:
        wanted = set(selector)
    result = []
    if not wanted:
        return result
    ids = tok.encode(text)
    pieces = [tok.decode([t]).strip("#") for t in ids][1:len(ids) - 1]
    chars, w = 0, 0
    for pos in range(len(pieces)):
        chars = chars + len(pieces[pos])
        if w in wanted:
            result.append(pos + 1)
        if chars >= len(words[w]):
            w, chars = w + 1, 0
    return result


def needleman_wunsch(a, b):
    """seq_aligner.py:46-76: score 0-gap / +1 match / -1 mismatch, trace 1 left 2 up 3 diag."""
    rows, cols = len(a) + 1, len(b) + 1
    score = [[0] * cols for _ in range(rows)]
    trace = [[0] * cols for _ in range(rows)]
    for j in range(cols):
        trace[0][j] = 1
    for i in range(rows):
        trace[i][0] = 2
    trace[0][0] = 4
    for i in range(1, rows):
        for j in range(1, cols):
            left = score[i][j - 1]
            up = score[i - 1][j]
            diag = score[i - 1][j - 1] + (1 if a[i - 1] == b[j - 1] else -1)
            best = max(left, up, diag)
            score[i][j] = best
            if best == left:
                trace[i][j] = 1
            elif best == up:
                trace[i][j] = 2
            else:
                trace[i][j] = 3
    return trace


def y_to_x(a, b, trace):
    """seq_aligner.py:79-104: for every token of b, the aligned token of a (or -1)."""
    i, j = len(a), len(b)
    out = []
    while i > 0 or j > 0:
        t = trace[i][j]
        if t == 3:
            i -= 1
            j -= 1
            out.append((j, i))
        elif t == 1:
            j -= 1
            out.append((j, -1))
        elif t == 2:
            i -= 1
        else:
            break
    return out[::-1]


def refinement(prompts, tok, n=77):
    """seq_aligner.py:107-128 -> (mapper [E, n] int64, alphas [E, n] f32)."""
    src = tok.encode(prompts[0])
    maps, alphas = [], []
    for p in prompts[1:]:
        tgt = tok.encode(p)
        pairs = y_to_x(src, tgt, needleman_wunsch(src, tgt))
        m = [x for (_, x) in pairs] + [len(tgt) + k for k in range(n - len(tgt))]
        a = [0.0 if x == -1 else 1.0 for (_, x) in pairs] + [1.0] * (n - len(pairs))
        maps.append(m)
        alphas.append(a)
    return torch.tensor(maps, dtype=torch.int64), torch.tensor(alphas, dtype=torch.float32)


def replacement(prompts, tok, n=77):
    """seq_aligner.py:152-195 -> [E, n, n] f32, including the (j, j) tail quirk."""
    out = []
    src = prompts[0]
    sw = src.split(" ")
    for p in prompts[1:]:
        tw = p.split(" ")
        if len(sw) != len(tw):
            raise ValueError("attention replacement edit can only be applied on prompts with the same length")
        changed = [k for k in range(len(tw)) if tw[k] != sw[k]]
        s_ind = [word_positions(src, k, tok) for k in changed]
        t_ind = [word_positions(p, k, tok) for k in changed]
        M = [[0.0] * n for _ in range(n)]
        i = j = c = 0
        while i < n and j < n:
            if c < len(s_ind) and s_ind[c][0] == i:
                s, t = s_ind[c], t_ind[c]
                if len(s) == len(t):
                    for a, b in zip(s, t):
                        M[a][b] = 1.0
                else:
                    for b in t:
                        for a in s:
                            M[a][b] = 1.0 / len(t)
                c += 1
                i += len(s)
                j += len(t)
            else:
                if c < len(s_ind):
                    M[i][j] = 1.0
                else:
                    M[j][j] = 1.0
                i += 1
                j += 1
        out.append(M)
    return torch.tensor(out, dtype=torch.float64).float()


def time_word_alpha(prompts, num_steps, spec, tok, n=77):
    """ptp_utils.py:266-297 -> [num_steps + 1, E, 1, 1, n]."""
    if not isinstance(spec, dict):
        spec = {"default_": spec}
    if "default_" not in spec:
        spec["default_"] = (0.0, 1.0)
    R = num_steps + 1
    E = len(prompts) - 1
    A = [[[0.0] * n for _ in range(E)] for _ in range(R)]

    def apply(bounds, e, cols):
        if isinstance(bounds, float):
            bounds = (0.0, bounds)
        lo, hi = int(bounds[0] * R), int(bounds[1] * R)
        for r in range(R):
            v = 1.0 if lo <= r < hi else 0.0
            for col in cols:
                A[r][e][col] = v

    for e in range(E):
        apply(spec["default_"], e, range(n))
    for word, bounds in spec.items():
        if word == "default_":
            continue
        for e in range(E):
            cols = word_positions(prompts[e + 1], word, tok)
            if cols:
                apply(bounds, e, cols)
    return torch.tensor(A, dtype=torch.float32).reshape(R, E, 1, 1, n)


def equalizer_main(text, select, values, tok, n=77):
    """main.py:281-290."""
    if isinstance(select, (int, str)):
        select = (select,)
    eq = torch.ones(len(values), n)
    for w in select:
        cols = word_positions(text, w, tok)
        eq[:, cols] = torch.tensor(values, dtype=torch.float32)
    return eq


def equalizer_null(text, select, values, tok, n=77):
    """null_text.py:340-349."""
    if isinstance(select, (int, str)):
        select = (select,)
    eq = torch.ones(1, n)
    for w, v in zip(select, values):
        eq[:, word_positions(text, w, tok)] = v
    return eq


def blend_alpha(prompts, words, tok, n=77):
    """main.py:58-64 / null_text.py:78-84: [B, n] 0/1 word selection."""
    a = torch.zeros(len(prompts), n)
    for i, (p, ws) in enumerate(zip(prompts, words)):
        for w in ([ws] if isinstance(ws, str) else ws):
            for col in word_positions(p, w, tok):
                a[i, col] = 1.0
    return a
