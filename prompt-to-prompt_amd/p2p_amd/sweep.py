"""Seed sweeps over edit groups, one process per GPU (BASELINE.json configs[3]).

The reference sweeps seeds in a sequential Python loop (main.py:425-444).  Edit groups are
independent -- a source prompt and its edits must share a GPU because the edits read the
source's probabilities inside the attention kernel -- so the sweep shards whole groups
across ranks (round-robin by seed, weak scaling) with no collective on the data path, and
gathers each group's results once at the end: the final latents AND the reduced stored maps
(aggregate_attention's 16x16 cross maps per prompt, main.py:293-307), packed into ONE
all-gather (RCCL over xGMI on GPUs, gloo on CPU).
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple, Union

import torch
import torch.distributed as dist

Result = Union[torch.Tensor, Tuple[torch.Tensor, ...]]


def partition(seeds: Sequence[int], rank: int, world: int) -> List[int]:
    """Round-robin shard: rank r gets seeds[r], seeds[r + world], ..."""
    return list(seeds[rank::world])


def gather_latents(local: torch.Tensor, n_total: int, world: int) -> torch.Tensor:
    """All-gather per-rank stacks [n_local, ...] (ranks may hold one group fewer) and return
    them in global seed order [n_total, ...]."""
    if world == 1:
        return local
    per = (n_total + world - 1) // world
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    for r in range(world):
        idx = list(range(r, n_total, world))
        out[idx] = parts[r][: len(idx)]
    return out


def gather_results(local: Sequence[torch.Tensor], n_total: int, world: int) -> List[torch.Tensor]:
    """Several per-group results ([n_local, ...] each, e.g. latents and reduced maps) in ONE
    collective: flattened side by side into one f32 [n_local, F] buffer, all-gathered, split."""
    local = [t.float() for t in local]
    n_local = local[0].shape[0]
    if any(t.shape[0] != n_local for t in local):
        raise ValueError("every result needs one row per local group")
    if world == 1:
        return list(local)
    widths = [int(t[0].numel()) if n_local else int(torch.Size(t.shape[1:]).numel()) for t in local]
    packed = torch.cat([t.reshape(n_local, w) for t, w in zip(local, widths)], dim=1)
    full = gather_latents(packed, n_total, world)
    outs, off = [], 0
    for t, w in zip(local, widths):
        outs.append(full[:, off:off + w].reshape((n_total,) + tuple(t.shape[1:])))
        off += w
    return outs


def run_sweep(seeds: Sequence[int], run_group: Callable[[int], Result], rank: int = 0,
              world: int = 1) -> Result:
    """Run this rank's share of the groups; every rank returns every group's results in seed
    order.  run_group(seed) returns one tensor (the final latents) or a tuple of tensors
    (latents, reduced maps, ...); the return value has the same structure, stacked over seeds."""
    mine = partition(seeds, rank, world)
    outs = [run_group(s) for s in mine]
    if not outs:
        outs_probe = run_group(seeds[0])
        single = isinstance(outs_probe, torch.Tensor)
        probe = (outs_probe,) if single else tuple(outs_probe)
        local = [p.new_zeros((0,) + tuple(p.shape)) for p in probe]
    else:
        single = isinstance(outs[0], torch.Tensor)
        cols = [(o,) if single else tuple(o) for o in outs]
        local = [torch.stack([c[i] for c in cols]) for i in range(len(cols[0]))]
    if single:
        return gather_latents(local[0], len(seeds), world)
    return tuple(gather_results(local, len(seeds), world))
