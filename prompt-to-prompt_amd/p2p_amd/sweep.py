"""Seed sweeps over edit groups, one process per GPU (BASELINE.json configs[3]).

The reference sweeps seeds in a sequential Python loop (main.py:425-444).  Edit groups are
independent -- a source prompt and its edits must share a GPU because the edits read the
source's probabilities inside the attention kernel -- so the sweep shards whole groups
across ranks (round-robin by seed, weak scaling) with no collective on the data path, and
gathers the final latents once at the end (RCCL all-gather over xGMI on GPUs, gloo on CPU).
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import torch
import torch.distributed as dist


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


def run_sweep(seeds: Sequence[int], run_group: Callable[[int], torch.Tensor], rank: int = 0,
              world: int = 1) -> torch.Tensor:
    """Run this rank's share of the groups; every rank returns all final latents in seed order."""
    mine = partition(seeds, rank, world)
    local = torch.stack([run_group(s) for s in mine]) if mine else None
    if local is None:
        probe = run_group(seeds[0])
        local = probe.new_zeros((0,) + tuple(probe.shape))
    return gather_latents(local, len(seeds), world)
