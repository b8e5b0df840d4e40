"""Seed sweeps over edit groups, one process per GPU (BASELINE.json configs[3]).

The reference sweeps seeds in a sequential Python loop (main.py:425-444).  Edit groups are
independent -- a source prompt and its edits must share a GPU because the edits read the
source's probabilities inside the attention kernel -- so the sweep shards whole groups
across ranks (round-robin by seed, weak scaling) with no collective on the data path, and
gathers each group's results once at the end: the final latents AND the reduced stored maps
(aggregate_attention's 16x16 cross maps per prompt, main.py:293-307), packed into ONE
all-gather (RCCL over xGMI on GPUs, gloo on CPU).  Inside a process group the gather runs even at
world size 1 (torchrun with one rank: the same collective path as the 8-GPU node).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist

Result = Union[torch.Tensor, Tuple[torch.Tensor, ...]]


def _in_group() -> bool:
    return dist.is_available() and dist.is_initialized()


def partition(seeds: Sequence[int], rank: int, world: int) -> List[int]:
    """Round-robin shard: rank r gets seeds[r], seeds[r + world], ..."""
    return list(seeds[rank::world])


def gather_latents(local: torch.Tensor, n_total: int, world: int) -> torch.Tensor:
    """All-gather per-rank stacks [n_local, ...] (ranks may hold one group fewer) and return
    them in global seed order [n_total, ...]."""
    if world == 1 and not _in_group():
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
    if world == 1 and not _in_group():
        return list(local)
    widths = [int(t[0].numel()) if n_local else int(torch.Size(t.shape[1:]).numel()) for t in local]
    packed = torch.cat([t.reshape(n_local, w) for t, w in zip(local, widths)], dim=1)
    full = gather_latents(packed, n_total, world)
    outs, off = [], 0
    for t, w in zip(local, widths):
        outs.append(full[:, off:off + w].reshape((n_total,) + tuple(t.shape[1:])))
        off += w
    return outs


def batches(seeds: Sequence[int], rank: int, world: int, groups_per_call: int) -> List[List[int]]:
    """This rank's seeds (round-robin shard) cut into batches of at most groups_per_call groups,
    each batch one U-Net call per denoising step (controllers.GroupBatch)."""
    mine = partition(seeds, rank, world)
    return [mine[i:i + groups_per_call] for i in range(0, len(mine), groups_per_call)]


def run_batched_sweep(seeds: Sequence[int], run_batch: Callable[[List[int]], Sequence[torch.Tensor]],
                      out_shapes: Sequence[Tuple[int, ...]], rank: int = 0, world: int = 1,
                      groups_per_call: int = 1, device=None,
                      on_batch: Optional[Callable[[int, int], None]] = None) -> Tuple[torch.Tensor, ...]:
    """The sweep bench.py times (configs[3]) and tests/test_distributed.py runs over gloo: this
    rank's share of the groups in batches of groups_per_call, then ONE all-gather of every
    result.  run_batch(seeds) returns one tensor per result, each [len(seeds), *out_shapes[i]]
    (e.g. final latents and reduced maps).  Every rank returns every group's results in seed
    order, as f32 [len(seeds), *out_shapes[i]].  A rank with no seeds contributes empty stacks
    of the given shapes (nothing is run to learn them)."""
    todo = batches(seeds, rank, world, groups_per_call)
    outs = []
    for i, b in enumerate(todo):
        res = tuple(run_batch(b))
        if len(res) != len(out_shapes) or any(tuple(r.shape) != (len(b),) + tuple(sh)
                                               for r, sh in zip(res, out_shapes)):
            raise ValueError(f"run_batch returned {[tuple(r.shape) for r in res]}, expected "
                             f"{[(len(b),) + tuple(sh) for sh in out_shapes]}")
        outs.append(res)
        if on_batch is not None:
            on_batch(i, len(todo))
    if outs:
        local = [torch.cat([o[j].float() for o in outs]) for j in range(len(out_shapes))]
    else:
        local = [torch.zeros((0,) + tuple(sh), device=device) for sh in out_shapes]
    return tuple(gather_results(local, len(seeds), world))


def run_sweep(seeds: Sequence[int], run_group: Callable[[int], Result], out_shapes: Sequence[Tuple[int, ...]],
              rank: int = 0, world: int = 1, device=None) -> Tuple[torch.Tensor, ...]:
    """One group per call: run_group(seed) returns a tensor or a tuple of tensors of out_shapes."""
    def run_batch(b):
        r = run_group(b[0])
        r = (r,) if isinstance(r, torch.Tensor) else tuple(r)
        return tuple(t[None] for t in r)
    return run_batched_sweep(seeds, run_batch, out_shapes, rank, world, 1, device)
