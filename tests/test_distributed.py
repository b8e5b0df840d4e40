"""Multi-rank sweep path on CPU (gloo, world size 2 and 3): seed sharding and the final
all-gather must reproduce the single-process sweep exactly."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from p2p_amd import sweep


def fake_group(seed: int) -> torch.Tensor:
    """Stand-in for a 50-step edit group: a deterministic latent per seed ([4, 4, 8, 8])."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(4, 4, 8, 8, generator=g) * (1 + seed)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, seeds, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lat = sweep.run_sweep(seeds, fake_group, rank, world)
        if rank == 0:
            torch.save(lat, out_path)
    finally:
        dist.destroy_process_group()


def test_partition_round_robin():
    seeds = list(range(10))
    parts = [sweep.partition(seeds, r, 4) for r in range(4)]
    assert parts == [[0, 4, 8], [1, 5, 9], [2, 6], [3, 7]]
    assert sorted(sum(parts, [])) == seeds


@pytest.mark.parametrize("world,n", [(2, 6), (3, 7)])
def test_gloo_sweep_matches_single_process(tmp_path, world, n):
    seeds = [11 * i + 3 for i in range(n)]
    out = str(tmp_path / "lat.pt")
    mp.spawn(_worker, args=(world, _free_port(), seeds, out), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    want = sweep.run_sweep(seeds, fake_group)
    assert got.shape == (n, 4, 4, 8, 8)
    assert torch.equal(got, want)
