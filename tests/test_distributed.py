"""Multi-rank sweep path on CPU (gloo, world size 2 and 3): seed sharding and the ONE final
all-gather of latents + reduced maps must reproduce the single-process sweep exactly.

The edit group each rank runs is a real (tiny) one: an SD-topology U-Net with small channels and
a 32x32 latent, denoised with the oracle's eager attention + AttentionReplace controller + DDIM
(the product's kernels need a GPU); its result is the final latents and the store's reduced
16x16 cross maps (controllers.reduce_maps, aggregate_attention per prompt).  bench.py runs the
same partition / gather code over RCCL with the product's HIP path.
"""
import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from p2p_amd import sweep

STEPS = 3


def tiny_model():
    from p2p_amd.ddim import DDIMScheduler
    from p2p_amd.pipeline import SyntheticTextEncoder
    from p2p_amd.tokenizer import default_tokenizer
    from p2p_amd.unet import UNet2DConditionModel
    torch.manual_seed(0)
    unet = UNet2DConditionModel(block_out_channels=(32, 64, 64, 64)).eval()
    for p in unet.parameters():
        p.requires_grad_(False)
    return SimpleNamespace(tokenizer=default_tokenizer(), text_encoder=SyntheticTextEncoder(), unet=unet,
                           scheduler=DDIMScheduler(beta_start=0.00085, beta_end=0.012, beta_schedule="scaled_linear",
                                                   clip_sample=False, set_alpha_to_one=False),
                           device=torch.device("cpu"))


def real_group(model, seed: int):
    """One 1-source + 3-edit AttentionReplace group, STEPS DDIM steps: (latents, reduced maps)."""
    from oracle_runs import oracle_controller, oracle_group
    from p2p_amd import controllers
    from p2p_amd import pipeline as pl
    prompts = pl.north_star_prompts()
    ctrl = oracle_controller("replace", prompts, model.tokenizer, STEPS, model.device)
    g = torch.Generator().manual_seed(seed)
    lat = oracle_group(model, prompts, torch.randn((1, 4, 32, 32), generator=g), ctrl, STEPS)
    store = controllers.AttentionStore()               # the product's reduction over the oracle's store
    store.attention_store, store.cur_step = ctrl.attention_store, ctrl.cur_step
    return lat, controllers.reduce_maps(store, 16, ["up", "down"], True, len(prompts))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


OUT_SHAPES = [(4, 4, 32, 32), (4, 16, 16, 77)]


def run_batch(model, seeds):
    """A batch of groups, as bench.py's batch(): results stacked [len(seeds), ...]."""
    res = [real_group(model, s) for s in seeds]
    return torch.stack([r[0] for r in res]), torch.stack([r[1] for r in res])


def _worker(rank, world, port, seeds, gpc, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = tiny_model()
        # the function bench.py times: shard, batches of gpc groups, ONE all-gather
        lat, maps = sweep.run_batched_sweep(seeds, lambda b: run_batch(model, b), OUT_SHAPES, rank, world, gpc)
        if rank == 0:
            torch.save({"lat": lat, "maps": maps}, out_path)
    finally:
        dist.destroy_process_group()


def test_partition_round_robin():
    seeds = list(range(10))
    parts = [sweep.partition(seeds, r, 4) for r in range(4)]
    assert parts == [[0, 4, 8], [1, 5, 9], [2, 6], [3, 7]]
    assert sorted(sum(parts, [])) == seeds


def test_gather_results_single_process_is_identity():
    a, b = torch.randn(3, 4, 2), torch.randn(3, 5)
    x, y = sweep.gather_results([a, b], 3, 1)
    assert torch.equal(x, a) and torch.equal(y, b)


def test_batches_cover_every_seed_once():
    seeds = list(range(11))
    got = [sweep.batches(seeds, r, 3, 2) for r in range(3)]
    assert got[0] == [[0, 3], [6, 9]] and got[2] == [[2, 5], [8]]
    assert sorted(s for r in got for b in r for s in b) == seeds


def test_rank_without_seeds_runs_nothing():
    """A rank whose shard is empty contributes empty stacks of the declared shapes; no group
    is run to learn them (the gloo cases below cover such a rank inside a real gather)."""
    calls = []
    out = sweep.run_batched_sweep([], lambda b: calls.append(b), OUT_SHAPES)
    assert calls == [] and [tuple(t.shape) for t in out] == [(0,) + s for s in OUT_SHAPES]


@pytest.mark.parametrize("world,n,gpc", [(2, 3, 1), (3, 4, 1), (2, 5, 2), (3, 2, 1)])   # (3, 2): rank 2 empty
def test_gloo_sweep_real_groups_matches_single_process(tmp_path, world, n, gpc):
    seeds = [11 * i + 3 for i in range(n)]
    out = str(tmp_path / "res.pt")
    mp.spawn(_worker, args=(world, _free_port(), seeds, gpc, out), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    threads = torch.get_num_threads()
    torch.set_num_threads(2)        # the workers' thread count: same CPU reduction order, same bits
    try:
        model = tiny_model()
        want_lat, want_maps = sweep.run_sweep(seeds, lambda s: real_group(model, s), OUT_SHAPES)
    finally:
        torch.set_num_threads(threads)
    assert got["lat"].shape == (n, 4, 4, 32, 32)
    assert got["maps"].shape == (n, 4, 16, 16, 77)
    assert torch.equal(got["lat"], want_lat.float())
    assert torch.equal(got["maps"], want_maps.float())
    # the source prompt's reduced maps are step/head/layer averages of probability rows (an edit's
    # rows are P0 . M, whose mapper rows need not sum to 1 -- seq_aligner.py:180-183)
    assert (got["maps"][:, 0].sum(-1) - 1).abs().max().item() < 1e-4
