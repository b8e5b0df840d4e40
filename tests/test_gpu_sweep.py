"""configs[3] on a GPU: the seed sweep exactly as bench.py --seeds S --groups-per-call 8 times it
(sweep.run_batched_sweep over pipeline.sweep_batch_runner; main.py:425-444 is the reference's
sequential seed loop), at world size 1 on the box's single GPU.  The multi-rank partition + gather
of the same function runs over gloo in tests/test_distributed.py.

16 seeds in batches of 8 groups per U-Net call (bf16 U-Net, bf16 kernels, 50 DDIM steps, 1 source
+ 3 AttentionReplace edits + LocalBlend per group).  Two sampled groups -- one from each batch --
against single-group ORACLE runs on the same weights (fp32 eager attention + reference controller
+ LocalBlend + DDIM): final latents cosine >= 0.999 per prompt, the edit-effect cosine against the
oracle's no-edit run >= 0.70 (a no-edit negative control must fail it), and the gathered 16x16
cross maps within 3e-3 (two bf16-U-Net trajectories; test_gpu_bench_config.py); every source
prompt's gathered map row sums to 1.
"""
import pytest
import torch

from oracle import control as oc
from oracle_runs import (EFFECT_BAR_BF16_UNET, base_group, check_effect, check_negative, cosine, oracle_controller,
                         oracle_group)
from p2p_amd import config, controllers, sweep
from p2p_amd import pipeline as pl

pytestmark = pytest.mark.gpu

SEEDS, GPC, STEPS = 16, 8, 50


def test_config3_sweep_world1_vs_oracle(cuda, tok):
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.bfloat16)
    prompts = pl.north_star_prompts()
    B = len(prompts)
    run = pl.sweep_batch_runner(model, prompts, STEPS, device=cuda)
    seeds = list(range(SEEDS))
    done = []
    with config.compute_mode("bf16"):
        lat, maps = sweep.run_batched_sweep(seeds, run, run.out_shapes, rank=0, world=1, groups_per_call=GPC,
                                            device=cuda, on_batch=lambda i, n: done.append(i))
    torch.cuda.synchronize()
    assert done == [0, 1]
    assert lat.shape == (SEEDS, B, 4, 64, 64) and maps.shape == (SEEDS, B, 16, 16, 77)
    assert torch.isfinite(lat).all() and torch.isfinite(maps).all()
    row_err = (maps[:, 0].sum(-1) - 1).abs().max().item()
    print(f"configs[3] sweep: {SEEDS} groups, source map rows sum to 1 within {row_err:.2e}", flush=True)
    assert row_err < 1e-3
    for s in (3, 12):
        lb = oc.OracleLocalBlend("null", prompts, pl.BLEND_WORDS, tok)
        lb.alpha = lb.alpha.to(cuda)
        octrl = oracle_controller("replace", prompts, tok, STEPS, cuda, local_blend=lb)
        want = oracle_group(model, prompts, pl.seed_latent(s), octrl, STEPS)
        cos = cosine(lat[s], want)
        store = controllers.AttentionStore()            # the product's reduction over the oracle's store
        store.attention_store, store.cur_step = octrl.attention_store, octrl.cur_step
        want_maps = controllers.reduce_maps(store, 16, ["up", "down"], True, B)
        dmap = (maps[s] - want_maps).abs().max().item()
        print(f"  seed {s}: latent cosine per prompt {[round(c, 6) for c in cos.tolist()]}, "
              f"16x16 map |diff| {dmap:.2e}", flush=True)
        assert cos.min().item() >= 0.999, cos
        assert dmap < 3e-3
        # the edit's effect against the oracle's no-edit run (bf16 U-Net bar, tests/oracle_runs.py)
        base = base_group(model, prompts, pl.seed_latent(s), STEPS)
        check_effect(f"  seed {s}", lat[s], want, base, EFFECT_BAR_BF16_UNET)
        if s == 3:     # negative control: that seed's group without the edit must fail the bar
            with config.compute_mode("bf16"):
                neg = pl.run_edit_group(model, prompts, controllers.EmptyControl(), pl.seed_latent(s), num_steps=STEPS)
            check_negative("no edit", neg, want, base, EFFECT_BAR_BF16_UNET)


def test_bench_under_torchrun_world1_rccl(cuda):
    """bench.py as the driver launches it on a node (torch.distributed.run, one rank per GPU), with
    ONE rank on this box's GPU: the RCCL process group init, barriers, the packed all-gather of
    the final latents + maps and the max-over-ranks all-reduce all run on hardware (at world 1 the
    collectives are identities, but the nccl path is the one the 8-GPU scaling run takes).  2 DDIM
    steps per group keep it short."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--ddim-steps", "2", "--no-cpu-baseline"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    print("torchrun world-1 bench:", line["value"], "edit-groups/s at 2 DDIM steps", flush=True)
    assert line["n_gpus"] == 1 and line["config"]["groups_total"] == 2 and line["value"] > 0
    # the default loop replays HIP graphs; the per-launch timing pass that follows ran eagerly
    assert line["loop"].startswith("HIP graphs") and line["eager_value"]["groups"] == 2
    assert line["roofline"]["launches"] > 0
