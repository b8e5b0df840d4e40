#!/usr/bin/env python
"""Edit-groups/sec of the Prompt-to-Prompt attention-control path on MI355X.

One "step" = one complete edit group of BASELINE.json configs[1]: SD-v1.4-shaped U-Net
(random init), 512x512 (64x64 latent), 1 source + 3 AttentionReplace edits with
null_text-form LocalBlend, CFG 7.5 (U-Net batch 8), 50 DDIM steps, cross_replace 0.8,
self_replace 0.4 -- every attention call is one fused HIP kernel (edits + store in it).
Text encoding is replaced by a synthetic context, no VAE decode.

Multi-GPU: one process per GPU (torchrun); edit groups (seeds) are partitioned across ranks
(weak scaling, no data-path collective); the final latents are all-gathered over RCCL once
at the end of the timed region.  Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# Algorithmic work of the dominant kernel: the 64x64 self-attention (G1/G7), per launch
# 4 * P * K * C * N FLOP (QK^T + PV, unpadded d), P = K = 4096, C = 320, N = 8.
MFMA_PEAK_BF16_TFLOPS = 2500.0   # dense, MI355X_MICROARCH.md:43
MFMA_PEAK_F32_TFLOPS = 157.3


class DominantKernelTimer:
    """HIP events around every launch of the dominant kernel, on the launch stream."""

    def __init__(self, n_query=4096):
        self.n_query = n_query
        self.pairs = []
        self.flops = []
        self._pending = None
        self.enabled = False

    def before(self, kind, t):
        if self.enabled and kind == "self" and t.n_query == self.n_query:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._pending = (ev, 4.0 * t.n_query * t.n_key * t.n_heads * t.head_dim * t.n_batch)

    def after(self, kind, t):
        if self._pending is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.pairs.append((self._pending[0], ev))
            self.flops.append(self._pending[1])
            self._pending = None

    def summary(self):
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in self.pairs]
        if not ms:
            return None, None, 0
        avg_ms = sum(ms) / len(ms)
        flops = sum(self.flops) / len(self.flops)
        return avg_ms, flops, len(ms)


def pmc_traffic():
    """HBM bytes per launch of the dominant kernel from the newest committed PMC pass
    (profiles/rNN/pmc_g1.json, written from tools/gpu_pmc.sh: FETCH_SIZE x2 per the gfx950
    correction + WRITE_SIZE).  bench.py cannot collect counters itself (rocprofv3 --pmc is a
    separate run), so it reports the committed measurement of the same kernel and names it."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_g1.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def cpu_baseline(num_ddim_steps: int):
    """The oracle's fp32 CPU restatement of the same workload on the host cores: ONE denoising
    step (U-Net at batch 8 with the eager patched attention + reference controller +
    LocalBlend + DDIM), extrapolated to the 50-step group."""
    from oracle import control as oc
    from oracle import forward as ofw
    from p2p_amd import pipeline as pl
    from p2p_amd.tokenizer import StandInTokenizer
    cores = torch.get_num_threads()
    tok = StandInTokenizer()
    model = pl.SyntheticStableDiffusion(device="cpu", dtype=torch.float32)
    prompts = pl.north_star_prompts()
    lb = oc.OracleLocalBlend("null", prompts, pl.BLEND_WORDS, tok, start_blend=0.0)
    ctrl = oc.OracleController("null", "replace", prompts, num_ddim_steps, 0.8, 0.4, tok, local_blend=lb,
                               store_self=False)
    ofw.install(model, ctrl)
    ids = model.tokenizer(prompts, padding="max_length", max_length=77, return_tensors="pt").input_ids
    uids = model.tokenizer([""] * 4, padding="max_length", max_length=77, return_tensors="pt").input_ids
    ctx = torch.cat([model.text_encoder(uids)[0], model.text_encoder(ids)[0]])
    lat = pl.seed_latent(0).expand(4, 4, 64, 64).clone()
    model.scheduler.set_timesteps(num_ddim_steps)
    t = model.scheduler.timesteps[0]
    with torch.no_grad():
        t0 = time.perf_counter()
        eps = model.unet(torch.cat([lat] * 2), t, encoder_hidden_states=ctx)["sample"]
        eu, ec = eps.chunk(2)
        lat = model.scheduler.step(eu + 7.5 * (ec - eu), t, lat)["prev_sample"]
        lat = ctrl.step_callback(lat)
        dt = time.perf_counter() - t0
    per_group = dt * num_ddim_steps
    return {"value": 1.0 / per_group, "unit": "edit-groups/s", "cores": cores, "kind": "port",
            "sample": f"1 of {num_ddim_steps} DDIM steps (U-Net N=8 fp32 + oracle eager attention/edits/"
                      f"store + LocalBlend + DDIM) timed = {dt:.2f} s, x{num_ddim_steps} extrapolated"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="edit groups timed per rank")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--ddim-steps", type=int, default=50)
    ap.add_argument("--unet-dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--compute", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--groups-per-call", type=int, default=1,
                    help="edit groups denoised per U-Net call (controllers.GroupBatch; a step = one such\n                         batch); 1 = configs[1] as quoted")
    ap.add_argument("--store-self", action="store_true",
                    help="also keep the 32x32/16x16/8x8 SELF maps (main.py AttentionStore default); the\n                         north-star workload keeps only the maps AttentionStore/LocalBlend read")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from p2p_amd import _hip, config
    from p2p_amd import pipeline as pl
    config.set_compute(args.compute)
    _hip.lib()

    dtype = torch.bfloat16 if args.unet_dtype == "bf16" else torch.float32
    model = pl.SyntheticStableDiffusion(device=dev, dtype=dtype)
    prompts = pl.north_star_prompts()
    timer = DominantKernelTimer()
    _hip.LAUNCH_OBSERVER = timer

    G = args.groups_per_call

    def make_ctrl():
        return pl.make_replace_controller(prompts, args.ddim_steps, device=dev, store_self_maps=args.store_self)

    def batch(seeds):
        # one step: G edit groups (each 1 source + 3 edits, its own seed), one U-Net call per DDIM step
        if G == 1:
            return pl.run_edit_group(model, prompts, make_ctrl(), pl.seed_latent(seeds[0]),
                                     num_steps=args.ddim_steps)[None]
        from p2p_amd import controllers
        ctrl = controllers.GroupBatch([make_ctrl() for _ in seeds])
        lat = pl.run_edit_groups(model, [prompts] * G, ctrl, [pl.seed_latent(s) for s in seeds],
                                 num_steps=args.ddim_steps)
        return lat.reshape(G, len(prompts), *lat.shape[1:])

    # groups (seeds) partitioned across ranks round-robin: no collective on the data path
    from p2p_amd import sweep
    all_seeds = list(range(world * (args.warmup + args.steps) * G))
    mine = sweep.partition(all_seeds, rank, world)
    batches = [mine[i * G:(i + 1) * G] for i in range(args.warmup + args.steps)]
    for b in batches[:args.warmup]:
        batch(b)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    timer.enabled = True
    t0 = time.perf_counter()
    finals = torch.cat([batch(b) for b in batches[args.warmup:]]).float()   # [steps * G, 4, 4, 64, 64]
    # one RCCL all-gather of the final latents at the end (the only inter-GPU traffic)
    gathered = sweep.gather_latents(finals, world * args.steps * G, world)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timer.enabled = False
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    assert gathered.shape[0] == world * args.steps * G and torch.isfinite(gathered).all()

    avg_ms, flops, n_launch = timer.summary()
    if rank == 0:
        peak = MFMA_PEAK_BF16_TFLOPS if args.compute == "bf16" else MFMA_PEAK_F32_TFLOPS
        achieved = flops / (avg_ms * 1e-3) / 1e12 if avg_ms else None
        traffic, traffic_src = pmc_traffic() if G == 1 else (None, "no PMC pass at N = 8G")
        roofline = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                    "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                    "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                    "algorithmic_bytes": 4.0 * 8 * G * 4096 * 320 * 2,
                    "kernel": f"self_attn_fused_kernel G1/G7 (P=K=4096, d=40, N={8 * G}, H=8)",
                    "avg_launch_ms": avg_ms, "launches": n_launch,
                    "flop_per_launch": flops}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.ddim_steps)
        total = world * args.steps * G
        line = {
            "metric": "edit-groups/sec (src+3 edits, SD1.4 512², 50 DDIM)",
            "value": total / elapsed, "unit": "edit-groups/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1000.0 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.compute,
            "data": "synthetic (random-init SD-v1.4-shaped U-Net, seeded x_T, stand-in text context)",
            "config": {"workload": "configs[1]: SD-v1.4 512x512 AttentionReplace + LocalBlend, 1 source + 3 edits, "
                                   f"{args.ddim_steps} DDIM, CFG 7.5", "global_batch": 8 * G * world, "groups_per_call": G,
                       "unet_dtype": args.unet_dtype, "self_maps_kept": args.store_self, "parallelism": f"replicas x{world} (groups by seed)"},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
