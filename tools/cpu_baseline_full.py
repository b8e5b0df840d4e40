"""Validate bench.py's CPU baseline: time ONE full 50-step edit group of the oracle's
fp32 CPU restatement on the host cores and compare it with the 2-step x25 extrapolation that
bench.py reports.  Same workload as bench.cpu_baseline (SD-v1.4-shaped U-Net N = 8, eager patched
attention + reference controller/store + LocalBlend + DDIM), one progress line per step.
Usage: python tools/cpu_baseline_full.py [steps]  -> JSON line"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main(n_steps=50):
    from oracle import control as oc
    from oracle import forward as ofw
    from p2p_amd import pipeline as pl
    from p2p_amd.tokenizer import StandInTokenizer
    cores = torch.get_num_threads()
    tok = StandInTokenizer()
    model = pl.SyntheticStableDiffusion(device="cpu", dtype=torch.float32)
    prompts = pl.north_star_prompts()
    lb = oc.OracleLocalBlend("null", prompts, pl.BLEND_WORDS, tok, start_blend=0.0)   # as bench.cpu_baseline: the blend runs every step
    ctrl = oc.OracleController("null", "replace", prompts, n_steps, 0.8, 0.4, tok, local_blend=lb, store_self=False)
    ofw.install(model, ctrl)
    ids = model.tokenizer(prompts, padding="max_length", max_length=77, return_tensors="pt").input_ids
    uids = model.tokenizer([""] * 4, padding="max_length", max_length=77, return_tensors="pt").input_ids
    ctx = torch.cat([model.text_encoder(uids)[0], model.text_encoder(ids)[0]])
    lat = pl.seed_latent(0).expand(4, 4, 64, 64).clone()
    model.scheduler.set_timesteps(n_steps)
    per_step = []
    with torch.no_grad():
        t_all = time.perf_counter()
        for i, t in enumerate(model.scheduler.timesteps):
            t0 = time.perf_counter()
            eps = model.unet(torch.cat([lat] * 2), t, encoder_hidden_states=ctx)["sample"]
            eu, ec = eps.chunk(2)
            lat = model.scheduler.step(eu + 7.5 * (ec - eu), t, lat)["prev_sample"]
            lat = ctrl.step_callback(lat)
            per_step.append(time.perf_counter() - t0)
            print(f"[cpu baseline] step {i + 1}/{n_steps}: {per_step[-1]:.2f} s", flush=True)
        total = time.perf_counter() - t_all
    extrap = (per_step[0] + per_step[1]) / 2 * n_steps
    out = {"kind": "port", "cores": cores, "ddim_steps": n_steps, "full_group_s": total,
           "full_group_value": 1.0 / total, "unit": "edit-groups/s",
           "two_step_extrapolation_s": extrap, "extrapolation_error": extrap / total - 1.0,
           "per_step_s": [round(x, 3) for x in per_step],
           "note": "oracle fp32 port on the host cores, full 50-step group vs bench.py's 2-step x25 rule"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
