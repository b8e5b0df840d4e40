"""BASELINE.json configs[2] throughput: G edit groups (AttentionReweight chained on AttentionRefine,
every 16/32-res cross map stored) per U-Net call through controllers.GroupBatch, bf16 U-Net, 50 DDIM
steps -- against the same groups run one per call.  Prints edit-groups/s for both."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import controllers, pipeline as pl  # noqa: E402


def main(G=8, steps=50):
    dev = torch.device("cuda")
    model = pl.SyntheticStableDiffusion(device=dev, dtype=torch.bfloat16)
    prompts = [pl.REFINE_SOURCE] + pl.REFINE_EDITS
    seeds = list(range(G))

    def batched():
        batch = controllers.GroupBatch([pl.make_refine_reweight_controller(prompts, steps, device=dev)
                                        for _ in seeds])
        return pl.run_edit_groups(model, [prompts] * G, batch, [pl.seed_latent(s) for s in seeds], steps)

    def sequential():
        return [pl.run_edit_group(model, prompts, pl.make_refine_reweight_controller(prompts, steps, device=dev),
                                  pl.seed_latent(s), steps) for s in seeds]

    for name, fn in (("batched", batched), ("sequential", sequential)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"config": "configs[2] Refine+Reweight, cross maps stored", "mode": name, "groups": G,
                          "ddim_steps": steps, "seconds": round(dt, 3), "edit_groups_per_s": round(G / dt, 4)}),
              flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
