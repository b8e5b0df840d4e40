"""LocalBlend coverage probe (GPU, oracle only): the configs[1] oracle run (null_text LocalBlend,
main.py:35-52 / null_text.py:41-70) with the normalised pooled word map recorded at every blended
step, printed as the fraction of pixels above a range of thresholds -- which thresholds make the
mask partial (neither all-ones nor empty) on the random-init and on the sharpened U-Net.

    python -u tools/blend_probe.py [gain ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "prompt-to-prompt_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import control as oc  # noqa: E402
from oracle_runs import oracle_controller, oracle_group, sharpen_attention  # noqa: E402
from p2p_amd import pipeline as pl  # noqa: E402
from p2p_amd.tokenizer import StandInTokenizer  # noqa: E402

THS = (0.3, 0.5, 0.6, 0.7, 0.8, 0.9)


def main():
    gains = [float(g) for g in sys.argv[1:]] or [1.0, 4.0]
    dev = torch.device("cuda:0")
    tok = StandInTokenizer()
    prompts = pl.north_star_prompts()
    for gain in gains:
        model = pl.SyntheticStableDiffusion(device=dev, dtype=torch.bfloat16)
        sharpen_attention(model, gain)
        lb = oc.OracleLocalBlend("null", prompts, pl.BLEND_WORDS, tok)
        lb.alpha = lb.alpha.to(dev)
        fields = []
        orig = lb._mask

        def rec(maps, alpha, pool, th, size):
            m = (maps * alpha).sum(-1).mean(1)
            if pool:
                m = F.max_pool2d(m, (3, 3), (1, 1), padding=(1, 1))
                m = F.interpolate(m, size=size)
                fields.append((m / m.max(2, keepdim=True)[0].max(3, keepdim=True)[0]).float())
            return orig(maps, alpha, pool, th, size)

        lb._mask = rec
        ctrl = oracle_controller("replace", prompts, tok, 50, dev, local_blend=lb)
        oracle_group(model, prompts, pl.seed_latent(0), ctrl, 50)
        print(f"gain {gain}: {len(fields)} blended steps; coverage of the edit prompts' masks (m[:1] | m) by threshold")
        for i in (0, len(fields) // 2, len(fields) - 1):
            f = fields[i]
            m = [((f[:1] > th) | (f > th))[1:].float().mean().item() for th in THS]
            print(f"  step {i + 11}: " + "  ".join(f"th {th}: {c:.3f}" for th, c in zip(THS, m)) +
                  f"   field min {f.min().item():.3f}", flush=True)


if __name__ == "__main__":
    main()
