"""GraphedEditRunner against the eager runner (pipeline.sweep_batch_runner): (1) bit-identity of
the final latents and reduced maps for two batches after the capture (deterministic MIOpen, as
tests/test_gpu_pipeline.py runs its bit-identity tests), (2) wall time per batch, eager and
graphed alternated.  Usage: python tools/graph_probe.py [groups_per_call] [rounds] [--identity]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from p2p_amd import pipeline as pl  # noqa: E402


def timed(fn, seeds):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn(seeds)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, out


def main(G=1, rounds=3):
    model = pl.SyntheticStableDiffusion(device="cuda", dtype=torch.bfloat16)
    prompts = pl.north_star_prompts()
    identity = "--identity" in sys.argv
    if not identity:
        eager = pl.sweep_batch_runner(model, prompts, 50, device=model.device)
        graphed = pl.sweep_batch_runner(model, prompts, 50, device=model.device, graphed=True)
        t, _ = timed(eager, [3 * 10 ** 6 + i for i in range(G)])
        print(f"first eager batch (library first-use searches): {t:.2f} s", flush=True)
        graphed([2 * 10 ** 6 + i for i in range(G)])
        print(f"graphed first batch: eager {graphed.first_seconds[0]:.2f} s, capture {graphed.first_seconds[1]:.2f} s",
              flush=True)
    else:
        # (deterministic MIOpen first: toggling the flag later in the same process made MIOpen's
        # immediate mode fall back to naive convolutions, ~60 s per batch)
        torch.backends.cudnn.deterministic = True
        eager = pl.sweep_batch_runner(model, prompts, 50, device=model.device)
        graphed = pl.sweep_batch_runner(model, prompts, 50, device=model.device, graphed=True)
        t, _ = timed(graphed, [10 ** 6 + i for i in range(G)])
        print(f"first batch: {t:.2f} s (eager on the capture stream {graphed.first_seconds[0]:.2f} s, capture of the "
              f"50 steps {graphed.first_seconds[1]:.2f} s)", flush=True)
        for b in range(2):
            seeds = [b * G + i for i in range(G)]
            _, (le, me) = timed(eager, seeds)
            _, (lg, mg) = timed(graphed, seeds)
            print(f"batch {b}: latents equal {torch.equal(le, lg)} (max |d| {(le - lg).abs().max().item():.3g}), "
                  f"maps equal {torch.equal(me, mg)} (max |d| {(me - mg).abs().max().item():.3g})", flush=True)
        return
    te, tg = [], []
    for r in range(rounds):
        seeds = [100 + r * G + i for i in range(G)]
        te.append(timed(eager, seeds)[0])
        tg.append(timed(graphed, seeds)[0])
        print(f"round {r}: eager {te[-1] * 1e3:.1f} ms, graphed {tg[-1] * 1e3:.1f} ms per batch of {G}", flush=True)
    me, mg = sorted(te)[len(te) // 2], sorted(tg)[len(tg) // 2]
    print(f"median: eager {me * 1e3:.1f} ms ({G / me:.3f} groups/s), graphed {mg * 1e3:.1f} ms ({G / mg:.3f} groups/s), "
          f"{(me / mg - 1) * 100:+.1f} %")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(int(args[0]) if args else 1, int(args[1]) if len(args) > 1 else 3)
