#!/usr/bin/env python
"""Edit-groups/sec of the Prompt-to-Prompt attention-control path on MI355X.

One "step" = one complete edit group of BASELINE.json configs[1]: SD-v1.4-shaped U-Net
(random init), 512x512 (64x64 latent), 1 source + 3 AttentionReplace edits with
null_text-form LocalBlend, CFG 7.5 (U-Net batch 8), 50 DDIM steps, cross_replace 0.8,
self_replace 0.4 -- every attention call is one fused HIP kernel (edits + store in it).
Text encoding is replaced by a synthetic context, no VAE decode.  By default each batch's 50
DDIM steps replay HIP graphs captured once (pipeline.GraphedEditRunner, during the warm-up);
the per-launch kernel timing (roofline, clock, attention totals) comes from an eager pass of the
same batches right after the timed region (--eager: time the eager loop itself).

Multi-GPU: one process per GPU (torchrun); edit groups (seeds) are partitioned across ranks
(weak scaling, no data-path collective); the final latents are all-gathered over RCCL once
at the end of the timed region.  Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import subprocess
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


HBM_PEAK_GBPS = 8000.0          # spec, MI355X_MICROARCH.md:36 (6.29 TB/s measured copy)


class FenceFreeEvent:
    """A HIP event created with hipEventDisableSystemFence, recorded on torch's current stream.
    torch.cuda.Event records with a system-scope release: an L2 writeback + invalidate at every
    record, which the next kernel pays as a cold cache -- hip_runtime_api.h documents the flag as
    the timing-only event that avoids "the cost of cache writeback and invalidation, and the
    performance impact of those actions on the execution of following work".  The timer reads
    the events only after torch.cuda.synchronize(), so the fence is not needed for correctness.
    Same record()/elapsed_time() surface as torch.cuda.Event; the events are created and recorded
    by the HIP runtime torch itself loaded (found in this process's mappings, whatever its soname)
    and destroyed with the object."""
    _hip = None

    @staticmethod
    def _runtime_path():
        """The libamdhip64 torch has mapped into this process (torch links it; no fixed soname)."""
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6 and os.path.basename(parts[5]).startswith("libamdhip64.so"):
                    return parts[5]
        raise RuntimeError("no HIP runtime (libamdhip64) mapped into this process")

    @classmethod
    def _lib(cls):
        if cls._hip is None:
            import ctypes
            L = ctypes.CDLL(cls._runtime_path())
            L.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            L.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            L.hipEventDestroy.argtypes = [ctypes.c_void_p]
            cls._hip = L
        return cls._hip

    def __init__(self, flags=0x20000000):   # hipEventDisableSystemFence
        import ctypes
        self._ctypes = ctypes
        self.ev = ctypes.c_void_p()
        rc = self._lib().hipEventCreateWithFlags(ctypes.byref(self.ev), flags)
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags failed: {rc}")

    def __del__(self):
        # may run at interpreter shutdown (after the HIP runtime is gone) or after a failed __init__
        ev, hip = getattr(self, "ev", None), FenceFreeEvent._hip
        if ev is None or not ev.value or hip is None:
            return
        try:
            hip.hipEventDestroy(ev)
        except Exception:
            pass
        self.ev = None

    def record(self):
        rc = self._lib().hipEventRecord(self.ev, ctypes_stream())
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed: {rc}")

    def elapsed_time(self, end) -> float:
        ms = self._ctypes.c_float()
        rc = self._lib().hipEventElapsedTime(self._ctypes.byref(ms), self.ev, end.ev)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime failed: {rc}")
        return ms.value


def ctypes_stream():
    import ctypes
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


NOMINAL_SCLK_MHZ = 2400.0       # the clock the dense peak assumes: 256 CU x 4 SIMD x 1024 FLOP/cycle x 2.4 GHz


class ClockProbe:
    """The shader clock the chip holds during the timed run (p2p_clock_probe, include/p2p_hip.h):
    8 one-wave workgroups (consecutive workgroups go to the 8 XCDs) each count shader cycles
    against the constant 100 MHz counter.  Two kinds of sample, each the median over the 8:
    * "during": every `every`-th dominant-kernel (G1/G7) launch, a probe of `ticks_during` (100 us,
      about half the kernel) on a second stream released together with the kernel, so it runs
      on 8 CUs while G1/G7 holds the other 248: the clock the chip holds under that kernel's load.
      Those launches lose 8 CUs (512 workgroups then need a third round: +30 %), so they leave
      every average (dominant kernel and all-attention totals) and are reported on their own;
    * "start" / "end": a 10 us probe on the launch stream at the start / end of the timed region
      (the chip at rest between launches)."""

    def __init__(self, device, max_samples=512, every=25, ticks=1000, ticks_during=10000):
        from p2p_amd import _hip
        self._hip = _hip
        self.buf = torch.zeros(max_samples, 8, 2, dtype=torch.int64, device=device)
        self.side = torch.cuda.Stream(device)
        self.tags, self.every, self.ticks, self.ticks_during, self.n_dominant = [], every, ticks, ticks_during, 0

    def sample(self, tag, ticks=None):
        if len(self.tags) < self.buf.shape[0]:
            self._hip.clock_probe(self.buf[len(self.tags)], ticks or self.ticks)
            self.tags.append(tag)
            return True
        return False

    def during_dominant(self) -> bool:
        """Called right before a dominant-kernel launch: True when this launch is probed."""
        self.n_dominant += 1
        if self.n_dominant % self.every or len(self.tags) >= self.buf.shape[0]:
            return False
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)           # released when the kernel before G1/G7 ends
        with torch.cuda.stream(self.side):
            self.sample("during", self.ticks_during)
        return True

    def summary(self):
        torch.cuda.synchronize()
        n = len(self.tags)
        if not n:
            return None
        b = self.buf[:n].double().cpu()
        mhz = (b[..., 0] / b[..., 1].clamp(min=1) * 100.0).median(dim=1).values.tolist()
        during = sorted(m for m, t in zip(mhz, self.tags) if t == "during")
        edge = {t: round(m, 1) for m, t in zip(mhz, self.tags) if t != "during"}
        return {"sclk_mhz": (during[len(during) // 2] if during else sorted(mhz)[n // 2]),
                "during_samples": len(during), "during_min_mhz": during[0] if during else None,
                "during_max_mhz": during[-1] if during else None, **{f"{k}_mhz": v for k, v in edge.items()}}


class LaunchTimer:
    """HIP events around the launches of interest, on the launch stream (torch's current stream,
    which the binding launches on):
    * "dominant": the G1/G7 self-attention (FLOP);
    * "attn": EVERY attention launch of the path (self and cross, all seven geometries), with its
      algorithmic FLOP 4 P K C N (K = 77 unpadded for cross), for the aggregate roofline
      the north star names ("45 % of bf16 peak in the attention kernels"), plus a per-geometry split;
    * the HBM-bound launches (the G2/G6 cross calls that keep their maps, --store-self's kept self
      maps, the LocalBlend mask and the latent step) with their algorithmic bytes.
    Every record also carries the index of the batch (edit group) it ran in, so per-batch
    averages show clock droop over a long run."""

    def __init__(self, n_query=4096, mode="ext"):
        self.n_query = n_query
        # "ext": the kernels' own dispatch timestamps (p2p_set_launch_events -> hipExtLaunchKernel; no
        # marker packets between the launches); "fence-free" / "torch": events recorded around the call
        self.mode = mode
        self.event = FenceFreeEvent if mode != "torch" else (lambda: torch.cuda.Event(enable_timing=True))
        self.rec = {}            # name -> list of (start event, end event, work, batch)
        self._pending = None     # (start event, [(name, work), ...])
        self.enabled = False
        self.batch = 0
        self.batch_marks = []    # one event at the end of each timed batch
        self.cross_group_kernel = {}   # geometry name -> True when the group cross kernel ran
        self.clock = None              # a ClockProbe sampled during the dominant kernel

    @staticmethod
    def _bytes(kind, t, info):
        """Algorithmic HBM bytes of one launch: q, k, v read once, o written once (bf16 or f32),
        and the kept maps: f32 [stored * H, P, K] written on the first step, read + written after."""
        es = 2 if t.io_dtype == 1 else 4
        C = t.n_heads * t.head_dim
        io = es * t.n_batch * C * (2 * t.n_query + 2 * t.n_key)
        maps = 4.0 * info["stored"] * t.n_heads * t.n_query * t.n_key * (2 if info["accumulate"] else 1)
        return io + maps

    def _names(self, kind, t, info):
        flop = 4.0 * t.n_query * t.n_key * t.n_heads * t.head_dim * t.n_batch
        geo = f"{kind}:P{t.n_query}:d{t.head_dim}"
        out = [("attn", flop), (f"attn:{geo}", flop), (f"bytes:{geo}", self._bytes(kind, t, info))]
        if kind == "self" and t.n_query == self.n_query and info["stored"] == 0:
            out.append(("dominant", flop))
        if t.n_query == 1024 and info["stored"] > 0 and info["accumulate"]:
            out.append((f"{kind}_store_p1024", self._bytes(kind, t, info)))
        return out

    def before(self, kind, t, info=None):
        if not self.enabled:
            return
        info = info or {"stored": 0, "accumulate": False}
        names = self._names(kind, t, info)
        if self.clock is not None and any(n == "dominant" for n, _ in names) and self.clock.during_dominant():
            # a probed launch runs on 248 CUs (a third round of workgroups): it leaves every average
            names = [("dominant_probed", w) for n, w in names if n == "dominant"]
        self._open(names)
        if kind == "cross" and "n_groups" in info:
            self.cross_group_kernel[f"attn:cross:P{t.n_query}:d{t.head_dim}"] = bool(info.get("group_kernel"))

    def _open(self, names):
        if self.mode == "ext":
            from p2p_amd import _hip
            start, stop = FenceFreeEvent(flags=0), FenceFreeEvent(flags=0)
            _hip.lib().p2p_set_launch_events(start.ev, stop.ev)
            self._pending = (start, names, stop)
        else:
            ev = self.event()
            ev.record()
            self._pending = (ev, names, None)

    def after(self, kind, t, info=None):
        if self._pending is not None:
            start, names, ev = self._pending
            if ev is not None:
                from p2p_amd import _hip
                _hip.lib().p2p_set_launch_events(None, None)
            else:
                ev = self.event()
                ev.record()
            for name, work in names:
                self.rec.setdefault(name, []).append((start, ev, work, self.batch))
            self._pending = None

    def before_aux(self, name, nbytes):
        """The LocalBlend mask and latent-step launches (HBM-type helpers), with their bytes."""
        if self.enabled:
            self._open([(name, float(nbytes))])

    def after_aux(self, name):
        self.after(name, None)

    def end_batch(self):
        if self.enabled:
            ev = self.event()
            ev.record()
            self.batch_marks.append(ev)
            self.batch += 1

    def summary(self, name="dominant", batch=None):
        """(average ms per launch, average work per launch, launches)"""
        torch.cuda.synchronize()
        pairs = [r for r in self.rec.get(name, []) if batch is None or r[3] == batch]
        pairs = [(r, self._ms(r)) for r in pairs]
        pairs = [(r, ms) for r, ms in pairs if ms is not None]
        if not pairs:
            return None, None, 0
        return (sum(ms for _, ms in pairs) / len(pairs), sum(r[2] for r, _ in pairs) / len(pairs), len(pairs))

    @staticmethod
    def _ms(r):
        """One record's launch time; None for a bracket whose call launched no kernel (ext events
        never bound)."""
        try:
            return r[0].elapsed_time(r[1])
        except RuntimeError:
            return None

    def attn_total(self, peak, unet_calls):
        """Aggregate roofline of ALL attention launches: summed algorithmic FLOP / summed HIP-event
        time, and the per-geometry split (average launch, its FLOP and fraction of peak)."""
        torch.cuda.synchronize()
        recs = [(r, self._ms(r)) for r in self.rec.get("attn", [])]
        recs = [(r, ms) for r, ms in recs if ms is not None]
        if not recs:
            return None
        tot_ms = sum(ms for _, ms in recs)
        tot_flop = sum(r[2] for r, _ in recs)
        achieved = tot_flop / (tot_ms * 1e-3) / 1e12
        by = []
        kind_ms, kind_flop, kind_bytes = {}, {}, {}
        for name in sorted(k for k in self.rec if k.startswith("attn:")):
            avg_ms, flop, n = self.summary(name)
            _, nbytes, _ = self.summary("bytes:" + name[5:])
            tf = flop / (avg_ms * 1e-3) / 1e12
            gbps = nbytes / (avg_ms * 1e-3) / 1e9
            d = {"geometry": name[5:], "launches": n, "avg_launch_ms": avg_ms, "flop_per_launch": flop,
                 "achieved_tflops": tf, "frac": tf / peak, "share_of_attn_time": avg_ms * n / tot_ms,
                 "algorithmic_bytes_per_launch": nbytes, "achieved_gbps": gbps, "hbm_frac": gbps / HBM_PEAK_GBPS}
            if name in self.cross_group_kernel:
                d["kernel"] = "cross_group_kernel" if self.cross_group_kernel[name] else "cross_attn_kernel"
            by.append(d)
            kind = name.split(":")[1]
            kind_ms[kind] = kind_ms.get(kind, 0.0) + avg_ms * n
            kind_flop[kind] = kind_flop.get(kind, 0.0) + flop * n
            kind_bytes[kind] = kind_bytes.get(kind, 0.0) + nbytes * n
        # the self kernels are MFMA work (judged by their MFMA fraction), the cross kernels (K = 77:
        # 3.6 % of the FLOP) are q / o / map traffic (judged by their HBM fraction)
        self_ms = kind_ms.get("self")
        by_kind = {
            "self": None if not self_ms else {
                "bound": "mfma", "achieved": kind_flop["self"] / (self_ms * 1e-3) / 1e12, "peak": peak,
                "unit": "TFLOP/s", "frac": kind_flop["self"] / (self_ms * 1e-3) / 1e12 / peak,
                "ms_per_unet_call": self_ms / unet_calls if unet_calls else None},
            "cross": None if not kind_ms.get("cross") else {
                "bound": "hbm", "achieved": kind_bytes["cross"] / (kind_ms["cross"] * 1e-3) / 1e9,
                "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": kind_bytes["cross"] / (kind_ms["cross"] * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                "ms_per_unet_call": kind_ms["cross"] / unet_calls if unet_calls else None,
                "bytes_model": "algorithmic lower bound: q + k + v read once, o written once, kept maps read + "
                               "written; the edits' re-reads of the source rows and their mapper tiles are "
                               "not counted (PMC FETCH_SIZE / WRITE_SIZE per launch: profiles/r05/pmc/table.md)"},
        }
        return {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                "by_kind": by_kind,
                "launches": len(recs), "attn_ms_total": tot_ms,
                "attn_ms_per_unet_call": tot_ms / unet_calls if unet_calls else None,
                "flop_per_unet_call": tot_flop / unet_calls if unet_calls else None,
                "rule": "sum over every self/cross attention launch of the timed run of 4 P K C N FLOP "
                        "(K = 77 unpadded for cross; SURVEY §8d) / sum of their HIP-event launch times",
                "by_geometry": by}

    def per_batch(self):
        """Per-batch GPU ms (event to event) and the dominant kernel's average launch per batch."""
        torch.cuda.synchronize()
        out = []
        for i in range(1, len(self.batch_marks)):
            dom, _, _ = self.summary("dominant", batch=i)
            out.append((i, self.batch_marks[i - 1].elapsed_time(self.batch_marks[i]), dom))
        return out

    def hbm_lines(self):
        out = []
        labels = {"cross_store_p1024": "cross-attention G2/G6 (P=1024, d=80, K=77) with the kept cross maps "
                                       "(read-add-write)",
                  "self_store_p1024": "self-attention G2/G6 (P=K=1024, d=80) with the kept self maps: fused "
                                      "pass (lse) + self_maps_kernel read-add-write",
                  "localblend": "LocalBlend mask (blend_finalize_kernel: folded word sums -> pooled, thresholded "
                                "64x64 mask)",
                  "latent_step": "latent_step_kernel (CFG + DDIM + LocalBlend blend with a precomputed mask)",
                  "latent_blend": "latent_blend_kernel: LocalBlend in one launch with the latent update (folded word "
                                  "sums -> mean, 3x3 max-pool, upsample, normalise, threshold -> blend) + CFG + DDIM"}
        rules = {"localblend": "word sums read (B x 2 x L*H x 16^2 f32) + mask written (B x 64^2 u8)",
                 "latent_step": "eps read (2B x 4 x 64^2, bf16) + latents read and written (f32) + mask read",
                 "latent_blend": "eps read (2B x 4 x 64^2, bf16) + latents read and written (f32) + folded word sums "
                                 "read once (B x 2 x L*H x 16^2 f32)"}
        for name in ("cross_store_p1024", "self_store_p1024", "localblend", "latent_step", "latent_blend"):
            avg_ms, nbytes, n = self.summary(name)
            if not n:
                continue
            gbps = nbytes / (avg_ms * 1e-3) / 1e9
            label = labels[name]
            if name == "cross_store_p1024":
                label = (("cross_group_kernel" if self.cross_group_kernel.get("attn:cross:P1024:d80") else
                          "cross_attn_kernel") + " " + label)
            out.append({"kernel": label, "avg_launch_ms": avg_ms, "launches": n,
                        "algorithmic_bytes": nbytes, "achieved": gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": gbps / HBM_PEAK_GBPS,
                        "bytes_rule": rules.get(name, "q + o + k + v (io dtype) + kept maps f32 x2 (read + write, "
                                                      "steps >= 1)")})
        return out


def _clock_fields(clk, frac):
    """roofline.sclk_mhz (the measured shader clock) and frac_at_measured_clock (the same achieved
    rate against the peak scaled to that clock): what separates box-to-box clock spread from a
    kernel change."""
    if not clk:
        return {"sclk_mhz": None, "frac_at_measured_clock": None}
    return {"sclk_mhz": clk["sclk_mhz"], "nominal_sclk_mhz": NOMINAL_SCLK_MHZ,
            "frac_at_measured_clock": frac * NOMINAL_SCLK_MHZ / clk["sclk_mhz"] if frac else None,
            "clock_probe": {**clk, "rule": "p2p_clock_probe: 8 one-wave workgroups count shader cycles against the "
                                           "100 MHz counter; 'during' = a 100 us probe on a second stream running "
                                           "beside every 25th G1/G7 launch (those launches leave the average); "
                                           "start / end = 10 us probes at the edges of the timed region; sclk = "
                                           "median of the 'during' samples"}}


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


def cpu_baseline(num_ddim_steps: int, sample_steps: int = 2):
    """The oracle's fp32 CPU restatement of the same workload on the host cores -- the reference
    itself is not importable here (no diffusers), so this is the port: ``sample_steps``
    consecutive denoising steps (U-Net at batch 8 with the eager patched attention + reference
    controller + LocalBlend + DDIM) timed and extrapolated x(num_ddim_steps / sample_steps)
    to the 50-step group (2 steps x 25)."""
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
    with torch.no_grad():
        t0 = time.perf_counter()
        for t in model.scheduler.timesteps[:sample_steps]:
            eps = model.unet(torch.cat([lat] * 2), t, encoder_hidden_states=ctx)["sample"]
            eu, ec = eps.chunk(2)
            lat = model.scheduler.step(eu + 7.5 * (ec - eu), t, lat)["prev_sample"]
            lat = ctrl.step_callback(lat)
        dt = time.perf_counter() - t0
    per_group = dt / sample_steps * num_ddim_steps
    return {"value": 1.0 / per_group, "unit": "edit-groups/s", "cores": cores, "kind": "port",
            "sample": f"{sample_steps} of {num_ddim_steps} DDIM steps timed = {dt:.2f} s, "
                      f"x{num_ddim_steps / sample_steps:g} extrapolated; oracle port (fp32 torch on the host: "
                      f"U-Net N=8 + eager attention + reference controller/store + LocalBlend + DDIM) -- the "
                      f"reference itself is not importable here (no diffusers)"}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="batches of --groups-per-call edit groups timed per rank")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--ddim-steps", type=int, default=50)
    ap.add_argument("--unet-dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--compute", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--launch-events", default="ext", choices=["ext", "fence-free", "torch"],
                    help="per-launch timing: the kernels' own dispatch timestamps through hipExtLaunchKernel\n"
                         "events (default; p2p_set_launch_events), HIP events recorded around each call without\n"
                         "the system-scope fence, or torch.cuda.Event (an L2 writeback + invalidate per record)")
    ap.add_argument("--groups-per-call", type=int, default=1,
                    help="edit groups denoised per U-Net call (controllers.GroupBatch; a step = one such\n"
                         "batch); 1 = configs[1] as quoted")
    ap.add_argument("--seeds", type=int, default=0,
                    help="configs[3] sweep: time ALL of seeds 0..S-1, partitioned over the ranks and run\n"
                         "--groups-per-call at a time (--steps is then ignored); value = S / wall")
    ap.add_argument("--eager", action="store_true",
                    help="time the eager denoising loop for value (default: the DDIM steps replay HIP graphs\n"
                         "captured after the first batch, pipeline.GraphedEditRunner; the per-launch kernel\n"
                         "timing then comes from an eager pass of --instrumented batches right after)")
    ap.add_argument("--instrumented", type=int, default=3,
                    help="batches of the eager per-launch timing pass that follows a graphed timed region")
    ap.add_argument("--store-self", action="store_true",
                    help="also keep the 32x32/16x16/8x8 SELF maps (main.py AttentionStore default); the\n"
                         "north-star workload keeps only the maps AttentionStore/LocalBlend read")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: start torchrun as a CHILD before anything touches the GPU (never
        # exec from a process that may have), wait, and exit with its status
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(cmd, env=env))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} launched with WORLD_SIZE={world}")
    # every rank torchrun starts joins an RCCL process group -- world 1 included, so a one-GPU box
    # runs the same init / barrier / all-gather / all-reduce path the 8-GPU node does
    distributed = "WORLD_SIZE" in os.environ
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from p2p_amd import _hip, config, sweep
    from p2p_amd import pipeline as pl
    config.set_compute(args.compute)
    _hip.lib()
    _hip.check_source_hash()

    dtype = torch.bfloat16 if args.unet_dtype == "bf16" else torch.float32
    model = pl.SyntheticStableDiffusion(device=dev, dtype=dtype)
    prompts = pl.north_star_prompts()
    B = len(prompts)
    timer = LaunchTimer(mode=args.launch_events)
    _hip.LAUNCH_OBSERVER = timer

    G = args.groups_per_call

    # one step = one batch of G groups: the runner the configs[3] GPU test drives through the same sweep
    graphed = not args.eager
    batch = pl.sweep_batch_runner(model, prompts, args.ddim_steps, store_self_maps=args.store_self, device=dev,
                                  graphed=graphed)
    # the same batches without graphs (the per-launch timing pass of a graphed run)
    eager_batch = batch.eager_run if graphed else batch

    # groups (seeds) partitioned across ranks round-robin: no collective on the data path.  A
    # graphed run always warms up once: its first batch is the eager run + the capture
    n_warm = max(args.warmup, 1 if graphed else 0)
    if args.seeds > 0:
        all_seeds = list(range(args.seeds))
        warm_seeds = [10 ** 6 + i for i in range(n_warm * G)]
    else:
        all_seeds = list(range(world * args.steps * G))
        warm_seeds = [10 ** 6 + rank * n_warm * G + i for i in range(n_warm * G)]
    for i in range(n_warm):
        batch(warm_seeds[i * G:(i + 1) * G])
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    clock = ClockProbe(dev)
    timer.clock = clock

    def max_over_ranks(x):
        if distributed:
            tt = torch.tensor([x], device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            return tt.item()
        return x

    timer.enabled = not graphed   # graph replays make no per-launch calls: the eager pass below times them
    t0 = time.perf_counter()
    clock.sample("start")
    timer.end_batch()     # (batch 0's start mark)

    def progress(i, n):   # a progress line per batch (stderr; host-side only) + the batch's end event
        timer.end_batch()
        if n > 4:
            print(f"[bench rank {rank}] batch {i + 1}/{n} host {1e3 * (time.perf_counter() - t0):.0f} ms",
                  file=sys.stderr, flush=True)

    # the sweep tests/test_distributed.py runs over gloo: this rank's batches, then ONE RCCL
    # all-gather of the final latents and the reduced maps (the only inter-GPU traffic)
    lat_all, maps_all = sweep.run_batched_sweep(all_seeds, batch, batch.out_shapes, rank, world, G,
                                                device=dev, on_batch=progress)
    clock.sample("end")
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    timer.enabled = False
    n_total = len(all_seeds)

    eager_line = None
    mine = sweep.batches(all_seeds, rank, world, G)
    inst = mine[:args.instrumented] if graphed else mine
    if graphed:
        # the per-launch timing pass: the same batches (this rank's first --instrumented), eager,
        # every hot-path launch bracketed by the kernels' own HIP events, the clock probed under
        # G1/G7; its wall time is reported beside value as eager_value
        timer.enabled = True
        t1 = time.perf_counter()
        clock.sample("start")
        timer.end_batch()
        for i, b in enumerate(inst):
            eager_batch(b)
            timer.end_batch()
        clock.sample("end")
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier()
        elapsed_inst = max_over_ranks(time.perf_counter() - t1)
        timer.enabled = False
        n_inst = sum(len(b) for b in inst)
        if distributed:
            tn = torch.tensor([float(n_inst)], device=dev)
            dist.all_reduce(tn)
            n_inst = int(tn.item())
        eager_line = {"value": n_inst / elapsed_inst, "groups": n_inst, "seconds": elapsed_inst,
                      "loop": "eager, every hot-path launch bracketed by its kernels' HIP events and the "
                              "clock probed beside every 25th G1/G7 launch"}
    assert lat_all.shape == (n_total, B, 4, 64, 64) and maps_all.shape == (n_total, B, 16, 16, 77)
    assert torch.isfinite(lat_all).all() and torch.isfinite(maps_all).all()
    # each source prompt's gathered map row is an average of probability rows: it sums to 1
    assert (maps_all[:, 0].sum(-1) - 1).abs().max().item() < 1e-2

    avg_ms, flops, n_launch = timer.summary()
    peak = MFMA_PEAK_BF16_TFLOPS if args.compute == "bf16" else MFMA_PEAK_F32_TFLOPS
    # per-batch GPU time and the dominant kernel's average launch in that batch (stderr): clock
    # droop over a long run shows up here, not in the one-line average
    for i, ms_b, dom in timer.per_batch():
        print(f"[bench rank {rank}] batch {i} gpu {ms_b:.1f} ms  dominant avg "
              f"{dom * 1e3 if dom else float('nan'):.1f} us", file=sys.stderr, flush=True)
    unet_calls = len(inst) * args.ddim_steps   # this rank's U-Net calls in the per-launch timing pass
    attn_total = timer.attn_total(peak, unet_calls)
    if rank == 0:
        achieved = flops / (avg_ms * 1e-3) / 1e12 if avg_ms else None
        traffic, traffic_src = pmc_traffic() if G == 1 else (None, "no PMC pass at N = 8G")
        roofline = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                    "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                    "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                    "algorithmic_bytes": 4.0 * 8 * G * 4096 * 320 * 2,
                    "kernel": f"self40_kernel G1/G7, F16 form (P=K=4096, d=40, N={8 * G}, H=8; 8 waves x 2 x 32 queries, "
                              f"256-key tiles, software-pipelined 32x32 blocks)",
                    "avg_launch_ms": avg_ms, "launches": n_launch,
                    "probed_launches": {"avg_launch_ms": timer.summary("dominant_probed")[0],
                                        "launches": timer.summary("dominant_probed")[2]},
                    "flop_per_launch": flops,
                    **_clock_fields(clock.summary(), (achieved / peak) if achieved else None),
                    "timing": {"ext": "HIP events bound to each launch's kernels (hipExtLaunchKernel start / stop "
                                      "events: the kernels' own dispatch timestamps, as rocprofv3's kernel trace), "
                                      "on the launch stream",
                               "fence-free": "HIP events recorded around each launch on its stream, created with "
                                             "hipEventDisableSystemFence",
                               "torch": "torch.cuda.Event around each launch"}[args.launch_events]}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.ddim_steps)
        n_steps = max(1, len(sweep.batches(all_seeds, 0, world, G)))
        workload = ("configs[3]: seed sweep of " + str(n_total) + " edit groups, " if args.seeds > 0 else
                    "configs[1]: ")
        line = {
            "metric": "edit-groups/sec (src+3 edits, SD1.4 512², 50 DDIM)",
            "value": n_total / elapsed, "unit": "edit-groups/s", "n_gpus": world, "steps": n_steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1000.0 / n_steps, "higher_is_better": True,
            "scaling": "weak" if args.seeds == 0 else "strong", "vs_baseline": None, "dtype": args.compute,
            "data": "synthetic (random-init SD-v1.4-shaped U-Net, seeded x_T, stand-in text context)",
            "config": {"workload": workload + "SD-v1.4 512x512 AttentionReplace + LocalBlend, 1 source + 3 edits, "
                                   f"{args.ddim_steps} DDIM, CFG 7.5", "global_batch": 8 * G * world,
                       "groups_per_call": G, "groups_total": n_total, "unet_dtype": args.unet_dtype,
                       "self_maps_kept": args.store_self, "gathered": "final latents + 16x16 cross maps (1 all-gather)",
                       "parallelism": f"replicas x{world} (groups by seed)"},
            "loop": ("HIP graphs: the 50 DDIM steps of each batch replay graphs captured once per batch size "
                     "(pipeline.GraphedEditRunner; bit-identical to the eager loop, tests/test_gpu_pipeline.py)"
                     if graphed else "eager"),
            # graphed runs: the eager loop's throughput over the per-launch timing pass that follows
            # (the same batches' first --instrumented of this rank; every roofline field comes from it)
            "eager_value": eager_line,
            "roofline": roofline, "cpu_baseline": cpu,
            # every attention launch of the timed run together (north star: ">= 45 % of bf16 MFMA peak
            # in the attention kernels"), HIP-event timed, with the per-geometry split
            "roofline_attn_total": attn_total,
            # the HBM-bound launches of the path (north star: "achieved HBM GB/s for the map and blend
            # kernels"), HIP-event timed in the same run; algorithmic bytes, not PMC
            "roofline_hbm": timer.hbm_lines(),
        }
        print(json.dumps(line))
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
