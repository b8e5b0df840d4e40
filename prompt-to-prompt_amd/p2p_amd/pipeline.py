"""Synthetic SD-v1.4 pipeline: the callers around the hot path (sampling loop inputs).

No checkpoints, tokenizer vocabularies or text encoders are available offline, so the
"model" object that ptp_utils.text2image_ldm_stable expects (``tokenizer``,
``text_encoder``, ``unet``, ``scheduler``, ``device``; main.py:29) is assembled from
stand-ins: the deterministic tokenizer, a seeded embedding-table text encoder that maps
identical prompts to identical contexts (as CLIP does for the shared "" uncond rows), the
random-init SD-shaped U-Net and the DDIM scheduler of null_text.py:16-20.
"""
from __future__ import annotations

import time
from typing import List, Optional, Sequence

import torch
import torch.nn as nn

from .ddim import DDIMScheduler
from .tokenizer import default_tokenizer
from .unet import UNet2DConditionModel

VOCAB = 49408


class SyntheticTextEncoder(nn.Module):
    def __init__(self, dim=768, max_len=77, seed=1):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.register_buffer("token", torch.randn(VOCAB, dim, generator=g))
        self.register_buffer("pos", 0.1 * torch.randn(max_len, dim, generator=g))

    def forward(self, ids):
        return (self.token[ids] + self.pos[None, : ids.shape[1]],)


class SyntheticStableDiffusion:
    def __init__(self, device="cuda", dtype=torch.float32, seed=0):
        self.device = torch.device(device)
        self.tokenizer = default_tokenizer()
        torch.manual_seed(seed)
        self.unet = UNet2DConditionModel().to(self.device, dtype).eval()
        for p in self.unet.parameters():
            p.requires_grad_(False)
        self.text_encoder = SyntheticTextEncoder().to(self.device)
        self.scheduler = DDIMScheduler(beta_start=0.00085, beta_end=0.012, beta_schedule="scaled_linear",
                                       clip_sample=False, set_alpha_to_one=False)
        self.vae = None


class SyntheticLatentDiffusion:
    """LDM-256 (BASELINE.json configs[0]): the "model" ptp_utils.text2image_ldm expects
    (``tokenizer``, ``bert``, ``unet``, ``scheduler``, ``vqvae``, ``device``;
    ptp_utils.py:98-126).  The ldm-text2im-large-256 U-Net is the SD topology with a 1280-d
    LDMBert context and a 32x32 latent (diffusers config -- external knowledge, not in the
    container), so every attention layer has P <= 1024 and main.py:131 stores all of them.
    Random-init weights, seeded embedding-table "LDMBert", DDIM scheduler; no VQ-VAE."""

    def __init__(self, device="cuda", dtype=torch.float32, seed=0):
        self.device = torch.device(device)
        self.tokenizer = default_tokenizer()
        torch.manual_seed(seed)
        self.unet = UNet2DConditionModel(cross_attention_dim=1280).to(self.device, dtype).eval()
        for p in self.unet.parameters():
            p.requires_grad_(False)
        self.bert = SyntheticTextEncoder(dim=1280, seed=2).to(self.device)
        self.scheduler = DDIMScheduler(beta_start=0.00085, beta_end=0.012, beta_schedule="scaled_linear",
                                       clip_sample=False, set_alpha_to_one=False)
        self.vqvae = None


LDM_PROMPTS = ["A painting of a squirrel eating a burger", "A painting of a squirrel eating a lasagna"]


def ldm_seed_latent(seed: int) -> torch.Tensor:
    """x_T for the 256x256 LDM (init_latent, ptp_utils.py:88-95: [1, 4, 32, 32])."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn((1, 4, 32, 32), generator=g)


# The north-star workload (BASELINE.json configs[1]): 1 source + 3 single-word replacements.
SOURCE = "a painting of a squirrel eating a burger"
EDITS = ["a painting of a lion eating a burger", "a painting of a cat eating a burger",
         "a painting of a squirrel eating a lasagna"]
BLEND_WORDS = (("squirrel", "burger"), ("lion",), ("cat",), ("lasagna",))


def north_star_prompts() -> List[str]:
    return [SOURCE] + EDITS


def seed_latent(seed: int) -> torch.Tensor:
    """x_T exactly as main.py:427-428 draws it (CPU generator)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn((1, 4, 64, 64), generator=g)


def make_replace_controller(prompts: Sequence[str], num_steps: int = 50, cross_replace_steps=0.8,
                            self_replace_steps=0.4, blend_words=BLEND_WORDS, store_self_maps=False,
                            device=None, blend_th=(.3, .3)):
    from . import null_text
    lb = (null_text.LocalBlend(list(prompts), blend_words, th=blend_th, device=device)
          if blend_words is not None else None)
    ctrl = null_text.AttentionReplace(list(prompts), num_steps, cross_replace_steps=cross_replace_steps,
                                      self_replace_steps=self_replace_steps, local_blend=lb, device=device)
    ctrl.store_self_maps = store_self_maps
    return ctrl


@torch.no_grad()
def run_edit_group(model: SyntheticStableDiffusion, prompts: Sequence[str], controller, x_T: torch.Tensor,
                   num_steps: int = 50, guidance_scale: float = 7.5):
    from . import ptp_utils
    latents, _ = ptp_utils.text2image_ldm_stable(model, list(prompts), controller, num_inference_steps=num_steps,
                                                 guidance_scale=guidance_scale, latent=x_T)
    return latents


@torch.no_grad()
def run_edit_groups(model: SyntheticStableDiffusion, prompt_groups: Sequence[Sequence[str]], controller,
                    x_Ts: Sequence[torch.Tensor], num_steps: int = 50, guidance_scale: float = 7.5):
    """G prompt groups (each 1 source + edits, its own seed) denoised in ONE U-Net batch
    (BASELINE.json configs[2]) with a controllers.GroupBatch: ptp_utils.text2image_ldm_stable's
    loop (ptp_utils.py:129-172) over the concatenated prompts, the groups' x_T expanded per group
    (init_latent, ptp_utils.py:88-95).  Returns the final latents [G * B, 4, 64, 64]."""
    from . import ptp_utils
    prompts = [p for grp in prompt_groups for p in grp]
    B = len(prompt_groups[0])
    if any(len(grp) != B for grp in prompt_groups):
        raise ValueError("every prompt group needs the same number of prompts")
    ptp_utils.register_attention_control(model, controller)
    text = ptp_utils._encode(model, prompts, model.text_encoder)
    uncond = ptp_utils._encode(model, [""] * len(prompts), model.text_encoder)
    context = ptp_utils.unet_context(model, torch.cat([uncond, text]))
    latents = torch.cat([x.reshape(1, 4, 64, 64).expand(B, 4, 64, 64) for x in x_Ts]).to(model.device)
    model.scheduler.set_timesteps(num_steps)
    for t in model.scheduler.timesteps:
        latents = ptp_utils.diffusion_step(model, controller, latents, context, t, guidance_scale)
    return latents


def sweep_batch_runner(model: SyntheticStableDiffusion, prompts: Sequence[str], num_steps: int = 50,
                       store_self_maps: bool = False, device=None, graphed: bool = False):
    """The unit of work bench.py times and the configs[3] sweep runs (sweep.run_batched_sweep):
    run(seeds) denoises len(seeds) edit groups -- each 1 source + 3 AttentionReplace edits with
    LocalBlend and its own seed -- one U-Net call per DDIM step (controllers.GroupBatch when
    len(seeds) > 1), and returns the final latents [g, B, 4, 64, 64] and each group's reduced
    stored maps [g, B, 16, 16, 77] (aggregate_attention's 16x16 cross average per prompt,
    main.py:293-307).  ``graphed``: the DDIM steps replay HIP graphs captured after the first
    batch of each size (GraphedEditRunner) -- the same launches, without the per-kernel gaps."""
    def make_ctrl():
        return make_replace_controller(prompts, num_steps, device=device, store_self_maps=store_self_maps)
    return edit_batch_runner(model, prompts, make_ctrl, num_steps, graphed=graphed)


def edit_batch_runner(model: SyntheticStableDiffusion, prompts: Sequence[str], make_ctrl, num_steps: int = 50,
                      graphed: bool = False, map_res: int = 16):
    """run(seeds) for any edit controller: ``make_ctrl()`` builds one group's controller (an
    AttentionStore subclass: its maps are reduced at ``map_res``); len(seeds) groups of ``prompts``
    share each U-Net call (controllers.GroupBatch when more than one).  Returns the final latents
    [g, B, 4, 64, 64] and the reduced cross maps [g, B, map_res, map_res, 77].  ``graphed``: a
    GraphedEditRunner around the same run."""
    from . import controllers
    B = len(prompts)

    def run(seeds):
        if len(seeds) == 1:
            ctrl = make_ctrl()
            lat = run_edit_group(model, prompts, ctrl, seed_latent(seeds[0]), num_steps=num_steps)
            return lat[None], controllers.reduce_maps(ctrl, map_res, ["up", "down"], True, B)[None]
        members = [make_ctrl() for _ in seeds]
        lat = run_edit_groups(model, [prompts] * len(seeds), controllers.GroupBatch(members),
                              [seed_latent(s) for s in seeds], num_steps=num_steps)
        maps = torch.stack([controllers.reduce_maps(m, map_res, ["up", "down"], True, B) for m in members])
        return lat.reshape(len(seeds), B, *lat.shape[1:]), maps

    run.out_shapes = [(B, 4, 64, 64), (B, map_res, map_res, 77)]
    if not graphed:
        return run
    return GraphedEditRunner(model, prompts, num_steps, make_ctrl, run, map_res=map_res)


class GraphedEditRunner:
    """edit_batch_runner's run(seeds) with every DDIM step replayed from a HIP graph.

    The first batch of each size runs eagerly on the runner's capture stream (it returns real
    results, and it makes every first-use library search -- MIOpen's convolution find, hipBLASLt's
    heuristics -- and every host table of the controllers happen outside a capture).  Then fresh
    controllers for that batch size are built and the 50 steps of ptp_utils.diffusion_step are
    captured, one graph per step, into one memory pool: each step's host plan (the controller's
    counters, cross_replace_alpha row, R_ONLY hint, self-injection window, store add / overwrite,
    LocalBlend start) is decided while capturing, exactly as the eager loop decides it at that step,
    and baked into that step's launches.  A later batch refills the static inputs -- x_T and the
    re-encoded text context -- and replays the 50 graphs in order; the captured controllers' running
    sums then hold that batch's maps (they are overwritten at step 0 as in an eager run), and their
    host state (cur_step = 50) is the state an eager run ends in, so reduce_maps reads them as usual.

    The graphs read the model's weights (and the stacked projection weights built from them) where
    they were at capture: after changing any weight, call release() -- the next batch of each size
    then runs eagerly and captures again.

    Not captured: the text encoder (runs eagerly per batch, its output copied into the static
    context).  The cross K / V projections are captured in step 0's graph and read by the later
    steps' (ptp_utils._cross_kv's capture rules), so every replayed batch projects its own context
    once, as an eager group does."""

    def __init__(self, model, prompts, num_steps, make_ctrl, eager_run, guidance_scale=7.5, map_res=16):
        self.map_res = map_res
        self.model, self.prompts, self.num_steps = model, list(prompts), num_steps
        self.make_ctrl, self.eager_run, self.guidance_scale = make_ctrl, eager_run, guidance_scale
        self.out_shapes = eager_run.out_shapes
        self.B = len(prompts)
        self.stream = None
        self.plans = {}

    def release(self):
        """Drop every captured plan (graphs, memory pool, controllers)."""
        self.plans = {}

    def __call__(self, seeds):
        seeds = list(seeds)
        plan = self.plans.get(len(seeds))
        if plan is None:
            return self._first(seeds)
        return self._replay(plan, seeds)

    # ------------------------------------------------------------------ first batch of a size
    def _first(self, seeds):
        dev = self.model.device
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=dev)
        cur = torch.cuda.current_stream(dev)
        self.stream.wait_stream(cur)
        t0 = time.perf_counter()
        with torch.cuda.stream(self.stream):
            out = tuple(r.clone() for r in self.eager_run(seeds))
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            self.plans[len(seeds)] = self._capture(len(seeds))
        torch.cuda.synchronize(dev)
        for r in out:            # made on the capture stream, read on the caller's
            r.record_stream(cur)
        self.first_seconds = (t1 - t0, time.perf_counter() - t1)   # (eager batch, capture)
        return out

    def _context(self, G):
        from . import ptp_utils
        prompts = self.prompts * G
        text = ptp_utils._encode(self.model, prompts, self.model.text_encoder)
        uncond = ptp_utils._encode(self.model, [""] * len(prompts), self.model.text_encoder)
        return ptp_utils.unet_context(self.model, torch.cat([uncond, text]))

    @torch.no_grad()
    def _capture(self, G):
        from . import controllers
        from . import ptp_utils as pu
        model, dev, B = self.model, self.model.device, self.B
        members = [self.make_ctrl() for _ in range(G)]
        ctrl = members[0] if G == 1 else controllers.GroupBatch(members)
        for m in members:
            _prime_for_capture(m, dev)
        pu.register_attention_control(model, ctrl)
        ctx = self._context(G).clone()
        x = torch.zeros(G * B, 4, 64, 64, device=dev)
        model.scheduler.set_timesteps(self.num_steps)
        ts = list(model.scheduler.timesteps)
        t_dev = [torch.full((1,), int(t), dtype=torch.int64, device=dev) for t in ts]
        pool = torch.cuda.graph_pool_handle()
        graphs = []
        lat = x
        torch.cuda.synchronize(dev)
        for t, td in zip(ts, t_dev):
            g = torch.cuda.CUDAGraph()
            # thread-local capture: another thread's HIP calls (an RCCL proxy thread of a
            # multi-GPU run) do not invalidate this thread's capture
            with torch.cuda.graph(g, pool=pool, stream=self.stream, capture_error_mode="thread_local"):
                lat = pu.diffusion_step(model, ctrl, lat, ctx, t, self.guidance_scale, t_unet=td)
            graphs.append(g)
        # the captured K / V cache entries: their tensors are written by step 0's graph and read by
        # the others, so they live as long as the graphs (an eager call replaces the module's entry)
        kv = [mod.__dict__["_p2p_kv"] for mod in model.unet.modules()
              if "_p2p_kv" in mod.__dict__ and mod.__dict__["_p2p_kv"][5] and mod.__dict__["_p2p_kv"][0]() is ctx]
        return {"graphs": graphs, "x": x, "ctx": ctx, "out": lat, "ctrl": ctrl, "members": members,
                "t_dev": t_dev, "pool": pool, "kv": kv}

    # ------------------------------------------------------------------ later batches
    @torch.no_grad()
    def _replay(self, plan, seeds):
        from . import controllers
        G, B = len(seeds), self.B
        x_T = torch.cat([seed_latent(s).expand(B, 4, 64, 64) for s in seeds])
        plan["x"].copy_(x_T)
        plan["ctx"].copy_(self._context(G))
        for g in plan["graphs"]:
            g.replay()
        lat = plan["out"].clone().reshape(G, B, 4, 64, 64)
        maps = torch.stack([controllers.reduce_maps(m, self.map_res, ["up", "down"], True, B)
                            for m in plan["members"]])
        return lat, maps


def _prime_for_capture(ctrl, device):
    """Make an edit controller's first call free of host <-> device copies (which a capture cannot
    hold): its device edit program and the host copy of cross_replace_alpha are built now."""
    from . import controllers
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:   # the key the kernels' tensors give (cuda:N)
        device = torch.device("cuda", torch.cuda.current_device())
    if isinstance(ctrl, controllers.AttentionControlEdit):
        try:
            ctrl._device_program(device)
        except controllers.NotFusable:
            return
        ctrl._cross_step(device, ctrl.cross_replace_alpha.shape[-1])


# BASELINE.json configs[2]: AttentionRefine + AttentionReweight (equalizer) groups whose 16/32-res
# cross maps are all stored.  Each group refines the source prompt by inserted words and
# reweights one word of it.
REFINE_SOURCE = "a photo of a house on a mountain"
REFINE_EDITS = ["a photo of a house on a snowy mountain", "a photo of a wooden house on a mountain",
                "a photo of a house on a mountain at night"]


def make_refine_reweight_controller(prompts: Sequence[str], num_steps: int = 50, word="mountain", value=2.0,
                                    device=None, tokenizer=None):
    """AttentionReweight(equalizer) chained on AttentionRefine (main.py:233-278), maps of the
    16/32-res cross layers kept by the store (self maps off)."""
    from . import controllers as c
    tok = tokenizer or c.get_tokenizer()
    refine = c.AttentionRefine(list(prompts), num_steps, cross_replace_steps=0.8, self_replace_steps=0.4,
                               tokenizer=tok, device=device)
    eq = c.get_equalizer(prompts[0], (word,), (value,), tokenizer=tok)
    ctrl = c.AttentionReweight(list(prompts), num_steps, cross_replace_steps=0.8, self_replace_steps=0.4,
                               equalizer=eq, controller=refine, tokenizer=tok, device=device)
    ctrl.store_self_maps = False
    return ctrl
