"""ctypes binding of ``libp2p_hip.so`` (C ABI: ``include/p2p_hip.h``).

This module is the only place the product talks to the device kernels.  There is no
fallback: if the shared library is missing or a call is rejected, it raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libp2p_hip.so")
# A/B timing tools load the experiments build (make EXPERIMENTS=1 -> p2p_amd/exp/) instead; it is
# built from the same sources and stamped "<hash>-exp" (check_source_hash accepts it only here)
if os.environ.get("P2P_EXPERIMENTS_LIB") == "1":
    _LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "exp", "libp2p_hip.so")
_lib = None

# Optional launch observer (bench.py times the dominant kernel and the map-store launches with HIP
# events through it): an object with before(kind, tensors, info) / after(kind, tensors, info),
# called around each launch; info = {"stored": entries whose maps are kept, "accumulate": bool}.
LAUNCH_OBSERVER = None

P2P_DTYPE_F32 = 0
P2P_DTYPE_BF16 = 1
P2P_COMPUTE_BF16 = 0
P2P_COMPUTE_F32 = 1
MAX_BATCH = 64
MAX_GROUPS = 32
MAX_KEYS_CROSS = 96
PROGRAM_COLS = 128
PROGRAM_TMAX = 8
ABI_VERSION = 15
GROUP_F_R_ONLY = 2      # p2p_group.flags: every edit's blend coefficient A is 0 this call (P' = R)
GROUP_F_SHARED_KV = 4   # p2p_group.flags: every entry of the group has the first entry's K and V


class HipError(RuntimeError):
    pass


class AttnTensors(ctypes.Structure):
    _fields_ = [
        ("q", ctypes.c_void_p), ("k", ctypes.c_void_p), ("v", ctypes.c_void_p), ("o", ctypes.c_void_p),
        ("q_row_stride", ctypes.c_int64), ("k_row_stride", ctypes.c_int64),
        ("v_row_stride", ctypes.c_int64), ("o_row_stride", ctypes.c_int64),
        ("q_batch_stride", ctypes.c_int64), ("k_batch_stride", ctypes.c_int64),
        ("v_batch_stride", ctypes.c_int64), ("o_batch_stride", ctypes.c_int64),
        ("n_batch", ctypes.c_int32), ("n_query", ctypes.c_int32), ("n_key", ctypes.c_int32),
        ("n_heads", ctypes.c_int32), ("head_dim", ctypes.c_int32),
        ("io_dtype", ctypes.c_int32), ("compute", ctypes.c_int32),
        ("scale", ctypes.c_float),
    ]


class Group(ctypes.Structure):
    _fields_ = [("first", ctypes.c_int32), ("count", ctypes.c_int32),
                ("program", ctypes.c_void_p), ("alpha", ctypes.c_void_p), ("flags", ctypes.c_int32),
                ("n_edits", ctypes.c_int32), ("blend_sums", ctypes.c_void_p), ("blend_alpha", ctypes.c_void_p),
                ("blend_sub", ctypes.c_void_p), ("blend_col", ctypes.c_int32), ("blend_lh", ctypes.c_int32)]


class BlendArgs(ctypes.Structure):
    _fields_ = [
        ("maps", ctypes.c_void_p * 8), ("n_maps", ctypes.c_int32), ("heads_per_map", ctypes.c_int32),
        ("n_prompts", ctypes.c_int32), ("n_words", ctypes.c_int32), ("map_res", ctypes.c_int32),
        ("alpha_layers", ctypes.c_void_p), ("substruct_layers", ctypes.c_void_p),
        ("th_pool", ctypes.c_float), ("th_sub", ctypes.c_float),
        ("x_t", ctypes.c_void_p), ("channels", ctypes.c_int32), ("lat_h", ctypes.c_int32),
        ("lat_w", ctypes.c_int32), ("word_sums", ctypes.c_void_p), ("mask_out", ctypes.c_void_p),
        ("word_sums_ready", ctypes.c_int32),
    ]


class LatentArgs(ctypes.Structure):
    _fields_ = [
        ("eps", ctypes.c_void_p), ("eps_dtype", ctypes.c_int32), ("cfg", ctypes.c_int32),
        ("guidance", ctypes.c_float), ("x", ctypes.c_void_p), ("out", ctypes.c_void_p),
        ("n_prompts", ctypes.c_int32), ("channels", ctypes.c_int32), ("height", ctypes.c_int32),
        ("width", ctypes.c_int32), ("sqrt_beta_t", ctypes.c_float), ("sqrt_alpha_t", ctypes.c_float),
        ("sqrt_alpha_prev", ctypes.c_float), ("sqrt_one_minus_alpha_prev", ctypes.c_float),
        ("mask", ctypes.c_void_p), ("group_size", ctypes.c_int32), ("group_blend", ctypes.c_void_p),
        ("blend_sums", ctypes.c_void_p * MAX_GROUPS), ("blend_lh", ctypes.c_int32), ("blend_res", ctypes.c_int32),
        ("blend_th_pool", ctypes.c_float), ("blend_th_sub", ctypes.c_float), ("blend_sub", ctypes.c_int32),
    ]


def library_path() -> str:
    return _LIB_PATH


def lib():
    """Load the HIP library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise HipError(f"{_LIB_PATH} is missing: run __graft_entry__.build() (make -C prompt-to-prompt_amd/csrc)")
        L = ctypes.CDLL(_LIB_PATH)
        i32, vp, f32, i64 = ctypes.c_int32, ctypes.c_void_p, ctypes.c_float, ctypes.c_int64
        L.p2p_abi_version.restype = ctypes.c_int
        L.p2p_error_string.restype = ctypes.c_char_p
        L.p2p_source_hash.restype = ctypes.c_char_p
        L.p2p_error_string.argtypes = [ctypes.c_int]
        L.p2p_self_attn_fwd.argtypes = [ctypes.POINTER(AttnTensors), vp, vp, vp, i32, vp, vp]
        L.p2p_cross_attn_fwd.argtypes = [ctypes.POINTER(AttnTensors), vp, i32, vp, vp, i32, vp]
        L.p2p_attn_probs.argtypes = [ctypes.POINTER(AttnTensors), vp, vp, vp]
        L.p2p_attn_pv.argtypes = [ctypes.POINTER(AttnTensors), vp, vp]
        L.p2p_localblend.argtypes = [ctypes.POINTER(BlendArgs), vp]
        L.p2p_store_scale.argtypes = [vp, vp, f32, i64, vp]
        L.p2p_latent_step.argtypes = [ctypes.POINTER(LatentArgs), vp]
        L.p2p_attn_fwd_lse.argtypes = [ctypes.POINTER(AttnTensors), vp, vp]
        L.p2p_attn_bwd.argtypes = [ctypes.POINTER(AttnTensors), vp, vp, vp, vp, vp, vp, i32, vp, i64, vp]
        L.p2p_attn_bwd_workspace.argtypes = [ctypes.POINTER(AttnTensors)]
        L.p2p_attn_bwd_workspace.restype = ctypes.c_int64
        L.p2p_clock_probe.argtypes = [vp, i32, i32, vp]
        L.p2p_set_launch_events.argtypes = [vp, vp]
        for fn in ("p2p_self_attn_fwd", "p2p_cross_attn_fwd", "p2p_attn_probs", "p2p_attn_pv",
                   "p2p_localblend", "p2p_store_scale", "p2p_latent_step", "p2p_attn_fwd_lse", "p2p_attn_bwd",
                   "p2p_clock_probe", "p2p_set_launch_events"):
            getattr(L, fn).restype = ctypes.c_int
        if L.p2p_abi_version() != ABI_VERSION:
            raise HipError(f"libp2p_hip.so ABI {L.p2p_abi_version()} != {ABI_VERSION}")
        _lib = L
    return _lib


def check_source_hash() -> str:
    """Raise unless the loaded library was built from the HIP sources in this tree (the Makefile
    stamps _srchash.source_hash() into it).  smoke() and the GPU tests call this, so a stale
    prebuilt libp2p_hip.so cannot pass for the current sources."""
    from . import _srchash
    built = lib().p2p_source_hash().decode()
    tree = _srchash.source_hash()
    if os.environ.get("P2P_EXPERIMENTS_LIB") == "1":
        tree += "-exp"   # the experiments build stamps its flavour (a production process refuses it)
    if built != tree:
        raise HipError(f"libp2p_hip.so was built from sources {built}, the tree has {tree}: rebuild "
                       f"(make -C prompt-to-prompt_amd/csrc)")
    return built


EXPORTED_SYMBOLS = ("p2p_abi_version", "p2p_source_hash", "p2p_error_string", "p2p_self_attn_fwd", "p2p_cross_attn_fwd",
                    "p2p_attn_probs", "p2p_attn_pv", "p2p_localblend", "p2p_store_scale", "p2p_latent_step",
                    "p2p_attn_fwd_lse", "p2p_attn_bwd", "p2p_attn_bwd_workspace", "p2p_clock_probe",
                    "p2p_set_launch_events")


def clock_probe(out: torch.Tensor, ticks: int = 1000):
    """Measurement only (bench.py): one p2p_clock_probe launch on the current stream, one one-wave
    workgroup per row of ``out`` (int64 [n, 2] on the GPU: shader cycles, 100 MHz ticks); the
    shader clock of row w is out[w, 0] / out[w, 1] x 100 MHz, read after a synchronise."""
    _require_cuda(out)
    if out.dtype != torch.int64 or out.dim() != 2 or out.shape[1] != 2 or not out.is_contiguous():
        raise HipError("clock_probe needs a contiguous int64 [n, 2] tensor")
    _check(lib().p2p_clock_probe(out.data_ptr(), out.shape[0], int(ticks), _stream(out.device)), "p2p_clock_probe")
    return out


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().p2p_error_string(rc).decode()
        raise HipError(f"{what} failed: {msg} (code {rc})")


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return P2P_DTYPE_F32
    if t.dtype == torch.bfloat16:
        return P2P_DTYPE_BF16
    raise HipError(f"unsupported attention dtype {t.dtype} (float32 or bfloat16)")


_COMPUTE = {"bf16": P2P_COMPUTE_BF16, "f32": P2P_COMPUTE_F32}


def _require_cuda(*ts: Optional[torch.Tensor]):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise HipError("p2p_amd kernels need GPU tensors (no CPU path in the product)")


def make_tensors(q, k, v, o, heads: int, scale: float, compute: str) -> AttnTensors:
    """q/o: [N, P, H*d]; k/v: [N, K, H*d]; last dim contiguous."""
    ref = q if q is not None else v
    _require_cuda(q, k, v, o)
    for t in (q, k, v, o):
        if t is not None and (t.dim() != 3 or t.stride(-1) != 1):
            raise HipError("attention operands must be [batch, tokens, heads*dim] with a unit last stride")
    C = ref.shape[-1]
    if C % heads:
        raise HipError(f"channels {C} not divisible by heads {heads}")
    t = AttnTensors()

    def ptr(x):
        return x.data_ptr() if x is not None else None

    t.q, t.k, t.v, t.o = ptr(q), ptr(k), ptr(v), ptr(o)
    z = lambda x, i: x.stride(i) if x is not None else 0  # noqa: E731
    t.q_row_stride, t.k_row_stride, t.v_row_stride, t.o_row_stride = z(q, 1), z(k, 1), z(v, 1), z(o, 1)
    t.q_batch_stride, t.k_batch_stride, t.v_batch_stride, t.o_batch_stride = z(q, 0), z(k, 0), z(v, 0), z(o, 0)
    t.n_batch = ref.shape[0]
    t.n_query = (q if q is not None else o).shape[1]
    t.n_key = (k if k is not None else v).shape[1]
    t.n_heads = heads
    t.head_dim = C // heads
    t.io_dtype = _dtype_code(ref)
    t.compute = _COMPUTE[compute]
    t.scale = float(scale)
    return t


def _i32_array(vals: Sequence[int]):
    arr = (ctypes.c_int32 * len(vals))(*[int(x) for x in vals])
    return arr


def _lse_workspace(device, numel):
    """f32 scratch for the row log-sum-exp of a self launch that keeps maps: allocated per call
    from torch's caching allocator on the current stream (cheap), so launches on different
    streams -- or replays of a captured graph -- never share it; the allocator's stream
    ordering keeps it alive until the launch that reads it has run."""
    return torch.empty(numel, dtype=torch.float32, device=device)


def self_attn(q, k, v, o, heads, scale, compute="bf16", qk_src=None, store=None, store_slot=None,
              accumulate=False):
    t = make_tensors(q, k, v, o, heads, scale, compute)
    src = _i32_array(qk_src) if qk_src is not None else None
    slots = _i32_array(store_slot) if store_slot is not None else None
    if store is not None:
        _require_cuda(store)
        assert store.dtype == torch.float32 and store.is_contiguous()
    ws = None
    if store is not None and store_slot is not None and any(int(s) >= 0 for s in store_slot):
        ws = _lse_workspace(q.device, t.n_batch * t.n_heads * t.n_query).data_ptr()
    obs = LAUNCH_OBSERVER
    if obs is not None:
        info = {"stored": sum(1 for x in store_slot if int(x) >= 0) if ws is not None else 0,
                "accumulate": bool(accumulate)}
        obs.before("self", t, info)
    rc = lib().p2p_self_attn_fwd(ctypes.byref(t), src, store.data_ptr() if store is not None else None,
                                 slots, int(bool(accumulate)), ws, _stream(q.device))
    if obs is not None:
        obs.after("self", t, info)
    _check(rc, "p2p_self_attn_fwd")


def cross_group_dispatch(t: AttnTensors, groups) -> bool:
    """Whether p2p_cross_attn_fwd runs cross_group_kernel for these arguments: the rule of
    run_cross / cross_group_eligible (p2p_attn.hip, p2p_cross.hip) -- bf16 inputs and compute, no
    term-plane program, K <= 96, d = 40, and >= 512 workgroups (groups x heads x 128-row query
    tiles).  Labels only (bench.py); the library decides."""
    if t.io_dtype != P2P_DTYPE_BF16 or t.compute != P2P_COMPUTE_BF16 or t.n_key > MAX_KEYS_CROSS:
        return False
    if t.head_dim != 40:
        return False
    for grp in groups:
        prog, count = grp[2], int(grp[1])
        if prog is not None and count > 1 and not (int(getattr(prog, "p2p_flags", 0)) & 1):
            return False
    return len(groups) * t.n_heads * ((t.n_query + 127) // 128) >= 512


SHARED_KV_HINTS = os.environ.get("P2P_SHARED_KV", "1") != "0"   # (A/B switch: 0 = never hint)


def shared_kv_hint(k, v, first: int, count: int) -> int:
    """GROUP_F_SHARED_KV when the K and V rows first .. first + count - 1 are bit-identical, as
    recorded on the projection views by ptp_utils._project (kv_row_classes); else 0."""
    rows = getattr(k, "_p2p_rows", None)
    if not SHARED_KV_HINTS or count < 2 or rows is None or getattr(v, "_p2p_rows", None) is not rows or len(rows) != k.shape[0]:
        return 0
    return GROUP_F_SHARED_KV if all(r == rows[first] for r in rows[first:first + count]) else 0


def cross_attn(q, k, v, o, heads, scale, groups, compute="bf16", store=None, store_slot=None,
               accumulate=False):
    """groups: list of (first, count, program_tensor|None, alpha_tensor|None[, blend[, hints]]) with
    blend = None or (sums [count, 2, lh, n_query] f32, alpha [count, n_key] f32, sub [count, n_key] |
    None, col, lh): LocalBlend's word sums folded into the store epilogue (p2p_group.blend_*); hints:
    per-call p2p_group.flags bits OR'ed onto the program's (GROUP_F_R_ONLY)."""
    t = make_tensors(q, k, v, o, heads, scale, compute)
    G = (Group * len(groups))()
    for i, grp in enumerate(groups):
        first, count, prog, alpha = grp[:4]
        blend = grp[4] if len(grp) > 4 else None
        hints = int(grp[5]) if len(grp) > 5 else 0
        G[i].first, G[i].count = int(first), int(count)
        G[i].program = prog.data_ptr() if prog is not None else None
        G[i].alpha = alpha.data_ptr() if alpha is not None else None
        G[i].flags = (int(getattr(prog, "p2p_flags", 0)) | hints) if prog is not None else (hints & GROUP_F_SHARED_KV)
        G[i].n_edits = int(getattr(prog, "p2p_n_edits", 0)) if prog is not None else 0
        if blend is not None:
            sums, balpha, bsub, col, lh = blend
            _require_cuda(sums, balpha, bsub)
            assert sums.dtype == torch.float32 and sums.is_contiguous() and sums.numel() == count * 2 * lh * t.n_query
            assert balpha.dtype == torch.float32 and balpha.is_contiguous() and balpha.shape == (count, t.n_key)
            assert bsub is None or (bsub.dtype == torch.float32 and bsub.is_contiguous() and bsub.shape == balpha.shape)
            G[i].blend_sums, G[i].blend_alpha = sums.data_ptr(), balpha.data_ptr()
            G[i].blend_sub = bsub.data_ptr() if bsub is not None else None
            G[i].blend_col, G[i].blend_lh = int(col), int(lh)
    slots = _i32_array(store_slot) if store_slot is not None else None
    if store is not None:
        _require_cuda(store)
        assert store.dtype == torch.float32 and store.is_contiguous()
    obs = LAUNCH_OBSERVER
    if obs is not None:
        info = {"stored": sum(1 for x in store_slot if int(x) >= 0) if (store is not None and store_slot is not None)
                else 0, "accumulate": bool(accumulate), "n_groups": len(groups),
                "group_kernel": cross_group_dispatch(t, groups)}
        obs.before("cross", t, info)
    rc = lib().p2p_cross_attn_fwd(ctypes.byref(t), G, len(groups),
                                  store.data_ptr() if store is not None else None, slots,
                                  int(bool(accumulate)), _stream(q.device))
    if obs is not None:
        obs.after("cross", t, info)
    _check(rc, "p2p_cross_attn_fwd")


def attn_probs(q, k, heads, scale, probs, compute="bf16", key_mask=None):
    t = make_tensors(q, k, None, None, heads, scale, compute)
    _require_cuda(probs, key_mask)
    assert probs.dtype == torch.float32 and probs.is_contiguous()
    rc = lib().p2p_attn_probs(ctypes.byref(t), key_mask.data_ptr() if key_mask is not None else None,
                              probs.data_ptr(), _stream(q.device))
    _check(rc, "p2p_attn_probs")


def attn_pv(probs, v, o, heads, compute="bf16"):
    t = make_tensors(None, None, v, o, heads, 1.0, compute)
    t.n_query = o.shape[1]
    _require_cuda(probs)
    assert probs.dtype == torch.float32 and probs.is_contiguous()
    rc = lib().p2p_attn_pv(ctypes.byref(t), probs.data_ptr(), _stream(v.device))
    _check(rc, "p2p_attn_pv")


def localblend(maps, heads_per_map, alpha_layers, substruct_layers, th_pool, th_sub, x_t, word_sums,
               mask_out=None, word_sums_ready=False):
    """LocalBlend on device; x_t None with mask_out given = mask only (no blend).  word_sums_ready:
    word_sums already holds the folded word reductions (cross_attn blend); the maps are not read."""
    _require_cuda(x_t, alpha_layers, word_sums, substruct_layers, mask_out, *maps)
    a = BlendArgs()
    for i, m in enumerate(maps):
        assert m.dtype == torch.float32 and m.is_contiguous()
        a.maps[i] = m.data_ptr()
    B, W = alpha_layers.shape
    a.n_maps = len(maps)
    a.heads_per_map = heads_per_map
    a.n_prompts = B
    a.n_words = W
    a.map_res = int(round((maps[0].shape[1]) ** 0.5))
    a.alpha_layers = alpha_layers.data_ptr()
    a.substruct_layers = substruct_layers.data_ptr() if substruct_layers is not None else None
    a.th_pool, a.th_sub = float(th_pool), float(th_sub)
    if x_t is not None:
        assert x_t.dtype == torch.float32 and x_t.is_contiguous()
        a.x_t = x_t.data_ptr()
        a.channels, a.lat_h, a.lat_w = x_t.shape[1], x_t.shape[2], x_t.shape[3]
    else:
        assert mask_out is not None and mask_out.dtype == torch.uint8 and mask_out.is_contiguous()
        a.x_t = None
        a.channels, a.lat_h, a.lat_w = 0, mask_out.shape[-2], mask_out.shape[-1]
    a.word_sums = word_sums.data_ptr()
    a.mask_out = mask_out.data_ptr() if mask_out is not None else None
    a.word_sums_ready = int(bool(word_sums_ready))
    obs = LAUNCH_OBSERVER
    if obs is not None and hasattr(obs, "before_aux"):
        # algorithmic bytes: the word sums (or the maps) read, the mask written, x_t read + written
        LH, R2 = len(maps) * heads_per_map, a.map_res * a.map_res
        nbytes = (B * 2 * LH * R2 * 4 if word_sums_ready else sum(m.numel() * 4 for m in maps) + B * 2 * LH * R2 * 8)
        nbytes += B * a.lat_h * a.lat_w + (2 * x_t.numel() * 4 if x_t is not None else 0)
        obs.before_aux("localblend", nbytes)
    rc = lib().p2p_localblend(ctypes.byref(a), _stream((x_t if x_t is not None else mask_out).device))
    if obs is not None and hasattr(obs, "after_aux"):
        obs.after_aux("localblend")
    _check(rc, "p2p_localblend")


def store_scale(src: torch.Tensor, divisor: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _require_cuda(src)
    assert src.dtype == torch.float32 and src.is_contiguous()
    out = torch.empty_like(src) if out is None else out
    rc = lib().p2p_store_scale(src.data_ptr(), out.data_ptr(), float(divisor), src.numel(), _stream(src.device))
    _check(rc, "p2p_store_scale")
    return out


def latent_step(eps, x, out, coeffs, guidance=None, mask=None, group_size=0, group_blend=None, blend=None):
    """Fused CFG + DDIM step + LocalBlend blend (p2p_latent_step).  eps: [2B or B, C, H, W]
    (f32/bf16, uncond block first when guidance is given); x, out: f32 [B, C, H, W] (out may be
    x unless ``blend`` is given); coeffs: (sqrt_beta_t, sqrt_alpha_t, sqrt_alpha_prev,
    sqrt_one_minus_alpha_prev) floats; mask: uint8 [B, H, W] or None; group_size: prompts per
    prompt group (0 = one group), with group_blend (uint8 [B / group_size] or None = every group)
    selecting the groups that blend.  blend: instead of ``mask``, one entry per prompt group --
    None (no blend) or (sums f32 [group prompts, 2, lh, res^2], th_pool, th_sub, use_substruct):
    the folded LocalBlend word sums the mask is built from in the same launch."""
    _require_cuda(eps, x, out, mask)
    for t in (eps, x, out):
        assert t.is_contiguous()
    assert x.dtype == torch.float32 and out.dtype == torch.float32 and x.shape == out.shape
    B, C, H, W = x.shape
    assert eps.shape[1:] == x.shape[1:] and eps.shape[0] == (2 * B if guidance is not None else B)
    a = LatentArgs()
    a.eps, a.eps_dtype = eps.data_ptr(), _dtype_code(eps)
    a.cfg = 1 if guidance is not None else 0
    a.guidance = float(guidance) if guidance is not None else 0.0
    a.x, a.out = x.data_ptr(), out.data_ptr()
    a.n_prompts, a.channels, a.height, a.width = B, C, H, W
    a.sqrt_beta_t, a.sqrt_alpha_t, a.sqrt_alpha_prev, a.sqrt_one_minus_alpha_prev = [float(c) for c in coeffs]
    if mask is not None:
        assert mask.dtype == torch.uint8 and mask.is_contiguous() and mask.shape[-2:] == (H, W)
        a.mask = mask.data_ptr()
    else:
        a.mask = None
    a.group_size = int(group_size)
    if group_blend is not None:
        _require_cuda(group_blend)
        assert group_blend.dtype == torch.uint8 and group_blend.numel() * max(group_size, B) >= B
        a.group_blend = group_blend.data_ptr()
    else:
        a.group_blend = None
    sums_bytes = 0
    if blend is not None and any(e is not None for e in blend):
        if mask is not None or group_blend is not None or out.data_ptr() == x.data_ptr():
            raise HipError("latent_step: blend (folded sums) excludes mask / group_blend and out aliasing x")
        gs = group_size if group_size > 0 else B
        if len(blend) != B // gs or len(blend) > MAX_GROUPS:
            raise HipError(f"latent_step: {len(blend)} blend entries for {B // gs} prompt groups")
        ref = next(e for e in blend if e is not None)
        _, th_pool, th_sub, use_sub = ref
        lh, r2 = ref[0].shape[2], ref[0].shape[3]
        for g, e in enumerate(blend):
            if e is None:
                continue
            sums = e[0]
            _require_cuda(sums)
            if (sums.dtype != torch.float32 or not sums.is_contiguous() or tuple(sums.shape) != (gs, 2, lh, r2)
                    or tuple(e[1:]) != (th_pool, th_sub, use_sub)):
                raise HipError("latent_step: blend sums must be f32 [group, 2, lh, res^2] with one threshold set")
            a.blend_sums[g] = sums.data_ptr()
            sums_bytes += sums.numel() * 4
        a.blend_lh, a.blend_res = int(lh), int(round(r2 ** 0.5))
        a.blend_th_pool, a.blend_th_sub, a.blend_sub = float(th_pool), float(th_sub), int(bool(use_sub))
    obs = LAUNCH_OBSERVER
    if obs is not None and hasattr(obs, "before_aux"):
        # algorithmic bytes: eps read, x read, out written, mask (or the folded word sums) read
        obs.before_aux("latent_blend" if sums_bytes else "latent_step",
                       eps.numel() * eps.element_size() + 2 * x.numel() * 4 +
                       (mask.numel() if mask is not None else 0) + sums_bytes)
    rc = lib().p2p_latent_step(ctypes.byref(a), _stream(x.device))
    if obs is not None and hasattr(obs, "after_aux"):
        obs.after_aux("latent_blend" if sums_bytes else "latent_step")
    _check(rc, "p2p_latent_step")
    return out


def attn_fwd_lse(q, k, v, o, heads, scale, lse):
    """O and the row log-sum-exp (log2 domain, scale folded) for the backward pass."""
    t = make_tensors(q, k, v, o, heads, scale, "bf16")
    _require_cuda(lse)
    assert lse.dtype == torch.float32 and lse.is_contiguous() and lse.numel() == t.n_batch * heads * t.n_query
    _check(lib().p2p_attn_fwd_lse(ctypes.byref(t), lse.data_ptr(), _stream(q.device)), "p2p_attn_fwd_lse")


def attn_bwd(q, k, v, o, dout, lse, heads, scale, dq, dk, dv, delta, workspace=None):
    """dq (q's dtype and layout); dk / dv packed [N, K, H*d], written, in k's dtype or f32.
    workspace: p2p_attn_bwd_workspace bytes (allocated here when None)."""
    for x in (q, k, v, o, dout, dq, dk, dv):
        assert x.is_contiguous()
    assert dout.shape == o.shape == q.shape and dq.shape == q.shape
    assert dk.shape == k.shape and dv.shape == v.shape and dk.dtype == dv.dtype
    assert dk.dtype in (k.dtype, torch.float32)
    t = make_tensors(q, k, v, o, heads, scale, "bf16")
    _require_cuda(dout, lse, delta, dq, dk, dv)
    need = int(lib().p2p_attn_bwd_workspace(ctypes.byref(t)))
    if need > 0 and (workspace is None or workspace.numel() * workspace.element_size() < need):
        workspace = torch.empty(need, dtype=torch.uint8, device=q.device)
    ws_ptr = workspace.data_ptr() if need > 0 else None
    kv_f32 = int(dk.dtype == torch.float32)
    rc = lib().p2p_attn_bwd(ctypes.byref(t), dout.data_ptr(), lse.data_ptr(), delta.data_ptr(), dq.data_ptr(),
                            dk.data_ptr(), dv.data_ptr(), kv_f32, ws_ptr, need, _stream(q.device))
    _check(rc, "p2p_attn_bwd")
