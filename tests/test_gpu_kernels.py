"""HIP kernels vs plain fp32 references (GPU).

Tolerances (north star): attention probabilities within 1e-5 max-abs in the exact-f32 check
mode and 2e-3 at bf16; outputs O = P V are checked relative to max|V| (bf16 PV rounds P and
V to 8 significant bits: |dO| <= 2^-7 max|V|; f32: 1e-5 max|V|).
"""
import numpy as np
import pytest
import torch

from p2p_amd import _hip

pytestmark = pytest.mark.gpu


def ref_probs(q, k, heads, scale, qk_src=None):
    N, P, C = q.shape
    d = C // heads
    if qk_src is not None:
        q, k = q[qk_src], k[qk_src]
    qh = q.float().reshape(N, P, heads, d).permute(0, 2, 1, 3)
    kh = k.float().reshape(N, k.shape[1], heads, d).permute(0, 2, 1, 3)
    return (torch.einsum("nhid,nhjd->nhij", qh, kh) * scale).softmax(-1)      # [N, H, P, K]


def ref_out(probs, v, heads):
    N, K, C = v.shape
    vh = v.float().reshape(N, K, heads, C // heads).permute(0, 2, 1, 3)
    o = torch.einsum("nhij,nhjd->nhid", probs, vh)
    return o.permute(0, 2, 1, 3).reshape(N, probs.shape[2], C)


def o_tol(v, compute):
    return (2.0 ** -7 if compute == "bf16" else 1e-5) * v.float().abs().max().item()


def make_qkv(N, P, K, heads, d, dtype, qscale=1.0, seed=0, dev="cuda"):
    g = torch.Generator(device=dev).manual_seed(seed)
    C = heads * d
    q = (torch.randn(N, P, C, device=dev, generator=g) * qscale).to(dtype)
    k = torch.randn(N, K, C, device=dev, generator=g).to(dtype)
    v = torch.randn(N, K, C, device=dev, generator=g).to(dtype)
    return q, k, v


SELF_GEOMS = [  # (N, P, K, heads, d)
    (2, 4096, 4096, 2, 40), (2, 1024, 1024, 2, 80), (4, 256, 256, 8, 160), (4, 64, 64, 8, 160),
    (2, 100, 77, 2, 64), (2, 200, 130, 4, 16), (3, 33, 96, 2, 8),
]


@pytest.mark.parametrize("geom", SELF_GEOMS, ids=lambda g: "x".join(map(str, g)))
@pytest.mark.parametrize("compute", ["f32", "bf16"])
def test_self_attention_output(cuda, geom, compute):
    N, P, K, H, d = geom
    q, k, v = make_qkv(N, P, K, H, d, torch.float32)
    o = torch.empty_like(q)
    scale = d ** -0.5
    _hip.self_attn(q, k, v, o, H, scale, compute=compute)
    torch.cuda.synchronize()
    want = ref_out(ref_probs(q, k, H, scale), v, H)
    err = (o - want).abs().max().item()
    assert err < o_tol(v, compute), err


@pytest.mark.parametrize("compute,qscale,tol", [("f32", 1.0, 1e-5), ("f32", 12.0, 1e-5),
                                               ("bf16", 1.0, 2e-3), ("bf16", 8.0, 2e-3), ("bf16", 16.0, 2e-3)])
@pytest.mark.parametrize("geom", [(2, 1024, 1024, 2, 80), (2, 256, 256, 4, 160), (2, 64, 4096, 2, 40),
                                  (2, 40, 1100, 2, 64), (3, 16, 16, 2, 32)],
                         ids=lambda g: "x".join(map(str, g)))
def test_self_attention_store_probs(cuda, geom, compute, qscale, tol):
    """The AttentionStore epilogue writes exact probabilities (fused pass's lse + self_maps_kernel);
    ragged cases: a partial query tile (P = 40, 16), a partial last key block and two key groups
    (K = 1100 > 4 x 256), d without a padding column (64, 32)."""
    N, P, K, H, d = geom
    q, k, v = make_qkv(N, P, K, H, d, torch.float32, qscale=qscale, seed=3)
    o = torch.empty_like(q)
    scale = d ** -0.5
    store = torch.full((N * H, P, K), 7.0, device=cuda)
    slots = [n * H for n in range(N)]
    _hip.self_attn(q, k, v, o, H, scale, compute=compute, store=store, store_slot=slots, accumulate=False)
    p = ref_probs(q, k, H, scale)
    err = (store - p.reshape(N * H, P, K)).abs().max().item()
    assert err < tol, err
    # second call accumulates (running sum of AttentionStore.between_steps)
    _hip.self_attn(q, k, v, o, H, scale, compute=compute, store=store, store_slot=slots, accumulate=True)
    err2 = (store - 2 * p.reshape(N * H, P, K)).abs().max().item()
    assert err2 < 2 * tol, err2
    want = ref_out(p, v, H)
    assert (o - want).abs().max().item() < o_tol(v, compute)


def test_self_attention_injection_and_partial_store(cuda):
    N, P, K, H, d = 8, 256, 256, 8, 160
    q, k, v = make_qkv(N, P, K, H, d, torch.float32, seed=5)
    o = torch.empty_like(q)
    scale = d ** -0.5
    src = [0, 1, 2, 3, 4, 4, 4, 4]           # cond edits read the cond source's P (main.py:171)
    store = torch.zeros(4 * H, P, K, device=cuda)
    slots = [-1, -1, -1, -1, 0, H, 2 * H, 3 * H]
    _hip.self_attn(q, k, v, o, H, scale, compute="f32", qk_src=src, store=store, store_slot=slots)
    p = ref_probs(q, k, H, scale, qk_src=src)
    assert (o - ref_out(p, v, H)).abs().max().item() < o_tol(v, "f32")
    assert (store - p[4:].reshape(4 * H, P, K)).abs().max().item() < 1e-5


def test_bf16_inputs_exact_products(cuda):
    """bf16 inputs: one bf16 MFMA per k-step multiplies them exactly; the probabilities match
    an fp32 softmax of the same bf16 data to 2e-3 even on very peaky rows."""
    N, P, K, H, d = 2, 1024, 1024, 2, 80
    q, k, v = make_qkv(N, P, K, H, d, torch.bfloat16, qscale=16.0, seed=21)
    o = torch.empty_like(q)
    store = torch.zeros(N * H, P, K, device=cuda)
    _hip.self_attn(q, k, v, o, H, d ** -0.5, compute="bf16", store=store, store_slot=[0, H])
    p = ref_probs(q, k, H, d ** -0.5).reshape(N * H, P, K)
    assert (store - p).abs().max().item() < 2e-3


@pytest.mark.parametrize("case", ["plain", "peaky32", "k_past_f16", "q_past_f16", "late_peak", "remap", "ragged",
                                  "g1", "multi_late_peak"])
def test_self_attention_f16_form(cuda, case):
    """The d = 40 production form (bf16 inputs, P >= 2048; p2p_self40.hip): Q prescaled by
    scale*log2(e) in f16, K staged as f16, -m in Q's padding column, the reference point m taken
    from the first 32 keys.  Within the bf16 O bound on peaky rows; inputs past the f16 range
    (|k| >= 65520, |c q| >= 65520) and a logit far above m in a later tile (late_peak: c s ~ 5.7e5
    with q and k inside the f16 range) take the exact bf16 recompute and stay exact.  g1: the
    config-2 launch itself (N = 8, H = 8, P = K = 4096), held to o_tol + one bf16 output ulp."""
    N, P, K, H, d = {"ragged": (2, 2100, 2100, 2, 40), "g1": (8, 4096, 4096, 8, 40),
                     "multi_late_peak": (2, 2048, 200, 2, 40)}.get(case, (2, 2048, 2048, 2, 40))
    q, k, v = make_qkv(N, P, K, H, d, torch.bfloat16, qscale=32.0 if case == "peaky32" else 1.0, seed=31)
    if case == "k_past_f16":
        k[1, 100, 3] = 70000.0          # one key element of entry 1, head 0
        q[1, :, 3] = 1e-3               # keeps its logits finite and moderate
    if case == "q_past_f16":
        q[0, 5, 41] = 4.0e5             # c q ~ 9e4 > 65504 (entry 0, head 1)
        k[0, :, 41] = 1e-4
    if case == "late_peak":
        q[0, 7, :d] = 250.0             # entry 0, head 0, query 7: c q ~ 57
        k[0, 1500, :d] = 250.0          # key 1500 (tile 5): c s ~ 5.7e5, tile 0 stays ordinary
    if case == "multi_late_peak":
        # K < 256: the F16 multi-block kernel (one masked 256-key tile, per-sub-block reference
        # point); query 7's logits stay ordinary until key 150 (sub-block 4), where c q (~456) and
        # k (10) are inside the f16 range but c s ~ 1.8e5 > 65504: the recompute must take the
        # exact path.  (k is kept moderate: the F16 form's logit error grows with |c q| |k|, and a
        # large k would also perturb every other row -- that is the form's documented bound)
        q[0, 7, :d] = 2000.0
        k[0, 150, :d] = 10.0
    src = [0, 0] if case == "remap" else None
    o = torch.empty_like(q)
    _hip.self_attn(q, k, v, o, H, d ** -0.5, compute="bf16", qk_src=src)
    want = ref_out(ref_probs(q, k, H, d ** -0.5, qk_src=src), v, H)
    assert torch.isfinite(o.float()).all()
    # O within 2^-7 max|V| (the bf16 bound) plus one bf16 rounding of the stored output
    bound = o_tol(v, "bf16") + 2.0 ** -8 * want.abs().max().item()
    assert (o.float() - want).abs().max().item() < bound


@pytest.mark.parametrize("case", ["plain", "peaky32", "late_peak", "remap", "ragged", "g2"])
def test_self_attention_d80_pipelined(cuda, case):
    """The d = 80 production form (bf16 inputs, P >= 512, K >= 256; p2p_self40.hip, bf16 Q K^T
    with p = exp2(fma(s, c, -m)), m from the first 32 keys): within the bf16 O bound on peaky rows;
    a logit far above m in a later tile (late_peak) takes the exact recompute.  g2: the config-2
    G2/G6 launch (N = 8, H = 8, P = K = 1024)."""
    N, P, K, H, d = {"ragged": (2, 1100, 1100, 2, 80), "g2": (8, 1024, 1024, 8, 80)}.get(case, (2, 1024, 1024, 2, 80))
    q, k, v = make_qkv(N, P, K, H, d, torch.bfloat16, qscale=32.0 if case == "peaky32" else 1.0, seed=33)
    if case == "late_peak":
        q[0, 7, :d] = 60.0              # entry 0, head 0, query 7
        k[0, 700, :d] = 60.0            # key 700 (tile 5 of 128): c s ~ 3.3e4 log2 units
    src = [0, 0] if case == "remap" else None
    o = torch.empty_like(q)
    _hip.self_attn(q, k, v, o, H, d ** -0.5, compute="bf16", qk_src=src)
    want = ref_out(ref_probs(q, k, H, d ** -0.5, qk_src=src), v, H)
    assert torch.isfinite(o.float()).all()
    bound = o_tol(v, "bf16") + 2.0 ** -8 * want.abs().max().item()
    assert (o.float() - want).abs().max().item() < bound


@pytest.mark.parametrize("io", [torch.bfloat16])
def test_self_attention_bf16_io(cuda, io):
    N, P, K, H, d = 2, 1024, 1024, 8, 80
    q, k, v = make_qkv(N, P, K, H, d, io, seed=9)
    o = torch.empty_like(q)
    _hip.self_attn(q, k, v, o, H, d ** -0.5, compute="bf16")
    want = ref_out(ref_probs(q, k, H, d ** -0.5), v, H)
    assert o.dtype == io
    assert (o.float() - want).abs().max().item() < 2 * o_tol(v, "bf16")   # + bf16 output rounding


@pytest.mark.parametrize("compute,tol", [("f32", 1e-5), ("bf16", 2e-3)])
@pytest.mark.parametrize("geom", [(4, 4096, 77, 8, 40), (4, 256, 77, 8, 160), (6, 100, 77, 2, 16),
                                  (2, 1024, 1024, 2, 80), (2, 40, 1100, 2, 64), (2, 33, 130, 2, 8)],
                         ids=lambda g: "x".join(map(str, g)))
def test_probs_and_pv_materialise(cuda, geom, compute, tol):
    N, P, K, H, d = geom
    q, k, v = make_qkv(N, P, K, H, d, torch.float32, qscale=4.0, seed=11)
    scale = d ** -0.5
    probs = torch.empty(N * H, P, K, device=cuda)
    _hip.attn_probs(q, k, H, scale, probs, compute=compute)
    p = ref_probs(q, k, H, scale)
    assert (probs - p.reshape(N * H, P, K)).abs().max().item() < tol
    o = torch.empty_like(q)
    _hip.attn_pv(probs, v, o, H, compute=compute)
    want = ref_out(probs.reshape(N, H, P, K), v, H)
    assert (o - want).abs().max().item() < o_tol(v, compute)


@pytest.mark.parametrize("compute,tol", [("f32", 1e-5), ("bf16", 2e-3)])
@pytest.mark.parametrize("P", [1024, 100])
def test_cross_plain_groups(cuda, compute, tol, P):
    N, K, H, d = 8, 77, 8, 80
    q, k, v = make_qkv(N, P, K, H, d, torch.float32, qscale=12.0, seed=13)
    scale = d ** -0.5
    o = torch.empty_like(q)
    store = torch.zeros(N * H, P, K, device=cuda)
    groups = [(n, 1, None, None) for n in range(N)]
    _hip.cross_attn(q, k, v, o, H, scale, groups, compute=compute, store=store,
                    store_slot=[n * H for n in range(N)])
    p = ref_probs(q, k, H, scale)
    assert (store - p.reshape(N * H, P, K)).abs().max().item() < tol
    assert (o - ref_out(p, v, H)).abs().max().item() < o_tol(v, compute)


@pytest.mark.parametrize("weight", [0.5, 1.0 / 3.0], ids=["dense", "terms"])
@pytest.mark.parametrize("compute,tol", [("f32", 1e-5), ("bf16", 2e-3)])
@pytest.mark.parametrize("geom", [(4096, 40), (1024, 80)], ids=["G1", "G2"])
def test_cross_edit_paths(cuda, weight, compute, tol, geom):
    """Both edit paths of the cross kernel against the materialised einsum (main.py:217-218):
    a mapper whose weights are bf16 values (1, 1/2) carries the dense tile (bf16 kernels: R on
    the MFMA), one with 1/3 weights does not (LDS term-plane gather); the f32 check mode always
    gathers.  Group layout as the controllers launch it: [uncond | source, 3 edits], store on."""
    from p2p_amd import programs
    P, d = geom
    B, H, K = 4, 8, 77
    N = 2 * B
    q, k, v = make_qkv(N, P, K, H, d, torch.float32, qscale=6.0, seed=21)
    scale = d ** -0.5
    mapper = torch.zeros(B - 1, K, K)
    mapper[:, torch.arange(K), torch.arange(K)] = 1.0
    mapper[0, 3, 3] = mapper[0, 4, 3] = weight        # a 2-/3-token source word -> one target word
    if weight < 0.5:
        mapper[0, 5, 3] = weight
    mapper[1, 7, 7], mapper[1, 7, 8] = 0.0, 1.0       # swapped columns
    mapper[1, 8, 8], mapper[1, 8, 7] = 0.0, 1.0
    prog_host = programs.replace_program(mapper)
    assert (prog_host.dense_f16() is not None) == (weight == 0.5)
    prog = prog_host.to_device(cuda)
    alpha = torch.ones(B - 1, K, device=cuda)
    alpha[2, 10:20] = 0.0                             # word-time alpha 0: own probabilities
    o = torch.empty_like(q)
    store = torch.zeros(B * H, P, K, device=cuda)
    groups = [(0, B, None, None), (B, B, prog, alpha)]
    _hip.cross_attn(q, k, v, o, H, scale, groups, compute=compute, store=store,
                    store_slot=[-1] * B + [i * H for i in range(B)])
    p = ref_probs(q, k, H, scale)                     # [N, H, P, K]
    cond = p[B:].clone()
    base = cond[0]
    R = torch.einsum("hpw,bwn->bhpn", base, mapper.to(cuda))
    a = alpha[:, None, None, :]
    cond[1:] = R * a + (1 - a) * cond[1:]
    assert (store - cond.reshape(B * H, P, K)).abs().max().item() < tol
    want = torch.cat([p[:B], cond])
    assert (o - ref_out(want, v, H)).abs().max().item() < o_tol(v, compute)


@pytest.mark.parametrize("geom", [(2, 1024, 1024, 2, 80), (2, 256, 4096, 2, 40), (3, 64, 77, 4, 160)],
                         ids=lambda g: "x".join(map(str, g)))
def test_probs_and_pv_materialise_bf16_inputs(cuda, geom):
    """bf16 q/k/v (the production U-Net): one bf16 MFMA per k-step, exact products; probabilities
    within 2e-3 of an fp32 softmax of the same bf16 data even on peaky rows, rows summing to 1."""
    N, P, K, H, d = geom
    q, k, v = make_qkv(N, P, K, H, d, torch.bfloat16, qscale=8.0, seed=23)
    probs = torch.empty(N * H, P, K, device=cuda)
    _hip.attn_probs(q, k, H, d ** -0.5, probs)
    p = ref_probs(q, k, H, d ** -0.5).reshape(N * H, P, K)
    assert (probs - p).abs().max().item() < 2e-3
    assert (probs.sum(-1) - 1).abs().max().item() < 1e-4
    o = torch.empty_like(q)
    _hip.attn_pv(probs, v, o, H)
    want = ref_out(probs.reshape(N, H, P, K), v, H)
    assert (o.float() - want).abs().max().item() < 2 * o_tol(v, "bf16")


@pytest.mark.parametrize("K", [77, 1100])
def test_key_mask_materialise(cuda, K):
    """Partial masks zero the masked keys; a fully masked row is uniform (softmax of -finfo.max)."""
    N, P, H, d = 3, 64, 2, 16
    q, k, v = make_qkv(N, P, K, H, d, torch.float32, seed=17)
    mask = torch.ones(N, K, dtype=torch.bool, device=cuda)
    mask[0, 50:] = False
    mask[1, :10] = False
    mask[2, :] = False
    probs = torch.empty(N * H, P, K, device=cuda)
    _hip.attn_probs(q, k, H, d ** -0.5, probs, compute="f32", key_mask=mask.to(torch.uint8))
    # ptp_utils.py:197-201: rows (n*H + h) take mask row (n*H + h) % N (head-major repeat)
    sim = torch.einsum("nhid,nhjd->nhij", q.reshape(N, P, H, d).permute(0, 2, 1, 3),
                       k.reshape(N, K, H, d).permute(0, 2, 1, 3)).reshape(N * H, P, K) * d ** -0.5
    m = mask[:, None, :].repeat(H, 1, 1)
    sim.masked_fill_(~m, -torch.finfo(sim.dtype).max)
    assert (probs - sim.softmax(-1)).abs().max().item() < 1e-5


def test_store_scale(cuda):
    """get_average_attention divides by cur_step; on cuda:0 (the reference's device) torch
    multiplies by the f32 reciprocal, which the kernel reproduces bit for bit."""
    x = torch.randn(3, 1000, 77, device=cuda)
    for steps in (7, 50, 3):
        y = _hip.store_scale(x, float(steps))
        assert torch.equal(y, x / steps)


def _edit_mapper(B, K, weight=0.5):
    m = torch.zeros(B - 1, K, K)
    m[:, torch.arange(K), torch.arange(K)] = 1.0
    m[0, 3, 3] = m[0, 4, 3] = weight
    if B > 2:
        m[1, 7, 7], m[1, 7, 8] = 0.0, 1.0
        m[1, 8, 8], m[1, 8, 7] = 0.0, 1.0
    return m


# (P, d, K, heads, prompt groups, kernel the launch must dispatch to): run_cross takes
# cross_group_kernel only when n_groups x heads x ceil(P / 128) >= 512 (p2p_cross.hip
# cross_group_eligible), so the group-kernel cases are sized to clear that bar
CROSS_GROUP_CASES = [
    (4096, 40, 77, 8, 1, "group"), (4096, 40, 77, 8, 2, "group"),     # G1/G7
    (4000, 40, 96, 8, 2, "group"),                                    # ragged P, K = 96: no short key tail
    (4000, 40, 33, 8, 1, "group"),                                    # K = 33, ragged P
    (1024, 80, 77, 8, 4, "entry"),                                    # G2/G6 as configs[3] batches it: the
    (1000, 80, 77, 8, 4, "entry"),                                    # per-entry kernel at d = 80 / 160 at any
    (256, 160, 77, 16, 8, "entry"),                                   # size (measured faster, p2p_cross.hip)
    (1024, 80, 77, 8, 1, "entry"), (256, 160, 77, 8, 2, "entry"),     # G2-G4 at configs[1]: per-entry
    (64, 160, 77, 8, 1, "entry"), (100, 80, 96, 8, 2, "entry"), (333, 40, 33, 8, 1, "entry"),
    (64, 160, 77, 8, 8, "entry"),   # N = 64 entries in a 512-workgroup launch: the per-entry work order's
                                    # rotation must stay a bijection when N does not divide 32
]


@pytest.mark.parametrize("case", CROSS_GROUP_CASES, ids=lambda c: "P{}_d{}_K{}_H{}_g{}_{}".format(*c))
def test_cross_group_kernel_bf16(cuda, case):
    """The cross-attention kernels with bf16 inputs (p2p_cross.hip group kernel where the grid is
    large enough, cross_attn_kernel otherwise; the case states which and the test asserts the
    dispatch rule): [uncond groups | cond groups], each cond group a source + 3 dense Replace
    edits against its OWN source (main.py:185-193), the cond maps kept and accumulated over two
    calls, LocalBlend word sums folded in, against fp32 einsum on the same bf16 inputs.  The group
    kernel (d = 40 only) is covered at ragged P, K = 96 (no short tail) and K = 33."""
    from p2p_amd import programs
    P, d, K, H, n_groups, kernel = case
    B = 4
    N = 2 * B * n_groups
    q, k, v = make_qkv(N, P, K, H, d, torch.bfloat16, qscale=6.0, seed=31 + P)
    scale = d ** -0.5
    mappers = [_edit_mapper(B, K) if g % 2 == 0 else _edit_mapper(B, K).flip(0) for g in range(n_groups)]
    if n_groups > 1:
        # group 1: a target word gathering three source words (tmax 3): the group kernel copies that
        # program's dense mapper image instead of building the tile from two term planes
        mappers[1][0, :, 5] = 0.0
        mappers[1][0, 5, 5], mappers[1][0, 6, 5], mappers[1][0, 9, 5] = 0.25, 0.25, 0.5
    progs = [programs.replace_program(m).to_device(cuda) for m in mappers]
    assert n_groups == 1 or programs.replace_program(mappers[1]).tmax == 3
    alpha = torch.ones(B - 1, K, device=cuda)      # edit 0: alpha 1 everywhere (R only)
    alpha[1] = 0.0                                   # edit 1: alpha 0 everywhere (own P only)
    alpha[2, 10:20] = 0.0                            # edit 2: both halves
    lh = 5 * H
    bsums = [torch.zeros(B, 2, lh, P, device=cuda) for _ in range(n_groups)]
    balpha = torch.rand(B, K, device=cuda, generator=torch.Generator(device=cuda).manual_seed(5))
    bsub = torch.rand(B, K, device=cuda, generator=torch.Generator(device=cuda).manual_seed(6))
    BG = B * n_groups
    groups = [(g * B, B, None, None) for g in range(n_groups)]
    groups += [(BG + g * B, B, progs[g], alpha, (bsums[g], balpha, bsub if g == 0 else None, 2 * H, lh))
               for g in range(n_groups)]
    store = torch.zeros(BG * H, P, K, device=cuda)
    slots = [-1] * BG + [i * H for i in range(BG)]
    o = torch.empty_like(q)
    t = _hip.make_tensors(q, k, v, o, H, scale, "bf16")
    assert _hip.cross_group_dispatch(t, groups) == (kernel == "group")
    for acc in (False, True):
        _hip.cross_attn(q, k, v, o, H, scale, groups, store=store, store_slot=slots, accumulate=acc)
    p = ref_probs(q, k, H, scale)                                    # [N, H, P, K]
    want = p.clone()
    for g in range(n_groups):
        s0 = BG + g * B
        base = p[s0]
        R = torch.einsum("hpw,bwn->bhpn", base, mappers[g].to(cuda))
        a = alpha[:, None, None, :]
        want[s0 + 1:s0 + B] = R * a + (1 - a) * p[s0 + 1:s0 + B]
    cond = want[BG:]
    assert (store - 2 * cond.reshape(BG * H, P, K)).abs().max().item() < 2 * 2e-3
    assert (o.float() - ref_out(want, v, H)).abs().max().item() < o_tol(v, "bf16")
    for g in range(n_groups):
        c = cond[g * B:(g + 1) * B]                                  # [B, H, P, K]
        ws_a = torch.einsum("bhpk,bk->bhp", c, balpha)
        got = bsums[g][:, 0, 2 * H:3 * H]
        assert (got - 2 * ws_a).abs().max().item() < 2e-2
        got_s = bsums[g][:, 1, 2 * H:3 * H]
        ws_s = torch.einsum("bhpk,bk->bhp", c, bsub) if g == 0 else torch.zeros_like(ws_a)
        assert (got_s - 2 * ws_s).abs().max().item() < 2e-2
        assert bsums[g][:, :, :2 * H].abs().max().item() == 0.0 and bsums[g][:, :, 3 * H:].abs().max().item() == 0.0


@pytest.mark.parametrize("case", ["g3", "g4", "peaky32", "remap", "ragged", "k200", "k129", "k300", "k33", "k20"])
def test_self_attention_key_split_d160(cuda, case):
    """d = 160 with bf16 inputs, O only (p2p_selfsplit.hip): K <= 128 takes the key-split kernel (the
    waves of a 32-query workgroup split the keys and combine (O_w, m_w, l_w) in LDS), larger K the
    key-halves kernel up to K = 256 and the 4-stage DMA ring kernel past it.  g4 / g3: the config-2
    8x8 and 16x16 launches; ragged P / K, key-split wave counts 1 and 2 (K = 20, 33, 77), K = 200 (a
    partial last tile and a key half ending in a tile wholly past K), K = 129 (one key in the second
    half's first tile), K = 300 (the ring kernel), peaky rows (defer-max rescales), a source remap."""
    N, P, K, H, d = {"g3": (8, 256, 256, 8, 160), "g4": (8, 64, 64, 8, 160), "ragged": (3, 100, 77, 2, 160),
                     "k200": (2, 130, 200, 4, 160), "k129": (2, 97, 129, 2, 160),
                     "k300": (2, 70, 300, 2, 160), "k33": (2, 70, 33, 2, 160),
                     "k20": (2, 45, 20, 2, 160)}.get(case, (4, 256, 256, 4, 160))
    q, k, v = make_qkv(N, P, K, H, d, torch.bfloat16, qscale=32.0 if case == "peaky32" else 1.0, seed=41)
    src = [0, 1, 0, 0] if case == "remap" else None
    o = torch.empty_like(q)
    _hip.self_attn(q, k, v, o, H, d ** -0.5, compute="bf16", qk_src=src)
    want = ref_out(ref_probs(q, k, H, d ** -0.5, qk_src=src), v, H)
    assert torch.isfinite(o.float()).all()
    bound = o_tol(v, "bf16") + 2.0 ** -8 * want.abs().max().item()
    assert (o.float() - want).abs().max().item() < bound


@pytest.mark.parametrize("geom", [(1024, 80, 1), (256, 160, 1), (64, 160, 1), (256, 160, 8), (4096, 40, 1)],
                         ids=lambda g: "P{}_d{}_g{}".format(*g))
def test_cross_r_only_hint(cuda, geom):
    """p2p_group.flags GROUP_F_R_ONLY (ABI 14): the host's per-call hint that alpha makes every
    edit's blend coefficient A zero (a Replace step inside cross_replace_steps, main.py:189), so
    the dense kernels skip the edits' own Q / K loads and softmax.  With the hint the outputs, the
    stored maps and the LocalBlend word sums are bit-identical to the unhinted launch; a WRONG hint
    (alpha 0 on some words: A != 0) falls back inside the kernel and is bit-identical as well."""
    from p2p_amd import programs
    P, d, n_groups = geom
    B, H, K = 4, 8, 77
    BG = B * n_groups
    N = 2 * BG
    q, k, v = make_qkv(N, P, K, H, d, torch.bfloat16, qscale=6.0, seed=77 + P)
    scale = d ** -0.5
    prog = programs.replace_program(_edit_mapper(B, K)).to_device(cuda)
    lh = 5 * H
    balpha = torch.rand(B, K, device=cuda, generator=torch.Generator(device=cuda).manual_seed(8))

    def run(alpha, hints):
        o = torch.empty_like(q)
        store = torch.zeros(BG * H, P, K, device=cuda)
        bsums = [torch.zeros(B, 2, lh, P, device=cuda) for _ in range(n_groups)]
        groups = [(g * B, B, None, None) for g in range(n_groups)]
        groups += [(BG + g * B, B, prog, alpha, (bsums[g], balpha, None, 0, lh), hints) for g in range(n_groups)]
        for acc in (False, True):
            _hip.cross_attn(q, k, v, o, H, scale, groups, store=store, store_slot=[-1] * BG + [i * H for i in range(BG)],
                            accumulate=acc)
        return o, store, torch.stack(bsums)

    ones = torch.ones(B - 1, K, device=cuda)
    mixed = ones.clone()
    mixed[2, 10:20] = 0.0
    for alpha in (ones, mixed):
        plain = run(alpha, 0)
        hinted = run(alpha, _hip.GROUP_F_R_ONLY)
        for x, y in zip(plain, hinted):
            assert torch.equal(x, y), (x.float() - y.float()).abs().max().item()
    # and the hinted launch is the edit: edit rows' maps equal R = P0 . M_e (alpha 1)
    o, store, _ = run(ones, _hip.GROUP_F_R_ONLY)
    p = ref_probs(q, k, H, scale)
    R = torch.einsum("hpw,bwn->bhpn", p[BG], _edit_mapper(B, K).to(cuda))
    assert (store[H:B * H] - 2 * R.reshape((B - 1) * H, P, K)).abs().max().item() < 2 * 2e-3


@pytest.mark.parametrize("geom", [(4096, 40, 1, "group"), (4096, 40, 2, "group"), (4000, 40, 1, "group"),
                                  (1024, 80, 1, "entry"), (256, 160, 8, "entry")],
                         ids=lambda g: "P{}_d{}_g{}_{}".format(*g))
def test_cross_shared_kv_hint(cuda, geom):
    """p2p_group.flags GROUP_F_SHARED_KV (ABI 15): the caller's guarantee that every entry of a group
    has the first entry's K and V (the uncond prompts ""); the group kernel stages them once and a
    plain group drops its barriers between entries.  With equal uncond rows the hinted launch is
    bit-identical to the unhinted one -- plain steps, R_ONLY edit steps, and one uncond group of
    every prompt group's rows (GroupBatch) -- and the per-entry kernel ignores the flag."""
    from p2p_amd import programs
    P, d, n_groups, kernel = geom
    B, H, K = 4, 8, 77
    BG = B * n_groups
    N = 2 * BG
    q, k, v = make_qkv(N, P, K, H, d, torch.bfloat16, qscale=6.0, seed=91 + P)
    k[1:BG] = k[0]
    v[1:BG] = v[0]
    scale = d ** -0.5
    prog = programs.replace_program(_edit_mapper(B, K)).to_device(cuda)
    ones = torch.ones(B - 1, K, device=cuda)

    def run(uncond, edits, shared):
        o = torch.empty_like(q)
        hint = _hip.GROUP_F_SHARED_KV if shared else 0
        groups = [(f, c, None, None, None, hint) for f, c in uncond]
        groups += [(BG + g * B, B, prog, ones, None, _hip.GROUP_F_R_ONLY) if edits else (BG + g * B, B, None, None)
                   for g in range(n_groups)]
        _hip.cross_attn(q, k, v, o, H, scale, groups)
        return o, groups

    per_group = [(g * B, B) for g in range(n_groups)]
    for uncond in (per_group, [(0, BG)]):
        for edits in (False, True):
            want, groups = run(uncond, edits, False)
            got, _ = run(uncond, edits, True)
            t = _hip.make_tensors(q, k, v, want, H, scale, "bf16")
            if uncond is per_group:
                assert _hip.cross_group_dispatch(t, groups) == (kernel == "group")
            assert torch.equal(got, want), (got.float() - want.float()).abs().max().item()
    # and it is attention: the uncond rows against fp32 torch
    o, _ = run(per_group, True, True)
    p = ref_probs(q, k, H, scale)
    assert (o[:BG].float() - ref_out(p, v, H)[:BG]).abs().max().item() < o_tol(v, "bf16")
