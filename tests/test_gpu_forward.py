"""The product hook (ptp_utils.register_attention_control) + fused controllers on the golden
stand-in module tree: outputs must match what the REFERENCE's patched forward produced
(tests/golden/forward.npz), in the exact-f32 check mode (GPU)."""
import numpy as np
import pytest
import torch

from conftest import golden, golden_json
from test_oracle import FG, FM, forward_tree, run_tree

from p2p_amd import config
from p2p_amd import null_text as pn
from p2p_amd import ptp_utils

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", ["dummy", "replace", "refine"])
def test_hook_matches_reference_forward(cuda, tok, tag):
    model, pairs, xs, ctx = forward_tree()
    model = model.to(cuda)
    xs = [x.to(cuda) for x in xs]
    ctx = ctx.to(cuda)
    with config.compute_mode("f32"):
        if tag == "dummy":
            ctrl, steps = None, 1
        elif tag == "replace":
            ctrl = pn.AttentionReplace(FM["prompts"], 4, {"default_": .5, "lasagna": .25}, .5, tokenizer=tok,
                                       device=cuda)
            steps = 4
        else:
            ctrl = pn.AttentionRefine(FM["refine_prompts"], 4, .75, (.25, .75), tokenizer=tok, device=cuda)
            steps = 3
        ptp_utils.register_attention_control(model, ctrl)
        outs = run_tree(model, pairs, xs, ctx, steps)
    for (s, i, kind), y in outs.items():
        want = FG[f"{tag}_s{s}_p{i}_{kind}"]
        np.testing.assert_allclose(y.cpu().numpy(), want, rtol=0, atol=2e-5, err_msg=f"{tag} s{s} p{i} {kind}")
    if tag == "replace":
        assert ctrl.num_att_layers == int(FG["replace_num_att_layers"])
        for key, lst in ctrl.attention_store.items():
            for i, t in enumerate(lst):
                np.testing.assert_allclose(t.cpu().numpy(), FG[f"replace_store_{key}_{i}"], rtol=0, atol=1e-5)


def test_localblend_kernel_matches_reference(cuda, tok):
    from test_oracle import LG, LM, lb_store, lb_words
    from p2p_amd import controllers as pc
    for ci, case in enumerate(LM):
        kw = dict(case["kwargs"])
        if "th" in kw:
            kw["th"] = tuple(kw["th"])
        if "substruct_words" in kw:
            kw["substruct_words"] = lb_words(kw["substruct_words"])
        words = lb_words(case["words"])
        if case["flavour"] == "main":
            lb = pc.LocalBlend(case["prompts"], words, tokenizer=tok, device=cuda, **kw)
        else:
            lb = pn.LocalBlend(case["prompts"], words, tokenizer=tok, device=cuda, **kw)
        store = {k: [t.to(cuda) for t in v] for k, v in lb_store(ci).items()}
        x = torch.from_numpy(LG[f"case{ci}_x_t"]).to(cuda)
        for c in range(case["calls"]):
            x = lb(x, store)
            want = torch.from_numpy(LG[f"case{ci}_out{c}"]).to(cuda)
            agree = (x == want).all(dim=1).float().mean().item()
            assert agree >= 0.999, (ci, c, agree)
