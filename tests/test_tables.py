"""Host edit tables (A9), bit-exact against the reference's golden vectors.

Both the product's tables (p2p_amd.seq_aligner / ptp_words / get_equalizer) and the oracle's
restatement are checked against tests/golden/tables.npz (tools/gen_golden.py ran the
reference's seq_aligner.py / ptp_utils.py / main.py / null_text.py to make it).
"""
import numpy as np
import pytest
import torch

from conftest import golden, golden_json

from oracle import tables as otab
from p2p_amd import controllers, null_text, seq_aligner
from p2p_amd.ptp_words import get_time_words_attention_alpha, get_word_inds

G = golden("tables")
M = golden_json("tables")


def _form(f):
    return tuple(f) if isinstance(f, list) else (dict((k, tuple(v) if isinstance(v, list) else v)
                                                      for k, v in f.items()) if isinstance(f, dict) else f)


def test_token_ids_match_fixture(tok):
    for case in M["replace"] + M["refine"]:
        for p, ids in zip(case["prompts"], case["ids"]):
            assert tok.encode(p) == ids


@pytest.mark.parametrize("i", range(len(M["replace"])))
def test_replacement_mapper(tok, i):
    prompts = M["replace"][i]["prompts"]
    want = G[f"replace{i}"]
    got = seq_aligner.get_replacement_mapper(prompts, tok).numpy()
    assert got.dtype == want.dtype and np.array_equal(got, want)
    assert np.array_equal(otab.replacement(prompts, tok).numpy(), want)


@pytest.mark.parametrize("i", range(len(M["refine"])))
def test_refinement_mapper(tok, i):
    prompts = M["refine"][i]["prompts"]
    m, a = seq_aligner.get_refinement_mapper(prompts, tok)
    assert np.array_equal(m.numpy(), G[f"refine{i}_mapper"]) and m.dtype == torch.int64
    assert np.array_equal(a.numpy(), G[f"refine{i}_alphas"])
    om, oa = otab.refinement(prompts, tok)
    assert np.array_equal(om.numpy(), G[f"refine{i}_mapper"])
    assert np.array_equal(oa.numpy(), G[f"refine{i}_alphas"])


@pytest.mark.parametrize("i", range(len(M["words"])))
def test_word_inds(tok, i):
    case = M["words"][i]
    got = get_word_inds(case["text"], case["word"], tok)
    assert np.array_equal(got.astype(np.int64), G[f"words{i}"])
    assert np.array_equal(seq_aligner.get_word_inds(case["text"], case["word"], tok).astype(np.int64),
                          G[f"words{i}_sa"])
    assert otab.word_positions(case["text"], case["word"], tok) == list(G[f"words{i}"])


@pytest.mark.parametrize("j", range(len(M["alphas"])))
def test_time_word_alpha(tok, j):
    case = M["alphas"][j]
    form = _form(case["form"])
    arg = dict(form) if isinstance(form, dict) else form
    got = get_time_words_attention_alpha(case["prompts"], case["num_steps"], arg, tok)
    assert np.array_equal(got.numpy(), G[case["key"]])
    arg = dict(form) if isinstance(form, dict) else form
    assert np.array_equal(otab.time_word_alpha(case["prompts"], case["num_steps"], arg, tok).numpy(), G[case["key"]])


@pytest.mark.parametrize("i", range(len(M["eq_main"])))
def test_equalizer_main(tok, i):
    c = M["eq_main"][i]
    words = tuple(c["words"]) if isinstance(c["words"], list) else c["words"]
    got = controllers.get_equalizer(c["text"], words, tuple(c["values"]), tokenizer=tok)
    assert np.array_equal(got.numpy(), G[f"eq_main{i}"])
    assert np.array_equal(otab.equalizer_main(c["text"], words, tuple(c["values"]), tok).numpy(), G[f"eq_main{i}"])


@pytest.mark.parametrize("i", range(len(M["eq_null"])))
def test_equalizer_null(tok, i):
    c = M["eq_null"][i]
    words = tuple(c["words"]) if isinstance(c["words"], list) else c["words"]
    got = null_text.get_equalizer(c["text"], words, tuple(c["values"]), tokenizer=tok)
    assert np.array_equal(got.numpy(), G[f"eq_null{i}"])
    assert np.array_equal(otab.equalizer_null(c["text"], words, tuple(c["values"]), tok).numpy(), G[f"eq_null{i}"])


def test_replacement_rejects_length_mismatch(tok):
    with pytest.raises(ValueError):
        seq_aligner.get_replacement_mapper(["a cat", "a big cat"], tok)


def test_alpha_dict_is_completed_in_place(tok):
    spec = {"cat": 0.5}
    get_time_words_attention_alpha(["a cat", "a dog"], 10, spec, tok)
    assert spec["default_"] == (0., 1.)   # ptp_utils.py:284-285 mutates the caller's dict
