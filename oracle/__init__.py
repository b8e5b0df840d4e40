"""ORACLE -- CPU restatement of the reference's attention-control path.

TEST INFRASTRUCTURE ONLY.  Imported solely by ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg, always as the checker / baseline, never as the product
path.  The product (``prompt-to-prompt_amd/p2p_amd``) never imports it.

What it restates (each function cites the reference file:line it follows):
* ``tables``  -- seq_aligner.py / ptp_utils.py / main.py / null_text.py host tables, in pure
                 Python loops (integer/byte work, small cases);
* ``control`` -- the controllers' edit / store / LocalBlend semantics on materialised fp32
                 probability tensors (torch CPU), and the DDIM step;
* ``forward`` -- the patched CrossAttention.forward of ptp_utils.py:183-208 as plain fp32
                 torch on CPU, and a hook that installs it.

Pinning: every piece is checked against the golden vectors in ``tests/golden`` that
``tools/gen_golden.py`` produced by running the reference code itself in the build container
(tables bit-exact; controller outputs / patched forward / LocalBlend / DDIM on the reference's
own tensors).  The U-Net, DDIM beta schedule and CLIP tokenizer are external to the reference
(diffusers / transformers) -- those parts are parity unpinned, see DESIGN.md §6.
"""
