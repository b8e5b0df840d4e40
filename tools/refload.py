"""Load the reference implementation from /root/reference for golden-vector generation.

TEST INFRASTRUCTURE ONLY.  Used by ``tools/gen_golden.py`` in the build container; the
reference never leaves that container and nothing here runs on the GPU box.

* ``seq_aligner`` imports as-is.
* ``ptp_utils`` imports once two display-only modules are stubbed (``cv2``,
  ``IPython.display``; used only by ``text_under_image``/``view_images``,
  ``ptp_utils.py:17-62``).
* ``main.py`` / ``null_text.py`` load a diffusers pipeline at import time
  (``main.py:29``, ``null_text.py:28-31``), so their classes are taken by AST
  extraction: only imports (minus diffusers/tqdm), ``ClassDef`` and ``FunctionDef``
  nodes are executed, in a namespace pre-seeded with the module constants.
"""
from __future__ import annotations

import ast
import sys
import types

REF = "/root/reference"


def _stub_display_modules():
    if "cv2" not in sys.modules:
        sys.modules["cv2"] = types.ModuleType("cv2")
    if "IPython.display" not in sys.modules:
        ip = types.ModuleType("IPython")
        ipd = types.ModuleType("IPython.display")
        ipd.display = lambda *a, **k: None
        ip.display = ipd
        sys.modules["IPython"] = ip
        sys.modules["IPython.display"] = ipd


def load_ref_modules():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    _stub_display_modules()
    import ptp_utils as ref_ptp  # noqa: E402
    import seq_aligner as ref_sa  # noqa: E402
    return ref_ptp, ref_sa


def load_script_classes(filename: str, tokenizer, device="cpu", extra_globals=None):
    """Execute only the class/function definitions of a reference script."""
    import torch
    ref_ptp, ref_sa = load_ref_modules()
    with open(f"{REF}/{filename}") as f:
        tree = ast.parse(f.read(), filename=filename)
    keep = []
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            mod = getattr(node, "module", None) or ""
            names = [a.name for a in node.names]
            if "diffusers" in mod or "tqdm" in mod or any("diffusers" in n for n in names):
                continue
            keep.append(node)
        elif isinstance(node, (ast.ClassDef, ast.FunctionDef)):
            keep.append(node)
    module = ast.Module(body=keep, type_ignores=[])
    ns = {
        "__name__": f"ref_{filename.replace('.py', '')}",
        "LOW_RESOURCE": False,
        "NUM_DIFFUSION_STEPS": 100,
        "NUM_DDIM_STEPS": 50,
        "GUIDANCE_SCALE": 7.5,
        "MAX_NUM_WORDS": 77,
        "device": torch.device(device),
        "tokenizer": tokenizer,
        "ptp_utils": ref_ptp,
        "seq_aligner": ref_sa,
        "tqdm": lambda *a, **k: None,
    }
    if extra_globals:
        ns.update(extra_globals)
    exec(compile(module, f"{REF}/{filename}", "exec"), ns)
    return ns
