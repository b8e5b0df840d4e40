import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "prompt-to-prompt_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# MIOpen's default find mode benchmarks every convolution solver (naive ones included) the first
# time a shape is seen -- on a fresh GPU box that is minutes per U-Net batch size and dtype.  The
# tests compare product and oracle runs of the SAME U-Net in one process, so which solver MIOpen
# picks does not matter to them; FAST picks one from its heuristics at once.  (bench.py keeps the
# default: its warmup groups absorb the search.)
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def golden(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)


def golden_json(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def tok():
    from p2p_amd.tokenizer import StandInTokenizer
    return StandInTokenizer()


@pytest.fixture(scope="session")
def cuda():
    """Every -m gpu test takes this fixture.  No visible GPU is a FAILURE, not a skip: a GPU run
    whose device vanished must not exit 0 (the CPU suite deselects these tests with -m "not gpu")."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible to a -m gpu test (torch.cuda.is_available() is False)")
    from p2p_amd import _hip
    _hip.lib()
    _hip.check_source_hash()     # the loaded libp2p_hip.so was built from THIS tree
    return torch.device("cuda:0")
