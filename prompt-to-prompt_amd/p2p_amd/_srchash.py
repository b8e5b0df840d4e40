"""Content hash of the HIP sources that libp2p_hip.so is built from.

The Makefile stamps this value into the library (``p2p_source_hash()``); ``_hip.check_source_hash``
recomputes it from the tree at run time, so a stale prebuilt binary (the .so is git-ignored and
travels to the GPU box as a file) cannot pass ``smoke()`` or the GPU tests.
Run as a script it prints the hash (the Makefile's ``$(shell ...)``).
"""
import hashlib
import os

_CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
# every file whose text reaches the compiler or the link line, in a fixed order
FILES = ("p2p_attn.hip", "p2p_self40.hip", "p2p_selfsplit.hip", "p2p_cross.hip", "p2p_bwd.hip", "p2p_blend.hip", "p2p_capi.hip", "p2p_device.h", "p2p_kernels.h",
         "../../include/p2p_hip.h", "Makefile")


def source_hash() -> str:
    h = hashlib.sha256()
    for name in FILES:
        with open(os.path.join(_CSRC, name), "rb") as f:
            h.update(name.encode())
            h.update(b"\0")
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())
