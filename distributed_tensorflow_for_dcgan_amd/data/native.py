"""Loader for the host C++ runtime (``_dcgan_host``: TFRecord, Example, shuffling loader).

Built in-tree by ``csrc/build.py``; if the shared object is missing (fresh checkout, CPU test
run) it is compiled on first use with g++ (a few seconds)."""
from __future__ import annotations

import importlib
import threading

_EXT = None
_LOCK = threading.Lock()


def ext():
    global _EXT
    if _EXT is not None:
        return _EXT
    with _LOCK:
        if _EXT is None:
            try:
                _EXT = importlib.import_module("distributed_tensorflow_for_dcgan_amd._dcgan_host")
            except ImportError:
                import os
                import sys
                root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
                sys.path.insert(0, os.path.join(root, "csrc"))
                try:
                    import build as _b  # csrc/build.py
                finally:
                    sys.path.pop(0)
                _b.build_host()
                _EXT = importlib.import_module("distributed_tensorflow_for_dcgan_amd._dcgan_host")
    return _EXT


def crc32c(data: bytes, crc: int = 0) -> int:
    return ext().crc32c(data, crc)
