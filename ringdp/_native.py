"""Loader for the native extension ``ringdp._C`` (built in-tree by ``ringdp/_build.py``).

The extension is required: ringdp's stores, process groups, reducer and every GPU op live in it.
There is no pure-Python fallback - if it is missing we fail loudly with the build command.
Set ``RINGDP_AUTOBUILD=1`` to compile it on first import instead.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

import torch  # noqa: F401  (loads libtorch / the bundled HIP runtime before our .so)

_C = None


def load():
    global _C
    if _C is not None:
        return _C
    alt = os.environ.get("RINGDP_EXT_PATH")
    if alt:
        # an alternative build of the same extension (e.g. the ASan host build, tools/asan_check.sh)
        spec = importlib.util.spec_from_file_location("ringdp._C", alt)
        _C = importlib.util.module_from_spec(spec)
        sys.modules["ringdp._C"] = _C
        spec.loader.exec_module(_C)
        return _C
    try:
        _C = importlib.import_module("ringdp._C")
    except ImportError as e:
        if os.environ.get("RINGDP_AUTOBUILD", "0") == "1":
            from . import _build

            _build.build(verbose=True)
            _C = importlib.import_module("ringdp._C")
        else:
            raise ImportError(
                "ringdp native extension (ringdp/_C*.so) is not built: run "
                "`python __graft_entry__.py build` (or set RINGDP_AUTOBUILD=1)"
            ) from e
    return _C


C = load()
