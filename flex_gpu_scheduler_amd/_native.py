"""Loader for the in-tree native extensions.

The C++ core (`_xsched`) is mandatory: there is no Python fallback for the
scheduling path, so a missing build fails loudly with the command to run.
"""
from __future__ import annotations

import importlib

_mod = None


def native():
    global _mod
    if _mod is None:
        try:
            _mod = importlib.import_module("flex_gpu_scheduler_amd._xsched")
        except ImportError as e:  # pragma: no cover - exercised only on broken installs
            raise ImportError(
                "native core flex_gpu_scheduler_amd/_xsched*.so is not built; run "
                "`python -m flex_gpu_scheduler_amd.build_ext` (or __graft_entry__.build())"
            ) from e
    return _mod
