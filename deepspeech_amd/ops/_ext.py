"""Loader for the in-tree gfx950 extension ``deepspeech_amd._C``.

Policy: the HIP engine never silently falls back to PyTorch. If a GPU is present and the
extension is missing or stale, :func:`ext` raises with the build command. Set
``DS2_AUTOBUILD=1`` to build on first use (hipcc cross-compiles for gfx950 anywhere).
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import threading

_lock = threading.Lock()
_mod = None
_err = None


def _try_import():
    path = os.environ.get("DS2_EXT_SO")
    if path:
        # same-box A/B of a compile-time variant (build.py --variant): load that file as _C
        import sys
        spec = importlib.util.spec_from_file_location("deepspeech_amd._C", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules["deepspeech_amd._C"] = mod
        return mod
    return importlib.import_module("deepspeech_amd._C")


def ext():
    """Return the loaded extension module (raise loudly if unavailable)."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            _mod = _try_import()
            return _mod
        except ImportError as e:  # pragma: no cover - depends on build state
            _err = e
        if os.environ.get("DS2_AUTOBUILD", "0") == "1":
            import sys
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            sys.path.insert(0, root)
            import build as _build  # type: ignore
            _build.build()
            _mod = _try_import()
            return _mod
        raise RuntimeError(
            "deepspeech_amd._C (gfx950 kernels) is not built: run `python build.py` in the repo "
            "root (import error: %s)" % (_err,))


def available() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False


_dev_info = {}


def device_info(device_index: int = 0) -> dict:
    if device_index not in _dev_info:
        _dev_info[device_index] = ext().device_info(device_index)
    return _dev_info[device_index]


def num_cus(device_index: int = 0) -> int:
    env = os.environ.get("DS2_NUM_CUS")
    if env:
        return int(env)
    return int(device_info(device_index)["cus"])
