"""Loader for the native host runtime ``deepspeech_amd.runtime._native`` (C++/pybind11).

Contents: bucketed SortaGrad batch planner + threaded mmap batch loader (loader.cpp),
TFRecord / SequenceExample codec (tfrecord.cpp), greedy + prefix-beam CTC decoding and
edit distance (decoder.cpp). Built by ``python build.py``.
"""
from __future__ import annotations

import importlib

_mod = None


def load():
    global _mod
    if _mod is None:
        try:
            _mod = importlib.import_module("deepspeech_amd.runtime._native")
        except ImportError as e:
            raise RuntimeError("native runtime not built: run `python build.py` (%s)" % e)
    return _mod


def available() -> bool:
    try:
        load()
        return True
    except RuntimeError:
        return False
