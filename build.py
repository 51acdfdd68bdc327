#!/usr/bin/env python3
"""Build the deepspeech_amd native extension in-tree for gfx950.

Explicit hipcc invocations (no hipify, no setuptools CUDA shim):
  * every ``deepspeech_amd/csrc/*.hip`` -> object with ``--offload-arch=gfx950``
  * ``deepspeech_amd/csrc/bindings.cpp`` (torch/pybind11 glue, host only) -> object
  * link -> ``deepspeech_amd/_C<EXT_SUFFIX>`` next to the package (travels with gpurun)
  * ``deepspeech_amd/runtime/*.cpp`` (native host runtime: loader, beam search,
    TFRecord codec) -> ``deepspeech_amd/runtime/_native<EXT_SUFFIX>``

Objects are cached under build/ keyed by a hash of (source, included headers, flags),
so a no-op rebuild takes well under a second. ``python build.py --force`` rebuilds all.

Same-box A/B of a compile-time change: ``python build.py --variant NAME -D SYMBOL`` links
``ab/_C_NAME<EXT_SUFFIX>`` with the extra defines (the in-tree ``_C`` is left alone) and
``DS2_EXT_SO=ab/_C_NAME...so`` makes a process load it instead (``scripts/ab_so.sh``).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "deepspeech_amd")
CSRC = os.path.join(PKG, "csrc")
RTSRC = os.path.join(PKG, "runtime")
BUILD = os.path.join(ROOT, "build")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hash(paths, flags) -> str:
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed (%d): %s\n%s" % (r.returncode, " ".join(cmd), r.stdout))
    return r.stdout


def _local_deps(src, seen=None):
    """csrc files reached through #include "..." from ``src`` (transitively): an object is
    rebuilt only when one of the files it actually includes changes."""
    import re
    seen = set() if seen is None else seen
    with open(src, "r", errors="replace") as f:
        text = f.read()
    for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
        p = os.path.join(os.path.dirname(src), name)
        if os.path.exists(p) and p not in seen:
            seen.add(p)
            _local_deps(p, seen)
    return sorted(seen)


def _compile(src, obj_dir, flags, deps):
    stem = os.path.splitext(os.path.basename(src))[0]
    key = _hash([src] + deps, flags)
    obj = os.path.join(obj_dir, "%s.%s.o" % (stem, key))
    if not os.path.exists(obj):
        tmp = obj + ".tmp.o"
        _run(flags[:1] + ["-c", src, "-o", tmp] + flags[1:])
        os.replace(tmp, obj)
    return obj


def build(force: bool = False, verbose: bool = False, jobs: int = 0, defines=(), variant: str = "") -> str:
    inc, torch_lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    os.makedirs(BUILD, exist_ok=True)
    if force:
        for f in os.listdir(BUILD):
            if f.endswith(".o"):
                os.remove(os.path.join(BUILD, f))
    hip_srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    common = ["-O3", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-I" + CSRC]
    if os.environ.get("DS2_DEBUG", "0") == "1":
        # device-side DS2_DCHECKs (csrc/common.h) print failing conditions; objects are keyed
        # by their flags, so debug and release objects coexist in build/
        common += ["-DDS2_DEBUG=1", "-g"]
    common += ["-D" + d for d in defines]
    hip_flags = [HIPCC, "--offload-arch=" + ARCH, "-fno-gpu-rdc", "-munsafe-fp-atomics"] + common
    torch_defs = ["-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1",
                  "-D_GLIBCXX_USE_CXX11_ABI=%d" % abi]
    bind_flags = [HIPCC, "-x", "c++"] + common + torch_defs + ["-I" + p for p in inc] + [
        "-I" + py_inc, "-I" + os.path.join(ROCM, "include"), "-Wno-unused-result", "-Wno-deprecated-declarations"]
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, BUILD, hip_flags, _local_deps(s)) for s in hip_srcs]
        futs.append(ex.submit(_compile, os.path.join(CSRC, "bindings.cpp"), BUILD, bind_flags, []))
        objs = [f.result() for f in futs]
    out = os.path.join(PKG, "_C" + EXT)
    stamp = os.path.join(BUILD, "_C.link")
    if variant:
        os.makedirs(os.path.join(ROOT, "ab"), exist_ok=True)
        out = os.path.join(ROOT, "ab", "_C_%s%s" % (variant, EXT))
        stamp = os.path.join(BUILD, "_C_%s.link" % variant)
    link_key = _hash(objs, [ARCH])
    if force or not os.path.exists(out) or not os.path.exists(stamp) or open(stamp).read() != link_key:
        tmp = out + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", tmp] + objs + [
            "-L" + torch_lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-Wl,-rpath," + torch_lib])
        os.replace(tmp, out)
        with open(stamp, "w") as f:
            f.write(link_key)
    if verbose:
        print("built", out)
    if not variant:
        build_runtime(verbose=verbose)
    return out


def build_runtime(verbose: bool = False) -> str:
    """Native host runtime (pure C++/pybind11; no GPU code)."""
    import pybind11
    srcs = sorted(os.path.join(RTSRC, f) for f in os.listdir(RTSRC) if f.endswith(".cpp"))
    if not srcs:
        return ""
    hdrs = sorted(os.path.join(RTSRC, f) for f in os.listdir(RTSRC) if f.endswith(".h"))
    py_inc = sysconfig.get_paths()["include"]
    cxx = shutil.which("g++") or "c++"
    flags = [cxx, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-I" + RTSRC,
             "-I" + pybind11.get_include(), "-I" + py_inc, "-pthread"]
    objs = [_compile(s, BUILD, flags, hdrs) for s in srcs]
    out = os.path.join(RTSRC, "_native" + EXT)
    key = _hash(objs, ["rt"])
    stamp = os.path.join(BUILD, "_native.link")
    if not os.path.exists(out) or not os.path.exists(stamp) or open(stamp).read() != key:
        tmp = out + ".tmp"
        _run([cxx, "-shared", "-fPIC", "-pthread", "-o", tmp] + objs)
        os.replace(tmp, out)
        with open(stamp, "w") as f:
            f.write(key)
    if verbose:
        print("built", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--variant", default="", help="link ab/_C_<variant> instead of the in-tree _C")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra -D for a variant")
    a = ap.parse_args()
    if a.defines and not a.variant:
        ap.error("-D needs --variant (the in-tree _C is always the default build)")
    try:
        build(force=a.force, verbose=True, jobs=a.jobs, defines=a.defines, variant=a.variant)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
