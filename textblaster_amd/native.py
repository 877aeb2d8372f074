"""Native components: build and load.

* ``_tbhost`` — pybind11 extension (g++): text primitives, the CPU pipeline, batch resolver,
  output assembly, HTML decoding, device-plan building and the host emulation of the device
  algorithms. Links ICU4C (the segmentation oracle).
* ``libtbhip.so`` — HIP kernels for gfx950 (hipcc), C ABI, loaded with ctypes, plus the native
  HIP runtime layer (csrc/hip/runtime.hip: caching device / pinned allocators, streams, events,
  scans) that owns device memory and streams; PyTorch is only used for torch.distributed.

Both are built in-tree (``textblaster_amd/``) so they travel with the repository snapshot.
"""
from __future__ import annotations

import ctypes
import json
import os
import re
import subprocess
import sys
import sysconfig
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO_DIR, "csrc")
BUILD_DIR = os.path.join(REPO_DIR, "build")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX")
HOST_EXT = os.path.join(PKG_DIR, "_tbhost" + EXT_SUFFIX)
HIP_LIB = os.path.join(PKG_DIR, "libtbhip.so")
# A/B experiments: TB_HIP_LIB points at an alternative build of the kernels (tools/build_variant.sh)
_HIP_LIB_OVERRIDE = os.environ.get("TB_HIP_LIB")
GPU_ARCH = os.environ.get("TB_GPU_ARCH", "gfx950")

_lock = threading.Lock()
_host = None
_hip = None


def _sources(sub: str, ext: str) -> List[str]:
    d = os.path.join(CSRC, sub)
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(ext))


def _headers() -> List[str]:
    out = []
    for sub in ("common", "host", "hip"):
        d = os.path.join(CSRC, sub)
        if os.path.isdir(d):
            out += [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".inc"))]
    return out


def _newest(paths: List[str]) -> float:
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _run(cmd: List[str], verbose: bool) -> str:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


RESOURCES_JSON = os.path.join(BUILD_DIR, "hip", "kernel_resources.json")


def parse_resource_remarks(text: str) -> dict:
    """Per-kernel resources from hipcc's -Rpass-analysis=kernel-resource-usage remarks:
    {mangled name: {"VGPRs": .., "VGPRs Spill": .., "ScratchSize [bytes/lane]": .., "Occupancy
    [waves/SIMD]": .., ...}}."""
    out: dict = {}
    cur = None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z][^:]*): (\d+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return out


def build_host(verbose: bool = False, force: bool = False) -> str:
    import pybind11

    srcs = _sources("host", ".cpp")
    hdrs = _headers()
    if (not force and os.path.exists(HOST_EXT)
            and os.path.getmtime(HOST_EXT) >= _newest(srcs + hdrs)):
        return HOST_EXT
    os.makedirs(os.path.join(BUILD_DIR, "host"), exist_ok=True)
    inc = ["-I" + sysconfig.get_paths()["include"], "-I" + pybind11.get_include()]
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
             "-march=x86-64-v2"]
    objs = []

    def compile_one(src: str) -> str:
        obj = os.path.join(BUILD_DIR, "host", os.path.basename(src) + ".o")
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < _newest([src] + hdrs):
            _run(["g++", *flags, *inc, "-c", src, "-o", obj], verbose)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = HOST_EXT + ".tmp"
    _run(["g++", "-shared", "-o", tmp, *objs, "-licuuc", "-lpthread"], verbose)
    os.replace(tmp, HOST_EXT)
    return HOST_EXT


def hipcc_path() -> Optional[str]:
    for p in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if p and os.path.exists(p):
            return p
    return None


def build_hip(verbose: bool = False, force: bool = False) -> str:
    hipcc = hipcc_path()
    if hipcc is None:
        raise RuntimeError("hipcc not found (ROCm required to build the device library)")
    srcs = _sources("hip", ".hip")
    hdrs = _headers()
    if (not force and os.path.exists(HIP_LIB)
            and os.path.getmtime(HIP_LIB) >= _newest(srcs + hdrs)):
        return HIP_LIB
    os.makedirs(os.path.join(BUILD_DIR, "hip"), exist_ok=True)
    # no -ffast-math: the language-id decision (langid.h: explicit-fma exp, IEEE f64 division) and
    # the exact integer / bf16 MFMA paths must match the host bit for bit
    # (constexpr-steps: the word-break pair table of uax29.h is generated at compile time)
    flags = [f"--offload-arch={GPU_ARCH}", "-O3", "-std=c++17", "-fPIC", "-fno-gpu-rdc", "-fconstexpr-steps=200000000"]
    objs = []

    def compile_one(src: str) -> str:
        obj = os.path.join(BUILD_DIR, "hip", os.path.basename(src) + ".o")
        rep = obj + ".resources.json"
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < _newest([src] + hdrs):
            # the compiler's per-kernel register / spill / occupancy report comes with the build
            # (tests/test_kernel_resources.py checks it against csrc/hip/resource_budget.json)
            log = _run([hipcc, *flags, "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", obj], False)
            if verbose:
                print(f"{os.path.basename(src)}: built", flush=True)
            with open(rep, "w") as f:
                json.dump(parse_resource_remarks(log), f, indent=1, sort_keys=True)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    merged: dict = {}
    for o in objs:
        try:
            with open(o + ".resources.json") as f:
                merged.update(json.load(f))
        except OSError:
            pass
    with open(RESOURCES_JSON, "w") as f:
        json.dump(merged, f, indent=1, sort_keys=True)
    tmp = HIP_LIB + ".tmp"
    _run([hipcc, f"--offload-arch={GPU_ARCH}", "-shared", "-fPIC", "-o", tmp, *objs], verbose)
    os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_all(verbose: bool = False) -> None:
    build_host(verbose)
    build_hip(verbose)


def host():
    """The host extension module (built on first use if missing)."""
    global _host
    if _host is None:
        with _lock:
            if _host is None:
                if not os.path.exists(HOST_EXT):
                    build_host()
                from . import _tbhost  # type: ignore

                _host = _tbhost
    return _host


def hip() -> ctypes.CDLL:
    """The HIP kernel library (fails loudly if missing: the GPU path never silently falls back)."""
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                path = _HIP_LIB_OVERRIDE or HIP_LIB
                if not _HIP_LIB_OVERRIDE and not os.path.exists(HIP_LIB):
                    build_hip()
                _hip = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
                _declare_hip(_hip)
    return _hip


def _declare_hip(lib: ctypes.CDLL) -> None:
    from .ops import kernels

    kernels.declare(lib)


if __name__ == "__main__":  # python -m textblaster_amd.native [host|hip|all]
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("host", "all"):
        print(build_host(verbose=True, force="--force" in sys.argv))
    if what in ("hip", "all"):
        print(build_hip(verbose=True, force="--force" in sys.argv))
