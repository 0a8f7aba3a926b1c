#!/usr/bin/env python3
"""Build the native extensions in-tree (no JIT cache, no hipify, gfx950 only).

* ``_dcgan_hip``: the HIP kernel library (csrc/hip/*.hip, hipcc --offload-arch=gfx950) +
  pybind11 bindings of the recorded launch ``Program`` (csrc/bindings.cpp).
* ``_dcgan_host``: host-side C++ runtime -- TFRecord reader/writer (CRC32C), tf.train.Example
  parsing, multi-threaded shuffling loader with a pinned ring buffer (csrc/host/*.cpp).

Objects are cached in build/ keyed by a content hash (sha256 of the compile command and of every
source / header the object depends on, kept in ``<object>.sig``): a stale object survives neither
an edit nor a copied tree with shifted mtimes. ``--force`` rebuilds everything. The .so files land
next to the Python package so they travel with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "distributed_tensorflow_for_dcgan_amd")
BUILD = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("DCGAN_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


FORCE = False  # --force: rebuild every object and library


def _signature(src_list, cmd) -> str:
    h = hashlib.sha256()
    h.update("\0".join(cmd).encode())
    for s in sorted(src_list):
        h.update(b"\0" + os.path.basename(s).encode() + b"\0")
        with open(s, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale(src_list, dst, cmd) -> bool:
    """True when dst must be (re)built: missing, --force, or its recorded content hash differs."""
    sig = _signature(src_list, cmd)
    try:
        with open(dst + ".sig") as f:
            old = f.read().strip()
    except OSError:
        old = ""
    return FORCE or not os.path.exists(dst) or old != sig


def _mark(src_list, dst, cmd) -> None:
    with open(dst + ".sig", "w") as f:
        f.write(_signature(src_list, cmd) + "\n")


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed (%d): %s\n%s" % (r.returncode, " ".join(cmd), r.stdout))
    return r.stdout


VARIANTS = {"bf16": ("", []), "f16": (".f16", ["-DDCG_F16"]), "f32": (".f32", ["-DDCG_F32"])}


def _variants(path: str):
    """Element-type builds of one kernel file from its first line ``// dcg-variants: bf16 f16 f32``
    (bf16 = default symbols, fp16 = ``*_f16``, fp32 = ``*_f32``); files without the line get all."""
    with open(path) as f:
        first = f.readline()
    names = first.split(":", 1)[1].split() if first.startswith("// dcg-variants:") else list(VARIANTS)
    return [VARIANTS[n] for n in names]


_INCLUDE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(path: str, seen=None):
    """The file plus every quoted #include it pulls in, transitively (resolved next to the
    including file, then under csrc/): an edit rebuilds only the objects that see it."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path) as f:
        text = f.read()
    for inc in _INCLUDE.findall(text):
        for base in (os.path.dirname(path), CSRC):
            cand = os.path.normpath(os.path.join(base, inc))
            if os.path.exists(cand):
                _deps(cand, seen)
                break
    return seen


def build_hip(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(os.path.join(CSRC, "hip", f) for f in os.listdir(os.path.join(CSRC, "hip")) if f.endswith(".hip"))
    common = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=%s" % ARCH, "-I", CSRC]
    jobs_list = []  # (cmd, deps, obj)
    objs = []
    for s in srcs:  # every kernel file once per element type it declares (`// dcg-variants:`)
        deps = sorted(_deps(s))
        for tag, defs in _variants(s):
            o = os.path.join(BUILD, os.path.basename(s) + tag + ".o")
            objs.append(o)
            cmd = [HIPCC] + common + defs + ["-c", s, "-o", o]
            if _stale(deps, o, cmd):
                jobs_list.append((cmd, deps, o))
    binding = os.path.join(CSRC, "bindings.cpp")
    bo = os.path.join(BUILD, "bindings.o")
    objs.append(bo)
    inc = []
    for i in _py_includes():
        inc += ["-I", i]
    bcmd = [HIPCC, "-O2", "-fPIC", "-std=c++17", "--offload-arch=%s" % ARCH, "-I", CSRC] + inc + ["-c", binding, "-o", bo]
    bdeps = sorted(_deps(binding))
    if _stale(bdeps, bo, bcmd):
        jobs_list.append((bcmd, bdeps, bo))

    def job(j):
        cmd, deps, o = j
        out = _run(cmd)
        _mark(deps, o, cmd)
        return out

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for out in ex.map(job, jobs_list):
            if verbose and out.strip():
                print(out)
    so = os.path.join(PKG, "_dcgan_hip" + _ext_suffix())
    lcmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=%s" % ARCH] + objs + ["-o", so]
    if _stale(objs, so, lcmd):
        _run(lcmd)
        _mark(objs, so, lcmd)
    return so


def build_host(verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hsrc = os.path.join(CSRC, "host")
    srcs = sorted(os.path.join(hsrc, f) for f in os.listdir(hsrc) if f.endswith(".cpp"))
    hdrs = [os.path.join(hsrc, f) for f in os.listdir(hsrc) if f.endswith(".h")]
    so = os.path.join(PKG, "_dcgan_host" + _ext_suffix())
    if not srcs:
        return ""
    inc = []
    for i in _py_includes():
        inc += ["-I", i]
    flags = ["-O3", "-fPIC", "-std=c++17", "-shared", "-pthread", "-I", hsrc]
    if os.environ.get("DCGAN_HOST_SANITIZE"):
        flags = ["-O1", "-g", "-fPIC", "-std=c++17", "-shared", "-pthread", "-I", hsrc,
                 "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    cmd = ["g++"] + flags + inc + srcs + ["-o", so]
    if _stale(srcs + hdrs, so, cmd):
        _run(cmd)
        _mark(srcs + hdrs, so, cmd)
    return so


def main(argv=None) -> int:
    global FORCE
    argv = sys.argv[1:] if argv is None else argv
    verbose = "-v" in argv
    FORCE = "--force" in argv
    built = []
    if "--host-only" not in argv:
        built.append(build_hip(verbose))
    if "--hip-only" not in argv:
        h = build_host(verbose)
        if h:
            built.append(h)
    for b in built:
        print("built", os.path.relpath(b, ROOT))
    return 0


if __name__ == "__main__":
    sys.exit(main())
