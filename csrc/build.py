#!/usr/bin/env python3
"""Build the native extensions in-tree (no JIT cache, no hipify, gfx950 only).

* ``_dcgan_hip``: the HIP kernel library (csrc/hip/*.hip, hipcc --offload-arch=gfx950) +
  pybind11 bindings of the recorded launch ``Program`` (csrc/bindings.cpp).
* ``_dcgan_host``: host-side C++ runtime -- TFRecord reader/writer (CRC32C), tf.train.Example
  parsing, multi-threaded shuffling loader with a pinned ring buffer (csrc/host/*.cpp).

Objects are cached in build/ keyed by source mtime; the .so files land next to the Python
package so they travel with the repository snapshot to the GPU box.
"""
from __future__ import annotations

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


def _newer(src_list, dst) -> bool:
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(s) > t for s in src_list)


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
    jobs_list = []
    objs = []
    for s in srcs:  # every kernel file once per element type it declares (`// dcg-variants:`)
        deps = sorted(_deps(s))
        for tag, defs in _variants(s):
            o = os.path.join(BUILD, os.path.basename(s) + tag + ".o")
            objs.append(o)
            if _newer(deps, o):
                jobs_list.append([HIPCC] + common + defs + ["-c", s, "-o", o])
    binding = os.path.join(CSRC, "bindings.cpp")
    bo = os.path.join(BUILD, "bindings.o")
    objs.append(bo)
    if _newer(sorted(_deps(binding)), bo):
        inc = []
        for i in _py_includes():
            inc += ["-I", i]
        jobs_list.append([HIPCC, "-O2", "-fPIC", "-std=c++17", "--offload-arch=%s" % ARCH, "-I", CSRC] + inc +
                         ["-c", binding, "-o", bo])
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out.strip():
                print(out)
    so = os.path.join(PKG, "_dcgan_hip" + _ext_suffix())
    if _newer(objs, so):
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=%s" % ARCH] + objs + ["-o", so])
    return so


def build_host(verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hsrc = os.path.join(CSRC, "host")
    srcs = sorted(os.path.join(hsrc, f) for f in os.listdir(hsrc) if f.endswith(".cpp"))
    hdrs = [os.path.join(hsrc, f) for f in os.listdir(hsrc) if f.endswith(".h")]
    so = os.path.join(PKG, "_dcgan_host" + _ext_suffix())
    if not srcs:
        return ""
    if _newer(srcs + hdrs, so):
        inc = []
        for i in _py_includes():
            inc += ["-I", i]
        flags = ["-O3", "-fPIC", "-std=c++17", "-shared", "-pthread", "-I", hsrc]
        if os.environ.get("DCGAN_HOST_SANITIZE"):
            flags = ["-O1", "-g", "-fPIC", "-std=c++17", "-shared", "-pthread", "-I", hsrc,
                     "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
        _run(["g++"] + flags + inc + srcs + ["-o", so])
    return so


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    verbose = "-v" in argv
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
