"""In-tree build of the native library ``_pz_C.so`` (gfx950 HIP kernels + host C++ runtime).

Usage: ``python -m penr_oz_neural_network_torch_amd._build [--force] [-j N]``

* ``*.hip`` → ``hipcc --offload-arch=gfx950 -O3`` (device code, no torch headers: fast compiles)
* ``*.cpp`` → ``g++ -O3`` with the torch / ROCm include paths (operator bindings, JSON formatter)
* link  → ``hipcc -shared`` against libtorch / libc10_hip

Freshness is keyed on CONTENT, not mtimes: every object records the SHA-256 of its source, every
header and its compile command; the ``.so`` records the digest of all of them
(``build/manifest.json``). A stale object whose mtime happens to be newer is still rebuilt, and an
up-to-date ``.so`` needs no objects at all (they need not travel with the tree). The ``.so`` lands
next to this file so it travels with the repository snapshot (``gpurun``) and is the one the GPU
tests load. No hipify, no ``torch.utils.cpp_extension`` JIT cache.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "build")
OUT = os.path.join(PKG, "_pz_C.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _torch_paths():
    import torch
    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    return inc, os.path.join(root, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc() -> str:
    return shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")


MANIFEST = os.path.join(BUILD, "manifest.json")


def _digest(paths, extra: str = "") -> str:
    h = hashlib.sha256(extra.encode())
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _headers_digest() -> str:
    return _digest(sorted(glob.glob(os.path.join(CSRC, "*.h"))))


def _load_manifest() -> dict:
    try:
        with open(MANIFEST) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _compile_cmd(src: str, obj: str) -> list:
    if src.endswith(".hip"):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
               "-I", CSRC, "-ffp-contract=fast", "-Wno-unused-result"]
    else:
        inc, _, abi = _torch_paths()
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj, "-I", CSRC,
               "-I", os.path.join(ROCM, "include"), "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
               f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_pz_C", "-Wno-deprecated-declarations"]
        for i in inc:
            cmd += ["-isystem", i]
        cmd += ["-isystem", sysconfig.get_paths()["include"]]
    return cmd


def _object_key(src: str, hdr: str) -> str:
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    return _digest([src], hdr + " ".join(_compile_cmd(src, obj)))


def _compile(src: str, key: str, manifest: dict, force: bool) -> str:
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    name = os.path.basename(obj)
    if not force and os.path.exists(obj) and manifest.get("objects", {}).get(name) == key:
        return obj
    cmd = _compile_cmd(src, obj)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return obj


def _sources_and_keys():
    sources = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    hdr = _headers_digest()
    keys = {s: _object_key(s, hdr) for s in sources}
    return sources, keys, hashlib.sha256("".join(keys[s] for s in sources).encode()).hexdigest()


def is_fresh() -> bool:
    """True when the in-tree library was linked from exactly the current sources, headers and
    compile commands (content hashes, not mtimes)."""
    return os.path.exists(OUT) and _load_manifest().get("library") == _sources_and_keys()[2]


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    sources, keys, lib_key = _sources_and_keys()
    manifest = _load_manifest()
    if not force and os.path.exists(OUT) and manifest.get("library") == lib_key:
        if verbose:
            print(f"[pz build] up to date: {OUT}")
        return OUT
    jobs = jobs or min(len(sources), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, keys[s], manifest, force), sources))
    manifest["objects"] = {os.path.basename(s) + ".o": keys[s] for s in sources}
    manifest.pop("library", None)
    _, libdir, _ = _torch_paths()
    tmp = OUT + ".tmp"
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp, "-L", libdir,
           "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", f"-Wl,-rpath,{libdir}"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, OUT)
    manifest["library"] = lib_key
    with open(MANIFEST + ".tmp", "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    os.replace(MANIFEST + ".tmp", MANIFEST)
    if verbose:
        print(f"[pz build] built {OUT}")
    return OUT


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    args = ap.parse_args(argv)
    build(force=args.force, jobs=args.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
