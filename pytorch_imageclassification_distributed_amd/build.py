"""Build the native extension ``_C.so`` in-tree with hipcc for gfx950.

Layout:
* ``csrc/*.hip``      - kernels + ``extern "C"``-free C++ launchers; include only
                        HIP headers, so each TU compiles in seconds;
* ``csrc/bindings.cpp`` - the only TU that includes torch headers: argument
                        checking, allocation through the caching allocator,
                        current-stream lookup, pybind11 module ``_C``.

Objects are cached in ``build/`` by content hash of the source + flags, so an
unchanged kernel file is not recompiled.  The result
``pytorch_imageclassification_distributed_amd/_C.so`` is git-ignored but travels
to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(os.path.dirname(PKG), "build", "objs")
OUT = os.path.join(PKG, "_C.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

KERNEL_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                "-Wno-unused-result", "-D__HIP_PLATFORM_AMD__=1"]


def _torch_flags():
    import torch.utils.cpp_extension as ce
    inc = ce.include_paths(device_type="cuda")
    libs = ce.library_paths(device_type="cuda")
    cflags = ["-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
              "-D_GLIBCXX_USE_CXX11_ABI=1", f"-I{sysconfig.get_paths()['include']}",
              "-Wno-deprecated-declarations", "-Wno-unused-result"]
    cflags += [f"-I{p}" for p in inc]
    ldflags = [f"-L{p}" for p in libs] + [f"-Wl,-rpath,{p}" for p in libs]
    ldflags += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                "-lamdhip64", "-lz"]
    return cflags, ldflags


def _hash(path: str, flags: list[str]) -> str:
    h = hashlib.sha1()
    for f in [path] + sorted(glob.glob(os.path.join(CSRC, "*.h"))):
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _compile(src: str, flags: list[str], verbose: bool) -> str:
    base = os.path.splitext(os.path.basename(src))[0]
    obj = os.path.join(BUILD, f"{base}.{_hash(src, flags)}.o")
    if os.path.exists(obj):
        return obj
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def _check_loadable(path: str) -> None:
    """dlopen the freshly linked module with every symbol bound now: a shared-library link
    tolerates undefined symbols (a binding left pointing at a removed kernel), import does not."""
    code = ("import ctypes, os, torch; ctypes.CDLL(os.path.abspath(%r), mode=os.RTLD_NOW | os.RTLD_GLOBAL)" % path)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    if r.returncode != 0:
        os.remove(path)
        raise RuntimeError(f"linked module does not load:\n{r.stderr[-2000:]}")


def build(verbose: bool = False, jobs: int | None = None, defines: dict | None = None, out: str | None = None) -> str:
    """Compile and link the extension.  ``defines`` {source basename: [-D...]} adds compile-time switches to
    those kernel sources only and ``out`` names another library in the package directory: a variant build
    for a same-box A/B (loaded with IMGCLS_EXT=<name>, _ext.py)."""
    OUT = os.path.join(PKG, out) if out else globals()["OUT"]
    os.makedirs(BUILD, exist_ok=True)
    cflags, ldflags = _torch_flags()
    kernels = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    binds = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    jobs = jobs or min(8, os.cpu_count() or 4)
    defines = defines or {}
    with cf.ThreadPoolExecutor(jobs) as ex:
        # a define keyed "*" applies to every kernel source (the bounds-checked build: '*:-DIMGCLS_BOUNDS_CHECK')
        futs = [ex.submit(_compile, k, KERNEL_FLAGS + defines.get("*", []) + defines.get(os.path.basename(k), []),
                          verbose) for k in kernels]
        futs += [ex.submit(_compile, b, cflags, verbose) for b in binds]
        objs = [f.result() for f in futs]
    key = hashlib.sha1(" ".join(objs).encode()).hexdigest()[:16]
    stamp = OUT + ".stamp"
    if os.path.exists(OUT) and os.path.exists(stamp) and open(stamp).read() == key:
        return OUT
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", OUT + ".tmp"] + objs + ldflags
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
    _check_loadable(OUT + ".tmp")
    os.replace(OUT + ".tmp", OUT)
    with open(stamp, "w") as f:
        f.write(key)
    return OUT


if __name__ == "__main__":
    # python build.py [-v] [--out NAME.so SOURCE.hip:-DFLAG=V ...]  (variant build for an A/B)
    args = [a for a in sys.argv[1:] if a != "-v"]
    out, defs = None, {}
    if args and args[0] == "--out":
        out = args[1]
        for spec in args[2:]:
            src, flag = spec.split(":", 1)
            defs.setdefault(src, []).append(flag)
    print(build(verbose="-v" in sys.argv, defines=defs, out=out))
