"""In-tree build of the native libraries (no JIT cache, no hipify, no torch headers).

* ``csrc/kernels/*.hip``  -> ``rafiki_amd/_native/librafiki_kernels.so``  (hipcc, gfx950 only)
* ``csrc/runtime/*.cpp``  -> ``rafiki_amd/_native/librafiki_runtime.so``  (g++, host-only C++
  runtime: TFRecord reader/CRC32C, shared-memory message queues for inference workers)

Kernels are plain ``extern "C"`` launchers taking raw device pointers and the HIP stream, bound
from Python with ``ctypes`` (``rafiki_amd/ops/_lib.py``).  That keeps each kernel TU a few seconds
to compile and makes the `.so` the single artefact that travels to the GPU box.

Run ``python -m rafiki_amd._build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL_SRC = ROOT / "csrc" / "kernels"
RUNTIME_SRC = ROOT / "csrc" / "runtime"
OBJ_DIR = ROOT / "build" / "obj"
NATIVE_DIR = Path(__file__).resolve().parent / "_native"
KERNEL_LIB = NATIVE_DIR / "librafiki_kernels.so"
RUNTIME_LIB = NATIVE_DIR / "librafiki_runtime.so"
PYEXT_SRC = ROOT / "csrc" / "pyext"
PYLIST_LIB = NATIVE_DIR / "librafiki_pylist.so"

ARCH = os.environ.get("RAFIKI_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
CXX = os.environ.get("CXX", "g++")
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread"]


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(map(str, cmd)), flush=True)
    res = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{res.stdout}\n{res.stderr}")
    return res


def build_kernels(verbose: bool = False, jobs: int | None = None) -> Path:
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    NATIVE_DIR.mkdir(parents=True, exist_ok=True)
    headers = sorted(KERNEL_SRC.glob("*.h"))
    srcs = sorted(KERNEL_SRC.glob("*.hip"))
    if not srcs:
        raise RuntimeError(f"no HIP sources under {KERNEL_SRC}")
    objs, cmds = [], []
    for s in srcs:
        o = OBJ_DIR / (s.stem + ".o")
        objs.append(o)
        if _stale(o, [s, *headers]):
            cmds.append([HIPCC, *HIP_FLAGS, "-c", s, "-o", o])
    n = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=max(1, n)) as ex:
        for f in [ex.submit(_run, c, verbose) for c in cmds]:
            f.result()
    if cmds or _stale(KERNEL_LIB, objs):
        tmp = KERNEL_LIB.with_suffix(".so.tmp")
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp], verbose)
        os.replace(tmp, KERNEL_LIB)
    return KERNEL_LIB


def build_runtime(verbose: bool = False) -> Path | None:
    srcs = sorted(RUNTIME_SRC.glob("*.cpp"))
    if not srcs:
        return None
    NATIVE_DIR.mkdir(parents=True, exist_ok=True)
    headers = sorted(RUNTIME_SRC.glob("*.h"))
    if _stale(RUNTIME_LIB, [*srcs, *headers]):
        tmp = RUNTIME_LIB.with_suffix(".so.tmp")
        _run([CXX, *CXX_FLAGS, "-shared", *srcs, "-o", tmp, "-lrt", "-lpthread"], verbose)
        os.replace(tmp, RUNTIME_LIB)
    return RUNTIME_LIB


def build_pyext(verbose: bool = False) -> Path | None:
    """``csrc/pyext/*.cpp`` -> librafiki_pylist.so: C++ against the CPython headers, loaded with
    ctypes.PyDLL (GIL held), no libpython link (symbols resolve in the host interpreter)."""
    import sysconfig
    srcs = sorted(PYEXT_SRC.glob("*.cpp"))
    if not srcs:
        return None
    NATIVE_DIR.mkdir(parents=True, exist_ok=True)
    if _stale(PYLIST_LIB, srcs):
        tmp = PYLIST_LIB.with_suffix(".so.tmp")
        _run([CXX, *CXX_FLAGS, "-shared", f"-I{sysconfig.get_paths()['include']}", *srcs, "-o", tmp], verbose)
        os.replace(tmp, PYLIST_LIB)
    return PYLIST_LIB


TOOLS_SRC = ROOT / "csrc" / "tools"


def build_tools(verbose: bool = False) -> list:
    """``csrc/tools/*.cpp`` -> executables in ``_native/`` (benchmark load generators)."""
    out = []
    NATIVE_DIR.mkdir(parents=True, exist_ok=True)
    for src in sorted(TOOLS_SRC.glob("*.cpp")):
        exe = NATIVE_DIR / src.stem
        if _stale(exe, [src]):
            tmp = exe.with_suffix(".tmp")
            _run([CXX, *CXX_FLAGS, src, "-o", tmp], verbose)
            os.replace(tmp, exe)
        out.append(exe)
    return out


def build(verbose: bool = False) -> None:
    if shutil.which(HIPCC) is None and not Path(HIPCC).exists():
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    build_kernels(verbose=verbose)
    build_runtime(verbose=verbose)
    build_pyext(verbose=verbose)
    build_tools(verbose=verbose)


if __name__ == "__main__":
    build(verbose="-v" in sys.argv)
    print(f"built {KERNEL_LIB}" + (f" and {RUNTIME_LIB}" if RUNTIME_LIB.exists() else "")
          + (f" and {PYLIST_LIB}" if PYLIST_LIB.exists() else ""))
