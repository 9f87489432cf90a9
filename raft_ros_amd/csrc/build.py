"""In-tree build of the raft_ros_amd native extension (``raft_ros_amd/_C.so``).

Every ``*.hip`` translation unit is compiled by ``hipcc --offload-arch=gfx950``
(device code for MI355X only; no hipify step, no CUDA sources) and the
dispatcher bindings (``bindings.cpp``) are compiled as host C++ against the
installed PyTorch-ROCm headers.  Objects are cached by mtime under
``raft_ros_amd/csrc/_build`` and compiled in parallel.

Usage::

    python -m raft_ros_amd.csrc.build          # incremental
    python -m raft_ros_amd.csrc.build --clean  # full rebuild

The reference builds its single CUDA extension with setuptools/nvcc
(alt_cuda_corr/setup.py:5-14); this replaces it.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

CSRC = Path(__file__).resolve().parent
PKG = CSRC.parent
BUILD = CSRC / "_build"
TARGET = PKG / "_C.so"
ARCH = os.environ.get("RAFT_AMD_ARCH", "gfx950")


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = Path(rocm) / "bin" / "hipcc"
    return str(cand) if cand.exists() else "hipcc"


def _torch_paths():
    import torch

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    lib = root / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _common_flags():
    inc, _, abi = _torch_paths()
    flags = [
        "-O3",
        "-fPIC",
        "-std=c++17",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        f"-I{CSRC}",
    ]
    return flags, inc


def _sources():
    hips = sorted(CSRC.glob("*.hip"))
    cpps = sorted(CSRC.glob("*.cpp"))
    return hips, cpps


def _needs(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    deps = [src] + sorted(CSRC.glob("*.h"))
    return any(d.stat().st_mtime > obj.stat().st_mtime for d in deps)


def _compile(cmd):
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")
    return cmd[-1]


def build(clean: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    flags, torch_inc = _common_flags()
    py_inc = sysconfig.get_paths()["include"]
    hips, cpps = _sources()
    cmds = []
    objs = []
    for src in hips:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if _needs(obj, src):
            # device TUs include only hip_runtime: fast compiles, no torch headers
            cmds.append([hipcc, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *flags, "-x", "hip",
                         "-c", str(src), "-o", str(obj)])
    for src in cpps:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if _needs(obj, src):
            incs = [f"-I{p}" for p in torch_inc] + [f"-I{py_inc}"]
            cmds.append([hipcc, *flags, *incs, "-c", str(src), "-o", str(obj)])
    jobs = jobs or min(8, os.cpu_count() or 4)
    if cmds:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for done in ex.map(_compile, cmds):
                if verbose:
                    print("compiled", done)
    relink = cmds or not TARGET.exists() or any(o.stat().st_mtime > TARGET.stat().st_mtime for o in objs)
    if relink:
        _, tlib, _ = _torch_paths()
        # link to a temporary name and rename: a process (or a repo snapshot) that reads the
        # library meanwhile sees the old or the new file, never a partial one
        tmp = TARGET.with_name(TARGET.name + ".tmp")
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp),
                f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
                f"-Wl,-rpath,{tlib}"]
        _compile(link)
        os.replace(tmp, TARGET)
        if verbose:
            print("linked", TARGET)
    return TARGET


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args(argv)
    path = build(clean=args.clean, jobs=args.jobs, verbose=args.verbose)
    print(path)


if __name__ == "__main__":
    sys.exit(main())
