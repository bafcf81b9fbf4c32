"""In-tree native build for serverless_learn_amd.

Two artefacts, both written into ``serverless_learn_amd/_native/`` so they
travel with the repo snapshot to the GPU box (a JIT cache would not):

* ``libslkernels.so`` -- every HIP kernel under ``csrc/kernels`` compiled for
  gfx950 with ``hipcc --offload-arch=gfx950`` and exposed through a plain C ABI
  (loaded with ctypes by :mod:`serverless_learn_amd.ops._native`).
* ``_slcore.so`` -- the C++ runtime (wire codec, membership registry, pinned
  ingest ring, shard generator) as a pybind11 module.

The reference builds its three binaries with a 44-line Makefile driving
protoc + g++ (/root/reference/src/Makefile:1-44); there is no protoc/gRPC-C++
in this image, so the wire layer is descriptor-built in Python and the hot
codecs are hand-written C++.

Usage: ``python -m serverless_learn_amd.build [--force] [--only kernels|core]``
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE_DIR = os.path.join(ROOT, "serverless_learn_amd", "_native")
KERNEL_DIR = os.path.join(ROOT, "csrc", "kernels")
CORE_DIR = os.path.join(ROOT, "csrc", "core")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("SL_OFFLOAD_ARCH", "gfx950")

KERNELS_SO = os.path.join(NATIVE_DIR, "libslkernels.so")
# the same kernels built with -DSL_DETERMINISTIC=1 (fixed-point cross-workgroup sums, no
# split-K atomics): loaded instead when the SL_DETERMINISTIC environment variable is 1
KERNELS_DET_SO = os.path.join(NATIVE_DIR, "libslkernels_det.so")


def _core_so_name() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return "_slcore" + suffix


CORE_SO = os.path.join(NATIVE_DIR, _core_so_name())


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        sys.stderr.write(proc.stdout)
        raise RuntimeError("native build failed: " + " ".join(cmd[:3]) + " ...")


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found; the HIP kernels need ROCm (%s)" % ROCM)
    return p


def build_kernels(force: bool = False, jobs: int = 8, deterministic: bool = False) -> str:
    """Compile csrc/kernels/*.hip for gfx950 into one shared object (``deterministic``:
    the SL_DETERMINISTIC=1 build, :data:`KERNELS_DET_SO`)."""
    os.makedirs(NATIVE_DIR, exist_ok=True)
    so_path = KERNELS_DET_SO if deterministic else KERNELS_SO
    srcs = sorted(glob.glob(os.path.join(KERNEL_DIR, "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(KERNEL_DIR, "*.h")))
    if not force and not _stale(so_path, srcs + hdrs):
        return so_path
    objdir = os.path.join(ROOT, "build", "kernels_det" if deterministic else "kernels")
    os.makedirs(objdir, exist_ok=True)
    hipcc = _hipcc()
    flags = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-I" + KERNEL_DIR,
             "-munsafe-fp-atomics", "-Wno-unused-result"] + (["-DSL_DETERMINISTIC=1"] if deterministic else [])
    objs = []
    procs = []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            procs.append((src, subprocess.Popen([hipcc, *flags, "-c", src, "-o", obj],
                                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
        while len([p for _, p in procs if p.poll() is None]) >= jobs:
            procs[0][1].wait()
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out)
            raise RuntimeError("hipcc failed on " + src)
    tmp = so_path + ".tmp"
    _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", *objs, "-o", tmp])
    _check_stubs(tmp)
    os.replace(tmp, so_path)
    return so_path


def _check_stubs(so: str) -> None:
    """Refuse a kernel library with an undefined launch stub.  A template kernel whose body
    names a device-only builtin in a type-dependent expression fails host-side instantiation
    silently: its launch stub is left undefined and the library only fails at dlopen, on the
    GPU box (csrc/kernels/conv.hip `blds16` is the wrapper that avoids this)."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    proc = subprocess.run([nm, "-D", "--undefined-only", so], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                          text=True)
    missing = [ln.split()[-1] for ln in proc.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        raise RuntimeError("undefined kernel launch stubs in %s: %s" % (so, ", ".join(missing)))


def build_core(force: bool = False) -> str:
    """Compile the C++ runtime (pybind11) against the HIP runtime API."""
    os.makedirs(NATIVE_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CORE_DIR, "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CORE_DIR, "*.h")))
    if not srcs:
        return ""
    if not force and not _stale(CORE_SO, srcs + hdrs):
        return CORE_SO
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    cxx = shutil.which("g++") or "c++"
    tmp = CORE_SO + ".tmp"
    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-function",
           "-D__HIP_PLATFORM_AMD__", "-I" + pybind11.get_include(), "-I" + py_inc,
           "-I" + CORE_DIR, "-I" + os.path.join(ROCM, "include"),
           *srcs, "-o", tmp, "-L" + os.path.join(ROCM, "lib"), "-lamdhip64",
           "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-lpthread"]
    if os.environ.get("SL_SANITIZE"):
        cmd[1:1] = ["-fsanitize=" + os.environ["SL_SANITIZE"], "-g", "-fno-omit-frame-pointer"]
    _run(cmd)
    os.replace(tmp, CORE_SO)
    return CORE_SO


def build_all(force: bool = False) -> None:
    build_kernels(force=force)
    build_kernels(force=force, deterministic=True)
    build_core(force=force)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["kernels", "core"], default=None)
    args = ap.parse_args(argv)
    if args.only in (None, "kernels"):
        print(build_kernels(force=args.force))
        print(build_kernels(force=args.force, deterministic=True))
    if args.only in (None, "core"):
        print(build_core(force=args.force))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
