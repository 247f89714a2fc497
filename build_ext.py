#!/usr/bin/env python3
"""In-tree native build for flexflow_amd.

Builds two extension modules next to the Python sources (so they travel with the repo snapshot
to GPU boxes and are what the tests / bench import):

  flexflow_amd/_C.so     HIP kernels for gfx950 (hipcc --offload-arch=gfx950) + torch glue
  flexflow_amd/_core.so  native runtime core (PCG, simulator, Unity/MCMC search, substitutions,
                         strategy I/O, data-loader ring) — plain C++17 + pybind11, no GPU needed

No hipify and no torch.utils.cpp_extension JIT: each translation unit is compiled explicitly and
incrementally (an object is rebuilt when its source or any header in its directory is newer).
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
KDIR = os.path.join(ROOT, "csrc", "kernels")
CDIR = os.path.join(ROOT, "csrc", "core")
BUILD = os.path.join(ROOT, "build")
PKG = os.path.join(ROOT, "flexflow_amd")
ARCH = os.environ.get("FF_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# Per-file code generation flags. attention.hip: no SLP vectorisation — hipcc packed the backward's
# adjacent f32 multiplies / adds into v_pk_mul_f32 / v_pk_add_f32 (56 per 64-query tile), which
# beside MFMAs cost more issue cycles than the scalar pairs they replace (MI355X_MICROARCH.md,
# 'price of one filler beside MFMAs'). A flag change rebuilds the file (the command is hashed).
FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize"]}


def _torch_paths():
    import torch  # noqa: F401  (only to locate headers / libs)
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _pybind_inc():
    import pybind11
    return pybind11.get_include()


def _newer(src: str, obj: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + "\n")
        raise RuntimeError(f"compile failed: {cmd[-1] if cmd else ''}")


def _stamp_text(cmd) -> str:
    """The compile command with the tree's own path factored out: a copy of the tree elsewhere (the
    GPU box's snapshot) does not rebuild objects whose flags did not change."""
    return " ".join(cmd).replace(os.path.dirname(os.path.abspath(__file__)), "<root>")


def build_kernels(jobs: int = 8, verbose: bool = False) -> str:
    inc, tlib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    os.makedirs(os.path.join(BUILD, "kernels"), exist_ok=True)
    headers = [os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith(".h")]
    srcs = sorted(f for f in os.listdir(KDIR) if f.endswith(".hip") or f.endswith(".cpp"))
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", KDIR]
    jobs_list = []
    objs = []
    for s in srcs:
        src = os.path.join(KDIR, s)
        obj = os.path.join(BUILD, "kernels", s + ".o")
        objs.append(obj)
        if s.endswith(".hip"):
            cmd = [HIPCC, f"--offload-arch={ARCH}", *common, *FILE_FLAGS.get(s, []), "-c", src, "-o", obj]
        else:  # torch glue: host code only
            cmd = [HIPCC, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
                   "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-deprecated-declarations",
                   *sum([["-isystem", i] for i in inc], []), "-isystem", py_inc, "-c", src, "-o", obj]
        stamp = obj + ".cmd"  # the compile command: a flag change rebuilds the object
        prev = open(stamp).read() if os.path.exists(stamp) else ""
        if _newer(src, obj, headers) or prev != _stamp_text(cmd):
            jobs_list.append(cmd)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, jobs_list))
    for cmd in jobs_list:  # stamped once every compile succeeded
        with open(cmd[-1] + ".cmd", "w") as f:
            f.write(_stamp_text(cmd))
    out = os.path.join(PKG, "_C.so")
    if jobs_list or not os.path.exists(out):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-L", tlib, f"-Wl,-rpath,{tlib}",
              "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64",
              "-lhipblaslt",  # torch/lib copy (same soname as the one libtorch_hip loads)
              "-o", out + ".tmp"])
        os.replace(out + ".tmp", out)  # atomic: a concurrent tree snapshot never sees a partial .so
    if verbose:
        print(f"[build_ext] {len(jobs_list)} kernel objects rebuilt -> {out}")
    return out


def build_core(jobs: int = 8, verbose: bool = False) -> str | None:
    if not os.path.isdir(CDIR):
        return None
    srcs = sorted(f for f in os.listdir(CDIR) if f.endswith(".cc"))
    if not srcs:
        return None
    py_inc = sysconfig.get_paths()["include"]
    os.makedirs(os.path.join(BUILD, "core"), exist_ok=True)
    headers = [os.path.join(CDIR, f) for f in os.listdir(CDIR) if f.endswith(".h")]
    flags = ["-O2", "-g0", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-I", CDIR, "-isystem", _pybind_inc(),
             "-isystem", py_inc]
    cxx = os.environ.get("CXX", "g++")
    jobs_list, objs = [], []
    for s in srcs:
        src = os.path.join(CDIR, s)
        obj = os.path.join(BUILD, "core", s + ".o")
        objs.append(obj)
        if _newer(src, obj, headers):
            jobs_list.append([cxx, *flags, "-c", src, "-o", obj])
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, jobs_list))
    out = os.path.join(PKG, "_core.so")
    if jobs_list or not os.path.exists(out):
        _run([cxx, "-shared", "-fPIC", *objs, "-lpthread", "-o", out])
    if verbose:
        print(f"[build_ext] {len(jobs_list)} core objects rebuilt -> {out}")
    return out


def build_capi(verbose: bool = False) -> str | None:
    """libflexflow_c.so: the C API (csrc/capi) over an embedded CPython runtime."""
    src = os.path.join(ROOT, "csrc", "capi", "flexflow_c.cc")
    if not os.path.exists(src):
        return None
    out = os.path.join(PKG, "libflexflow_c.so")
    hdr = os.path.join(ROOT, "csrc", "capi", "flexflow_c.h")
    if _newer(src, out, [hdr]):
        paths = sysconfig.get_paths()
        libdir = sysconfig.get_config_var("LIBDIR")
        ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
        _run([os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-I", paths["include"], src,
              "-L", libdir, f"-lpython{ver}", f"-Wl,-rpath,{libdir}", "-o", out])
        if verbose:
            print(f"[build_ext] C API -> {out}")
    return out


def build_all(verbose: bool = True) -> None:
    jobs = min(8, os.cpu_count() or 4)
    build_core(jobs, verbose)
    build_kernels(jobs, verbose)
    build_capi(verbose)


if __name__ == "__main__":
    build_all()
