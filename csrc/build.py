"""Native build for dtfe: gfx950 HIP kernel library + C++ runtime module.

Produces (in-tree, so the artefacts travel with the repo snapshot to the GPU box):

  distributed-tensorflow-examples_amd/_C/libdtfe_kernels.so
      every csrc/kernels/*.hip (hipcc --offload-arch=gfx950) + csrc/bindings/*.cpp
      (torch.ops.dtfe.* registrations), linked against the ROCm build of torch.
  distributed-tensorflow-examples_amd/_C/_dtfe_rt<EXT_SUFFIX>
      csrc/runtime/*.cpp (crc32c, TF tensor-bundle checkpoint writer/reader,
      TFRecord/event writer, MNIST idx reader + batcher), a pybind11 module
      that needs no GPU.

Objects are cached under build/obj keyed by a hash of (source, headers, flags),
so rebuilds only recompile what changed.  Usage:

    python csrc/build.py [--only kernels|rt] [-j N] [--verbose]
    python csrc/build.py --ab REV FILE...    # A/B library: FILEs (csrc/kernels/*.hip) taken from git REV

The A/B build writes distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so (same bindings, the listed kernel sources as of
REV); DTFE_KERNEL_LIB=<that path> makes a process load it instead, so two code versions can be
timed alternately in one process pool on one GPU box (box-to-box spread is ~3 %).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "distributed-tensorflow-examples_amd")
OUT_DIR = os.path.join(PKG, "_C")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

KERNEL_LIB = os.path.join(OUT_DIR, "libdtfe_kernels.so")
RT_LIB = os.path.join(OUT_DIR, "_dtfe_rt" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def _torch_paths():
    import torch.utils.cpp_extension as ce
    import torch

    inc = ce.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    return inc, lib


def _hash_file(path: str, extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    with open(path, "rb") as f:
        h.update(f.read())
    # headers in the same tree: hash them all (cheap, conservative)
    for hdr in sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)):
        with open(hdr, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        sys.stderr.write(p.stdout)
        raise RuntimeError("command failed: " + " ".join(cmd[:3]) + " ... " + cmd[-1])
    return p.stdout


def _compile(src, flags, compiler, verbose):
    key = _hash_file(src, compiler + " ".join(flags))
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + "." + key + ".o")
    if not os.path.exists(obj):
        _run([compiler] + flags + ["-c", src, "-o", obj + ".tmp"], verbose)
        os.replace(obj + ".tmp", obj)
    return obj


def build_kernels(jobs: int, verbose: bool, ab_rev: str | None = None, ab_files=()) -> str:
    inc, libdir = _torch_paths()
    os.makedirs(OBJ_DIR, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    common = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wno-unused-result"]
    kflags = common + ["-I" + os.path.join(CSRC, "kernels")]
    bflags = common + ["-DUSE_ROCM", "-D__HIP_PLATFORM_AMD__", "-DTORCH_EXTENSION_NAME=dtfe"] + ["-I" + p for p in inc]
    kern_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    bind_srcs = sorted(glob.glob(os.path.join(CSRC, "bindings", "*.cpp")))
    out_lib = KERNEL_LIB
    if ab_rev:
        ab_dir = os.path.join(OUT_DIR, "ab")  # in-tree (travels with the gpurun snapshot; git-ignored)
        os.makedirs(os.path.join(ROOT, "build", "ab_src"), exist_ok=True)
        os.makedirs(ab_dir, exist_ok=True)
        # the A/B sources compile against the headers of the SAME revision (a struct that changed
        # between REV and HEAD would otherwise mix layouts silently): every csrc/kernels/*.h of REV
        # goes into build/ab_src, first on the include path
        ab_src = os.path.join(ROOT, "build", "ab_src")
        names = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", ab_rev, "csrc/kernels/"], check=True,
                               stdout=subprocess.PIPE, text=True).stdout.split()
        for rel in names:
            if rel.endswith(".h"):
                txt = subprocess.run(["git", "-C", ROOT, "show", "%s:%s" % (ab_rev, rel)], check=True,
                                     stdout=subprocess.PIPE).stdout
                with open(os.path.join(ab_src, os.path.basename(rel)), "wb") as fh:
                    fh.write(txt)
        kflags = common + ["-I" + ab_src, "-I" + os.path.join(CSRC, "kernels")]
        for f in ab_files:
            rel = os.path.relpath(os.path.abspath(f), ROOT)
            txt = subprocess.run(["git", "-C", ROOT, "show", "%s:%s" % (ab_rev, rel)], check=True,
                                 stdout=subprocess.PIPE).stdout
            dst = os.path.join(ROOT, "build", "ab_src", os.path.basename(rel))
            with open(dst, "wb") as fh:
                fh.write(txt)
            kern_srcs = [dst if os.path.abspath(k) == os.path.abspath(f) else k for k in kern_srcs]
        out_lib = os.path.join(ab_dir, "libdtfe_kernels.so")
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, kflags, HIPCC, verbose) for s in kern_srcs]
        futs += [ex.submit(_compile, s, bflags + ["-x", "hip"], HIPCC, verbose) for s in bind_srcs]
        objs = [f.result() for f in futs]
    link = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", out_lib + ".tmp"] + objs + [
        "-L" + libdir, "-Wl,-rpath," + libdir,
        "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lc10", "-lc10_hip",
        # RCCL: the librccl torch ships (same soname torch already loaded), for bindings/comm_ops.cpp
        "-lrccl",
    ]
    _run(link, verbose)
    os.replace(out_lib + ".tmp", out_lib)
    return out_lib


def build_runtime(jobs: int, verbose: bool) -> str:
    import pybind11

    os.makedirs(OBJ_DIR, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    py_inc = sysconfig.get_paths()["include"]
    flags = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-msse4.2",
             "-I" + pybind11.get_include(), "-I" + py_inc, "-I" + os.path.join(CSRC, "runtime")]
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, "g++", verbose), srcs))
    _run(["g++", "-shared", "-fPIC", "-o", RT_LIB + ".tmp"] + objs + ["-lz", "-lpthread"], verbose)
    os.replace(RT_LIB + ".tmp", RT_LIB)
    return RT_LIB


def build(only: str | None = None, jobs: int = 8, verbose: bool = False):
    out = []
    if only in (None, "rt"):
        out.append(build_runtime(jobs, verbose))
    if only in (None, "kernels"):
        out.append(build_kernels(jobs, verbose))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["kernels", "rt"], default=None)
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--ab", nargs="+", metavar=("REV", "FILE"), default=None,
                    help="A/B library: kernel sources FILE... as of git REV -> _C/ab/libdtfe_kernels.so")
    a = ap.parse_args()
    if a.ab:
        print("built", build_kernels(a.j, a.verbose, a.ab[0], a.ab[1:]))
        return
    for p in build(a.only, a.j, a.verbose):
        print("built", p)


if __name__ == "__main__":
    main()
