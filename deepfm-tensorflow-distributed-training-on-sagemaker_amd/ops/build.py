"""In-tree build of the native libraries (no JIT cache, no pip install).

* ``_lib/libhipfm_kernels.so`` — every ``csrc/kernels/*.hip`` compiled by ``hipcc
  --offload-arch=gfx950`` (cross-compiles without a GPU), C ABI, bound with ctypes.
* ``_lib/libhipfm_io.so``      — ``csrc/io/*.cpp`` (TFRecord framing + CRC32C, tf.train.Example
  decoder, libsvm parser, threaded batch loader), host-only C++17.

Objects are rebuilt when a source or header is newer than the object, or when the compile
command (flags, arch, compiler) differs from the one recorded in the object's ``.cmd`` stamp.
Usage: ``python -m hipfm.ops.build [--force]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
from ..utils.knobs import knob

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "_lib")
BUILD_DIR = os.path.join(REPO, "build", "obj")
ARCH = knob("HIPFM_ARCH")

KERNELS_SO = os.path.join(LIB_DIR, "libhipfm_kernels.so")
# experiment: packed-FP32 VALU ops left on (HIPFM_BUILD_PACKED=1 -> its own objects and library,
# loaded with HIPFM_KERNELS_SO; tests/test_gpu_determinism.py is the check)
PACKED = knob("HIPFM_BUILD_PACKED") == "1"
if PACKED:
    KERNELS_SO = os.path.join(LIB_DIR, "libhipfm_kernels_packed.so")
    BUILD_DIR = BUILD_DIR + "_packed"
# diagnostic: per-workgroup phase stamps (HIPFM_BUILD_STAMPS=1 -> -DHFM_STAMPS, own objects and
# library; tools/stamps.py loads it with HIPFM_KERNELS_SO and reads the stamp buffers)
STAMPS = knob("HIPFM_BUILD_STAMPS") == "1"
if STAMPS:
    KERNELS_SO = os.path.join(LIB_DIR, "libhipfm_kernels_stamps.so")
    BUILD_DIR = BUILD_DIR + "_stamps"
# diagnostic variants: HIPFM_BUILD_VARIANT=<tag>:<DEF1>,<DEF2> -> -D<DEF> for each, own objects and
# library libhipfm_kernels_<tag>.so (loaded with HIPFM_KERNELS_SO; delete it after the experiment)
VARIANT = knob("HIPFM_BUILD_VARIANT")
VDEFS = []
if VARIANT:
    _vtag, _, _vdefs = VARIANT.partition(":")
    KERNELS_SO = os.path.join(LIB_DIR, f"libhipfm_kernels_{_vtag}.so")
    BUILD_DIR = BUILD_DIR + "_" + _vtag
    VDEFS = ["-D" + d for d in _vdefs.split(",") if d and d != "PACKED"]
    PACKED = PACKED or "PACKED" in _vdefs.split(",")      # (a variant with packed-FP32 ops on)
IO_SO = os.path.join(LIB_DIR, "libhipfm_io.so")


# No packed-FP32 VALU ops (v_pk_add/mul/fma_f32) in device code.  Measured on MI355X: a
# v_pk_add_f32 whose result feeds a ds_bpermute (the __shfl_xor of a lane reduction) at once
# read stale lanes for one 16-lane quarter-wave now and then -- only with two workgroups per CU
# (tools/det5.py: the FM logit of 2 adjacent samples off by ~1e-5, a different pair every
# run; tower_kernel's gather reduction, and training was not bitwise reproducible).  Without
# the packed ops the same code is exact and deterministic (tests/test_gpu_determinism.py).
# (hipcc also hands the feature to the x86 host pass, which prints "'-packed-fp32-ops' is not a
# recognized feature for this target (ignoring feature)": expected and harmless; -Xarch_device
# cannot forward -Xclang pairs.)
NO_PACKED_F32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build hipfm kernels)")


def _newer(src_files, target) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_files)


def _stamp_ok(obj: str, cmd) -> bool:
    """The object was built by exactly this command (its ``.cmd`` stamp matches)."""
    try:
        with open(obj + ".cmd") as f:
            return f.read() == "\x00".join(cmd)
    except OSError:
        return False


def _write_stamp(obj: str, cmd) -> None:
    with open(obj + ".cmd", "w") as f:
        f.write("\x00".join(cmd))


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    os.makedirs(BUILD_DIR, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    hipcc = _hipcc()
    objs = []
    todo = []
    def cmd_of(s, o):
        return [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
                "-fvisibility=hidden", "-Wno-unused-result", *([] if PACKED else NO_PACKED_F32),
                *(["-DHFM_STAMPS"] if STAMPS else []), *VDEFS,
                "-c", s, "-o", o]

    for s in srcs:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer([s] + hdrs, o) or not _stamp_ok(o, cmd_of(s, o)):
            todo.append((s, o))

    def comp(so):
        s, o = so
        cmd = cmd_of(s, o)
        out = _run(cmd)
        _write_stamp(o, cmd)
        if verbose and out.strip():
            print(out)
        return o

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(comp, todo))
    if force or todo or _newer(objs, KERNELS_SO):
        tmp = KERNELS_SO + ".tmp"
        # librccl.so.1 resolves to the RCCL PyTorch already loaded (same SONAME) at run time
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs +
             ["-L/opt/rocm/lib", "-lrccl"])
        os.replace(tmp, KERNELS_SO)
    return KERNELS_SO


def build_io(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "io", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "io", "*.h")))
    if not srcs:
        return ""
    os.makedirs(LIB_DIR, exist_ok=True)
    if force or _newer(srcs + hdrs, IO_SO):
        cxx = os.environ.get("CXX", "g++")
        tmp = IO_SO + ".tmp"
        out = _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-msse4.2", "-pthread",
                    "-fvisibility=hidden", "-o", tmp] + srcs)
        if verbose and out.strip():
            print(out)
        os.replace(tmp, IO_SO)
    return IO_SO


def build_all(force: bool = False, verbose: bool = False):
    return build_kernels(force, verbose=verbose), build_io(force, verbose=verbose)


if __name__ == "__main__":
    print(build_all(force="--force" in sys.argv, verbose=True))
