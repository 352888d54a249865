"""In-tree native build for beforeholiday_amd (gfx950 only).

Produces ``beforeholiday_amd/_C<EXT_SUFFIX>`` from

* ``csrc/kernels/*.hip``  -- torch-free HIP device code, compiled by ``hipcc --offload-arch=gfx950``
* ``csrc/bindings/*.cpp`` -- the ATen/pybind11 front-end, compiled by the host C++ compiler

and links against the PyTorch-ROCm libraries (``libamdhip64`` resolves to the copy torch loaded,
both carry the soname ``libamdhip64.so.7``). The build is driven by a generated ``build.ninja``
so re-builds are incremental (header dependencies tracked through depfiles) and parallel.

Usage::

    python -m beforeholiday_amd._build            # build / incremental rebuild
    python -m beforeholiday_amd._build --clean    # wipe build dir first

Environment: ``BH_ARCH`` (default ``gfx950``), ``MAX_JOBS`` (ninja -j), ``BH_DEBUG=1`` (-O0 -g).
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(os.path.dirname(PKG_DIR), "build", "native")
EXT_NAME = "_C"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def ext_path() -> str:
    return os.path.join(PKG_DIR, EXT_NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    incs = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames else ce.include_paths(True)
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, libdir, abi


def _sources():
    hip = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp = sorted(glob.glob(os.path.join(CSRC, "bindings", "*.cpp")))
    return hip, cpp


# per-source extra hipcc flags. attn.hip: the flash kernels take fmaxf / sums of MFMA results in
# tight VALU budgets; without NaN semantics hipcc emits bare v_max3_f32 trees (no canonicalising
# v_max per operand), and without SLP it keeps f32 adds scalar (v_pk_add_f32 co-issues badly with
# MFMA). No kernel in that file tests for NaN.
_FILE_FLAGS = {"attn.hip": "-fno-honor-nans -fno-slp-vectorize"}


def write_ninja() -> str:
    arch = os.environ.get("BH_ARCH", "gfx950")
    debug = os.environ.get("BH_DEBUG", "0") == "1"
    incs, libdir, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    opt = "-O0 -g" if debug else "-O3"
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    cxx = os.environ.get("CXX", "g++")

    hip_flags = [
        opt, f"--offload-arch={arch}", "-std=c++17", "-fPIC", "-ffp-contract=fast",
        "-D__HIP_PLATFORM_AMD__=1", "-munsafe-fp-atomics", "-Wno-unused-result",
        f"-I{os.path.join(CSRC, 'include')}",
    ]
    cxx_flags = [
        "-O2" if not debug else "-O0 -g", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DHIPBLAS_V2", "-Wno-deprecated-declarations",
        f"-I{os.path.join(CSRC, 'include')}", f"-I{py_inc}",
    ] + [f"-isystem {p}" for p in incs]
    ldflags = [
        "-shared", "-fPIC", f"-L{libdir}", f"-Wl,-rpath,{libdir}",
        "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
        f"-L{os.path.join(ROCM, 'lib')}", "-lamdhip64",
    ]

    hip, cpp = _sources()
    os.makedirs(BUILD_DIR, exist_ok=True)
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"cxx = {cxx}",
        f"hip_flags = {' '.join(hip_flags)}",
        f"cxx_flags = {' '.join(cxx_flags)}",
        f"ldflags = {' '.join(ldflags)}",
        "",
        "rule hip",
        "  command = $hipcc -MD -MF $out.d $hip_flags -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "",
        "rule cxx",
        "  command = $cxx -MD -MF $out.d $cxx_flags -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "",
        "rule link",
        "  command = $hipcc $in $ldflags -o $out",
        "  description = LINK $out",
        "",
    ]
    objs = []
    for src in hip:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        objs.append(obj)
        lines.append(f"build {obj}: hip {src}")
        extra = _FILE_FLAGS.get(os.path.basename(src))
        if extra:
            lines.append(f"  hip_flags = $hip_flags {extra}")
    for src in cpp:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        objs.append(obj)
        lines.append(f"build {obj}: cxx {src}")
    lines.append(f"build {ext_path()}: link {' '.join(objs)}")
    lines.append(f"default {ext_path()}")
    path = os.path.join(BUILD_DIR, "build.ninja")
    content = "\n".join(lines) + "\n"
    old = open(path).read() if os.path.exists(path) else None
    if old != content:
        with open(path, "w") as f:
            f.write(content)
    return path


def build(clean: bool = False, verbose: bool = False) -> str:
    if clean and os.path.isdir(BUILD_DIR):
        shutil.rmtree(BUILD_DIR)
    ninja_file = write_ninja()
    jobs = os.environ.get("MAX_JOBS") or str(min(16, os.cpu_count() or 4))
    cmd = ["ninja", "-f", ninja_file, "-j", jobs]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True, cwd=BUILD_DIR)
    return ext_path()


if __name__ == "__main__":
    print(build(clean="--clean" in sys.argv, verbose="-v" in sys.argv))
