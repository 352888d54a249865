"""pip / setuptools entry point (reference: setup.py:241-854, ``--cpp_ext --cuda_ext`` and per-extension flags).

    pip install --no-build-isolation .                 # builds the gfx950 extension (ninja + hipcc)
    BH_PYTHON_ONLY=1 pip install --no-build-isolation . # python-only install (CPU reference paths)
    python setup.py build_ext --inplace                 # in-tree build, same as python -m beforeholiday_amd._build

Every native module of the reference (amp_C, syncbn, fused_layer_norm_cuda, fused_dense_cuda, mlp_cuda,
scaled_*softmax_cuda, fast_multihead_attn, xentropy_cuda, focal_loss_cuda, fused_index_mul_2d,
fused_adam_cuda, distributed_{adam,lamb}_cuda, transducer_{joint,loss}_cuda, peer_memory_cuda, ...) is a
submodule of the ONE extension ``beforeholiday_amd._C`` (nccl_p2p is python over torch.distributed's RCCL
communicators: ``beforeholiday_amd.contrib.nccl_p2p``), so there are no per-extension flags: the reference's flags selected which of its
~25 .so files to compile; here one ninja build compiles all kernels for gfx950 (incremental).
"""
import os

from setuptools import Extension, find_packages, setup
from setuptools.command.build_ext import build_ext

PYTHON_ONLY = os.environ.get("BH_PYTHON_ONLY", "0") == "1"


class NinjaBuild(build_ext):
    """Runs beforeholiday_amd._build (hipcc --offload-arch=gfx950 + host C++), then places _C where
    setuptools expects it (in-tree for --inplace / develop, in build_lib for wheels)."""

    def build_extension(self, ext):
        import shutil

        from beforeholiday_amd import _build

        built = _build.build()
        dest = self.get_ext_fullpath(ext.name)
        os.makedirs(os.path.dirname(dest), exist_ok=True)
        if os.path.abspath(built) != os.path.abspath(dest):
            shutil.copyfile(built, dest)


setup(
    name="beforeholiday_amd",
    version="0.1.0",
    description="MI355X-native (gfx950) mixed-precision and distributed training library with the Apex API",
    packages=find_packages(include=["beforeholiday_amd", "beforeholiday_amd.*"]),
    package_data={"beforeholiday_amd": ["utils/tuned/*.csv", "csrc/include/bh/*.h", "csrc/kernels/*.hip", "csrc/bindings/*.cpp",
                                        "csrc/bindings/*.h"]},
    ext_modules=[] if PYTHON_ONLY else [Extension("beforeholiday_amd._C", sources=[])],
    cmdclass={} if PYTHON_ONLY else {"build_ext": NinjaBuild},
    python_requires=">=3.9",
    install_requires=["torch"],
)
