"""Build the in-tree native extension `_pddl_native` (HIP kernels for gfx950 + torch bindings).

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

The built shared object is moved next to the Python package
(`parallel-and-distributed-deep-learning_amd/_pddl_native*.so`) by `pddl_build.py`;
`__graft_entry__.build()` drives both steps.
"""
import glob
import os

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CUDAExtension

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
ROOT = os.path.dirname(os.path.abspath(__file__))
kern = sorted(glob.glob(os.path.join("csrc", "kernels", "*.hip")))
srcs = [os.path.join("csrc", "bindings.cpp")] + kern

setup(
    name="pddl_native",
    ext_modules=[
        CUDAExtension(
            "_pddl_native",
            srcs,
            include_dirs=[os.path.join(ROOT, "csrc")],
            extra_compile_args={
                "cxx": ["-O2", "-std=c++17"],
                "nvcc": ["-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=fast"],
            },
        )
    ],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
