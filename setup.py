"""Build the in-tree native extension `_pddl_native` (HIP kernels for gfx950 + torch bindings).

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

The built shared object is moved next to the Python package
(`parallel-and-distributed-deep-learning_amd/_pddl_native*.so`) by `pddl_build.py`;
`__graft_entry__.build()` drives both steps.
"""
import glob
import os

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension, CUDAExtension

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
ROOT = os.path.dirname(os.path.abspath(__file__))
kern = sorted(glob.glob(os.path.join("csrc", "kernels", "*.hip")))
rt = sorted(glob.glob(os.path.join("csrc", "runtime", "*.cpp")))
srcs = [os.path.join("csrc", "bindings.cpp")] + rt + kern

setup(
    name="pddl_native",
    ext_modules=[
        CUDAExtension(
            "_pddl_native",
            srcs,
            include_dirs=[os.path.join(ROOT, "csrc"), "/opt/rocm/include"],
            library_dirs=["/opt/rocm/lib"],
            libraries=["rccl"],
            extra_link_args=["-Wl,-rpath,/opt/rocm/lib"],
            extra_compile_args={
                "cxx": ["-O2", "-std=c++17"],
                "nvcc": ["-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=fast"],
            },
        ),
        # Keras-layout .h5 checkpoints through the system HDF5 1.10 (separate module so the
        # kernels never depend on libhdf5 being loadable)
        CppExtension(
            "_pddl_h5",
            [os.path.join("csrc", "h5", "h5io.cpp")],
            include_dirs=["/opt/conda/include"],
            library_dirs=["/opt/conda/lib"],
            libraries=["hdf5"],
            extra_link_args=["-Wl,-rpath,/opt/conda/lib"],
            extra_compile_args=["-O2", "-std=c++17"],
        ),
    ],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
