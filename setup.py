"""Build the in-tree native extensions.

    python pddl_build.py                      (what __graft_entry__.build() runs)

`_pddl_native`: the gfx950 HIP kernels (csrc/kernels/*.hip) are compiled by hipcc directly
into position-independent objects -- no source translation step touches them -- and linked
with the host-side torch bindings and runtime (csrc/bindings.cpp, csrc/runtime/*.cpp), which
are plain C++ against the HIP runtime and PyTorch-ROCm headers.

`_pddl_io`: the ImageNet reader (TFRecord / JPEG decode via libjpeg, resize_with_crop_or_pad),
a separate module for the same reason.

`_pddl_h5`: Keras-layout .h5 checkpoints through the system HDF5 1.10 (separate module so the
kernels never depend on libhdf5 being loadable).

The built shared objects are moved next to the Python package by `pddl_build.py`.
"""
import glob
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension, include_paths, library_paths

ROOT = os.path.dirname(os.path.abspath(__file__))
ARCH = os.environ.get("PDDL_OFFLOAD_ARCH", "gfx950")
TEMP = os.environ.get("PDDL_BUILD_TEMP", os.path.join(os.environ.get("TMPDIR", "/tmp"), "pddl_build_temp"))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
HIP_FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-ffp-contract=fast", "-fPIC", "-I" + os.path.join(ROOT, "csrc")]
# A/B builds of compile-time kernel parameters, e.g. PDDL_HIP_DEFINES="-DIGEMM_MIN_BLOCKS_1=4"
# (use a separate PDDL_BUILD_TEMP: objects are rebuilt on source changes only)
HIP_FLAGS += os.environ.get("PDDL_HIP_DEFINES", "").split()


def compile_kernels():
    """hipcc -c every kernel translation unit (rebuilt when it or a kernel header changed)."""
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    hdrs = glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.h"))
    hdr_mtime = max(os.path.getmtime(h) for h in hdrs)
    odir = os.path.join(TEMP, "kernels", ARCH)
    os.makedirs(odir, exist_ok=True)

    def one(src):
        obj = os.path.join(odir, os.path.basename(src)[:-4] + ".o")
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
            return obj
        r = subprocess.run([HIPCC, *HIP_FLAGS, "-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        return obj
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        return list(ex.map(one, srcs))


kernel_objs = compile_kernels()
# PDDL_SANITIZE=1 (UBSan) or =<list> (e.g. address,undefined): host code (bindings, runtime, io)
# built with sanitizers for the CPU test suite (scripts/sanitize_host.sh); device code unaffected.
_san = os.environ.get("PDDL_SANITIZE", "")
SAN = ([f"-fsanitize={'undefined' if _san == '1' else _san}", "-fno-omit-frame-pointer", "-g"] if _san else [])
HOST_CFLAGS = (["-O1"] if SAN else ["-O2", "-g0"]) + ["-std=c++17"] + SAN
STRIP = [] if SAN else ["-Wl,--strip-debug"]
host_srcs = [os.path.join("csrc", "bindings.cpp")] + sorted(glob.glob(os.path.join("csrc", "runtime", "*.cpp")))

setup(
    name="pddl_native",
    ext_modules=[
        CppExtension(
            "_pddl_native",
            host_srcs,
            include_dirs=[os.path.join(ROOT, "csrc")] + include_paths(device_type="cuda"),
            library_dirs=library_paths(device_type="cuda"),
            libraries=["amdhip64", "c10_hip", "torch_hip", "rccl"],
            define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
            extra_objects=kernel_objs,
            extra_link_args=["-Wl,-rpath,/opt/rocm/lib"] + STRIP + SAN,
            extra_compile_args=HOST_CFLAGS,
        ),
        CppExtension(
            "_pddl_io",
            [os.path.join("csrc", "io", "imagenet_io.cpp")],
            include_dirs=[os.path.join(ROOT, "csrc"), "/opt/conda/include"],
            library_dirs=["/opt/conda/lib"],
            libraries=["jpeg"],
            extra_link_args=["-Wl,-rpath,/opt/conda/lib"] + STRIP + SAN,
            extra_compile_args=HOST_CFLAGS,
        ),
        CppExtension(
            "_pddl_h5",
            [os.path.join("csrc", "h5", "h5io.cpp")],
            include_dirs=["/opt/conda/include"],
            library_dirs=["/opt/conda/lib"],
            libraries=["hdf5"],
            extra_link_args=["-Wl,-rpath,/opt/conda/lib"] + STRIP + SAN,
            extra_compile_args=HOST_CFLAGS,
        ),
    ],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
