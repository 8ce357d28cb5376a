"""Op layer: native HIP kernels (GPU) and their PyTorch-CPU reference semantics."""
from .native import native, native_available, require_native  # noqa: F401
