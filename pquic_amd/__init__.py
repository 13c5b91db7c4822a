"""pquic_amd -- MI355X-native FEC engine for PQUIC's plugins/fec path.

The product is the C-ABI library pquic_amd/lib/libpquic_fec.so (HIP kernels for gfx950 +
C protoop adapters).  This package is a thin Python mirror used by tests and bench.py:
it loads that library with ctypes and passes device pointers (torch CUDA tensors are
used only as HBM allocations and for the HIP stream).  There is no CPU fallback: if the
library or a gfx950 device is missing, calls raise.
"""
from .engine import Engine, FecGpuError, HostPath, load_library, LIB_PATH  # noqa: F401
from .engine import BLOCK_RECOVERED, BLOCK_NOTHING, BLOCK_REF_UB  # noqa: F401

__all__ = ["Engine", "FecGpuError", "HostPath", "load_library", "LIB_PATH",
           "BLOCK_RECOVERED", "BLOCK_NOTHING", "BLOCK_REF_UB"]
