"""corda_amd — MI355X-native batch signature verification + tx-id engine for
Corda's verification hot path.

The compute lives in libcordagpu.so (HIP kernels for gfx950, C ABI in
include/cordagpu.h).  This package is the host-side mirror of the reference's
``Crypto`` batch surface (crypto.py), transaction helpers incl. filtered
transactions (transactions.py), CompositeKey fulfilment (composite.py) and the
multi-GPU sharding driver (dist.py).
"""
from ._lib import Context, CordaGpuError, load  # noqa: F401

__all__ = ["Context", "CordaGpuError", "load"]
