"""ctypes binding of libcordagpu (include/cordagpu.h).

The shared library is built in-tree (``corda_amd/libcordagpu.so``) by
``__graft_entry__.build()`` / ``make -C corda_amd/csrc``.  There is deliberately
no fallback: if the library or a gfx950 device is missing, opening a context
raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

LIB_PATH = os.environ.get("CORDA_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcordagpu.so")

# status codes
CG_OK = 0
CG_E_INVALID_ARGUMENT = -1
CG_E_NO_DEVICE = -2
CG_E_DEVICE = -3
CG_E_OUT_OF_MEMORY = -4
CG_E_MERKLE_EMPTY = -5

# verdicts
ACCEPT, REJECT, SIG_MALFORMED, KEY_INVALID, ARG_EMPTY, UNSUPPORTED = 0, 1, 2, 3, 4, 5
MODE_IS_VALID, MODE_DO_VERIFY = 0, 1
# FilteredTransaction.verify outcomes (cg_ftx_verify_batch)
FTX_TRUE, FTX_FALSE, FTX_NO_LEAVES, FTX_MALFORMED = 0, 1, 2, 3
# CompositeKey fulfilment (cg_composite_eval_batch)
COMPOSITE_LEAF, COMPOSITE_NODE, COMPOSITE_INVALID = 0, 1, 0x80
# per-tx codes of cg_tx_verify_batch / cg_tx_verify_signatures_except (>= 0: first bad signature)
TX_OK, TX_NO_SIGNATURES, TX_NO_COMPONENTS, TX_SIGNATURES_MISSING = -1, -2, -3, -4
# cg_set_debug options (test hooks)
DEBUG_FORCE_FULL_LENGTH, DEBUG_FAIL_ALLOC, DEBUG_THROW, DEBUG_FORCE_GLV_FALLBACK = 1, 2, 3, 4
ABI_VERSION = 4

# exported symbols and their prototypes: (restype, argtypes)
_u8p, _u32p, _u64p, _i32p = POINTER(c_uint8), POINTER(c_uint32), POINTER(c_uint64), POINTER(ctypes.c_int32)
PROTOTYPES = {
    "cg_abi_version": (c_int, []),
    "cg_device_count": (c_int, []),
    "cg_open": (c_int, [c_int, POINTER(c_void_p)]),
    "cg_close": (None, [c_void_p]),
    "cg_last_error": (c_char_p, [c_void_p]),
    "cg_verify_batch": (c_int, [c_void_p, c_size_t, c_int, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t,
                                c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cg_batch_create": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_void_p,
                                c_void_p, c_size_t, c_void_p, c_void_p, POINTER(c_void_p)]),
    "cg_batch_verify": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "cg_batch_size": (c_size_t, [c_void_p]),
    "cg_batch_destroy": (None, [c_void_p, c_void_p]),
    "cg_der_parse_batch": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "cg_txid_batch": (c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p]),
    "cg_tx_verify_batch": (c_int, [c_void_p, c_int, c_size_t, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_void_p,
                                   c_void_p, c_void_p, c_void_p]),
    "cg_tx_verify_signatures_except": (c_int, [c_void_p, c_int, c_size_t, c_void_p, c_size_t, c_void_p, c_void_p,
                                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p,
                                               c_size_t, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_void_p]),
    "cg_ftx_verify_batch": (c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cg_composite_eval_batch": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                        c_void_p]),
    "cg_register_host": (c_int, [c_void_p, c_void_p, c_size_t]),
    "cg_unregister_host": (c_int, [c_void_p, c_void_p]),
    "cg_release_cached": (c_int, [c_void_p]),
    "cg_set_profiling": (c_int, [c_void_p, c_int]),
    "cg_kernel_stats": (c_int, [c_void_p, c_char_p, POINTER(c_double), POINTER(c_uint64), POINTER(c_uint64)]),
    "cg_reset_stats": (c_int, [c_void_p]),
    "cg_set_debug": (c_int, [c_void_p, c_int, ctypes.c_int64]),
    "cg_set_option": (c_int, [c_void_p, c_char_p, c_char_p]),
}

_lib = None


class CordaGpuError(RuntimeError):
    """A libcordagpu call failed (non-zero cg_status)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"libcordagpu status {status}: {message}")
        self.status = status


def _share_torch_hip_runtime() -> None:
    """One HIP runtime per process.  The PyTorch-ROCm wheel bundles its own
    libamdhip64 (SONAME libamdhip64.so.7, but NEEDED by torch under the name
    libamdhip64.so).  If libcordagpu is loaded first, its libamdhip64.so.7
    resolves to /opt/rocm and a later ``import torch`` maps a second HIP/HSA
    runtime that then finds no GPU ("No HIP GPUs are available").  Importing
    torch first lets the dynamic loader bind libcordagpu's dependency to the
    runtime torch already mapped.  Without torch (a plain C-ABI host) the system
    runtime is used."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load() -> ctypes.CDLL:
    """Loads the in-tree library (raises OSError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built: run __graft_entry__.build() or make -C corda_amd/csrc")
        _share_torch_hip_runtime()
        lib = ctypes.CDLL(LIB_PATH)
        if lib.cg_abi_version() != ABI_VERSION:
            raise OSError(f"{LIB_PATH}: ABI version {lib.cg_abi_version()}, binding expects {ABI_VERSION} (rebuild)")
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def ptr(a):
    """Address of a numpy array (or None) for a c_void_p argument."""
    if a is None:
        return None
    return a.ctypes.data


class Context:
    """One libcordagpu context: one HIP device + stream (one per process/rank)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = c_void_p()
        st = self.lib.cg_open(device, ctypes.byref(h))
        if st != CG_OK:
            raise CordaGpuError(st, "cg_open failed (no gfx950 device?)")
        self.h = h
        self.device = device

    def check(self, st: int) -> int:
        if st not in (CG_OK,):
            raise CordaGpuError(st, (self.lib.cg_last_error(self.h) or b"").decode())
        return st

    def close(self):
        if getattr(self, "h", None):
            self.lib.cg_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_profiling(self, on):
        """False / True, or 2: only each cg_verify_batch's "call" span (its GPU time)."""
        self.check(self.lib.cg_set_profiling(self.h, 2 if on == 2 else 1 if on else 0))

    def kernel_stats(self, name: str):
        ms, launches, items = c_double(), c_uint64(), c_uint64()
        self.check(self.lib.cg_kernel_stats(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(launches),
                                            ctypes.byref(items)))
        return ms.value, launches.value, items.value

    def reset_stats(self):
        self.check(self.lib.cg_reset_stats(self.h))

    def set_debug(self, option: int, value: int):
        """Test hooks (cg_set_debug): forced full-length Ed25519 scalars, injected
        allocation failures, an injected exception."""
        self.check(self.lib.cg_set_debug(self.h, option, value))

    def set_option(self, key: str, value=None):
        """One run-time option of this context (cg_set_option): a
        CORDA_AMD_* knob, read from the environment only at cg_open.  value None: unset
        (the library default)."""
        self.check(self.lib.cg_set_option(self.h, key.encode(), None if value is None else str(value).encode()))

    def options(self, **kv):
        """Context manager: set options (CORDA_AMD_ prefix optional) for a block, unset
        them afterwards."""
        import contextlib

        @contextlib.contextmanager
        def scope():
            keys = [k if k.startswith("CORDA_AMD_") else "CORDA_AMD_" + k for k in kv]
            try:
                for k, v in zip(keys, kv.values()):
                    self.set_option(k, v)
                yield self
            finally:
                for k in keys:
                    self.set_option(k, None)
        return scope()

    def register_host(self, *arrays):
        """Page-locks numpy arrays the caller will pass again (cg_register_host)."""
        for a in arrays:
            if a is not None and a.nbytes:
                self.check(self.lib.cg_register_host(self.h, a.ctypes.data, a.nbytes))

    def unregister_host(self, *arrays):
        for a in arrays:
            if a is not None and a.nbytes:
                self.check(self.lib.cg_unregister_host(self.h, a.ctypes.data))
