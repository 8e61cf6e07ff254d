"""ctypes binding of the C-ABI declared in include/dmf_hip.h.

The reference (pure PyTorch) has no FFI; this module is
the seam a maintainer would otherwise write as a cgo/JNI stub. It loads the
in-tree ``libdmf_hip.so`` built by ``csrc/Makefile`` *after* torch, so the
library's ``libamdhip64.so.7`` dependency resolves to the HIP runtime torch
already mapped (one HIP runtime per process, shared device pointers and
streams).

There is no CPU fallback anywhere in the product path: if the library is
missing or a kernel reports an error, a RuntimeError is raised.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DMF_HIP_LIB", os.path.join(_HERE, "libdmf_hip.so"))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "dmf_hip.h")

F32, BF16, F16 = 0, 1, 2  # include/dmf_hip.h DMF_F32 / DMF_BF16 / DMF_F16
ACT_NONE, ACT_RELU, ACT_GELU, ACT_SIGMOID = 0, 1, 2, 3
# conv kernel bodies (dmf_conv_last_form, include/dmf_hip.h DMF_FORM_*)
FORMS = {0: "igemm", 1: "buf", 2: "buf_ina", 3: "wide", 4: "sq", 5: "ps", 6: "pp", 7: "stem"}

_lib = None
_lock = threading.Lock()

# name -> argtypes (restype is always c_int unless listed in _RESTYPES)
P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_longlong
F = ctypes.c_float
U64 = ctypes.c_ulonglong

_RESTYPES = {"dmf_last_error": ctypes.c_char_p}


def _ctype_of(decl):
    decl = decl.strip()
    if "*" in decl:
        return P
    decl = re.sub(r"\b(const|volatile)\b", "", decl)
    toks = decl.split()[:-1]  # drop the parameter name
    t = " ".join(toks)
    table = {
        "int": I,
        "long long": L,
        "unsigned long long": U64,
        "float": F,
        "double": ctypes.c_double,
    }
    if t not in table:
        raise RuntimeError(f"dmf_hip.h: unsupported parameter type {decl!r}")
    return table[t]


def _signatures():
    """argtypes for every entry point, parsed from include/dmf_hip.h (the
    header is the single source of truth for the ABI)."""
    with open(HEADER_PATH) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    sigs = {}
    for m in re.finditer(r"\b(int|long long|const char\*)\s+(dmf_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        if ret == "long long":
            _RESTYPES[name] = L
        if params in ("", "void"):
            sigs[name] = []
        else:
            sigs[name] = [_ctype_of(p) for p in params.split(",")]
    return sigs


def _header_constants():
    """Integer ``#define DMF_*`` constants of include/dmf_hip.h (workspace sizes and the like)."""
    with open(HEADER_PATH) as f:
        src = f.read()
    return {m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define\s+(DMF_[A-Z0-9_]+)\s+(0x[0-9a-fA-F]+|\d+)\s", src)}


globals().update(_header_constants())


def declared_symbols():
    """Names of every function include/dmf_hip.h declares (parsed)."""
    with open(HEADER_PATH) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dmf_[a-z0-9_]+)\s*\(", src)))


def load():
    """Load (once) and return the ctypes library handle."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"HIP extension not built: {LIB_PATH} is missing "
                "(run __graft_entry__.build() or `make -C csrc`)"
            )
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in _signatures().items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        lib.dmf_last_error.argtypes = []
        lib.dmf_last_error.restype = ctypes.c_char_p
        _lib = lib
    return _lib


def call(name, *args):
    """Invoke a C-ABI entry point; raise RuntimeError on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.dmf_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")
    return rc


class BnDesc(ctypes.Structure):
    """dmf_bn_desc of include/dmf_hip.h (a training-mode BatchNorm2d whose
    statistics a dmf_conv2d_fwd_acc launch accumulated)."""

    _fields_ = [("acc", ctypes.c_void_p), ("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p),
                ("running_mean", ctypes.c_void_p), ("running_var", ctypes.c_void_p),
                ("num_batches_tracked", ctypes.c_void_p), ("scale_shift", ctypes.c_void_p),
                ("save_mean_invstd", ctypes.c_void_p), ("count", ctypes.c_double), ("unbias_count", ctypes.c_double),
                ("momentum", ctypes.c_float), ("eps", ctypes.c_float), ("replicas", ctypes.c_int)]


def stream_ptr(device=None):
    """hipStream_t of torch's current stream (graph-capture aware)."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float16:
        return F16
    raise RuntimeError(f"unsupported dtype {dt} (expected float32, bfloat16 or float16)")


def require_cuda(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "dmf HIP ops need device tensors; got a CPU tensor "
                "(the product path has no CPU fallback)"
            )
