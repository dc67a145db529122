"""ctypes binding of libsrpde_hip.so (the C ABI declared in include/srpde.h).

The prototypes are parsed from ``include/srpde.h`` itself, so the header is the single
source of truth for argument types.  Every call raises ``RuntimeError`` with the
library's thread-local message on a non-zero return.  There is no fallback: if the
library is missing or no GPU is present the product path fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  -- load torch's HIP runtime first: the .so binds to the same libamdhip64

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
# SRPDE_LIB: an alternate build of the same ABI (same-box A/B timing of kernel changes, tools/gpu/conv_ab.sh)
LIB_PATH = os.environ.get("SRPDE_LIB") or os.path.join(PKG, "lib", "libsrpde_hip.so")
HEADER = os.path.join(ROOT, "include", "srpde.h")

_CTYPES = {
    "int": ctypes.c_int,
    "long long": ctypes.c_longlong,
    "size_t": ctypes.c_size_t,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "hipStream_t": ctypes.c_void_p,
    "void": None,
}


def _ctype(decl: str):
    decl = decl.strip()
    if "*" in decl:
        return ctypes.c_char_p if decl.replace(" ", "") == "constchar*" else ctypes.c_void_p
    decl = decl.replace("const ", "").strip()
    parts = decl.split()
    base = " ".join(parts[:-1]) if len(parts) > 1 else parts[0]
    if base not in _CTYPES:
        raise ValueError(f"unsupported C type in srpde.h: {decl!r}")
    return _CTYPES[base]


def parse_header(path: str = HEADER):
    """-> {name: (restype, [argtypes])} for every prototype in srpde.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    protos = {}
    for m in re.finditer(r"^([A-Za-z_][\w ]*?[\w\*]+)\s+\**\s*(srpde_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.M | re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        full_ret = text[m.start():m.start(2)].strip()
        restype = ctypes.c_char_p if "char" in full_ret and "*" in full_ret else (
            ctypes.c_void_p if "*" in full_ret else _CTYPES[full_ret.replace("const ", "").strip()])
        args = " ".join(args.split())
        argtypes = [] if args in ("void", "") else [_ctype(a) for a in args.split(",")]
        protos[name] = (restype, argtypes)
    return protos


_lib = None
_protos = None


def lib():
    global _lib, _protos
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -m superresolution_for_pdes_amd.build` "
                "(the HIP path has no CPU fallback)")
        cd = ctypes.CDLL(LIB_PATH)
        want = int(re.search(r"#define SRPDE_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
        have = cd.srpde_version()
        if have != want:   # a library built against another header would misread arguments
            raise RuntimeError(f"{LIB_PATH}: ABI version {have}, include/srpde.h declares {want}: rebuild it "
                               "(python -m superresolution_for_pdes_amd.build --force)")
        _lib = cd
        _protos = parse_header()
        for name, (res, args) in _protos.items():
            fn = getattr(_lib, name)
            fn.restype = res
            fn.argtypes = args
    return _lib


def last_error() -> str:
    return lib().srpde_last_error().decode(errors="replace")


def call(name: str, *args) -> int:
    fn = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed (rc={rc}): {last_error()}")
    return rc


def query(name: str, *args):
    return getattr(lib(), name)(*args)


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
