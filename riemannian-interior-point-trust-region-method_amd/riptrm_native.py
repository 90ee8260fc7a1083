"""ctypes binding of ``libriptrm_hip.so`` (the C-ABI declared in ``include/riptrm.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``hipcc --offload-arch=gfx950``).
There is no fallback: if the library is missing or no gfx950 device is visible, every entry
point raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Dict, List, Optional

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libriptrm_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "riptrm.h")

c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p
P_int32 = ctypes.POINTER(ctypes.c_int32)


class RiptrmOptions(ctypes.Structure):
    """Mirror of ``riptrm_options`` (include/riptrm.h)."""
    _fields_ = [
        ("struct_size", c_int32), ("maxiter", c_int32), ("inner_maxiter", c_int32),
        ("tcg_mininner", c_int32), ("save_inner_iteration", c_int32), ("manvio_kind", c_int32),
        ("log_capacity", c_int32), ("restart_every", c_int32),
        ("maxtime", c_double), ("inner_maxtime", c_double), ("tolresid", c_double),
        ("initial_tr_radius", c_double), ("minimal_initial_tr_radius", c_double),
        ("maximal_tr_radius", c_double), ("rho", c_double), ("reduction_regularization", c_double),
        ("gamma", c_double), ("tcg_theta", c_double), ("tcg_kappa", c_double),
        ("const_left", c_double), ("const_right", c_double),
        ("trs_solver", c_int32), ("second_order_stationarity", c_int32), ("trs_tolhardcase", c_double),
        ("tol2_table", c_void_p),
    ]


class RiptrmSIProblem(ctypes.Structure):
    """Mirror of ``riptrm_si_problem`` (include/riptrm.h)."""
    _fields_ = [
        ("struct_size", c_int32), ("d", c_int32), ("N", c_int32), ("m", c_int32), ("h", c_double),
        ("X", c_void_p), ("XP", c_void_p), ("data_stride", c_int64), ("cons", c_void_p),
        ("cons_stride", c_int64),
    ]


# (restype, argtypes) of every exported symbol
SIGNATURES: Dict[str, tuple] = {
    "riptrm_abi_version": (c_int32, []),
    "riptrm_ctx_create": (c_int32, [ctypes.POINTER(c_void_p), c_int32, c_void_p]),
    "riptrm_ctx_destroy": (c_int32, [c_void_p]),
    "riptrm_last_error": (c_char_p, [c_void_p]),
    "riptrm_ctx_set_stream": (c_int32, [c_void_p, c_void_p]),
    "riptrm_nonnegpca_ld": (c_int64, [c_int32]),
    "riptrm_nonnegpca_rows": (c_int64, [c_int32]),
    "riptrm_nonnegpca_s_elems": (c_int64, [c_int32, c_int32]),
    "riptrm_workspace_bytes": (c_int64, [c_int32, c_int32, c_int32, c_int32]),
    "riptrm_workspace_offset": (c_int64, [c_int32, c_int32, c_int32, c_int32, c_int32]),
    "riptrm_nonnegpca_pack": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p,
                                        c_int32, c_int64]),
    "riptrm_nonnegpca_bind": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int64,
                                        c_void_p, c_int64, c_int32]),
    "riptrm_nonnegpca_hvp": (c_int32, [c_void_p, c_void_p, c_void_p, c_double, c_void_p, c_void_p, c_int64]),
    "riptrm_nonnegpca_operator_aw": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64]),
    "riptrm_tcg": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, P_int32, P_int32, c_int32]),
    "riptrm_solve_begin": (c_int32, [c_void_p, ctypes.POINTER(RiptrmOptions), c_void_p, c_void_p, c_int64,
                                     c_void_p, c_void_p, c_void_p, c_int32]),
    "riptrm_solve_advance": (c_int32, [c_void_p, c_int32, c_int32, P_int32]),
    "riptrm_device_clock_hz": (c_double, [c_void_p]),
    "riptrm_log_rebase": (c_int32, [c_void_p]),
    "riptrm_set_stream_groups": (c_int32, [c_void_p, c_int32]),
    "riptrm_set_graphs": (c_int32, [c_void_p, c_int32]),
    "riptrm_set_persistent": (c_int32, [c_void_p, c_int32]),
    "riptrm_get_persistent": (c_int32, [c_void_p, P_int32, P_int32]),
    "riptrm_persist_fallbacks": (c_int32, [c_void_p, P_int32]),
    "riptrm_trs_workspace_bytes": (ctypes.c_int64, [c_int32, c_int32]),
    "riptrm_trs_bind_workspace": (c_int32, [c_void_p, c_void_p, ctypes.c_int64, c_int32, c_int32]),
    "riptrm_trs_cache_bytes": (ctypes.c_int64, [c_int32, c_int32]),
    "riptrm_trs_bind_cache": (c_int32, [c_void_p, c_void_p, ctypes.c_int64, c_int32, c_int32]),
    "riptrm_trs_cache_stats": (c_int32, [c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "riptrm_trs_skip_stats": (c_int32, [c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "riptrm_sym_tridiag": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                                     c_int64, c_void_p]),
    "riptrm_sym_eig": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p,
                                 c_int32]),
    "riptrm_trs_backend_status": (c_int32, [ctypes.c_char_p, c_int32]),
    "riptrm_persist_trace": (c_int32, [c_void_p, c_void_p, c_int32]),
    "riptrm_set_spass_kind": (c_int32, [c_void_p, c_int32]),
    "riptrm_get_spass_calibration": (c_int32, [c_void_p, ctypes.POINTER(c_double), ctypes.POINTER(c_double), P_int32]),
    "riptrm_profile_enable": (c_int32, [c_void_p, c_int32]),
    "riptrm_profile_read": (c_int32, [c_void_p, ctypes.POINTER(c_double), ctypes.POINTER(c_int64),
                                      ctypes.POINTER(c_double), ctypes.POINTER(c_int64)]),
    "riptrm_si_workspace_bytes": (c_int64, [c_int32, c_int32, c_int32, c_int32, c_int32]),
    "riptrm_si_workspace_offset": (c_int64, [c_int32, c_int32, c_int32, c_int32, c_int32, c_int32]),
    "riptrm_si_bind": (c_int32, [c_void_p, ctypes.POINTER(RiptrmSIProblem), c_int32, c_void_p, c_int64, c_int32]),
    "riptrm_si_hvp": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "riptrm_si_tcg": (c_int32, [c_void_p, ctypes.POINTER(RiptrmOptions), c_void_p, c_void_p, c_void_p, c_void_p]),
    "riptrm_si_profile_enable": (c_int32, [c_void_p, c_int32]),
    "riptrm_si_profile_read": (c_int32, [c_void_p, ctypes.POINTER(c_double)]),
    "riptrm_stiefel_inner": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int64, c_void_p, c_void_p, c_void_p,
                                       c_void_p]),
    "riptrm_stiefel_proj": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int64, c_void_p, c_void_p, c_void_p]),
    "riptrm_stiefel_retr": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int64, c_void_p, c_void_p, c_void_p]),
    "riptrm_stiefel_ehess2rhess": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int64, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_void_p]),
    "riptrm_trs_gep": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p,
                                 c_double, c_void_p, c_void_p, c_void_p, c_void_p]),
    "riptrm_si_solve": (c_int32, [c_void_p, ctypes.POINTER(RiptrmOptions), c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_int32]),
}


def header_symbols(path: str = HEADER_PATH) -> List[str]:
    """Function names declared in include/riptrm.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(riptrm_[a-z0-9_]+)\s*\(", txt)))


def header_constants(path: str = HEADER_PATH) -> Dict[str, int]:
    """#define NAME <int> and enum members of include/riptrm.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out: Dict[str, int] = {}
    for name, val in re.findall(r"#define\s+(RIPTRM_[A-Z0-9_]+)\s+(-?\d+)", txt):
        out[name] = int(val)
    for body in re.findall(r"enum\s+\w+\s*\{(.*?)\}", txt, flags=re.S):
        cur = -1
        for item in body.split(","):
            item = item.strip()
            if not item:
                continue
            if "=" in item:
                nm, v = [t.strip() for t in item.split("=")]
                cur = int(v)
            else:
                nm = item
                cur += 1
            out[nm] = cur
    return out


CONST = header_constants() if os.path.exists(HEADER_PATH) else {}

_lib: Optional[ctypes.CDLL] = None


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load the HIP library (cached).  Raises RuntimeError if it is missing.  RIPTRM_LIB names an
    alternative in-tree build (A/B measurements of compile-time variants)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("RIPTRM_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"libriptrm_hip.so not built at {path}; run __graft_entry__.build() "
                           "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.riptrm_abi_version() != CONST.get("RIPTRM_ABI_VERSION", 1):
        raise RuntimeError("libriptrm_hip.so ABI version mismatch with include/riptrm.h")
    _lib = lib
    return lib


class Context:
    """Owns one ``riptrm_ctx`` (one per GPU per process)."""

    def __init__(self, device: int = 0, stream: int = 0):
        self.lib = load()
        h = c_void_p()
        rc = self.lib.riptrm_ctx_create(ctypes.byref(h), int(device), c_void_p(stream or None))
        if rc != 0:
            raise RuntimeError(f"riptrm_ctx_create failed (code {rc}): no gfx950 device {device}?")
        self.h = h

    def check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.riptrm_last_error(self.h)
            raise RuntimeError(f"{what} failed (code {rc}): {msg.decode() if msg else ''}")

    def set_stream(self, stream: int):
        self.check(self.lib.riptrm_ctx_set_stream(self.h, c_void_p(stream or None)), "riptrm_ctx_set_stream")

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.riptrm_ctx_destroy(self.h)
            self.h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
