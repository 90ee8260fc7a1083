"""Exact_RepMat trust-region subproblem solver on the MI355X (csrc/riptrm_trs.hip, riptrm_trs.h).

``TRSgep(A, a, B, Del, tolhardcase)`` keeps the reference's signature and return value
(src/solver/RIPTRM.py:218-299: ``(x, lam1, type)``); ``trs_gep_batched`` solves a batch of
subproblems held as torch tensors on the GPU (dim <= RIPTRM_TRS_DIM_MAX: one launch, the matrix in
LDS; larger: the HBM path — up to dim 149 the hand-written eigensolver and SciPy's CG restated in its
eigen-coordinates, 150..1024 the cooperative tridiagonalisation and the subproblem in T's coordinates,
rocSOLVER dsyevd above and for hard cases; the secular Newton — every subproblem of the batch in one
pass when the scratch budget allows).  Only B = I is supported — the one call site passes ``np.eye(xdim)``
(RIPTRM.py:441).  No CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import numpy as np
import torch

import riptrm_native as N
from engine import _stream_handle, trs_workspace_slots

C = N.CONST
KIND_NAMES = {C["RIPTRM_TRS_BOUNDARY"]: "boundary", C["RIPTRM_TRS_INTERIOR"]: "interior",
              C["RIPTRM_TRS_HARDCASE_1"]: "hardcase_1"}
DIM_MAX = C["RIPTRM_TRS_DIM_MAX"]

_ctx = {}


def _context(device: torch.device) -> N.Context:
    c = _ctx.get(device.index)
    if c is None:
        c = _ctx[device.index] = N.Context(device.index, _stream_handle(device))
    c.set_stream(_stream_handle(device))
    return c


_ws = {}


def bind_trs_workspace(ctx: N.Context, device: torch.device, order: int, slots: int = 1) -> torch.Tensor:
    """Allocate (or reuse) and bind the HBM scratch of Exact_RepMat above RIPTRM_TRS_DIM_MAX for
    matrices of order `order` (riptrm_trs_workspace_bytes / riptrm_trs_bind_workspace).  The
    tensor is kept alive with the context."""
    key = (id(ctx), device.index)
    have = _ws.get(key)
    if have is None or have[1] < order or have[2] < slots:
        nbytes = int(ctx.lib.riptrm_trs_workspace_bytes(int(order), int(slots)))
        buf = torch.empty(nbytes + 256, dtype=torch.uint8, device=device)
        have = _ws[key] = (buf, int(order), int(slots))
    buf, o, sl = have
    base = buf.data_ptr()
    ptr = base + (-base) % 256
    ctx.check(ctx.lib.riptrm_trs_bind_workspace(ctx.h, ctypes.c_void_p(ptr), buf.numel() - (ptr - base), o, sl),
              "riptrm_trs_bind_workspace")
    return buf


def trs_gep_batched(A: torch.Tensor, a: torch.Tensor, Delta: torch.Tensor, tolhardcase: float = 1e-8
                    ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """A: (batch, dim, dim) symmetric, a: (batch, dim), Delta: (batch,), fp64 contiguous on one GPU.
    Returns (x (batch, dim), lam1 (batch,), kind (batch,) int32 RIPTRM_TRS_*, mineig (batch,))."""
    if not torch.cuda.is_available():
        raise RuntimeError("trs_gep_batched needs a ROCm GPU (gfx950); there is no CPU fallback")
    if A.dim() != 3 or A.shape[1] != A.shape[2] or a.shape != A.shape[:2] or Delta.shape != A.shape[:1]:
        raise ValueError("expected A (batch, dim, dim), a (batch, dim), Delta (batch,)")
    dev = A.device
    for t in (A, a, Delta):
        if t.dtype != torch.float64 or t.device != dev or not t.is_contiguous():
            raise ValueError("expected contiguous float64 tensors on one GPU")
    B, dim = A.shape[0], A.shape[1]
    if dim < 1:
        raise ValueError("dim must be >= 1")
    ctx = _context(dev)
    if dim > DIM_MAX:   # HBM path: one slot of order dim per subproblem of a pass (riptrm_trs_workspace_bytes)
        bind_trs_workspace(ctx, dev, dim, trs_workspace_slots(ctx.lib, dim, B))
    x = torch.empty((B, dim), dtype=torch.float64, device=dev)
    lam1 = torch.empty(B, dtype=torch.float64, device=dev)
    kind = torch.empty(B, dtype=torch.int32, device=dev)
    mineig = torch.empty(B, dtype=torch.float64, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    ctx.check(ctx.lib.riptrm_trs_gep(ctx.h, dim, B, p(A), dim, dim * dim, p(a), dim, p(Delta), float(tolhardcase),
                                     p(x), p(lam1), p(kind), p(mineig)), "riptrm_trs_gep")
    return x, lam1, kind, mineig


def TRSgep(A, a, B, Del, tolhardcase=1e-4):
    """RIPTRM.py:218-299 on the GPU: returns (x, lam1, type) as numpy / float / str."""
    A = np.asarray(A, dtype=np.float64)
    if B is not None and not np.array_equal(np.asarray(B), np.eye(A.shape[0])):
        raise NotImplementedError("TRSgep on the GPU supports B = I only (the call site RIPTRM.py:441)")
    dev = torch.device("cuda", torch.cuda.current_device())
    At = torch.as_tensor(A, device=dev).reshape(1, *A.shape).contiguous()
    at = torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev).reshape(1, -1).contiguous()
    Dt = torch.tensor([float(Del)], dtype=torch.float64, device=dev)
    x, lam1, kind, _ = trs_gep_batched(At, at, Dt, tolhardcase)
    torch.cuda.synchronize(dev)
    k = int(kind[0])
    return x[0].cpu().numpy(), (0 if k == C["RIPTRM_TRS_INTERIOR"] else float(lam1[0])), KIND_NAMES[k]


def sym_eig(A: torch.Tensor, vectors: bool = True) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Batched symmetric eigendecomposition on the GPU (riptrm_sym_eig, csrc/riptrm_eig.h: the
    eigensolver the Exact_RepMat HBM service uses for manifold.dim 97..199).  A: (batch, dim, dim)
    symmetric float64 on one GPU, dim <= 199.  Returns (w (batch, dim) ascending, V (batch, dim, dim)
    with eigenvector j in row j -- V[k] @ A[k] @ V[k].T = diag(w[k]) -- or None, info (batch,))."""
    if not torch.cuda.is_available():
        raise RuntimeError("sym_eig needs a ROCm GPU (gfx950); there is no CPU fallback")
    if A.dim() != 3 or A.shape[1] != A.shape[2] or A.dtype != torch.float64 or not A.is_cuda:
        raise ValueError("expected A (batch, dim, dim) float64 on a GPU")
    B, dim = A.shape[0], A.shape[1]
    V = A.contiguous().clone()
    w = torch.empty((B, dim), dtype=torch.float64, device=A.device)
    info = torch.empty(B, dtype=torch.int32, device=A.device)
    ctx = _context(A.device)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    ctx.check(ctx.lib.riptrm_sym_eig(ctx.h, dim, B, p(V), dim, dim * dim, p(w), dim, p(info), 1 if vectors else 0),
              "riptrm_sym_eig")
    return w, (V if vectors else None), info


def sym_tridiag(A: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Batched tridiagonal reduction on the GPU (riptrm_sym_tridiag, csrc/riptrm_tri.h k_tridiag_dist: the
    first stage of the Exact_RepMat HBM service from order 150 on; dsytd2 lower).  A: (batch, dim, dim)
    symmetric float64 on one GPU, 64 <= dim <= 1024.  Returns (d (batch, dim), e (batch, dim) with
    e[:, :dim - 1] the off-diagonal, info (batch,))."""
    if not torch.cuda.is_available():
        raise RuntimeError("sym_tridiag needs a ROCm GPU (gfx950); there is no CPU fallback")
    if A.dim() != 3 or A.shape[1] != A.shape[2] or A.dtype != torch.float64 or not A.is_cuda:
        raise ValueError("expected A (batch, dim, dim) float64 on a GPU")
    A = A.contiguous()
    B, dim = A.shape[0], A.shape[1]
    d = torch.empty((B, dim), dtype=torch.float64, device=A.device)
    e = torch.zeros((B, dim), dtype=torch.float64, device=A.device)
    info = torch.empty(B, dtype=torch.int32, device=A.device)
    ctx = _context(A.device)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    ctx.check(ctx.lib.riptrm_sym_tridiag(ctx.h, dim, B, p(A), dim, dim * dim, p(d), p(e), dim, p(info)),
              "riptrm_sym_tridiag")
    return d, e, info
