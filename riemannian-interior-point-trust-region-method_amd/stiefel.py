"""Batched Stiefel(n, p) manifold operations on the MI355X (csrc/riptrm_stiefel.hip).

SURVEY.md §8a A14: required by north_star ("the Sphere/Stiefel projection+retraction from pymanopt
re-implemented as HIP kernels") although the reference's problems do not use Stiefel; the API
mirrors pymanopt's ``Stiefel`` methods on batches of (n, p) matrices held as torch tensors on the
GPU (shape (batch, n, p), fp64, contiguous).  No CPU fallback.
"""
from __future__ import annotations

import ctypes
import math

import torch

import riptrm_native as N
from engine import _stream_handle


class StiefelBatch:
    """pymanopt.manifolds.Stiefel(n, p) operations on `batch` points at once."""

    def __init__(self, n: int, p: int, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("StiefelBatch needs a ROCm GPU (gfx950); there is no CPU fallback")
        if not (1 <= p <= N.CONST["RIPTRM_STIEFEL_PMAX"] and p <= n):
            raise ValueError("need 1 <= p <= min(n, 64)")
        self.lib = N.load()
        self.n, self.p = int(n), int(p)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.ctx = N.Context(self.device.index, _stream_handle(self.device))
        self.dim = n * p - p * (p + 1) // 2
        self.typical_dist = math.sqrt(p)

    def _chk(self, *ts):
        for t in ts:
            if t.dtype != torch.float64 or t.device != self.device or not t.is_contiguous() or \
                    t.dim() != 3 or t.shape[1:] != (self.n, self.p) or t.shape[0] != ts[0].shape[0]:
                raise ValueError(f"expected contiguous float64 (batch, {self.n}, {self.p}) tensors on {self.device}")
        self.ctx.set_stream(_stream_handle(self.device))
        return ts[0].shape[0]

    def _ptr(self, t):
        return ctypes.c_void_p(t.data_ptr())

    def inner_product(self, X, U, V) -> torch.Tensor:
        B = self._chk(X, U, V)
        out = torch.empty(B, dtype=torch.float64, device=self.device)
        self.ctx.check(self.lib.riptrm_stiefel_inner(self.ctx.h, self.n, self.p, B, self.n * self.p, self._ptr(X),
                                                     self._ptr(U), self._ptr(V), self._ptr(out)), "riptrm_stiefel_inner")
        return out

    def projection(self, X, U) -> torch.Tensor:
        B = self._chk(X, U)
        out = torch.empty_like(U)
        self.ctx.check(self.lib.riptrm_stiefel_proj(self.ctx.h, self.n, self.p, B, self.n * self.p, self._ptr(X),
                                                    self._ptr(U), self._ptr(out)), "riptrm_stiefel_proj")
        return out

    to_tangent_space = projection
    euclidean_to_riemannian_gradient = projection

    def retraction(self, X, U) -> torch.Tensor:
        B = self._chk(X, U)
        out = torch.empty_like(X)
        self.ctx.check(self.lib.riptrm_stiefel_retr(self.ctx.h, self.n, self.p, B, self.n * self.p, self._ptr(X),
                                                    self._ptr(U), self._ptr(out)), "riptrm_stiefel_retr")
        return out

    def euclidean_to_riemannian_hessian(self, X, G, H, U) -> torch.Tensor:
        B = self._chk(X, G, H, U)
        out = torch.empty_like(X)
        self.ctx.check(self.lib.riptrm_stiefel_ehess2rhess(self.ctx.h, self.n, self.p, B, self.n * self.p,
                                                           self._ptr(X), self._ptr(G), self._ptr(H), self._ptr(U),
                                                           self._ptr(out)), "riptrm_stiefel_ehess2rhess")
        return out
