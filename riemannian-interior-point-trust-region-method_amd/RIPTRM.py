"""Drop-in ``RIPTRM`` solver plugin (MI355X / gfx950).

Same plugin contract as the reference ``src/solver/RIPTRM.py``: the simulator imports the
module named ``RIPTRM`` from its solver path and calls ``RIPTRM(option).run(problem)``
(``src/base/base_simulator.py:51-67``), getting an ``Output(name, x, option, log, ineqLagmult,
eqLagmult)`` whose ``log`` has the reference's columns, one row per inner iteration
(``RIPTRM.py:812-818``).  Differences, all explicit errors rather than silent fallbacks:

* ``TRS_solver='tCG'`` (what every shipped config selects) and ``'Exact_RepMat'`` (the class
  default, with ``second_order_stationarity``) at any size: up to ``manifold.dim = 96`` the matrix
  of HwCur lives in LDS (csrc/riptrm_trs.h), beyond that in HBM (csrc/riptrm_trs_big.hip), with the
  hand-written batched eigensolver (csrc/riptrm_eig.h) up to order 149, the hand-written
  distributed tridiagonalisation with the subproblem solved in T's coordinates (csrc/riptrm_tri.h)
  for orders 150..1024, and rocSOLVER's dsyevd only for that path's hard cases and above 1024;
* the problem is a structured descriptor (``problems.NonnegPCAProblem`` or
  ``si.SIProblem`` for StableIdentification) instead of a list of autograd closures, because
  closures cannot execute on the GPU;
* ``manviofun`` must be 0 or the problem's simulator function (NonnegPCA ``||x|| - 1``,
  StableIdentification's symmetry / definiteness violation); ``callbackfun`` and wandb are not
  supported;
* ``do_euclidean_lincomb`` (RIPTRM.py:480-482, :514-517, :543-545) is accepted for both problems:
  the device evaluates the Lagrangian's derivatives in closed form, which is what both branches
  compute (the conversions are linear), up to rounding.  ``is_euclidean_embedded``
  (:567-568) is accepted for NonnegPCA (on the Sphere <egrad g_i, dx> = <rgrad g_i, dx> for
  tangent dx) and raises for StableIdentification (a different operator on the SPD factors).

``run_batch(problems)`` solves many instances of the same size at once (the reference runs its
Hydra multi-run axis one after another, ``config_simulation.yaml:35-42``).
"""
from __future__ import annotations

import copy
import warnings
from typing import Any, Dict, List, Sequence

import numpy as np
import torch

from engine import NonnegPCABatch, REFERENCE_DEFAULTS, manvio_kind, resolve_options
from problems import NonnegPCAProblem
from si import SIBatch, SIProblem, si_manvio_kind
from solver_base import Output, Solver


def _any_manvio_kind(f):
    try:
        return manvio_kind(f)
    except Exception:
        return si_manvio_kind(f)


class RIPTRM(Solver):
    """Riemannian interior point trust region method, tCG subproblem solver on the GPU."""

    def __init__(self, option: Dict[str, Any]):
        merged = dict(REFERENCE_DEFAULTS)
        merged.update(option)
        self.option = merged
        self.excluded_time = 0
        self.log: Dict[str, list] = {}
        self.name = f"RIPTRM_{self.option['TRS_solver']}"
        self.initialize_wandb()
        # validate early (raises on unsupported options)
        resolve_options(self.option, np.pi, 1, manvio_classifier=_any_manvio_kind)
        self.last_batch = None

    def run(self, problem) -> Output:
        return self.run_batch([problem])[0]

    SI_LOG_BYTES = 8e9   # upper bound of the StableIdentification device log per batch

    def run_batch(self, problems: Sequence[Any], log_capacity: int | None = None) -> List[Output]:
        """NonnegPCA: the device log is drained to the host whenever it is half full, so logs of
        any length are complete (log_capacity = rows of the device ring, default 8192).
        StableIdentification runs each solve in one launch: its log keeps the first
        log_capacity/2 and the latest records.  Its capacity is the requested one (default 65536
        rows per instance), capped so the batch's log stays within SI_LOG_BYTES (256 B per row)."""
        problems = list(problems)
        if not problems:
            return []
        if all(isinstance(p, SIProblem) for p in problems):
            req = 65536 if log_capacity is None else int(log_capacity)
            cap = max(16, min(req, int(self.SI_LOG_BYTES // (256 * len(problems)))))
            return self._run_batch_si(problems, cap)
        if log_capacity is None:
            log_capacity = 8192
        for p in problems:
            if not isinstance(p, NonnegPCAProblem):
                raise NotImplementedError(
                    f"RIPTRM (MI355X) needs a structured problem (problems.NonnegPCAProblem), got {type(p).__name__}")
            if p.has_eqconstraints:
                warnings.warn("Equality constraints detecred. Currently, RIPTRM does not support equality "
                              "constraints and will completely ignore them.", Warning)
        n = problems[0].n
        if any(p.n != n for p in problems):
            raise ValueError("run_batch needs instances of equal dimension n (group them by n)")
        B = len(problems)
        Zs = [np.asarray(p.Z.cpu() if hasattr(p.Z, "cpu") else p.Z, dtype=np.float64) for p in problems]
        # multi-start (the problem_initialpoint axis): one Z for every problem -> one shared S,
        # S-pass on the matrix cores
        shared = B > 1 and all(z is Zs[0] or np.array_equal(z, Zs[0]) for z in Zs[1:])
        eng = NonnegPCABatch(n, B, log_capacity=log_capacity, layout="shared" if shared else "sym")
        eng.load_Z(Zs[0] if shared else np.stack(Zs))
        self.last_layout = eng.layout_name
        x0 = np.stack([np.asarray(p.initialpoint, dtype=np.float64) for p in problems])
        y0 = np.stack([np.asarray(p.initialineqLagmult, dtype=np.float64) for p in problems])
        res = eng.solve(x0, y0, self.option)
        self.last_batch = res
        xs = res.x.cpu().numpy()
        ys = res.y.cpu().numpy()
        return self._outputs(res, [xs[b].copy() for b in range(B)], ys, log_capacity)

    def _run_batch_si(self, problems: List[SIProblem], log_capacity: int) -> List[Output]:
        """StableIdentification (src/StableIdentification/coordinator.py): one workgroup per
        problem, every solve of the batch in one launch."""
        p0 = problems[0]
        d, N_, m = p0.d, p0.N, p0.m
        if any((p.d, p.N, p.m) != (d, N_, m) for p in problems):
            raise ValueError("run_batch needs StableIdentification problems of equal (d, N, m)")
        for p in problems:
            if p.has_eqconstraints:
                warnings.warn("Equality constraints detecred. Currently, RIPTRM does not support equality "
                              "constraints and will completely ignore them.", Warning)
        if self.option.get('is_euclidean_embedded'):
            # RIPTRM.py:567-568: <egrad g_i, dx> in the manifold metric; on the SPD factors that is
            # tr(X^-1 G X^-1 dX), not <rgrad g_i, dx> = tr(sym(G) dX): a different operator
            raise NotImplementedError("is_euclidean_embedded=True changes Gxajfun on the SPD factors and is not "
                                      "implemented for StableIdentification on the device")
        B = len(problems)
        eng = SIBatch(d, N_, m, B, log_capacity=log_capacity)

        def _same(a, b):   # `is` only as a per-field fast path
            return a is b or np.array_equal(a, b)

        same = all(_same(p.X, p0.X) and _same(p.XP, p0.XP) and _same(p.cons, p0.cons) and p.h == p0.h
                   for p in problems)
        if same:   # the problem_initialpoint axis: one data set, many starts
            eng.load(p0.X, p0.XP, p0.h, p0.cons)
        else:
            if any(p.h != p0.h for p in problems):
                raise ValueError("run_batch needs one h per batch")
            eng.load(np.stack([p.X for p in problems]), np.stack([p.XP for p in problems]), p0.h,
                     np.stack([p.cons for p in problems]))
        self.last_layout = "si-shared" if same else "si"
        x0 = np.stack([p.point_array() for p in problems])
        y0 = np.stack([np.asarray(p.initialineqLagmult, dtype=np.float64) for p in problems])
        res = eng.solve(x0, y0, self.option)
        self.last_batch = res
        xs = res.x.cpu().numpy()
        ys = res.y.cpu().numpy()
        return self._outputs(res, [[xs[b, 0].copy(), xs[b, 1].copy(), xs[b, 2].copy()] for b in range(B)], ys,
                             log_capacity)

    def _outputs(self, res, xs, ys, log_capacity) -> List[Output]:
        outs = []
        B = len(xs)
        for b in range(B):
            opt = copy.copy(self.option)
            err = res.error(b)
            if err is not None:   # RIPTRM.py:961-966: print the error, no stoppingcriterion
                print(f"Error: {err}")
            reason = res.stopping_criterion(b)
            if reason is not None:
                opt["stoppingcriterion"] = reason
            dropped = int(res.dropped[b]) if res.dropped is not None else 0
            if dropped > 0:
                warnings.warn(f"instance {b}: log capacity {log_capacity} exceeded within one device launch; "
                              f"{dropped} records from the middle of the log were dropped (the first and the "
                              f"latest records are kept)")
            log = res.log(b)
            if self.option.get("verbosity", 0) == 1:
                for it, c, r, m, st in zip(log["iteration"], log["cost"], log["residual"], log["mu"],
                                           log["inner_status"]):
                    if st in (None, "converged", "max-time-exceeded", "max-iter-exceeded"):
                        print(f"Outer iteration: {it}, Cost: {c}, KKT residual: {r}, mu: {m}")
                if reason:
                    print(reason)
            outs.append(Output(name=self.name, x=xs[b], option=opt, log=log,
                               ineqLagmult=ys[b].copy(), eqLagmult=[]))
        self.log = outs[0].log if B == 1 else {}
        return outs
