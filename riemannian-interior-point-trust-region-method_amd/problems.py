"""Structured problem descriptors consumed by the HIP path.

The reference hands its solver a ``utils.NonlinearProblem`` holding n autograd closures
(``src/NonnegPCA/coordinator.py:17-95``).  Closures cannot run on the GPU, so the drop-in takes
the *data* that defines the problem instead:

* ``NonnegPCAProblem`` — Sphere(n), cost ``-x^T Z x`` (``coordinator.py:46-56``), constraints
  ``-x_i <= 0`` for every i (``coordinator.py:59-77``), initial point and multipliers
  (``coordinator.py:84-95``).
* ``Coordinator`` — loads it from the reference's dataset layout
  (``dataset/NonnegPCA/<instance>/{dim,Z,initx_<point>,initineqLagmult}.csv``,
  ``src/base/problem_coordinator.py:20``), i.e. what ``Coordinator(cfg).run()`` returns there.
* ``manviofun`` — the NonnegPCA simulator's manifold violation ``||x|| - 1``
  (``src/NonnegPCA/simulator.py:12-14``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any

import numpy as np


@dataclass
class NonnegPCAProblem:
    Z: Any                      # (n, n) fp64, numpy or torch
    initialpoint: Any           # (n,)
    initialineqLagmult: Any     # (n,)
    initialeqLagmult: Any = field(default_factory=lambda: np.array([]))

    @property
    def n(self) -> int:
        return int(self.Z.shape[0])

    @property
    def num_ineqconstraints(self) -> int:
        return self.n

    @property
    def has_eqconstraints(self) -> bool:
        return False

    # Sphere(n) facts used by the solver (RIPTRM.py:447, :857)
    @property
    def manifold_dim(self) -> int:
        return self.n - 1

    @property
    def typical_dist(self) -> float:
        return float(np.pi)

    def cost(self, x):
        """f(x) = -x^T Z x (host-side helper, coordinator.py:52-54)."""
        Z = np.asarray(self.Z.cpu() if hasattr(self.Z, "cpu") else self.Z, dtype=np.float64)
        x = np.asarray(x, dtype=np.float64)
        return -x @ Z @ x


def manviofun(problem, x):
    """Manifold violation of the sphere, src/NonnegPCA/simulator.py:12-14."""
    return np.linalg.norm(np.asarray(x)) - 1


class Coordinator:
    """Problem coordinator for NonnegPCA with the reference's cfg keys and dataset layout."""

    def __init__(self, cfg, root: str = "."):
        for key in ("problem_name", "problem_instance", "problem_initialpoint"):
            if not _has(cfg, key):
                raise AssertionError(f"cfg lacks '{key}'")
        self.cfg = cfg
        self.dataset_path = os.path.join(root, f"dataset/{_get(cfg, 'problem_name')}/{_get(cfg, 'problem_instance')}")

    def run(self) -> NonnegPCAProblem:
        p = self.dataset_path
        dim = int(np.loadtxt(f"{p}/dim.csv"))
        Z = np.loadtxt(f"{p}/Z.csv")
        x0 = np.loadtxt(f"{p}/initx_{_get(self.cfg, 'problem_initialpoint')}.csv")
        y0 = np.loadtxt(f"{p}/initineqLagmult.csv")
        if Z.shape != (dim, dim) or x0.shape != (dim,) or y0.shape != (dim,):
            raise ValueError(f"inconsistent NonnegPCA dataset at {p}")
        return NonnegPCAProblem(Z=Z, initialpoint=x0, initialineqLagmult=y0)


def _has(cfg, key):
    return (key in cfg) if isinstance(cfg, dict) else hasattr(cfg, key)


def _get(cfg, key):
    return cfg[key] if isinstance(cfg, dict) else getattr(cfg, key)
