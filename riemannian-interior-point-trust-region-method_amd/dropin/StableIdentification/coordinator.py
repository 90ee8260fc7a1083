"""Drop-in ``coordinator`` module for the reference's StableIdentification simulator.

Same mechanism as ``dropin/NonnegPCA/coordinator.py``: the reference's Simulator imports the
module named by ``cfg.problem_coordinator_name`` (``src/base/base_simulator.py:44-49``); with this
directory first on ``sys.path`` it gets ``si.SICoordinator``, which reads the files of
``src/StableIdentification/coordinator.py:13-152`` (noisyX_<i> / X_<i>, dim, constset,
init{J,R,Q}_<point>, initineqLagmult) and returns an ``si.SIProblem`` for the MI355X ``RIPTRM``.
"""
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(1, _PKG)

from si import SICoordinator as _StructuredCoordinator  # noqa: E402


class Coordinator(_StructuredCoordinator):
    """``coordinator.Coordinator(cfg)`` as the reference's Simulator constructs it (one argument)."""

    def __init__(self, cfg, root: str = "."):
        if not (hasattr(cfg, "problem_coordinator_name") or (isinstance(cfg, dict) and "problem_coordinator_name" in cfg)):
            raise AssertionError("cfg lacks 'problem_coordinator_name'")   # problem_coordinator.py:16
        super().__init__(cfg, root=root)
