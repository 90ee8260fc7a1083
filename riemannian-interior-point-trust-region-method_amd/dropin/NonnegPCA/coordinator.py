"""Drop-in ``coordinator`` module for the reference's NonnegPCA simulator.

The reference's ``Simulator.set_coordinator`` (``src/base/base_simulator.py:44-49``) does
``importlib.import_module(cfg.problem_coordinator_name).Coordinator(cfg)`` with
``problem_coordinator_name: "coordinator"`` (``src/NonnegPCA/config_simulation.yaml``).  Put this
directory first on ``sys.path`` and that lookup returns the structured
coordinator below: ``Coordinator(cfg).run()`` reads the same files as
``src/NonnegPCA/coordinator.py:17-95`` (``dataset/NonnegPCA/<instance>/{dim,Z,initx_<point>,
initineqLagmult}.csv``, relative to the working directory as in
``src/base/problem_coordinator.py:20``) and returns a ``problems.NonnegPCAProblem`` that the
MI355X ``RIPTRM`` consumes.
"""
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(1, _PKG)

from problems import Coordinator as _StructuredCoordinator  # noqa: E402


class Coordinator(_StructuredCoordinator):
    """``coordinator.Coordinator(cfg)`` as the reference's Simulator constructs it (one argument)."""

    def __init__(self, cfg, root: str = "."):
        if not (hasattr(cfg, "problem_coordinator_name") or (isinstance(cfg, dict) and "problem_coordinator_name" in cfg)):
            raise AssertionError("cfg lacks 'problem_coordinator_name'")   # problem_coordinator.py:16
        super().__init__(cfg, root=root)
