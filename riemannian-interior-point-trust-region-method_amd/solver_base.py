"""Solver plugin surface: the ``Solver`` / ``BaseOutput`` / ``Output`` contract of the reference.

Mirrors the behaviour of ``src/base/base_solver.py:6-107`` (option merge, dict-of-lists log,
time/iteration stopping test) and ``src/solver/utils.py:13-16`` (``Output`` adds the Lagrange
multipliers), so that ``Simulator.save_output`` (``src/base/base_simulator.py:75-95``) and the
analyzer notebooks read our outputs unchanged.  wandb logging is not supported (no network);
``wandb_logging=True`` raises.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class BaseOutput:
    name: str
    x: Any = field(default_factory=list)
    option: Optional[Dict] = None
    log: Optional[Dict] = None


@dataclass
class Output(BaseOutput):
    ineqLagmult: Any = field(default_factory=list)
    eqLagmult: Any = field(default_factory=list)


class Solver:
    """Base solver: ``Solver(option)``; subclasses implement ``run(problem) -> Output``."""

    def __init__(self, solver_option: Dict[str, Any], *args, **kwargs):
        opts = {
            'maxtime': 100,
            'maxiter': 100,
            'wandb_logging': False,
            'callbackfun': lambda problem, xCur, option, eval: eval,
        }
        opts.update(solver_option)
        self.option = opts
        self.log: Dict[str, list] = {}
        self.name = type(self).__name__
        self.initialize_wandb()

    def initialize_wandb(self):
        if self.option.get("wandb_logging"):
            raise NotImplementedError("wandb logging is not available in this build (no network)")

    def run(self, problem):  # pragma: no cover - abstract
        raise NotImplementedError

    def add_log(self, iteration, start_time, eval, solver_status, excluded_time=0):
        """Append one row; the first row (iteration 0) creates the columns with time 0."""
        if iteration == 0:
            self.log = {"iteration": [0], "time": [0]}
            for k, v in list(eval.items()) + list(solver_status.items()):
                self.log[k] = [v]
            return
        self.log["iteration"].append(iteration)
        self.log["time"].append(time.time() - start_time - excluded_time)
        for k, v in list(eval.items()) + list(solver_status.items()):
            self.log[k].append(v)

    def check_stoppingcriterion(self, start_time, iteration, stopping_criteria, excluded_time=0):
        run_time = time.time() - start_time - excluded_time
        return stop_reason(self.option, run_time, iteration, stopping_criteria)


def stop_reason(option, run_time, iteration, stopping_criteria):
    """The stopping rule of base_solver.py:85-107: time, then iteration count; any extra
    (flag, message) criterion that holds overrides the reason."""
    stop, reason = False, None
    if run_time >= option["maxtime"]:
        stop, reason = True, f"Max time exceeded; runtime={run_time:.2f} and maxtime={option['maxtime']}"
    elif iteration >= option["maxiter"]:
        stop, reason = True, f"Max iteration count reached; maxiter={option['maxiter']} after {run_time:.2f} seconds"
    for flag, msg in stopping_criteria:
        if flag:
            stop, reason = True, f"{msg} after {run_time:.2f} seconds"
    return stop, reason
