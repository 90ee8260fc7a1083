"""NonnegPCA simulator flow + CSV writer with the reference's file layout.

``Simulator(cfg).run()`` follows ``src/NonnegPCA/simulator.py:21-42``: build the problem with the
coordinator, merge ``solver_option.common`` with ``solver_option.<name>`` and the NonnegPCA
``manviofun`` (``src/base/base_simulator.py:51-67``, ``src/NonnegPCA/simulator.py:16-19``),
run the solver, and write ``<output_path>/<output.name>_<attr>.csv`` for every attribute of the
Output exactly as ``Simulator.save_output`` does (``src/base/base_simulator.py:75-95``):
arrays with ``np.savetxt``, dicts through a one-row-per-entry pandas DataFrame (scalars wrapped
in lists first), anything else with ``csv.writer.writerows``.  Only ``RIPTRM`` is available as a
solver here; the reference's other solvers are out of scope.
"""
from __future__ import annotations

import copy
import csv
import logging
import os
from typing import Any, Dict, Iterable, List

import numpy as np

from problems import Coordinator, manviofun


def _cfg_get(cfg, key, default=None):
    if isinstance(cfg, dict):
        return cfg.get(key, default)
    return getattr(cfg, key, default)


def save_output(output_path: str, solver_name: str, output) -> List[str]:
    """Write every attribute of ``output`` like base_simulator.Simulator.save_output."""
    os.makedirs(output_path, exist_ok=True)
    written = []
    for attr, content in vars(output).items():
        path = f"{output_path}/{solver_name}_{attr}.csv"
        if isinstance(content, (np.matrix, np.ndarray)):
            np.savetxt(path, content)
        elif isinstance(content, dict):
            import pandas as pd
            content = dict(content)
            for key, value in content.items():
                if not isinstance(value, list):
                    content[key] = [value]
            pd.DataFrame(content).to_csv(path, index=False)
        else:
            with open(path, "w") as fh:
                csv.writer(fh).writerows(content)
        written.append(path)
    return written


class Simulator:
    """Runs the configured solvers on one NonnegPCA instance/initial point and saves the CSVs."""

    def __init__(self, cfg, root: str = "."):
        for key in ("problem_name", "problem_instance", "problem_initialpoint", "solver_name", "solver_option"):
            if _cfg_get(cfg, key) is None:
                raise AssertionError(f"cfg lacks '{key}'")
        self.cfg = cfg
        self.root = root
        self.logger = logging.getLogger(__name__)

    def solver_option(self, name: str) -> Dict[str, Any]:
        so = _cfg_get(self.cfg, "solver_option")
        option = copy.deepcopy(dict(_cfg_get(so, "common", {}) or {}))
        specific = _cfg_get(so, name)
        if specific is not None:
            option.update(dict(specific))
        option["manviofun"] = manviofun          # src/NonnegPCA/simulator.py:17-19
        return option

    def output_path(self) -> str:
        p = _cfg_get(self.cfg, "output_path")
        if p is None:
            p = (f"intermediate/{_cfg_get(self.cfg, 'problem_name')}/{_cfg_get(self.cfg, 'problem_instance')}/"
                 f"{_cfg_get(self.cfg, 'problem_initialpoint')}")
        return os.path.join(self.root, p)

    def run(self):
        problem = Coordinator(self.cfg, root=self.root).run()
        outputs = []
        names: Iterable[str] = _cfg_get(self.cfg, "solver_name")
        if isinstance(names, str):
            names = [names]
        for name in names:
            if name != "RIPTRM":
                raise NotImplementedError(f"solver {name!r}: only RIPTRM is implemented on the MI355X path")
            from RIPTRM import RIPTRM
            output = RIPTRM(self.solver_option(name)).run(copy.deepcopy(problem))
            save_output(self.output_path(), output.name, output)
            outputs.append(output)
        return outputs
