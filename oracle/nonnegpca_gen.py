"""NonnegPCA synthetic instance recipe (CPU) — TEST INFRASTRUCTURE ONLY.

Restates ``src/NonnegPCA/generator.py:9-65`` (ZGenerator, InitialPointGenerator 'feasible',
InitialIneqLagMultGenerator) with numpy's legacy RandomState and the same call order as the
reference generator's ``main`` (``generator.py:67-74``), seeded per instance so that the
reference's unseeded runs become reproducible: instance b uses ``RandomState(seed0 + b)``.
Defaults snr=0.5, delta=0.7 are ``src/NonnegPCA/config_dataset.yaml:7-8``.
"""
from __future__ import annotations

import numpy as np

SEED0 = 20251212


def generate_instance(n: int, seed: int, snr: float = 0.5, delta: float = 0.7,
                      initialpoints_type: str = "feasible"):
    rs = np.random.RandomState(seed)
    samplesize = np.floor(delta * n)
    S = rs.choice(n, samplesize.astype(int), replace=False)          # generator.py:20
    v = np.zeros(n)
    v[S] = 1 / np.sqrt(samplesize)                                    # generator.py:22
    Z = np.sqrt(snr) * np.outer(v, v)                                 # generator.py:23-24
    noise = rs.randn(n, n) / np.sqrt(n)                               # generator.py:25
    for ii in range(n):                                               # generator.py:26-27
        noise[ii, ii] = rs.randn() * 2 / np.sqrt(n)
    Z = Z + noise
    x0 = rs.rand(n)                                                   # generator.py:42-50
    x0 = x0 / np.linalg.norm(x0)
    if initialpoints_type == "feasible":
        x0 = np.abs(x0)
    y0 = np.ones(n)                                                   # generator.py:63
    return Z, x0, y0


def generate_batch(n: int, batch: int, seed0: int = SEED0, **kw):
    Zs, xs, ys = [], [], []
    for b in range(batch):
        Z, x0, y0 = generate_instance(n, seed0 + b, **kw)
        Zs.append(Z)
        xs.append(x0)
        ys.append(y0)
    return np.stack(Zs), np.stack(xs), np.stack(ys)
