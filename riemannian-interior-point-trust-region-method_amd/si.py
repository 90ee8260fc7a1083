"""StableIdentification on the MI355X: problem descriptor, coordinator and batched engine.

The reference (``src/StableIdentification/coordinator.py:13-187``) builds a pymanopt Product
(SkewSymmetric(d), SPD(d), SPD(d)) problem whose cost and m box constraints are autograd closures
over the trajectory data X / XP.  The drop-in takes the data instead (``SIProblem``) and runs every
RIPTRM solve of a batch (the ``problem_initialpoint`` / ``problem_instance`` axes) inside ONE HIP
launch, one workgroup per instance (``csrc/riptrm_si.hip``: a 64-lane wave up to d = 8, one thread per
element of a d x d block above, d <= RIPTRM_SI_DMAX).  No CPU fallback.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

import riptrm_native as N
from engine import BatchResult, C, NSTAT, NLOG, ResolvedOptions, TCG_NAMES, _stream_handle, assemble_log, resolve_options


def expand_constset(constset) -> np.ndarray:
    """constset.csv rows -> (m, 5) table [kind, r, c, p0, p1] in the reference's constraint order
    (coordinator.py:132-152): type 0/1 -> (-A_rc + ls, A_rc - rs); type 2 -> -(A_rc - c)^2 + k^2."""
    rows = []
    for row in np.atleast_2d(np.asarray(constset, dtype=np.float64)):
        t, r, c = row[0], int(row[1]), int(row[2])
        if t == 0 or t == 1:
            rows.append((0, r, c, row[3], 0.0))
            rows.append((1, r, c, row[4], 0.0))
        elif t == 2:
            rows.append((2, r, c, row[3], row[4] ** 2))
        else:
            raise ValueError("Invalid constraint type")
    return np.asarray(rows, dtype=np.float64).reshape(-1, 5)


@dataclass
class SIProblem:
    """Structured StableIdentification problem (coordinator.py:49-179)."""
    X: Any                      # (d, N): trajectories without their last column, stacked
    XP: Any                     # (d, N): without their first column
    h: float
    constset: Any               # constset.csv rows
    initialpoint: Any           # [J, R, Q] (d x d each)
    initialineqLagmult: Any     # (m,)
    initialeqLagmult: Any = field(default_factory=lambda: np.array([]))

    @property
    def d(self) -> int:
        return int(np.asarray(self.X).shape[0])

    @property
    def N(self) -> int:
        return int(np.asarray(self.X).shape[1])

    @property
    def cons(self) -> np.ndarray:
        return expand_constset(self.constset)

    @property
    def m(self) -> int:
        return int(self.cons.shape[0])

    @property
    def num_ineqconstraints(self) -> int:
        return self.m

    @property
    def has_eqconstraints(self) -> bool:
        return False

    @property
    def manifold_dim(self) -> int:
        d = self.d
        return d * (d - 1) // 2 + d * (d + 1)

    @property
    def typical_dist(self) -> float:
        # Product.typical_dist = sqrt(sum typical_dist_i^2), each sqrt(dim_i) (pymanopt)
        return math.sqrt(self.manifold_dim)

    def point_array(self) -> np.ndarray:
        return np.stack([np.asarray(a, dtype=np.float64) for a in self.initialpoint])


def synthetic_problem(d: int, seed: int, starts: int = 1, N: int = 20, Xset=(1, 2, 3, 4, 5),
                       oneboxratio: float = 0.2, twoboxratio: float = 0.1, snr: float = 10.0, h: float = 0.02):
    """A StableIdentification instance of block size d by the reference's dataset recipe
    (src/StableIdentification/generator.py:18-134, config_dataset.yaml: N 20, one-box ratio 0.2,
    two-box ratio 0.1, snr 10 dB, h 0.02, 5 trajectories), seeded (numpy legacy RandomState):
      * true (J, R, Q): skew / SPD random points, A = (J - R) Q (:55-64);
      * constraints on floor(ratio d^2) random entries of A (:66-109): one-box [A - a|A|, A + b|A|],
        two-box [-|A| - a|A|, |A| + b|A|] plus -(A - c)^2 + k^2 <= 0 with c = cc A;
      * trajectories x_i = exp(i h A) x_0 ELEMENTWISE (np.exp, as :124) from x_0 ~ U(-1000, 1000)^d,
        AWGN at snr dB (:111-120), normalised (:127-128); X / XP = the noisy ones without their
        last / first column, stacked (coordinator.py:54-90).
    One deviation: the reference draws the constraint values around the true A and then finds
    strictly interior starts with RALM (:136-207, out of scope).  Here a start is the true point
    congruence-perturbed (J + 0.05 skew noise, R, Q -> E R E^T with E = I + 0.05 sym noise), the
    constraint values are drawn around start 0's A (so it is strictly feasible: the two-box radius
    is k = kc |A - c| with kc in [0.2, 0.8)), and further starts (start 0 perturbed the same way at
    2e-3) are kept only if strictly feasible.
    y0 = ones(m).  Returns (X, XP, h, constset rows, [(x0, y0), ...])."""
    rs = np.random.RandomState(seed)

    def skew_pt():
        a = rs.randn(d, d)
        return (a - a.T) / 2

    def spd_pt():
        q, _ = np.linalg.qr(rs.randn(d, d))
        return (q * rs.uniform(0.5, 2.0, d)) @ q.T

    J, R, Q = skew_pt(), spd_pt(), spd_pt()
    A = (J - R) @ Q

    def perturb(x, eps=0.05):
        e = np.eye(d) + eps * (lambda b: (b + b.T) / 2)(rs.randn(d, d))
        return np.stack([x[0] + eps * skew_pt(), e @ x[1] @ e.T, e @ x[2] @ e.T])

    x_first = perturb(np.stack([J, R, Q]))
    A0 = (x_first[0] - x_first[1]) @ x_first[2]
    nel = d * d
    n1, n2 = int(nel * oneboxratio), int(nel * twoboxratio)
    idx = rs.permutation(nel)[:n1 + n2]
    rows = []
    for t, cind in enumerate(idx):
        r, c = cind % d, cind // d
        av = A0[r, c]
        aa = abs(av)
        if t < n1:
            rows.append([0, r, c, av - rs.uniform(0.2, 0.8) * aa, av + rs.uniform(0.2, 0.8) * aa])
        else:
            cc = rs.uniform(0.2, 0.8) * av
            k = rs.uniform(0.2, 0.8) * abs(av - cc)
            rows.append([1, r, c, -aa - rs.uniform(0.2, 0.8) * aa, aa + rs.uniform(0.2, 0.8) * aa])
            rows.append([2, r, c, cc, k])
    constset = np.asarray(rows, dtype=np.float64)
    Xs = XPs = None
    for _ in Xset:
        x0 = -1000 + 2000 * rs.rand(d)
        Xt = np.zeros((d, N))
        Xn = np.zeros((d, N))
        for i in range(N):
            xi = x0 if i == 0 else np.exp(i * h * A) @ x0
            Xt[:, i] = xi
            p = np.mean(np.abs(xi) ** 2) / 10 ** (snr / 10)
            Xn[:, i] = xi + np.sqrt(p) * rs.randn(d)
        Xn = Xn / np.linalg.norm(Xn[:, 0])
        Xs = Xn[:, :N - 1] if Xs is None else np.hstack((Xs, Xn[:, :N - 1]))
        XPs = Xn[:, 1:] if XPs is None else np.hstack((XPs, Xn[:, 1:]))
    cons = expand_constset(constset)

    def feasible(x):
        Ax = (x[0] - x[1]) @ x[2]
        for kind, r, c, p0, p1 in cons:
            kind, r, c = int(kind), int(r), int(c)
            a = Ax[r, c]
            g = (-a + p0) if kind == 0 else ((a - p0) if kind == 1 else (-(a - p0) ** 2 + p1))
            if not g < 0:
                return False
        return bool(np.all(np.linalg.eigvalsh(x[1]) > 0) and np.all(np.linalg.eigvalsh(x[2]) > 0))

    assert feasible(x_first), "start 0 must be strictly feasible by construction"
    m = cons.shape[0]
    out = [(x_first, np.ones(m))]
    tries = 0
    while len(out) < starts and tries < 100 * starts:
        tries += 1
        x = perturb(x_first, 2e-3)
        if feasible(x):
            out.append((x, np.ones(m)))
    assert len(out) == starts, "could not draw enough strictly feasible starts"
    return Xs, XPs, h, constset, out


def si_manviofun(problem, x):
    """src/StableIdentification/simulator.py:11-32 (host copy; the device computes its own)."""
    J, R, Q = x[0], x[1], x[2]
    manvio = 0
    manvio += np.linalg.norm(J + J.T)
    manvio += np.linalg.norm(R - R.T)
    manvio += np.linalg.norm(Q - Q.T)
    if not np.all(np.linalg.eigvalsh(R) > 0):
        print("R is not positive definite.")
        manvio = np.inf
    if not np.all(np.linalg.eigvalsh(Q) > 0):
        print("Q is not positive definite.")
        manvio = np.inf
    return manvio


def si_manvio_kind(f) -> int:
    """Classify 'manviofun' for the product manifold: 0 (identically zero) or the SI simulator's."""
    if f is None:
        return C["RIPTRM_MANVIO_ZERO"]
    good = [np.zeros((3, 3)), np.eye(3), np.eye(3)]
    bad = [np.ones((3, 3)), np.eye(3), np.eye(3)]
    a, b = f(None, good), f(None, bad)
    if a == 0 and b == 0:
        return C["RIPTRM_MANVIO_ZERO"]
    if a == 0 and abs(b - 6.0) < 1e-12:
        return C["RIPTRM_MANVIO_SI"]
    raise NotImplementedError("manviofun must be 0 or the StableIdentification simulator's "
                              "(src/StableIdentification/simulator.py:11-32)")


class SICoordinator:
    """coordinator.py:13-179 with the reference's cfg keys and dataset layout
    (dataset/StableIdentification/<instance>/...)."""

    def __init__(self, cfg, root: str = "."):
        for key in ("problem_name", "problem_instance", "problem_initialpoint"):
            if not _has(cfg, key):
                raise AssertionError(f"cfg lacks '{key}'")
        self.cfg = cfg
        self.dataset_path = os.path.join(root, f"dataset/{_get(cfg, 'problem_name')}/{_get(cfg, 'problem_instance')}")

    def run(self) -> SIProblem:
        p = self.dataset_path
        noisy = bool(_get(self.cfg, "is_X_noisy", True))
        Xset = list(_get(self.cfg, "Xset", [1, 2, 3, 4, 5]))
        h = float(_get(self.cfg, "h", 0.02))
        X = XP = None
        for i in Xset:   # coordinator.py:71-88
            Xo = np.loadtxt(f"{p}/{'noisyX' if noisy else 'X'}_{i}.csv")
            n = Xo.shape[1]
            Xc, XPc = Xo[:, :n - 1], Xo[:, 1:n]
            X = Xc if X is None else np.hstack((X, Xc))
            XP = XPc if XP is None else np.hstack((XP, XPc))
        dim = int(np.loadtxt(f"{p}/dim.csv"))
        if X.shape[0] != dim:
            raise ValueError(f"inconsistent StableIdentification dataset at {p}")
        pt = _get(self.cfg, "problem_initialpoint")
        x0 = [np.loadtxt(f"{p}/init{c}_{pt}.csv") for c in "JRQ"]
        y0 = np.atleast_1d(np.loadtxt(f"{p}/initineqLagmult.csv"))
        return SIProblem(X=X, XP=XP, h=h, constset=np.loadtxt(f"{p}/constset.csv"), initialpoint=x0,
                         initialineqLagmult=y0)


def _has(cfg, key):
    return (key in cfg) if isinstance(cfg, dict) else hasattr(cfg, key)


def _get(cfg, key, default=None):
    if isinstance(cfg, dict):
        return cfg.get(key, default)
    return getattr(cfg, key, default)


class SIBatch:
    """A batch of StableIdentification solves on one GPU: one workgroup per instance, one launch."""

    def __init__(self, d: int, N_: int, m: int, batch: int, device: Optional[int] = None, log_capacity: int = 4096):
        if not torch.cuda.is_available():
            raise RuntimeError("SIBatch needs a ROCm GPU (gfx950); there is no CPU fallback")
        self.lib = N.load()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.d, self.N, self.m, self.batch, self.cap = int(d), int(N_), int(m), int(batch), int(log_capacity)
        self.dd = self.d * self.d
        nbytes = int(self.lib.riptrm_si_workspace_bytes(self.d, self.N, self.m, self.batch, self.cap))
        if nbytes < 0:
            raise ValueError(f"need 1 <= d <= {N.CONST['RIPTRM_SI_DMAX']}, 1 <= m <= 64 (d <= 8) or "
                             f"m <= 64 ceil(d^2 / 64) (d > 8), batch >= 1")
        self.ctx = N.Context(self.device.index, _stream_handle(self.device))
        self.ws = torch.zeros(nbytes + 256, dtype=torch.uint8, device=self.device)
        base = self.ws.data_ptr()
        self._pad = (-base) % 256
        self.ws_ptr = base + self._pad
        self.ws_bytes = nbytes
        self._keep: List[torch.Tensor] = []
        self.ro: Optional[ResolvedOptions] = None
        self._trs_ws = None   # (buffer, order, slots): Exact_RepMat at d >= 8 (manifold.dim > 96)

    def _view(self, kind: int, shape):
        off = int(self.lib.riptrm_si_workspace_offset(self.d, self.N, self.m, self.batch, self.cap, kind))
        count = int(np.prod(shape))
        start = self._pad + off
        return self.ws[start:start + count * 8].view(torch.float64).view(*shape)

    def x(self):
        return self._view(0, (self.batch, 3, self.d, self.d))

    def y(self):
        return self._view(1, (self.batch, self.m))

    def eta(self):
        return self._view(2, (self.batch, 3, self.d, self.d))

    def heta(self):
        return self._view(3, (self.batch, 3, self.d, self.d))

    def stats(self) -> np.ndarray:
        return self._view(4, (self.batch, NSTAT)).cpu().numpy().copy()

    def log_rows(self, count: int) -> np.ndarray:
        lg = self._view(5, (self.batch, self.cap, NLOG))
        return lg[:, :max(0, min(count, self.cap))].cpu().numpy()

    def _dev(self, a, shape) -> torch.Tensor:
        t = torch.as_tensor(np.asarray(a, dtype=np.float64)).reshape(shape)
        return t.to(self.device).contiguous()

    def load(self, X, XP, h: float, cons) -> "SIBatch":
        """X, XP: (d, N) shared by the batch or (batch, d, N); cons: (m, 5) or (batch, m, 5)."""
        X, XP, cons = np.asarray(X, np.float64), np.asarray(XP, np.float64), np.asarray(cons, np.float64)
        shared_data = X.ndim == 2
        shared_cons = cons.ndim == 2
        self.Xd = self._dev(X, X.shape)
        self.XPd = self._dev(XP, XP.shape)
        self.consd = self._dev(cons, cons.shape)
        pr = N.RiptrmSIProblem()
        pr.struct_size = ctypes.sizeof(N.RiptrmSIProblem)
        pr.d, pr.N, pr.m, pr.h = self.d, self.N, self.m, float(h)
        pr.X, pr.XP = self.Xd.data_ptr(), self.XPd.data_ptr()
        pr.data_stride = 0 if shared_data else self.d * self.N
        pr.cons = self.consd.data_ptr()
        pr.cons_stride = 0 if shared_cons else self.m * 5
        self.ctx.set_stream(_stream_handle(self.device))
        self.ctx.check(self.lib.riptrm_si_bind(self.ctx.h, ctypes.byref(pr), self.batch, ctypes.c_void_p(self.ws_ptr),
                                               self.ws_bytes, self.cap), "riptrm_si_bind")
        self._prob = pr
        return self

    def hvp(self, x, y, mu, v) -> torch.Tensor:
        X = self._dev(x, (self.batch, 3, self.d, self.d))
        Y = self._dev(y, (self.batch, self.m))
        V = self._dev(v, (self.batch, 3, self.d, self.d))
        M = self._dev(np.broadcast_to(np.asarray(mu, np.float64), (self.batch,)).copy(), (self.batch,))
        out = torch.zeros_like(X)
        self.ctx.set_stream(_stream_handle(self.device))
        self.ctx.check(self.lib.riptrm_si_hvp(self.ctx.h, ctypes.c_void_p(X.data_ptr()), ctypes.c_void_p(Y.data_ptr()),
                                              ctypes.c_void_p(M.data_ptr()), ctypes.c_void_p(V.data_ptr()),
                                              ctypes.c_void_p(out.data_ptr())), "riptrm_si_hvp")
        torch.cuda.synchronize(self.device)
        return out

    def tcg(self, x, y, mu, Delta):
        X = self._dev(x, (self.batch, 3, self.d, self.d))
        Y = self._dev(y, (self.batch, self.m))
        M = self._dev(np.broadcast_to(np.asarray(mu, np.float64), (self.batch,)).copy(), (self.batch,))
        D = self._dev(np.broadcast_to(np.asarray(Delta, np.float64), (self.batch,)).copy(), (self.batch,))
        self.ctx.set_stream(_stream_handle(self.device))
        self.ctx.check(self.lib.riptrm_si_tcg(self.ctx.h, None, ctypes.c_void_p(X.data_ptr()),
                                              ctypes.c_void_p(Y.data_ptr()), ctypes.c_void_p(M.data_ptr()),
                                              ctypes.c_void_p(D.data_ptr())), "riptrm_si_tcg")
        torch.cuda.synchronize(self.device)
        st = self.stats()
        js = st[:, C["RIPTRM_STAT_TCG_LAST_J"]].astype(int)
        stops = [TCG_NAMES[int(s)] for s in st[:, C["RIPTRM_STAT_TCG_LAST_STOP"]]]
        return self.eta().clone(), self.heta().clone(), js, stops

    def begin(self, x0, y0, option: Dict[str, Any], restart_every: int = 0) -> ResolvedOptions:
        d = self.d
        typical = math.sqrt(d * (d - 1) // 2 + d * (d + 1))
        ro = resolve_options(option, typical, self.cap, restart_every, manvio_classifier=si_manvio_kind)
        X = self._dev(x0, (self.batch, 3, d, d))
        Y = self._dev(y0, (self.batch, self.m))
        tdim = d * (d - 1) // 2 + d * (d + 1)
        if ro.exact and tdim > C["RIPTRM_TRS_DIM_MAX"]:
            # d >= 8: the subproblem's matrix (manifold.dim squared) no longer fits LDS; instances park
            # at each subproblem and the host's batched service (riptrm_trs_big.hip) solves them in
            # caller-owned HBM scratch, one slot per instance of a pass (riptrm_trs_bind_workspace)
            from engine import bind_trs_scratch, trs_workspace_slots
            slots = trs_workspace_slots(self.lib, tdim, self.batch)
            self._trs_ws = bind_trs_scratch(self.ctx, self.lib, self.device, self._trs_ws, tdim, slots)
        tabs = ro.device_tables(self.device)
        self._keep = [X, Y] + tabs
        self.ctx.set_stream(_stream_handle(self.device))
        self.ctx.check(self.lib.riptrm_si_solve(self.ctx.h, ctypes.byref(ro.c_opt), ctypes.c_void_p(X.data_ptr()),
                                                ctypes.c_void_p(Y.data_ptr()), ctypes.c_void_p(tabs[0].data_ptr()),
                                                ctypes.c_void_p(tabs[1].data_ptr()), ctypes.c_void_p(tabs[2].data_ptr()),
                                                len(ro.mu_tab)), "riptrm_si_solve")
        self.ro = ro
        return ro

    def trs_skip_stats(self):
        """(subproblems whose CG was decided on their eigenpairs, CGs skipped) since the context was
        created (riptrm_trs_skip_stats)."""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        self.ctx.check(self.lib.riptrm_trs_skip_stats(self.ctx.h, ctypes.byref(a), ctypes.byref(b)), "riptrm_trs_skip_stats")
        return int(a.value), int(b.value)

    def trs_cache_stats(self):
        """(subproblems served from the keyed eigendecomposition cache, subproblems served) of the
        last solve on the HBM Exact_RepMat path (riptrm_trs_cache_stats)."""
        h, t = ctypes.c_int64(0), ctypes.c_int64(0)
        self.ctx.check(self.lib.riptrm_trs_cache_stats(self.ctx.h, ctypes.byref(h), ctypes.byref(t)), "riptrm_trs_cache_stats")
        return int(h.value), int(t.value)

    def profile_enable(self, on: bool = True):
        self.ctx.check(self.lib.riptrm_si_profile_enable(self.ctx.h, 1 if on else 0), "riptrm_si_profile_enable")

    def profile_read(self) -> Dict[str, float]:
        out = (ctypes.c_double * C["RIPTRM_SI_PROF_NFIELDS"])()
        self.ctx.check(self.lib.riptrm_si_profile_read(self.ctx.h, out), "riptrm_si_profile_read")
        names = ("total", "prepare", "tcg", "hvp", "trial", "eval")
        return {k: float(out[i]) for i, k in enumerate(names)}

    def solve(self, x0, y0, option: Dict[str, Any], restart_every: int = 0) -> BatchResult:
        self.begin(x0, y0, option, restart_every)
        return self.result()

    def result(self) -> BatchResult:
        torch.cuda.synchronize(self.device)
        st = self.stats()
        count = st[:, C["RIPTRM_STAT_LOG_COUNT"]].astype(np.int64)
        cap = min(self.cap, int(self.ro.c_opt.log_capacity))
        slots = self.log_rows(int(count.max()) if self.batch else 0)
        logs, dropped = [], []
        for b in range(self.batch):   # one launch per solve: no draining, head + latest records kept
            rows, drop = assemble_log(slots[b], int(count[b]), cap)
            logs.append(rows.copy())
            dropped.append(drop)
        return BatchResult(x=self.x().clone(), y=self.y().clone(), stats=st, raw_log=logs, ro=self.ro,
                           dropped=np.array(dropped))
