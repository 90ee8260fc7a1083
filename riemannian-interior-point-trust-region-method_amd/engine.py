"""Batched NonnegPCA RIPTRM engine on one MI355X: device memory + the C-ABI calls.

PyTorch owns the device memory (S, workspace, tables) and the stream; every operation on the
hot path is a HIP kernel in ``libriptrm_hip.so``.  Layout in HBM:

* ``S``   one flat fp64 buffer, ``S_b = Z_b + Z_b^T`` per instance in one of two layouts:
  ``"sym"`` (default) = the upper triangle as 128 x 128 tiles, ~4 n^2 bytes per instance
  (69 MB at n = 4000, 8.9 GB for 128 instances); ``"full"`` = row-major n x n padded to 128
  columns, 8 n^2 bytes (131 MB at n = 4000).
* workspace: 16 state vectors per instance (batch, ld) fp64, per-instance scalars, stats and the
  per-inner-iteration log rows, active lists.

Host-side option handling mirrors ``RIPTRM.__init__`` (``src/solver/RIPTRM.py:305-365``): the
option callables (forcing functions, barrier schedule) are evaluated here into per-outer-
iteration tables, so the device reproduces the reference's mu sequence bit-exactly.
"""
from __future__ import annotations

import ctypes
import math
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

import riptrm_native as N

C = N.CONST
NLOG = C["RIPTRM_LOG_NFIELDS"]
NSTAT = C["RIPTRM_STAT_NFIELDS"]

TRS_NAMES = {C["RIPTRM_TRS_BOUNDARY"]: "boundary", C["RIPTRM_TRS_INTERIOR"]: "interior",
             C["RIPTRM_TRS_HARDCASE_1"]: "hardcase_1"}
TCG_NAMES = {C["RIPTRM_TCG_MAX_INNER_ITER"]: "MAX_INNER_ITER",
             C["RIPTRM_TCG_NEGATIVE_CURVATURE"]: "NEGATIVE_CURVATURE",
             C["RIPTRM_TCG_EXCEEDED_TR"]: "EXCEEDED_TR",
             C["RIPTRM_TCG_MODEL_INCREASED"]: "MODEL_INCREASED",
             C["RIPTRM_TCG_REACHED_TARGET_LINEAR"]: "REACHED_TARGET_LINEAR",
             C["RIPTRM_TCG_REACHED_TARGET_SUPERLINEAR"]: "REACHED_TARGET_SUPERLINEAR",
             C["RIPTRM_TCG_NONFINITE"]: "NONFINITE", C["RIPTRM_TCG_EIGFAIL"]: "EIGFAIL"}
ERROR_TEXT = {C["RIPTRM_ERR_NO_TCG_ITER"]: "manifold dimension 0: truncated CG cannot iterate",
              C["RIPTRM_ERR_BARRIER_TIMEOUT"]: "persistent lock-step: a peer workgroup did not arrive within 2 s",
              C["RIPTRM_ERR_NONFINITE"]: ("non-finite value (NaN/Inf) in the KKT residual, the tCG residual, the "
                                          "trust-region radius or <delta, H delta>; returning the iterate the outer "
                                          "step started from (the completed iterate when the residual at the outer "
                                          "loop head is the non-finite value)"),
              C["RIPTRM_ERR_EIGEN"]: ("Exact_RepMat: the eigendecomposition did not converge (eigensolver info != 0; "
                                      "scipy.linalg.eig raises LinAlgError); returning the iterate the outer step "
                                      "started from")}
STATUS_NAMES = {0: None, 1: "initial", 2: "converged", 3: "primal_infeasible", 4: "successful",
                5: "unsuccessful", 6: "max-time-exceeded", 7: "max-iter-exceeded"}
RU_NAMES = {0: None, 1: "reduced", 2: "expanded", 3: "unchanged"}

def assemble_log(slots: np.ndarray, k: int, cap: int):
    """Records of one instance in chronological order from its device log slots, given k records
    written since the last rebase into a log of `cap` slots (include/riptrm.h "Log slots": slot k
    while k < cap, then the first cap/2 slots keep the head and the rest is a ring of the latest
    records).  Returns (rows, dropped): dropped = records lost from the middle (0 unless k > cap)."""
    if k <= cap:
        return slots[:k], 0
    h = cap // 2
    t = cap - h
    k0 = k - t                                   # oldest record still in the ring
    order = [h + ((k0 - h + i) % t) for i in range(t)]
    return np.concatenate([slots[:h], slots[order]]), k - cap


def dxtype_name(code: int) -> str:
    """inner_info['dxtype'] (RIPTRM.py:734): TRSgep's type or f"tCG_{stop_tCG}"."""
    return TRS_NAMES[code] if code in TRS_NAMES else f"tCG_{TCG_NAMES[code]}"


# RIPTRM default_option (src/solver/RIPTRM.py:305-358)
REFERENCE_DEFAULTS: Dict[str, Any] = {
    'maxtime': 240, 'maxiter': 100, 'tolresid': 1e-15,
    'inner_maxiter': None, 'inner_maxtime': None,
    'initial_TR_radius': None, 'minimal_initial_TR_radius': 1e-15, 'maximal_TR_radius': 10,
    'rho': 0.1, 'reduction_regularization': 1e3, 'gamma': 0.25,
    'forcing_function_Lagrangian': lambda mu: max(mu, 1e-14),
    'forcing_function_complementarity': lambda mu: max(1e-3 * mu, 1e-14),
    'forcing_function_second_order': lambda mu: mu,
    'min_barrier_parameter': 1e-15,
    'TRS_solver': 'Exact_RepMat', 'second_order_stationarity': True,
    'do_euclidean_lincomb': False, 'is_euclidean_embedded': False,
    'TRS_tolresid': 1e-12, 'TRS_tolhardcase': 1e-8,
    'tCG_theta': 1, 'tCG_kappa': 0.1, 'tCG_mininner': 1,
    'checkTRSoptimality': False,
    'initial_barrier_parameter': 0.1,
    'barrier_parameter_update_r': 0.01, 'barrier_parameter_update_c': 0.5,
    'barrier_parameter_update_b': 0.8, 'do_simple_barrier_parameter_update': True,
    'const_left': 0.5, 'const_right': 1e+20,
    'basisfun': None,
    'verbosity': 0,
    'manviofun': lambda problem, x: 0,
    'callbackfun': None,
    'save_inner_iteration': True, 'wandb_logging': False,
    'do_exit_on_error': True,
}


def mu_schedule(o: Dict[str, Any], maxlen: int) -> List[float]:
    """mu_0, mu_1, ... exactly as RIPTRM.py:852 and :890-893 compute them (Python floats),
    truncated once the sequence reaches a fixed point (the device then repeats the last one)."""
    mu = o['initial_barrier_parameter']
    out = [mu]
    while len(out) < maxlen:
        if o['do_simple_barrier_parameter_update']:
            nxt = max(o['min_barrier_parameter'],
                      o['barrier_parameter_update_c'] * (mu ** (1 + o['barrier_parameter_update_r'])))
        else:
            nxt = max(o['min_barrier_parameter'],
                      min(o['barrier_parameter_update_b'] * mu,
                          o['barrier_parameter_update_c'] * (mu ** (1 + o['barrier_parameter_update_r']))))
        out.append(nxt)
        if nxt == mu:
            break
        mu = nxt
    return out


def manvio_kind(f) -> int:
    """Classify the 'manviofun' option numerically: 0 (identically zero) or 1 (||x|| - 1)."""
    if f is None:
        return C["RIPTRM_MANVIO_ZERO"]
    a = f(None, np.array([3.0, 4.0]))
    b = f(None, np.array([0.6, 0.8]))
    if abs(a) == 0 and abs(b) == 0:
        return C["RIPTRM_MANVIO_ZERO"]
    if abs(a - 4.0) < 1e-12 and abs(b) < 1e-12:
        return C["RIPTRM_MANVIO_SPHERE"]
    raise NotImplementedError("manviofun must be 0 or ||x||-1 (the NonnegPCA simulator's); "
                              "arbitrary Python callables cannot run on the device")


@dataclass
class ResolvedOptions:
    option: Dict[str, Any]
    c_opt: N.RiptrmOptions
    mu_tab: List[float]
    tolL_tab: List[float]
    tolC_tab: List[float]
    tol2_tab: List[float]

    @property
    def exact(self) -> bool:
        return self.c_opt.trs_solver == C["RIPTRM_TRS_SOLVER_EXACT_REPMAT"]

    def device_tables(self, device) -> List[torch.Tensor]:
        """(mu, tolL, tolC[, tol2]) tables on the device; tol2's pointer goes into c_opt.  The
        caller keeps the tensors alive while the solve runs."""
        tabs = [torch.tensor(t, dtype=torch.float64, device=device) for t in (self.mu_tab, self.tolL_tab, self.tolC_tab)]
        if self.exact and self.c_opt.second_order_stationarity:
            t2 = torch.tensor(self.tol2_tab, dtype=torch.float64, device=device)
            tabs.append(t2)
            self.c_opt.tol2_table = t2.data_ptr()
        else:
            self.c_opt.tol2_table = None
        return tabs


def resolve_options(option: Dict[str, Any], typical_dist: float, log_capacity: int,
                    restart_every: int = 0, manvio_classifier=None) -> ResolvedOptions:
    o = dict(REFERENCE_DEFAULTS)
    o.update(option or {})
    if o['TRS_solver'] not in ('tCG', 'Exact_RepMat'):
        raise ValueError(f"TRS_solver {o['TRS_solver']} is not supported.")   # RIPTRM.py:453-454
    if o.get('checkTRSoptimality'):
        raise NotImplementedError("checkTRSoptimality (a diagnostic print, RIPTRM.py:367-391) is not on the device path")
    if o.get('use_rand'):
        raise NotImplementedError("use_rand tCG start is not on the reference's path (RIPTRM.py:450)")
    if o.get('callbackfun') is not None:
        raise NotImplementedError("callbackfun cannot run on the device")
    if o.get('wandb_logging'):
        raise NotImplementedError("wandb logging is not available")
    maxiter = int(o['maxiter'])
    tab = mu_schedule(o, maxlen=max(2, maxiter + 2))
    tolL = [float(o['forcing_function_Lagrangian'](m)) for m in tab]
    tolC = [float(o['forcing_function_complementarity'](m)) for m in tab]
    exact = o['TRS_solver'] == 'Exact_RepMat'
    sos = bool(exact and o['second_order_stationarity'])
    tol2 = [float(o['forcing_function_second_order'](m)) for m in tab] if sos else []
    c = N.RiptrmOptions()
    c.struct_size = ctypes.sizeof(N.RiptrmOptions)
    c.maxiter = min(maxiter, 2 ** 31 - 2)
    c.inner_maxiter = -1 if o['inner_maxiter'] is None else int(o['inner_maxiter'])
    c.tcg_mininner = int(o['tCG_mininner'])
    c.save_inner_iteration = 1 if o['save_inner_iteration'] else 0
    c.manvio_kind = (manvio_classifier or manvio_kind)(o['manviofun'])
    c.log_capacity = int(log_capacity)
    c.restart_every = int(restart_every)
    c.maxtime = float(o['maxtime']) if o['maxtime'] is not None else math.inf
    c.inner_maxtime = -1.0 if o['inner_maxtime'] is None else float(o['inner_maxtime'])
    c.tolresid = float(o['tolresid'])
    c.initial_tr_radius = (typical_dist / 8) if o['initial_TR_radius'] is None else float(o['initial_TR_radius'])
    c.minimal_initial_tr_radius = float(o['minimal_initial_TR_radius'])
    c.maximal_tr_radius = float(o['maximal_TR_radius'])
    c.rho = float(o['rho'])
    c.reduction_regularization = float(o['reduction_regularization'])
    c.gamma = float(o['gamma'])
    c.tcg_theta = float(o['tCG_theta'])
    c.tcg_kappa = float(o['tCG_kappa'])
    c.const_left = float(o['const_left'])
    c.const_right = float(o['const_right'])
    c.trs_solver = C["RIPTRM_TRS_SOLVER_EXACT_REPMAT"] if exact else C["RIPTRM_TRS_SOLVER_TCG"]
    c.second_order_stationarity = 1 if sos else 0
    c.trs_tolhardcase = float(o['TRS_tolhardcase'])
    return ResolvedOptions(o, c, tab, tolL, tolC, tol2)


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


EXACT_BIG_CHUNK = 4        # lock-step iterations per advance on the HBM Exact_RepMat path
TRS_WS_BUDGET = 16 << 30   # bytes of HBM the Exact_RepMat scratch may take (RIPTRM_TRS_WS_GB overrides)


def trs_hbm_path(n: int) -> bool:
    """Exact_RepMat's subproblems go to the HBM service: above the LDS solver's size (manifold.dim =
    n - 1 > RIPTRM_TRS_DIM_MAX), or at every n with RIPTRM_TRS_HBM=1 (A/B; riptrm_solve_begin reads it)."""
    import os
    return n - 1 > C["RIPTRM_TRS_DIM_MAX"] or os.environ.get("RIPTRM_TRS_HBM", "") == "1"


def bind_trs_scratch(ctx, lib, device, have, order: int, slots: int):
    """Bind the HBM scratch of Exact_RepMat above RIPTRM_TRS_DIM_MAX (riptrm_trs_bind_workspace) for
    `slots` matrices of order `order`.  `have` is the (buffer, order, slots) this caller bound before
    (or None): it is reused when it is large enough and reallocated otherwise (a later begin() may ask
    for more slots once RIPTRM_TRS_WS_GB or the batch changed).  Returns the (buffer, order, slots)
    to keep."""
    if have is None or have[1] < order or have[2] < slots:
        nbytes = int(lib.riptrm_trs_workspace_bytes(int(order), int(slots)))
        have = (torch.empty(nbytes + 256, dtype=torch.uint8, device=device), int(order), int(slots))
    buf = have[0]
    base = buf.data_ptr()
    ptr = base + (-base) % 256
    ctx.check(lib.riptrm_trs_bind_workspace(ctx.h, ctypes.c_void_p(ptr), buf.numel() - (ptr - base), int(order),
                                            int(slots)), "riptrm_trs_bind_workspace")
    return have


def trs_workspace_slots(lib, order: int, want: int) -> int:
    """Slots of order `order` for the HBM Exact_RepMat path: one per subproblem served in the same
    pass (`want`), as many as the budget holds, at least one."""
    import os
    budget = int(float(os.environ.get("RIPTRM_TRS_WS_GB", TRS_WS_BUDGET / 2 ** 30)) * 2 ** 30)
    per = int(lib.riptrm_trs_workspace_bytes(int(order), 1))
    return max(1, min(int(want), budget // max(per, 1)))


TRS_CACHE_BUDGET = 16 << 30   # bytes of HBM the eigendecomposition cache may take (RIPTRM_TRS_CACHE_GB)


def trs_cache_wanted(lib, order: int, batch: int) -> int:
    """Bytes of the HBM Exact_RepMat path's eigendecomposition cache (riptrm_trs_bind_cache), or 0
    when RIPTRM_TRS_CACHE=0 or the whole batch does not fit the budget (the cache is all or none)."""
    import os
    if os.environ.get("RIPTRM_TRS_CACHE", "1") == "0":
        return 0
    budget = int(float(os.environ.get("RIPTRM_TRS_CACHE_GB", TRS_CACHE_BUDGET / 2 ** 30)) * 2 ** 30)
    nbytes = int(lib.riptrm_trs_cache_bytes(int(order), int(batch)))
    return nbytes if 0 < nbytes <= budget else 0


LAYOUTS = {"full": C["RIPTRM_LAYOUT_FULL"], "sym": C["RIPTRM_LAYOUT_SYMTILE"], "shared": C["RIPTRM_LAYOUT_SHARED"]}


class NonnegPCABatch:
    """A batch of NonnegPCA instances with a common n, resident on one GPU.

    layout "sym" (default) / "full": one S = Z + Z^T per instance.  layout "shared": ONE S for the
    whole batch (multi-start: same Z, different initial points — the reference's
    problem_initialpoint axis), S-pass on the fp64 matrix cores."""

    def __init__(self, n: int, batch: int, device: Optional[int] = None, log_capacity: int = 4096,
                 layout: str = "sym", stream_groups: int = 0, spass_kind: int = 1, drain_logs: bool = True,
                 persistent: int = 1):
        if not torch.cuda.is_available():
            raise RuntimeError("NonnegPCABatch needs a ROCm GPU (gfx950); there is no CPU fallback")
        if n < 2 or batch < 1:
            raise ValueError("need n >= 2 and batch >= 1")
        self.lib = N.load()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.n, self.batch, self.cap = int(n), int(batch), int(log_capacity)
        if layout not in LAYOUTS:
            raise ValueError(f"layout must be one of {sorted(LAYOUTS)}")
        self.layout_name = layout
        self.layout = LAYOUTS[layout]
        self.ld = int(self.lib.riptrm_nonnegpca_ld(self.n))
        self.rows = int(self.lib.riptrm_nonnegpca_rows(self.n))
        self.shared = layout == "shared"
        self.inst_stride = int(self.lib.riptrm_nonnegpca_s_elems(self.n, self.layout))
        self.ctx = N.Context(self.device.index, _stream_handle(self.device))
        self.ctx.check(self.lib.riptrm_set_stream_groups(self.ctx.h, int(stream_groups)), "riptrm_set_stream_groups")
        self.ctx.check(self.lib.riptrm_set_spass_kind(self.ctx.h, int(spass_kind)), "riptrm_set_spass_kind")
        # small symmetric-tile batches: the whole lock-step loop in one launch per chunk (k_persist)
        self.ctx.check(self.lib.riptrm_set_persistent(self.ctx.h, int(persistent)), "riptrm_set_persistent")
        self.S = torch.zeros((1 if self.shared else self.batch, self.inst_stride), dtype=torch.float64,
                             device=self.device)
        nbytes = int(self.lib.riptrm_workspace_bytes(self.n, self.batch, self.cap, self.layout))
        self.ws = torch.zeros(nbytes + 256, dtype=torch.uint8, device=self.device)
        base = self.ws.data_ptr()
        self._ws_pad = (-base) % 256
        self.ws_ptr = base + self._ws_pad
        self.ws_bytes = nbytes
        self.bound = False
        self._keep: List[torch.Tensor] = []
        self._trs_ws = None   # (buffer, order, slots) of Exact_RepMat above RIPTRM_TRS_DIM_MAX
        self._trs_cache: Optional[torch.Tensor] = None   # its eigendecomposition cache
        # log records copied to the host by drain_logs() (riptrm_log_rebase), per instance
        self.drain = bool(drain_logs)
        self._drained: List[List[np.ndarray]] = [[] for _ in range(self.batch)]
        self._dropped = np.zeros(self.batch, dtype=np.int64)

    # ---- views into the workspace -------------------------------------------------------
    def _view(self, kind: int, shape, dtype=torch.float64):
        off = int(self.lib.riptrm_workspace_offset(self.n, self.batch, self.cap, self.layout, kind))
        count = int(np.prod(shape))
        start = self._ws_pad + off
        return self.ws[start:start + count * 8].view(dtype).view(*shape)

    def vec(self, kind: int) -> torch.Tensor:
        """kind 0 = x, 1 = y, 2 = eta, 3 = Heta (batch, n) views (no copy)."""
        return self._view(kind, (self.batch, self.ld))[:, :self.n]

    def stats(self) -> np.ndarray:
        return self._view(4, (self.batch, NSTAT)).cpu().numpy().copy()

    def log_rows(self, count: int) -> np.ndarray:
        lg = self._view(5, (self.batch, self.cap, NLOG))
        return lg[:, :max(0, min(count, self.cap))].cpu().numpy()

    def _pending_logs(self, st: np.ndarray):
        """Per instance: the records written since the last rebase, in order, and how many of them
        the slots dropped."""
        k = (st[:, C["RIPTRM_STAT_LOG_COUNT"]] - st[:, C["RIPTRM_STAT_LOG_BASE"]]).astype(np.int64)
        cap = min(self.cap, int(self.ro.c_opt.log_capacity)) if getattr(self, "ro", None) else self.cap
        kmax = int(k.max()) if self.batch else 0
        slots = self.log_rows(kmax)
        out = []
        for b in range(self.batch):
            out.append(assemble_log(slots[b], int(k[b]), cap) if k[b] > 0 else (slots[b, :0], 0))
        return out

    def drain_logs(self):
        """Copy every instance's new log records to the host and rebase the device log
        (riptrm_log_rebase), so a solve of any length keeps its whole log."""
        torch.cuda.synchronize(self.device)
        st = self.stats()
        for b, (rows, dropped) in enumerate(self._pending_logs(st)):
            if len(rows):
                self._drained[b].append(rows.copy())
            self._dropped[b] += dropped
        self._sync_stream()
        self.ctx.check(self.lib.riptrm_log_rebase(self.ctx.h), "riptrm_log_rebase")

    # ---- data ---------------------------------------------------------------------------
    def _sync_stream(self):
        self.ctx.set_stream(_stream_handle(self.device))

    def load_Z(self, Z) -> "NonnegPCABatch":
        """Z: (batch, n, n) fp64 (numpy or torch).  S_b = Z_b + Z_b^T packed on the device.
        Shared layout: one (n, n) (or (1, n, n)) Z for the whole batch."""
        if isinstance(Z, np.ndarray) and not Z.flags.writeable:   # torch wants writable host memory
            Z = Z.copy()
        Zt = torch.as_tensor(Z, dtype=torch.float64)
        if self.shared:
            if Zt.dim() == 3 and Zt.shape[0] == 1:
                Zt = Zt[0]
            if Zt.shape != (self.n, self.n):
                raise ValueError(f"shared layout: Z must be {(self.n, self.n)}, got {tuple(Zt.shape)}")
            self.pack_one(Zt.to(self.device).contiguous(), 0)
            torch.cuda.synchronize(self.device)
            self.bind()
            return self
        if Zt.shape != (self.batch, self.n, self.n):
            raise ValueError(f"Z must be {(self.batch, self.n, self.n)}, got {tuple(Zt.shape)}")
        tmp = torch.empty((self.n, self.n), dtype=torch.float64, device=self.device)
        for b in range(self.batch):
            tmp.copy_(Zt[b])
            self.pack_one(tmp, b)
        torch.cuda.synchronize(self.device)
        self.bind()
        return self

    def pack_one(self, Zdev: torch.Tensor, slot: int):
        """S[slot] <- pack(Z + Z^T) from a contiguous (n, n) device tensor (riptrm_nonnegpca_pack)."""
        assert Zdev.is_contiguous() and Zdev.shape == (self.n, self.n) and Zdev.device == self.device
        self._sync_stream()
        self.ctx.check(self.lib.riptrm_nonnegpca_pack(self.ctx.h, ctypes.c_void_p(Zdev.data_ptr()), self.n,
                                                      self.n * self.n, self.n, 1,
                                                      ctypes.c_void_p(self.S[slot].data_ptr()), self.layout,
                                                      self.inst_stride), "riptrm_nonnegpca_pack")

    def unpack(self, slot: int) -> np.ndarray:
        """Host copy of S[slot] as a dense n x n matrix (tests / inspection)."""
        raw = self.S[slot].cpu().numpy()
        n, ld = self.n, self.ld
        if self.layout != LAYOUTS["sym"]:
            return raw[: self.rows * ld].reshape(self.rows, ld)[:n, :n].copy()
        ts, nt = 128, ld // 128
        wl = -(-(n - (nt - 1) * ts) // 32) * 32     # stored columns of the last tile column
        full = np.zeros((ld, ld))
        F = ts * ts
        for I in range(nt):
            base = F * (I * (nt - 1) - I * (I - 1) // 2) + I * ts * wl
            for J in range(I, nt):
                off = base + (J - I) * F
                rT = wl if I == nt - 1 else ts
                cT = wl if J == nt - 1 else ts
                blk = raw[off:off + rT * cT].reshape(rT, cT)
                full[I * ts:I * ts + rT, J * ts:J * ts + cT] = blk
                full[J * ts:J * ts + cT, I * ts:I * ts + rT] = blk.T
        return full[:n, :n].copy()

    def bind(self):
        self._sync_stream()
        self.ctx.check(self.lib.riptrm_nonnegpca_bind(self.ctx.h, ctypes.c_void_p(self.S.data_ptr()), self.n,
                                                      self.batch, self.layout, 0 if self.shared else self.inst_stride,
                                                      ctypes.c_void_p(self.ws_ptr), self.ws_bytes, self.cap),
                       "riptrm_nonnegpca_bind")
        self.bound = True

    def generate_synthetic(self, seed0: int = 20251212, snr: float = 0.5, delta: float = 0.7,
                           ids: Optional[Sequence[int]] = None):
        """Synthetic instances with the reference recipe's distribution
        (src/NonnegPCA/generator.py:9-65) drawn on the device with torch's Philox generator:
        Z = sqrt(snr) v v^T + N(0,1)/sqrt(n) with diagonal N(0,1)*2/sqrt(n), v = 1/sqrt(|S|) on a
        random floor(delta n)-subset; feasible x0 = |u|/||u||, u ~ U[0,1)^n; y0 = 1.
        Slot b uses seed ``seed0 + ids[b]`` (ids defaults to 0..batch-1, i.e. global instance
        ids, so a sharded run draws the same instances as an unsharded one).
        Shared layout: Z (and the first start) from ``seed0``; start b's x0 from its own
        generator seeded ``seed0 + 1000003 * (ids[b] + 1)``.
        Returns (x0, y0) device tensors (batch, n)."""
        n = self.n
        k = int(np.floor(delta * n))
        x0 = torch.empty((self.batch, n), dtype=torch.float64, device=self.device)
        y0 = torch.ones((self.batch, n), dtype=torch.float64, device=self.device)
        ids = list(range(self.batch)) if ids is None else list(ids)
        if len(ids) != self.batch:
            raise ValueError("ids must have one entry per batch slot")
        Zb = torch.empty((n, n), dtype=torch.float64, device=self.device)
        if self.shared:
            self._draw_Z(Zb, int(seed0), k, snr)
            self.pack_one(Zb, 0)
            for b in range(self.batch):
                g = torch.Generator(device=self.device)
                g.manual_seed(int(seed0) + 1000003 * (int(ids[b]) + 1))
                u = torch.rand(n, dtype=torch.float64, device=self.device, generator=g)
                x0[b] = (u / torch.linalg.vector_norm(u)).abs()
            torch.cuda.synchronize(self.device)
            self.bind()
            return x0, y0
        for b in range(self.batch):
            g = self._draw_Z(Zb, int(seed0) + int(ids[b]), k, snr)
            u = torch.rand(n, dtype=torch.float64, device=self.device, generator=g)
            x0[b] = (u / torch.linalg.vector_norm(u)).abs()
            self.pack_one(Zb, b)
        torch.cuda.synchronize(self.device)
        self.bind()
        return x0, y0

    def _draw_Z(self, Zb: torch.Tensor, seed: int, k: int, snr: float) -> torch.Generator:
        n = self.n
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        idx = torch.randperm(n, generator=g, device=self.device)[:k]
        v = torch.zeros(n, dtype=torch.float64, device=self.device)
        v[idx] = 1.0 / math.sqrt(k)
        Zb.normal_(0.0, 1.0, generator=g).div_(math.sqrt(n))
        dg = torch.randn(n, dtype=torch.float64, device=self.device, generator=g) * 2 / math.sqrt(n)
        Zb.diagonal().copy_(dg)
        Zb.add_(math.sqrt(snr) * torch.outer(v, v))
        return g

    # ---- operators ----------------------------------------------------------------------
    def _padded(self, a) -> torch.Tensor:
        t = torch.as_tensor(a, dtype=torch.float64)
        if t.dim() == 1:
            t = t.unsqueeze(0)
        if t.shape != (self.batch, self.n):
            raise ValueError(f"expected {(self.batch, self.n)}, got {tuple(t.shape)}")
        out = torch.zeros((self.batch, self.ld), dtype=torch.float64, device=self.device)
        out[:, :self.n] = t.to(self.device)
        return out

    def spass_calibration(self) -> Dict[str, Any]:
        """riptrm_get_spass_calibration: the S-pass kernel of wide launches (and, for spass_kind 3
        only, the bind-time timing that chose it; zeros otherwise)."""
        t, u, k = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
        self.ctx.check(self.lib.riptrm_get_spass_calibration(self.ctx.h, ctypes.byref(t), ctypes.byref(u),
                                                             ctypes.byref(k)), "riptrm_get_spass_calibration")
        return {"ms_per_launch_tile": t.value, "ms_per_launch_super": u.value,
                "kernel": "k_spass_sup" if k.value == 1 else "k_spass_sym"}

    def trs_skip_stats(self):
        """(Exact_RepMat subproblems whose CG went through the certified skip test, CGs skipped) since
        the context was created (riptrm_trs_skip_stats; the tridiagonal path from order 150 on counts
        here, the eigen-coordinate path below does not)."""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        self.ctx.check(self.lib.riptrm_trs_skip_stats(self.ctx.h, ctypes.byref(a), ctypes.byref(b)), "riptrm_trs_skip_stats")
        return int(a.value), int(b.value)

    def persistent_state(self) -> Dict[str, bool]:
        """riptrm_get_persistent: whether the bound shape runs k_persist on this device, and whether
        the current solve / tCG run uses it."""
        pos, act, fb = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self.ctx.check(self.lib.riptrm_get_persistent(self.ctx.h, ctypes.byref(pos), ctypes.byref(act)),
                       "riptrm_get_persistent")
        self.ctx.check(self.lib.riptrm_persist_fallbacks(self.ctx.h, ctypes.byref(fb)), "riptrm_persist_fallbacks")
        return {"possible": bool(pos.value), "active": bool(act.value), "fallbacks": int(fb.value)}

    def hvp(self, x, y, mu: float, v) -> torch.Tensor:
        """HwCur(v) at (x, y, mu) for every instance (RIPTRM.py:729)."""
        assert self.bound
        X, Y, V = self._padded(x), self._padded(y), self._padded(v)
        out = torch.zeros_like(X)
        self._sync_stream()
        self.ctx.check(self.lib.riptrm_nonnegpca_hvp(self.ctx.h, ctypes.c_void_p(X.data_ptr()),
                                                     ctypes.c_void_p(Y.data_ptr()), float(mu),
                                                     ctypes.c_void_p(V.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                     self.ld), "riptrm_nonnegpca_hvp")
        torch.cuda.synchronize(self.device)
        return out[:, :self.n]

    def operator_aw(self, x, z, s, v) -> torch.Tensor:
        """RIPM's OperatorAw(v) at (x, z, s) for every instance (src/solver/RIPM.py:485-487)."""
        assert self.bound
        X, Zt, St, V = self._padded(x), self._padded(z), self._padded(s), self._padded(v)
        out = torch.zeros_like(X)
        self._sync_stream()
        self.ctx.check(self.lib.riptrm_nonnegpca_operator_aw(self.ctx.h, ctypes.c_void_p(X.data_ptr()),
                                                             ctypes.c_void_p(Zt.data_ptr()), ctypes.c_void_p(St.data_ptr()),
                                                             ctypes.c_void_p(V.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                             self.ld), "riptrm_nonnegpca_operator_aw")
        torch.cuda.synchronize(self.device)
        return out[:, :self.n]

    def tcg(self, x, y, mu, Delta, max_steps: int = 0):
        """truncated_conjugate_gradient at (x_b, y_b, mu_b, Delta_b) (RIPTRM.py:41-216 via
        compute_direction :445-452).  Returns (eta, Heta, j, stop_names)."""
        assert self.bound
        X, Y = self._padded(x), self._padded(y)
        mu_t = torch.as_tensor(np.broadcast_to(np.asarray(mu, dtype=np.float64), (self.batch,)).copy(),
                               device=self.device)
        de_t = torch.as_tensor(np.broadcast_to(np.asarray(Delta, dtype=np.float64), (self.batch,)).copy(),
                               device=self.device)
        it = (ctypes.c_int32 * self.batch)()
        st = (ctypes.c_int32 * self.batch)()
        self._sync_stream()
        self.ctx.check(self.lib.riptrm_tcg(self.ctx.h, ctypes.c_void_p(X.data_ptr()), ctypes.c_void_p(Y.data_ptr()),
                                           self.ld, ctypes.c_void_p(mu_t.data_ptr()), ctypes.c_void_p(de_t.data_ptr()),
                                           it, st, int(max_steps)), "riptrm_tcg")
        eta = self.vec(2).clone()
        heta = self.vec(3).clone()
        return eta, heta, np.array(list(it)), [TCG_NAMES[s] for s in st]

    # ---- full solve ---------------------------------------------------------------------
    def begin(self, x0, y0, option: Dict[str, Any], restart_every: int = 0) -> ResolvedOptions:
        assert self.bound
        ro = resolve_options(option, math.pi, self.cap, restart_every)
        if ro.exact and trs_hbm_path(self.n):
            # Exact_RepMat beyond the LDS solver: the frame matrices (n x n) live in HBM scratch, one
            # slot per instance served in the same pass (riptrm_trs_bind_workspace;
            # csrc/riptrm_trs_big.hip), as many as trs_workspace_slots allows
            slots = trs_workspace_slots(self.lib, self.n, self.batch)
            self._trs_ws = bind_trs_scratch(self.ctx, self.lib, self.device, self._trs_ws, self.n, slots)
            # with the second-order test every trial point's eigenpairs are computed anyway; a
            # subproblem at that same point (step accepted without dual clipping) then skips its
            # eigensolve (RIPTRM.py:686-692 keeps HwNewmatrix the same way)
            cbytes = trs_cache_wanted(self.lib, self.n, self.batch) if ro.c_opt.second_order_stationarity else 0
            if cbytes and (self._trs_cache is None or self._trs_cache.numel() < cbytes + 256):
                self._trs_cache = torch.empty(cbytes + 256, dtype=torch.uint8, device=self.device)
            if cbytes:
                base = self._trs_cache.data_ptr()
                ptr = base + (-base) % 256
                self.ctx.check(self.lib.riptrm_trs_bind_cache(self.ctx.h, ctypes.c_void_p(ptr), cbytes, self.n,
                                                              self.batch), "riptrm_trs_bind_cache")
            else:
                self.ctx.check(self.lib.riptrm_trs_bind_cache(self.ctx.h, None, 0, 0, 0), "riptrm_trs_bind_cache")
        X, Y = self._padded(x0), self._padded(y0)
        tabs = ro.device_tables(self.device)
        self._keep = [X, Y] + tabs
        self._sync_stream()
        self.ctx.check(self.lib.riptrm_solve_begin(self.ctx.h, ctypes.byref(ro.c_opt), ctypes.c_void_p(X.data_ptr()),
                                                   ctypes.c_void_p(Y.data_ptr()), self.ld,
                                                   ctypes.c_void_p(tabs[0].data_ptr()), ctypes.c_void_p(tabs[1].data_ptr()),
                                                   ctypes.c_void_p(tabs[2].data_ptr()), len(ro.mu_tab)),
                       "riptrm_solve_begin")
        self.ro = ro
        self._target = 2 ** 31 - 1
        self._drained = [[] for _ in range(self.batch)]
        self._dropped = np.zeros(self.batch, dtype=np.int64)
        return ro

    def trs_cache_stats(self):
        """(cache hits, subproblems served) of the HBM Exact_RepMat path since begin()."""
        h, t = ctypes.c_int64(0), ctypes.c_int64(0)
        self.ctx.check(self.lib.riptrm_trs_cache_stats(self.ctx.h, ctypes.byref(h), ctypes.byref(t)),
                       "riptrm_trs_cache_stats")
        return int(h.value), int(t.value)

    def advance(self, steps: int, outer_target: Optional[int] = None) -> int:
        tgt = 2 ** 31 - 1 if outer_target is None else int(outer_target)
        act = ctypes.c_int32(0)
        self._sync_stream()
        self.ctx.check(self.lib.riptrm_solve_advance(self.ctx.h, int(steps), tgt, ctypes.byref(act)),
                       "riptrm_solve_advance")
        return int(act.value)

    def run_until(self, outer_target: Optional[int] = None, max_chunk: int = 512, timeout_s: float = 1e9) -> int:
        """Advance until every instance is finished or paused at ``outer_target``.  With log draining
        on, a chunk is at most a quarter of the log capacity in lock-step iterations (each writes at
        most one record per instance on the tCG path) and the device log is drained once half full."""
        chunk, t0 = 4, time.time()
        cap = min(self.cap, int(self.ro.c_opt.log_capacity))
        if self.ro.exact and trs_hbm_path(self.n):
            # the HBM Exact_RepMat path parks every instance a few lock-step iterations after each
            # service (subproblem -> trial point -> trial eigenvalue): short chunks, so the parked
            # instances are served as soon as they all wait
            max_chunk = min(max_chunk, EXACT_BIG_CHUNK)
        if self.drain:
            max_chunk = max(1, min(max_chunk, cap // 4))
        act = self.advance(0, outer_target)
        while act > 0:
            act = self.advance(min(chunk, max_chunk), outer_target)
            chunk = min(chunk * 2, max_chunk)
            if self.drain and cap > 0:
                st = self.stats()
                pend = st[:, C["RIPTRM_STAT_LOG_COUNT"]] - st[:, C["RIPTRM_STAT_LOG_BASE"]]
                if pend.max() > cap // 2:
                    self.drain_logs()
            if time.time() - t0 > timeout_s:
                raise TimeoutError("RIPTRM device solve exceeded the host timeout")
        return act

    def solve(self, x0, y0, option: Dict[str, Any]) -> "BatchResult":
        self.begin(x0, y0, option)
        self.run_until(None)
        return self.result()

    def result(self) -> "BatchResult":
        torch.cuda.synchronize(self.device)
        st = self.stats()
        x = self.vec(0).clone()
        y = self.vec(1).clone()
        logs, dropped = [], []
        for b, (rows, drop) in enumerate(self._pending_logs(st)):
            logs.append(np.concatenate(self._drained[b] + [rows]) if self._drained[b] else rows.copy())
            dropped.append(int(self._dropped[b]) + drop)
        return BatchResult(x=x, y=y, stats=st, raw_log=logs, ro=self.ro, dropped=np.array(dropped))


@dataclass
class BatchResult:
    x: torch.Tensor
    y: torch.Tensor
    stats: np.ndarray
    raw_log: List[np.ndarray]        # per instance: its log records in order (NLOG doubles each)
    ro: ResolvedOptions
    dropped: Optional[np.ndarray] = None   # per instance: records lost from the middle of the log

    def stat(self, b: int, name: str) -> float:
        return float(self.stats[b, C[f"RIPTRM_STAT_{name}"]])

    def error(self, b: int) -> Optional[str]:
        """The instance's error (RIPTRM_STAT_ERROR) as the text the reference prints after
        "Error: " when outer_step raises (RIPTRM.py:961-966), or None."""
        code = int(self.stat(b, "ERROR"))
        return None if code == C["RIPTRM_ERR_NONE"] else ERROR_TEXT.get(code, f"device error code {code}")

    def stopping_criterion(self, b: int) -> Optional[str]:
        code = int(self.stat(b, "STOP_CODE"))
        rt = self.stat(b, "STOP_RUNTIME")
        o = self.ro.option
        if code == C["RIPTRM_STOP_MAXTIME"]:
            return f"Max time exceeded; runtime={rt:.2f} and maxtime={o['maxtime']}"
        if code == C["RIPTRM_STOP_MAXITER"]:
            return f"Max iteration count reached; maxiter={o['maxiter']} after {rt:.2f} seconds"
        if code == C["RIPTRM_STOP_TOLRESID"]:
            res = np.float64(self.stat(b, "FINAL_RESIDUAL"))
            return ("KKT residual tolerance reached; current residual=" + str(res)
                    + " and tolresid=" + str(o['tolresid']) + f" after {rt:.2f} seconds")
        return None

    def log(self, b: int) -> Dict[str, list]:
        """Instance b's log in the reference's column schema (base_solver.py:58-76,
        utils.py:356-364, RIPTRM.py:986-1023)."""
        rows = self.raw_log[b]
        save_inner = bool(self.ro.option['save_inner_iteration'])
        cols: Dict[str, list] = {k: [] for k in (
            "iteration", "time", "cost", "distance", "residual", "gradnorm", "complviolation",
            "dualviolation", "manviolation", "maxviolation", "meanviolation", "mu", "num_inner",
            "inner_status", "TR_radius")}
        extra = ("dxtype", "normdx", "minxfeasi", "minyfeasi", "compl", "mineigvalHw", "ared/pred",
                 "radius_update", "dual_clipping")
        if save_inner:
            for k in extra:
                cols[k] = []
        cols["maxabsLagmult"] = []
        F = lambda name: C[f"RIPTRM_LOG_{name}"]
        for r in rows:
            it = int(r[F("ITERATION")])
            cols["iteration"].append(it)
            cols["time"].append(0 if len(cols["time"]) == 0 else float(r[F("TIME")]))
            for k, f in (("cost", "COST"), ("distance", "DISTANCE"), ("residual", "RESIDUAL"),
                         ("gradnorm", "GRADNORM"), ("complviolation", "COMPLVIOLATION"),
                         ("dualviolation", "DUALVIOLATION"), ("manviolation", "MANVIOLATION"),
                         ("maxviolation", "MAXVIOLATION"), ("meanviolation", "MEANVIOLATION"),
                         ("mu", "MU")):
                cols[k].append(np.float64(r[F(f)]))
            has = r[F("HAS_INFO")] != 0
            cols["num_inner"].append(int(r[F("NUM_INNER")]) if has else None)
            cols["inner_status"].append(STATUS_NAMES[int(r[F("INNER_STATUS")])] if has else None)
            cols["TR_radius"].append(np.float64(r[F("TR_RADIUS")]) if has else None)
            if save_inner:
                cols["dxtype"].append(dxtype_name(int(r[F('DXTYPE')])) if has else None)
                cols["normdx"].append(np.float64(r[F("NORMDX")]) if has else None)
                cols["minxfeasi"].append(np.float64(r[F("MINXFEASI")]) if has else None)
                cols["minyfeasi"].append(np.float64(r[F("MINYFEASI")]) if has else None)
                cols["compl"].append(np.float64(r[F("COMPL")]) if has else None)
                cols["mineigvalHw"].append(np.float64(r[F("MINEIGVALHW")]) if has and r[F("HAS_MINEIG")] != 0 else None)
                hr = has and r[F("HAS_RATIO")] != 0
                cols["ared/pred"].append(np.float64(r[F("ARED_PRED")]) if hr else None)
                cols["radius_update"].append(RU_NAMES[int(r[F("RADIUS_UPDATE")])] if hr else None)
                dc = int(r[F("DUAL_CLIPPING")])
                cols["dual_clipping"].append(None if (not has or dc < 0) else bool(dc))
            cols["maxabsLagmult"].append(np.float64(r[F("MAXABSLAGMULT")]))
        return cols

    def tcg_iters_per_row(self, b: int) -> List[int]:
        return [int(v) for v in self.raw_log[b][:, C["RIPTRM_LOG_TCG_ITERS"]]]


def profile_enable(batch: NonnegPCABatch, on: bool = True):
    """HIP-event timing of every S-pass / state launch (riptrm_profile_enable)."""
    batch.ctx.check(batch.lib.riptrm_profile_enable(batch.ctx.h, 1 if on else 0), "riptrm_profile_enable")


def profile_read(batch: NonnegPCABatch) -> Dict[str, float]:
    gm, sm = ctypes.c_double(0), ctypes.c_double(0)
    gn, sn = ctypes.c_int64(0), ctypes.c_int64(0)
    batch.ctx.check(batch.lib.riptrm_profile_read(batch.ctx.h, ctypes.byref(gm), ctypes.byref(gn),
                                                  ctypes.byref(sm), ctypes.byref(sn)), "riptrm_profile_read")
    return {"gemv_ms": gm.value, "gemv_launches": gn.value, "state_ms": sm.value, "state_launches": sn.value}
