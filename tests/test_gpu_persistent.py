"""Persistent lock-step mode (k_persist, csrc/riptrm_kernels.hip) against the lock-step kernels
(k_spass_sym + k_state) on the same inputs: bitwise identical iterates, logs (except the time
column) and counters.  k_persist runs the reference's tCG loop (RIPTRM.py:41-216) and the inner /
outer loops (:707-896) of small symmetric-tile batches in one launch per chunk: every stored tile
of S stays in LDS, every workgroup of an instance runs a replica of the instance's state machine,
and the S-pass partial sums are exchanged through write-through stores + one arrival counter per
instance.  The arithmetic (tile products, partial-sum order, reductions) is the lock-step path's,
so the bar is equality, not a tolerance.  Shapes: n <= 1024 (2 elements per thread) and
1024 < n <= 2048 (4 per thread), one tile (no exchange) up to 136 tiles, up to 7 instances.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import nonnegpca_gen as G


def _opt(**kw):
    from problems import manviofun
    o = {"TRS_solver": "tCG", "second_order_stationarity": False, "manviofun": manviofun,
         "tolresid": 0.0, "maxtime": 1e9}
    o.update(kw)
    return o


def _solve(insts, persistent, **kw):
    import engine
    n, B = insts[0][0].shape[0], len(insts)
    eng = engine.NonnegPCABatch(n, B, log_capacity=4096, persistent=persistent)
    eng.load_Z(np.stack([z for z, _, _ in insts]))
    res = eng.solve(np.stack([x for _, x, _ in insts]), np.stack([y for _, _, y in insts]), _opt(**kw))
    return eng, res


def _assert_same(ra, rb, B):
    import engine
    assert torch.equal(ra.x, rb.x) and torch.equal(ra.y, rb.y)
    for b in range(B):
        la, lb = ra.log(b), rb.log(b)
        assert list(la.keys()) == list(lb.keys())
        for k in la:
            if k != "time":
                assert la[k] == lb[k] or np.array_equal(np.array(la[k], float), np.array(lb[k], float)), (b, k)
        for f in ("OUTER_ITERS", "INNER_ITERS", "TCG_ITERS", "PASSES", "STOP_CODE"):
            assert ra.stat(b, f) == rb.stat(b, f), (b, f)


@pytest.mark.parametrize("n,B,K", [(37, 5, 10), (200, 4, 10), (1000, 1, 10), (1000, 7, 6), (1500, 1, 6),
                                   (2048, 1, 5)])
def test_persistent_matches_lockstep_bitwise(n, B, K):
    insts = [G.generate_instance(n, 900 + b) for b in range(B)]
    e1, r1 = _solve(insts, 1, maxiter=K)
    st = e1.persistent_state()
    assert st["possible"] and st["active"] and st["fallbacks"] == 0
    e0, r0 = _solve(insts, 0, maxiter=K)
    assert e0.persistent_state()["active"] is False
    _assert_same(r1, r0, B)


def test_persistent_teacher_forced_tcg_bitwise():
    """riptrm_tcg (MODE_TCG_ONLY) through k_persist == through the lock-step kernels."""
    import engine
    n, B = 1000, 3
    Z, x0, _ = G.generate_instance(n, 77)
    rs = np.random.RandomState(4)
    xs = np.stack([np.abs(rs.rand(n)) for _ in range(B)])
    xs /= np.linalg.norm(xs, axis=1, keepdims=True)
    ys = rs.rand(B, n) + 0.1
    mus, deltas = np.array([0.1, 1e-3, 1e-6]), np.array([np.pi / 8, 1e-3, 5.0])
    out = []
    for mode in (1, 0):
        eng = engine.NonnegPCABatch(n, B, persistent=mode)
        eng.load_Z(np.broadcast_to(Z, (B, n, n)))
        out.append(eng.tcg(xs, ys, mus, deltas))
    (e1, h1, j1, s1), (e0, h0, j0, s0) = out
    assert torch.equal(e1, e0) and torch.equal(h1, h0)
    assert list(j1) == list(j0) and s1 == s0


def test_persistent_pause_resume_and_drain():
    """outer_target pauses, resumes and host log drains between persistent launches change nothing."""
    import engine
    n, B = 1000, 2
    insts = [G.generate_instance(n, 950 + b) for b in range(B)]
    Z = np.stack([z for z, _, _ in insts])
    X0 = np.stack([x for _, x, _ in insts])
    Y0 = np.stack([y for _, _, y in insts])
    ref = engine.NonnegPCABatch(n, B, log_capacity=4096, persistent=0)
    ref.load_Z(Z)
    r0 = ref.solve(X0, Y0, _opt(maxiter=9))
    eng = engine.NonnegPCABatch(n, B, log_capacity=16, persistent=1)   # 16 slots: drained every few chunks
    eng.load_Z(Z)
    eng.begin(X0, Y0, _opt(maxiter=9))
    for tgt in (2, 5, None):
        eng.run_until(tgt)
    r1 = eng.result()
    assert eng.persistent_state()["active"]
    _assert_same(r1, r0, B)


def test_persistent_not_used_when_too_large():
    """Shapes beyond one workgroup per tile per CU keep the lock-step kernels."""
    import engine
    eng = engine.NonnegPCABatch(2176, 1)   # n > 2048
    Z, x0, y0 = G.generate_instance(2176, 3)
    eng.load_Z(Z[None])
    assert eng.persistent_state()["possible"] is False
    eng2 = engine.NonnegPCABatch(1000, 8)  # 8 x 36 tiles > 256 workgroups
    eng2.load_Z(np.broadcast_to(Z[:1000, :1000], (8, 1000, 1000)))
    assert eng2.persistent_state()["possible"] is False


def test_refused_persistent_launch_falls_back_to_lockstep():
    """A persistent launch the runtime refuses before the solve's first persistent step (mode 3
    simulates it) hands the solve to the lock-step kernels: same results bitwise, one fallback."""
    n, B = 1000, 3
    insts = [G.generate_instance(n, 960 + b) for b in range(B)]
    e3, r3 = _solve(insts, 3, maxiter=6)
    st = e3.persistent_state()
    assert st["possible"] and not st["active"] and st["fallbacks"] == 1
    e0, r0 = _solve(insts, 0, maxiter=6)
    _assert_same(r3, r0, B)


def test_plain_launch_mode_matches():
    """Mode 2 (plain launch, the round-2 path; A/B only) gives the same bits as the cooperative one."""
    n, B = 200, 4
    insts = [G.generate_instance(n, 970 + b) for b in range(B)]
    e2, r2 = _solve(insts, 2, maxiter=8)
    assert e2.persistent_state()["active"]
    e1, r1 = _solve(insts, 1, maxiter=8)
    _assert_same(r2, r1, B)


def test_two_persistent_solves_on_concurrent_streams():
    """Two batches whose persistent grids together exceed the CUs (2 x 7 x 36 = 504 workgroups of one
    CU each), solved at the same time from two threads on two streams: the cooperative launches may
    not interleave their workgroups (the in-launch barriers would spin against each other), so both
    must finish without a barrier timeout and match the lock-step results."""
    import threading
    import engine
    n, B = 1000, 7
    sets = [[G.generate_instance(n, 980 + 10 * k + b) for b in range(B)] for k in range(2)]
    refs = [_solve(s_, 0, maxiter=4)[1] for s_ in sets]
    out, errs = [None, None], []

    def run(k):
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                eng = engine.NonnegPCABatch(n, B, log_capacity=4096, persistent=1)
                eng.load_Z(np.stack([z for z, _, _ in sets[k]]))
                res = eng.solve(np.stack([x for _, x, _ in sets[k]]), np.stack([y for _, _, y in sets[k]]),
                                _opt(maxiter=4))
                torch.cuda.current_stream().synchronize()
                out[k] = (eng.persistent_state(), res)
        except Exception as e:   # reported below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    for k in range(2):
        st, res = out[k]
        assert st["possible"]
        for b in range(B):
            assert res.stat(b, "ERROR") == 0
        _assert_same(res, refs[k], B)


@pytest.mark.timeout(900)
def test_cfg1_bench_window_matches_oracle(capsys):
    """BASELINE configs[1] as `bench.py --dim 1000 --batch 1 --warmup 5 --steps 20` runs it: one
    instance at n = 1000 drawn on the device (seed 20251212 + id), the persistent k_persist path
    (asserted active), options maxiter = 45 and restart_every = 20, paused at outer targets as the
    bench's warm-up / timed regions do.  The bench times positions 6..20 and, after the restart, 1..5:
    * the first 20 outer iterations (every position the bench times) against the oracle built from
      the device's own S under the null-calibrated bar (tests/parity.py check_null / assert_null),
      twelve instances (ids 0..11; id 0 is the bench's own) pooled into one rank test;
    * the restart: x, y after outer iteration 25 (restart position 5) are bitwise the x, y after outer
      iteration 5 of the same run (RIPTRM.py:785-976 from (x0, y0, mu0, Delta0) again).
    RIPTRM.py:98-214 (tCG), 631-705 (acceptance), 785-976 (loops)."""
    import engine
    from parity import assert_null, check_instances_parallel
    from problems import manviofun
    import os
    n, K, ids = 1000, 20, list(range(12))
    oracle_opt = dict(tolresid=0.0, maxtime=1e9, maxiter=K)
    from oracle import riptrm_oracle as O
    oracle_opt["manviofun"] = O.sphere_manvio
    opt = {"maxiter": 45, "tolresid": 0.0, "maxtime": 1e9, "manviofun": manviofun, "TRS_solver": "tCG",
           "second_order_stationarity": False}
    items = []
    for k in ids:
        eng = engine.NonnegPCABatch(n, 1, log_capacity=2048, drain_logs=False)
        x0, y0 = eng.generate_synthetic(20251212, ids=[k])
        eng.begin(x0, y0, opt, restart_every=20)
        eng.run_until(5)
        torch.cuda.synchronize()
        st = eng.persistent_state()
        assert st["possible"] and st["active"] and st["fallbacks"] == 0, st
        x5, y5 = eng.vec(0).clone(), eng.vec(1).clone()
        eng.run_until(K)
        res = eng.result()
        assert int(res.stat(0, "OUTER_ITERS")) == K
        eng.run_until(25)
        torch.cuda.synchronize()
        assert torch.equal(eng.vec(0), x5) and torch.equal(eng.vec(1), y5), k
        items.append(dict(gl=res.log(0), S=eng.unpack(0), x0=x0[0].cpu().numpy(), y0=y0[0].cpu().numpy(),
                          gpu_x=res.x[0].cpu().numpy()[:n], gpu_y=res.y[0].cpu().numpy()[:n],
                          gpu_tcg=res.tcg_iters_per_row(0)[1:], name=f"bench id {k}"))
        del eng
    with capsys.disabled():
        print("[cfg1] 12 GPU solves done", flush=True)
        results = check_instances_parallel(items, oracle_opt, progress=lambda m: print(m, flush=True))
        names = [it["name"] for it in items]
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity", "cfg1.json")
        assert_null([results[nm] for nm in names], names, path)
