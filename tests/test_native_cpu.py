"""CPU-side checks of the C-ABI library and the host logic (no GPU compute calls)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

import riptrm_native as N


def test_library_exports_every_header_symbol(built_lib):
    syms = N.header_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(built_lib, s)]
    assert not missing, missing
    # and the ctypes signature table covers exactly the header
    assert sorted(N.SIGNATURES) == syms


def test_abi_version_and_no_device(built_lib):
    assert built_lib.riptrm_abi_version() == N.CONST["RIPTRM_ABI_VERSION"]
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("a GPU is visible")
    h = ctypes.c_void_p()
    rc = built_lib.riptrm_ctx_create(ctypes.byref(h), 0, None)
    assert rc == N.CONST["RIPTRM_E_NODEV"]
    assert h.value is None


_BACKEND_PROBE = """
import ctypes, sys
sys.path.insert(0, {pkg!r})
import riptrm_native as N
lib = N.load()
buf = ctypes.create_string_buffer(512)
rc = lib.riptrm_trs_backend_status(buf, 512)
print(rc, buf.value.decode())
"""


@pytest.mark.parametrize("bogus", [False, True])
def test_trs_backend_load_failure_is_reported_not_fatal(built_lib, bogus):
    """riptrm_trs_big.hip loads rocBLAS / rocSOLVER with dlopen at first use.  A library that cannot
    be loaded must come back as RIPTRM_E_HIP with dlopen's message (dlerror() was called
    twice, the second NULL crashed the process).  Run in a child so the probe's cached state and the
    environment override stay there."""
    from conftest import PKG
    env = dict(os.environ)
    if bogus:
        env["RIPTRM_ROCSOLVER_LIB"] = "libriptrm_no_such_solver.so.0"
    r = subprocess.run([sys.executable, "-c", _BACKEND_PROBE.format(pkg=PKG)], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rc, msg = r.stdout.strip().split(" ", 1)
    if bogus:
        assert int(rc) == N.CONST["RIPTRM_E_HIP"]
        assert "libriptrm_no_such_solver.so.0" in msg and "cannot load" in msg
    elif int(rc) != 0:
        pytest.skip(f"rocSOLVER not loadable on this host: {msg}")
    else:
        assert "dsyevd" in msg


def test_layout_functions(built_lib):
    C = N.CONST
    for n in (2, 17, 50, 1000, 4000, 4001):
        ld = built_lib.riptrm_nonnegpca_ld(n)
        rows = built_lib.riptrm_nonnegpca_rows(n)
        assert ld >= n and ld % 128 == 0 and ld - n < 128
        assert rows >= n and rows % 32 == 0
        nt = ld // 128
        assert built_lib.riptrm_nonnegpca_s_elems(n, C["RIPTRM_LAYOUT_FULL"]) == rows * ld
        sym = built_lib.riptrm_nonnegpca_s_elems(n, C["RIPTRM_LAYOUT_SYMTILE"])
        wl = -(-(n - (nt - 1) * 128) // 32) * 32     # last tile column keeps its stored width
        assert sym == (nt - 1) * nt // 2 * 128 * 128 + (nt - 1) * 128 * wl + wl * wl
        assert sym >= n * (n + 1) // 2
        if n >= 1000:
            assert sym < 0.6 * n * n  # about half the bytes of the full matrix
        if n >= 4000:
            assert sym < 0.55 * n * n
        assert built_lib.riptrm_nonnegpca_s_elems(n, C["RIPTRM_LAYOUT_SHARED"]) == rows * ld
        # shared layout: 4 K-slice slabs x 2 right-hand sides of partial products per instance
        assert (built_lib.riptrm_workspace_bytes(n, 8, 0, C["RIPTRM_LAYOUT_SHARED"])
                - built_lib.riptrm_workspace_bytes(n, 8, 0, C["RIPTRM_LAYOUT_FULL"])) >= 4 * 2 * 8 * ld * 8
        for layout in (C["RIPTRM_LAYOUT_FULL"], C["RIPTRM_LAYOUT_SYMTILE"], C["RIPTRM_LAYOUT_SHARED"]):
            for B, cap in ((1, 0), (3, 10), (128, 4096)):
                tot = built_lib.riptrm_workspace_bytes(n, B, cap, layout)
                offs = [built_lib.riptrm_workspace_offset(n, B, cap, layout, k) for k in range(6)]
                assert all(0 <= o < tot for o in offs[:5])
                assert offs[0] == 0 and offs[1] == B * ld * 8
                assert offs[4] % 256 == 0 and offs[5] % 256 == 0
                assert offs[5] + B * cap * 32 * 8 <= tot
    assert built_lib.riptrm_workspace_bytes(0, 1, 1, 0) == -1
    assert built_lib.riptrm_workspace_bytes(10, 1, 1, 7) == -1
    assert built_lib.riptrm_workspace_offset(10, 1, 1, 0, 9) == -1
    assert built_lib.riptrm_nonnegpca_s_elems(10, 5) == -1


def test_exact_hbm_scratch_sizes(built_lib, monkeypatch):
    """Host-side sizing of the HBM Exact_RepMat path: the per-instance eigendecomposition cache
    (n^2 + 3 vpad(n) + 8 doubles per instance, vpad = n rounded up to 64, plus the compact
    eigenvectors' or the tridiagonal path's reflectors: m (m + 1) / 2 rounded up to 8, m = n up to
    order 1024, riptrm_tri.h TRI_MAX, else 199), the engine's all-or-none cache budget, and the SI
    workspace's extra regions once manifold.dim = d(d-1)/2 + d(d+1) exceeds RIPTRM_TRS_DIM_MAX
    (d >= 8: the subproblem matrix, coordinates, service outputs and resume records)."""
    import engine
    vpad = lambda n: -(-n // 64) * 64
    for n, B in ((98, 1), (200, 64), (1000, 3), (1025, 2)):
        m = n if n <= 1024 else 199
        refl = -(-(m * (m + 1) // 2) // 8) * 8
        assert built_lib.riptrm_trs_cache_bytes(n, B) == (n * n + 3 * vpad(n) + 8 + refl) * 8 * B
    assert built_lib.riptrm_trs_cache_bytes(0, 4) == 0 and built_lib.riptrm_trs_cache_bytes(4, 0) == 0
    assert engine.trs_cache_wanted(built_lib, 200, 64) == built_lib.riptrm_trs_cache_bytes(200, 64)
    monkeypatch.setenv("RIPTRM_TRS_CACHE_GB", "0.001")
    assert engine.trs_cache_wanted(built_lib, 200, 64) == 0   # the whole batch or nothing
    monkeypatch.delenv("RIPTRM_TRS_CACHE_GB")
    monkeypatch.setenv("RIPTRM_TRS_CACHE", "0")
    assert engine.trs_cache_wanted(built_lib, 200, 64) == 0
    ws = lambda d: built_lib.riptrm_si_workspace_bytes(d, 95, 16, 4, 64)
    dim = lambda d: d * (d - 1) // 2 + d * (d + 1)
    assert dim(7) <= N.CONST["RIPTRM_TRS_DIM_MAX"] < dim(8)
    nt = lambda d: 64 if d <= 8 else -(-d * d // 64) * 64
    for d in (8, 12, 16):
        # at least the 4 subproblem matrices and 4 resume records on top of the tCG layout's share
        extra = 4 * 8 * (dim(d) ** 2 + 32 + 21 * nt(d))
        assert ws(d) >= extra, d
    assert ws(8) - ws(7) > 4 * 8 * dim(8) ** 2


@pytest.mark.parametrize("cls,cname", [("RiptrmOptions", "riptrm_options"), ("RiptrmSIProblem", "riptrm_si_problem")])
def test_options_struct_layout_matches_c(tmp_path, cls, cname):
    """ctypes mirrors == the C structs (sizeof and every offset), compiled with gcc."""
    S = getattr(N, cls)
    fields = [f for f, _ in S._fields_]
    src = tmp_path / "probe.c"
    body = "\n".join(f'printf("%zu\\n", offsetof({cname}, {f}));' for f in fields)
    src.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "riptrm.h"\n'
                   f'int main(void){{printf("%zu\\n", sizeof({cname}));\n{body}\nreturn 0;}}\n')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    assert vals[0] == ctypes.sizeof(S)
    for f, off in zip(fields, vals[1:]):
        assert getattr(S, f).offset == off, f


def test_resolve_options_defaults_and_errors():
    import engine
    from problems import manviofun
    ro_d = engine.resolve_options({}, np.pi, 16)   # reference defaults: Exact_RepMat + second-order test
    assert ro_d.exact and ro_d.c_opt.second_order_stationarity == 1 and ro_d.c_opt.trs_tolhardcase == 1e-8
    assert ro_d.tol2_tab == ro_d.mu_tab                # forcing_function_second_order = mu (RIPTRM.py:322)
    with pytest.raises(ValueError):
        engine.resolve_options({"TRS_solver": "Lanczos"}, np.pi, 16)   # RIPTRM.py:453-454
    with pytest.raises(NotImplementedError):
        engine.resolve_options({"checkTRSoptimality": True}, np.pi, 16)
    ro = engine.resolve_options({"TRS_solver": "tCG", "manviofun": manviofun, "maxiter": 50}, np.pi, 16)
    c = ro.c_opt
    assert not ro.exact and c.trs_solver == N.CONST["RIPTRM_TRS_SOLVER_TCG"] and c.second_order_stationarity == 0
    assert c.struct_size == ctypes.sizeof(N.RiptrmOptions)
    assert c.maxiter == 50 and c.inner_maxiter == -1 and c.inner_maxtime == -1.0
    assert c.initial_tr_radius == np.pi / 8
    assert c.manvio_kind == N.CONST["RIPTRM_MANVIO_SPHERE"]
    assert c.rho == 0.1 and c.gamma == 0.25 and c.const_right == 1e20
    assert ro.tolL_tab[0] == 0.1 and ro.tolC_tab[0] == 1e-4
    assert ro.tolL_tab[-1] == 1e-14 and ro.tolC_tab[-1] == 1e-14
    ro0 = engine.resolve_options({"TRS_solver": "tCG"}, np.pi, 16)
    assert ro0.c_opt.manvio_kind == N.CONST["RIPTRM_MANVIO_ZERO"]
    with pytest.raises(NotImplementedError):
        engine.resolve_options({"TRS_solver": "tCG", "manviofun": lambda p, x: float(np.sum(x))}, np.pi, 16)
    with pytest.raises(NotImplementedError):
        engine.resolve_options({"TRS_solver": "tCG", "callbackfun": lambda *a: a[-1]}, np.pi, 16)


def test_log_decoding_schema_matches_oracle(fixture_n50):
    """A raw device log decodes into the reference's columns in the reference's order."""
    import engine
    from oracle import riptrm_oracle as O
    C = N.CONST
    Z, x0, y0 = fixture_n50
    ref = O.solve(Z, x0, y0, dict(maxiter=2, tolresid=0.0, maxtime=1e9, manviofun=O.sphere_manvio))
    ro = engine.resolve_options({"TRS_solver": "tCG", "maxiter": 2}, np.pi, 8)
    raw = np.zeros((1, 3, C["RIPTRM_LOG_NFIELDS"]))
    raw[0, 1, C["RIPTRM_LOG_HAS_INFO"]] = 1
    raw[0, 1, C["RIPTRM_LOG_INNER_STATUS"]] = C["RIPTRM_IS_SUCCESSFUL"]
    raw[0, 1, C["RIPTRM_LOG_HAS_RATIO"]] = 1
    raw[0, 1, C["RIPTRM_LOG_RADIUS_UPDATE"]] = C["RIPTRM_RU_EXPANDED"]
    raw[0, 1, C["RIPTRM_LOG_DUAL_CLIPPING"]] = 0
    raw[0, 2, C["RIPTRM_LOG_HAS_INFO"]] = 1
    raw[0, 2, C["RIPTRM_LOG_INNER_STATUS"]] = C["RIPTRM_IS_CONVERGED"]
    raw[0, 2, C["RIPTRM_LOG_DUAL_CLIPPING"]] = -1
    raw[0, 2, C["RIPTRM_LOG_DXTYPE"]] = C["RIPTRM_TCG_EXCEEDED_TR"]
    stats = np.zeros((1, C["RIPTRM_STAT_NFIELDS"]))
    stats[0, C["RIPTRM_STAT_LOG_COUNT"]] = 3
    stats[0, C["RIPTRM_STAT_STOP_CODE"]] = C["RIPTRM_STOP_MAXITER"]
    res = engine.BatchResult(x=None, y=None, stats=stats, raw_log=[raw[0]], ro=ro)
    log = res.log(0)
    assert list(log.keys()) == list(ref.log.keys())
    assert log["inner_status"] == [None, "successful", "converged"]
    assert log["radius_update"] == [None, "expanded", None]
    assert log["dual_clipping"] == [None, False, None]
    assert log["dxtype"][2] == "tCG_EXCEEDED_TR"
    assert log["time"][0] == 0
    assert res.stopping_criterion(0).startswith("Max iteration count reached; maxiter=2 after")


def test_product_path_has_no_oracle_dependency():
    """The shipped package must never import the oracle (no CPU fallback)."""
    pkg = os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            txt = open(os.path.join(pkg, fn)).read()
            assert "oracle" not in txt.replace("oracle/", ""), fn


def test_engine_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import engine
    with pytest.raises(RuntimeError):
        engine.NonnegPCABatch(10, 1)


def test_save_output_reference_layout(tmp_path):
    """CSV files as base_simulator.Simulator.save_output writes them (no GPU needed)."""
    import pandas as pd
    from simulator import save_output
    from solver_base import Output
    log = {"iteration": [0, 1, 1], "time": [0, 0.1, 0.2], "residual": [4.9, 0.5, 0.1],
           "inner_status": [None, "successful", "converged"], "dual_clipping": [None, False, None]}
    out = Output(name="RIPTRM_tCG", x=np.array([0.6, 0.8]), option={"maxiter": 3, "tolresid": 1e-16},
                 log=log, ineqLagmult=np.array([1.0, 2.0]), eqLagmult=[])
    files = save_output(str(tmp_path), out.name, out)
    names = sorted(os.path.basename(f) for f in files)
    assert names == sorted(f"RIPTRM_tCG_{a}.csv" for a in ("name", "x", "option", "log", "ineqLagmult", "eqLagmult"))
    np.testing.assert_array_equal(np.loadtxt(tmp_path / "RIPTRM_tCG_x.csv"), [0.6, 0.8])
    df = pd.read_csv(tmp_path / "RIPTRM_tCG_log.csv")
    assert list(df.columns) == list(log.keys())
    conv = df[(df["inner_status"] == "converged") | (df["inner_status"].isna())]   # analyzer.ipynb filter
    assert list(conv["residual"]) == [4.9, 0.1]
    opt = pd.read_csv(tmp_path / "RIPTRM_tCG_option.csv")
    assert opt["maxiter"][0] == 3
    assert open(tmp_path / "RIPTRM_tCG_eqLagmult.csv").read() == ""
    # csv.writerows on the name string: one character per row, as the reference writes it
    assert open(tmp_path / "RIPTRM_tCG_name.csv").read().split() == list("RIPTRM_tCG")


def test_log_slot_assembly_keeps_head_and_latest():
    """include/riptrm.h "Log slots": linear up to the capacity, then the first cap/2 records and a
    ring of the latest; assemble_log restores chronological order and counts the dropped middle."""
    import engine
    for cap in (1, 2, 7, 8):
        for k in range(0, 40):
            slots = np.full((cap, 1), -1.0)
            for r in range(k):       # the device's slot rule (riptrm_device.h log_slot)
                i = r if r < cap else cap // 2 + (r - cap // 2) % (cap - cap // 2)
                slots[i, 0] = r
            rows, dropped = engine.assemble_log(slots, k, cap)
            if k <= cap:
                assert dropped == 0 and list(rows[:, 0]) == list(range(k))
            else:
                h = cap // 2
                want = list(range(h)) + list(range(k - (cap - h), k))
                assert dropped == k - cap and list(rows[:, 0]) == want, (cap, k)


@pytest.mark.parametrize("problem", ["NonnegPCA", "StableIdentification"])
def test_dropin_coordinator_module_resolves_by_name(problem, tmp_path):
    """base_simulator.py:44-49: importlib.import_module(cfg.problem_coordinator_name).Coordinator(cfg)
    with 'coordinator' resolved through sys.path alone yields the structured problem (subprocess,
    so the module name 'coordinator' does not leak into this session)."""
    import shutil
    import subprocess
    import textwrap
    from conftest import GOLDEN
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(GOLDEN, "nonnegpca_1" if problem == "NonnegPCA" else "si_1")
    shutil.copytree(src, tmp_path / "dataset" / problem / "1")
    dropin = os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd", "dropin", problem)
    code = textwrap.dedent(f"""
        import importlib, sys, types
        sys.path.insert(0, {dropin!r})
        cfg = types.SimpleNamespace(problem_name={problem!r}, problem_instance=1, problem_initialpoint='a',
                                    problem_coordinator_name='coordinator', is_X_noisy=True,
                                    Xset=[1, 2, 3, 4, 5], h=0.02)
        mod = importlib.import_module(cfg.problem_coordinator_name)
        prob = mod.Coordinator(cfg).run()
        print(type(prob).__name__, mod.__file__)
    """)
    out = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    name, path = out.stdout.split()
    assert name == ("NonnegPCAProblem" if problem == "NonnegPCA" else "SIProblem")
    assert path.startswith(dropin)
