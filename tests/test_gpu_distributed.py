"""The multi-rank path on the GPU box: two processes on cuda:0 (the box has one GPU;
the 8-GPU run is the driver's), torch.distributed over gloo, distributed.solve_sharded (global
instance b on rank b % world, each rank solving its shard with the drop-in RIPTRM.run_batch) and
distributed.gather_rows (the only collective of the path).  The gathered x, y and per-instance
results must equal a single-process run_batch of the same global instances bitwise: an instance's
iterates do not depend on the batch it is solved in (fixed reduction orders, the S-pass kernel
chosen by n alone)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

N, TOTAL, K = 200, 5, 6


def _problems():
    from oracle import nonnegpca_gen as G
    from problems import NonnegPCAProblem
    out = []
    for b in range(TOTAL):
        Z, x0, y0 = G.generate_instance(N, 1200 + b)
        out.append(NonnegPCAProblem(Z=Z, initialpoint=x0, initialineqLagmult=y0))
    return out


def _option():
    from problems import manviofun
    return {"maxiter": K, "tolresid": 0.0, "maxtime": 1e9, "TRS_solver": "tCG", "second_order_stationarity": False,
            "manviofun": manviofun}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "riemannian-interior-point-trust-region-method_amd")]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed import gather_rows, solve_sharded
        outs, ids = solve_sharded(_problems(), _option())
        x = torch.tensor(np.stack([o.x for o in outs]), dtype=torch.float64)
        y = torch.tensor(np.stack([o.ineqLagmult for o in outs]), dtype=torch.float64)
        res = torch.tensor([[len(o.log["iteration"]), float(o.log["residual"][-1])] for o in outs], dtype=torch.float64)
        gx = gather_rows(x, TOTAL, world, rank)
        gy = gather_rows(y, TOTAL, world, rank)
        gr = gather_rows(res, TOTAL, world, rank)
        q.put((rank, ids, gx.numpy(), gy.numpy(), gr.numpy()))
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_match_single_process_bitwise():
    import torch.multiprocessing as mp
    from RIPTRM import RIPTRM
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = RIPTRM(_option()).run_batch(_problems())
    rx = np.stack([o.x for o in ref])
    ry = np.stack([o.ineqLagmult for o in ref])
    rr = np.array([[len(o.log["iteration"]), float(o.log["residual"][-1])] for o in ref])
    for rank, ids, gx, gy, gr in got:
        assert ids == list(range(rank, TOTAL, world))
        np.testing.assert_array_equal(gx, rx)
        np.testing.assert_array_equal(gy, ry)
        np.testing.assert_array_equal(gr, rr)


def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` (the driver's command form, no torchrun) starts two ranks itself
    (bench.launch_ranks) and reports the whole-job line: n_gpus 2, twice the per-GPU batch."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--same-device",
                        "--backend", "gloo", "--dim", "200", "--batch", "4", "--warmup", "1", "--steps", "3",
                        "--cpu-budget", "0"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["world_size"] == 2
    assert out["config"]["global_batch"] == 8
    assert out["value"] > 0


def test_bench_configs3_per_rank_shape_two_ranks():
    """BASELINE configs[3] (n = 4000, 128 instances per rank; src/NonnegPCA/config_simulation.yaml:35-42
    is the reference's multi-run axis) at its real per-rank shape through bench.py's own launcher:
    two ranks on the one GPU (2 x 8.5 GB of S), gloo standing in for RCCL on a 1-GPU box.  The line
    must report both ranks and the backend, and the gathered x / y of global instances spread over
    both shards must equal a single-process solve of the same instances bitwise."""
    import json
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    W, K, n, B, seed0 = 1, 2, 4000, 128, 20251212
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    with tempfile.TemporaryDirectory() as td:
        dump = os.path.join(td, "gathered.npz")
        r = subprocess.run([sys.executable, "-u", os.path.join(root, "bench.py"), "--gpus", "2", "--same-device",
                            "--backend", "gloo", "--dim", str(n), "--batch", str(B), "--warmup", str(W), "--steps", str(K),
                            "--cpu-budget", "0", "--dump", dump], env=env, capture_output=True, text=True, timeout=500)
        assert r.returncode == 0, r.stderr[-3000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        out = json.loads(lines[0])
        g = np.load(dump)
        gx, gy, gs = g["x"], g["y"], g["stats"]
    assert out["n_gpus"] == 2 and out["config"]["world_size"] == 2
    assert out["config"]["global_batch"] == 2 * B
    assert out["config"]["backend"] == "gloo"
    assert [c["rank"] for c in out["config"]["ranks"]] == [0, 1]
    assert all(c["world_size_seen"] == 2 for c in out["config"]["ranks"])
    assert gx.shape == (2 * B, n)
    import engine
    from problems import manviofun
    C = engine.C
    assert (gs[:, C["RIPTRM_STAT_OUTER_ITERS"]] == W + K).all()
    ids = [0, 1, 2 * B - 1, 137]          # rank 0: 0, 137 is odd -> rank 1 too; both shards covered
    eng = engine.NonnegPCABatch(n, len(ids), log_capacity=64, layout="sym", drain_logs=False)
    xg, yg = eng.generate_synthetic(seed0, ids=ids)
    opt = {"maxiter": W + 2 * K, "tolresid": 0.0, "maxtime": float("inf"), "manviofun": manviofun,
           "TRS_solver": "tCG", "second_order_stationarity": False}
    eng.begin(xg, yg, opt, restart_every=20)
    eng.run_until(W + K)
    res = eng.result()
    rx, ry = res.x.cpu().numpy(), res.y.cpu().numpy()
    for k, i in enumerate(ids):
        np.testing.assert_array_equal(gx[i], rx[k], err_msg=f"global instance {i}")
        np.testing.assert_array_equal(gy[i], ry[k], err_msg=f"global instance {i}")


def test_bench_rccl_one_rank_matches_no_dist_bitwise():
    """Every RCCL call site of the N-GPU bench path, executed on the one GPU: `bench.py --gpus 1
    --dist-at-1` initialises a one-rank "nccl" (RCCL) process group with device_id, so rank_census's
    device-tensor all_gather, the timing all_reduce(SUM / MAX) and distributed.gather_rows' final
    all_gather of x, y and the stats all run over RCCL at the configs[3] per-rank shape (n = 4000,
    128 instances).  The gathered x / y / stats must equal a run without a process group bitwise
    (the reference's multi-run axis, src/NonnegPCA/config_simulation.yaml:35-42)."""
    import json
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    base = [sys.executable, "-u", os.path.join(root, "bench.py"), "--gpus", "1", "--dim", "4000", "--batch", "128",
            "--warmup", "1", "--steps", "2", "--cpu-budget", "0"]
    with tempfile.TemporaryDirectory() as td:
        outs, dumps = [], []
        for extra in (["--dist-at-1"], []):
            dumps.append(os.path.join(td, f"g{len(dumps)}.npz"))
            r = subprocess.run(base + extra + ["--dump", dumps[-1]], env=env, capture_output=True, text=True, timeout=400)
            assert r.returncode == 0, r.stderr[-3000:]
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            assert len(lines) == 1, r.stdout
            outs.append(json.loads(lines[0]))
        a, b = np.load(dumps[0]), np.load(dumps[1])
        for key in ("x", "y"):
            np.testing.assert_array_equal(a[key], b[key], err_msg=key)
        import engine
        keep = [i for i in range(a["stats"].shape[1]) if i != engine.C["RIPTRM_STAT_STOP_RUNTIME"]]   # a clock
        np.testing.assert_array_equal(a["stats"][:, keep], b["stats"][:, keep], err_msg="stats")
    cfg = outs[0]["config"]
    assert cfg["backend"] == "nccl", cfg
    assert cfg["ranks"] == [{"rank": 0, "world_size_seen": 1, "device": 0, "rccl": True}], cfg["ranks"]
    assert outs[1]["config"]["backend"] is None and outs[1]["config"]["ranks"][0]["rccl"] is False
    assert outs[0]["n_gpus"] == 1 and outs[0]["config"]["global_batch"] == 128
