#!/usr/bin/env python3
"""Benchmark: outer RIPTRM iterations/sec on batched NonnegPCA n=4000 (BASELINE.json).

One process per GPU (torchrun sets RANK/LOCAL_RANK/WORLD_SIZE); every rank owns 128 independent
instances (global instance b -> rank b % WORLD_SIZE; weak scaling) generated on its own device.
A "step" is one outer RIPTRM iteration of every instance of the batch (RIPTRM.py:931-968).
``--warmup W`` outer iterations run untimed, then exactly ``--steps K`` outer iterations per
instance are timed between barriers + device syncs; the max over ranks is the time.  The only
collectives are the timing all_reduce and the final gather of per-instance results.

Window: the defaults (W=1, K=19) time outer iterations 2..20 of every instance, the BASELINE.md
window (20 outer iterations, mu 0.1 -> 1.4e-8).  Each instance restarts its solve from
(x0, y0, mu0, Delta0) after every 20 outer iterations (riptrm_options.restart_every), so any
--warmup/--steps keeps measuring that same workload instead of running into the mu floor.

The JSON line also carries:
* roofline: the S-pass kernel (k_gemv) timed with HIP events on the stream it runs on, over the
  timed region: algorithmic bytes (8 n^2 + 16 n per instance-pass) / summed kernel time,
  against the 8 TB/s HBM3E peak; ``traffic`` from a committed rocprofv3 PMC summary if present;
* cpu_baseline: the CPU oracle (vectorised NumPy "port") on a bounded sample of the same workload,
  the better of two variants: one instance with all BLAS threads, and --cpu-procs
  single-threaded processes with one instance each, over the same outer-iteration window.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "outer RIPTRM iterations/sec, batched NonnegPCA n=4000, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0
MM_KZ = 4  # K slices of the shared-layout MFMA S-pass (csrc/riptrm_device.h)
MFMA_F64_PEAK_TFS = 78.6  # MI355X dense FP64 matrix peak (spec); tools/mfma_bench.hip issue probe: 70 TFLOP/s


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def trs_options(trs: str) -> dict:
    """--trs: the reference's shipped path (tCG, config_simulation.yaml:21-22) or its class
    default (Exact_RepMat + second-order stationarity, RIPTRM.py:325-326)."""
    if trs == "Exact_RepMat":
        return {"TRS_solver": "Exact_RepMat", "second_order_stationarity": True}
    return {"TRS_solver": "tCG", "second_order_stationarity": False}


def window_positions(warmup: int, steps: int, cycle: int):
    """Solve positions (1..cycle) of the timed outer iterations warmup+1..warmup+steps: instances
    restart after every `cycle` outer iterations (riptrm_options.restart_every), so iteration k of
    the GPU window is outer iteration ((k - 1) mod cycle) + 1 of a solve."""
    c = cycle if cycle > 0 else warmup + steps
    return [((k - 1) % c) + 1 for k in range(warmup + 1, warmup + steps + 1)]


def _oracle_positions(n: int, seed: int, pmax: int, budget_s: float, trs: str, structured: bool = False):
    """Run the oracle on one instance through outer iteration pmax (or until the budget ends);
    returns the solver time of every completed outer iteration (evaluation excluded, as
    RIPTRM.py:932-941) keyed by its position 1..pmax."""
    from oracle import nonnegpca_gen as G
    from oracle import riptrm_oracle as O
    Z, x0, y0 = G.generate_instance(n, seed)
    orc = O.RIPTRMOracle(dict(maxiter=pmax, tolresid=0.0, maxtime=1e12, manviofun=O.sphere_manvio,
                              **trs_options(trs)), deadline=time.time() + budget_s)
    P = O.NonnegPCAStructured(Z) if structured else O.NonnegPCAVectorized(Z)
    try:
        orc.run(P, x0, y0)
    except O.BudgetExceeded:
        pass
    h = orc.outer_heads
    durs = {p: h[p] - h[p - 1] for p in range(1, pmax + 1) if p in h and p - 1 in h}
    _oracle_positions.inner_durations = list(orc.inner_durations)
    return durs


def _window_rate(durs, positions):
    """outer iterations/s over exactly the GPU window's multiset of positions (None if incomplete)."""
    if any(p not in durs for p in positions):
        return None
    t = sum(durs[p] for p in positions)
    return len(positions) / t if t > 0 else None


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max([d.get("num_threads", 1) for d in threadpool_info() if d.get("user_api") == "blas"] or [1])
    except Exception:
        return int(os.environ.get("OMP_NUM_THREADS", "1"))


def _inner_sampled(idurs, inner_per_outer, procs, cores, n, trs, who, budget_s, what=None):
    """A window the CPU cannot finish in its budget (Exact_RepMat at n = 1000: one 2n x 2n pencil
    per inner step): the solver seconds of the inner steps it completed, converted to outer
    iterations/s with the GPU window's own inner iterations per outer iteration."""
    if not idurs or not inner_per_outer:
        return None
    per_inner = sum(idurs) / len(idurs)
    return {"value": procs / (per_inner * inner_per_outer), "unit": "outer iterations/s", "cores": int(cores),
            "kind": "port",
            "sample": ((what or f"oracle/riptrm_oracle.py NonnegPCAVectorized, {who}, n={n}")
                       + (", TRS_solver=Exact_RepMat (trs_oracle: 2n x 2n pencil, scipy.linalg.eig)" if trs != "tCG" else "")
                       + f": the window does not complete in the {budget_s:.0f} s budget, so the rate is sampled per inner "
                         f"step -- {len(idurs)} inner steps of outer iteration 1.. at {per_inner:.2f} s each (evaluation "
                         f"excluded) -- times the GPU window's {inner_per_outer:.2f} inner iterations per outer iteration"
                       + (f", x {procs} processes" if procs > 1 else "")),
            "sampled_inner_s": per_inner}


def cpu_baseline(n: int, positions, budget_s: float, trs: str = "tCG", inner_per_outer=None):
    """SURVEY.md §8d variant (V), one process with all BLAS threads: the oracle (vectorised NumPy +
    OpenBLAS dsymv) on one instance, timed over the GPU window's own outer iterations."""
    from oracle import nonnegpca_gen as G
    durs = _oracle_positions(n, G.SEED0, max(positions), budget_s, trs)
    rate = _window_rate(durs, positions)
    cores = _blas_threads()
    if rate is None:
        return _inner_sampled(_oracle_positions.inner_durations, inner_per_outer, 1, cores, n, trs,
                              f"1 instance (seed {G.SEED0}), {cores} BLAS threads", budget_s)
    return {"value": rate, "unit": "outer iterations/s", "cores": int(cores), "kind": "port",
            "sample": (f"oracle/riptrm_oracle.py NonnegPCAVectorized, 1 instance n={n} (reference generator recipe, "
                       f"seed {G.SEED0}), timed over the GPU window's own outer-iteration positions "
                       f"{_pos_text(positions)} (evaluation time excluded as RIPTRM.py:932-941), NumPy + OpenBLAS dsymv "
                       f"(one triangle of S), {cores} threads"
                       + (", TRS_solver=Exact_RepMat (trs_oracle: 2n x 2n pencil, scipy.linalg.eig)" if trs != "tCG" else ""))}


def _pos_text(positions):
    """Compact text of a position multiset, e.g. '6..20 + 1..5'."""
    runs, start, prev = [], positions[0], positions[0]
    for p in positions[1:]:
        if p == prev + 1:
            prev = p
            continue
        runs.append((start, prev))
        start = prev = p
    runs.append((start, prev))
    return " + ".join(f"{a}..{b}" if a != b else f"{a}" for a, b in runs)


def _cpu_worker(argv):
    """One single-threaded oracle instance (run in its own process by cpu_baseline_pool)."""
    n, seed, pmax, budget, trs = int(argv[0]), int(argv[1]), int(argv[2]), float(argv[3]), argv[4]
    durs = _oracle_positions(n, seed, pmax, budget, trs)
    out = {str(k): v for k, v in durs.items()}
    out["inner"] = _oracle_positions.inner_durations
    print(json.dumps(out), flush=True)


def cpu_baseline_pool(n: int, positions, budget_s: float, procs: int, trs: str = "tCG", inner_per_outer=None):
    """SURVEY.md §8d variant (V) as a pool: `procs` single-threaded oracle processes, one instance
    each (seeds SEED0 + i), run concurrently, each timed over the GPU window's own positions;
    aggregate = sum of the per-process rates, over processes that completed the whole window."""
    import subprocess
    from oracle import nonnegpca_gen as G
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", str(n), str(G.SEED0 + i),
                            str(max(positions)), str(budget_s), trs], stdout=subprocess.PIPE,
                           stderr=subprocess.DEVNULL, env=env, text=True) for i in range(procs)]
    rates, inner = [], []
    for p in ps:
        out, _ = p.communicate(timeout=budget_s + 600)
        try:
            rec = json.loads(out.strip().splitlines()[-1])
            inner.extend(rec.pop("inner", []))
            durs = {int(k): v for k, v in rec.items()}
        except Exception:
            continue
        r = _window_rate(durs, positions)
        if r is not None:
            rates.append(r)
    if not rates:
        return _inner_sampled(inner, inner_per_outer, procs, procs, n, trs,
                              f"{procs} single-threaded processes, one instance each (seeds {G.SEED0}..)", budget_s)
    # every process runs the same amount of work, so the complete ones are a fair sample; scale the
    # aggregate to all `procs` cores (incomplete processes ran on cores too)
    agg = sum(rates) / len(rates) * procs
    return {"value": agg, "unit": "outer iterations/s", "cores": int(procs), "kind": "port",
            "sample": (f"oracle/riptrm_oracle.py NonnegPCAVectorized, {procs} single-threaded processes, one instance n={n} "
                       f"each (seeds {G.SEED0}..{G.SEED0 + procs - 1}), each timed over the GPU window's own positions "
                       f"{_pos_text(positions)} within a {budget_s:.0f} s budget; {len(rates)}/{procs} processes completed the "
                       f"window, aggregate = mean complete per-process rate x {procs}, evaluation time excluded as "
                       f"RIPTRM.py:932-941")}


def cpu_reference_structured(n: int, budget_s: float):
    """SURVEY.md §8d variant (R): the oracle's per-constraint restatement of the reference's wiring
    (NonnegPCAStructured: n constraint closures, per-constraint Gx/Gxaj/hessLagrangian loops as
    RIPTRM.py:475-571 runs them; no autograd, so a lower bound on the reference's own cost), one
    instance, outer iterations 1..k completed within the budget.  A stated extra, not the
    like-for-like baseline."""
    from oracle import nonnegpca_gen as G
    durs = _oracle_positions(n, G.SEED0, 20, budget_s, "tCG", structured=True)
    if not durs:
        return None
    k = max(durs)
    t = sum(durs[p] for p in range(1, k + 1))
    return {"value": k / t, "unit": "outer iterations/s", "cores": 1, "kind": "port",
            "sample": (f"oracle/riptrm_oracle.py NonnegPCAStructured (reference-structured, per-constraint loops), "
                       f"1 instance n={n} seed {G.SEED0}, outer iterations 1..{k} ({t:.1f} s) within a {budget_s:.0f} s "
                       f"budget")}


def host_cpu_info() -> dict:
    """lscpu model name and os.cpu_count() of the host the CPU legs ran on."""
    model, cores_per_socket, sockets = None, None, None
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            key, _, val = line.partition(":")
            key, val = key.strip(), val.strip()
            if key == "Model name" and model is None:
                model = val
            elif key == "Core(s) per socket":
                cores_per_socket = int(val)
            elif key == "Socket(s)":
                sockets = int(val)
    except Exception:
        pass
    if model is None:
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
        except Exception:
            pass
    phys = cores_per_socket * sockets if cores_per_socket and sockets else None
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "physical_cores": phys}


def core_rationale(cpu: dict, gpus_per_node: int = 8) -> dict:
    """Why the CPU legs use the cores they use, and what the whole host would give (SURVEY.md §8d:
    the baseline is context, not the target).  The GPU box leases this job one GPU and 16 of the
    host's CPUs (OMP_NUM_THREADS / MAX_JOBS are 16 there, and its process limits are sized for 16
    workers), which is also one GPU's share of an 8-GPU node's physical cores on the pool's hosts; a
    pool over the whole host is outside the lease, so it is extrapolated, not timed."""
    phys = cpu.get("physical_cores")
    out = {"core_rationale": (f"{cpu['cores']} cores = the CPU share the GPU box leases to one GPU's job (OMP_NUM_THREADS="
                              f"{os.environ.get('OMP_NUM_THREADS', '?')} there)"
                              + (f"; the host has {phys} physical cores / {cpu.get('os_cpu_count')} threads for "
                                 f"{gpus_per_node} GPUs = {phys / gpus_per_node:g} cores per GPU" if phys else "")
                              + "; a whole-host pool is outside the lease: whole_host_estimate scales the pool linearly "
                                "to every physical core (an upper bound, not measured)")}
    if phys and cpu.get("cores"):
        out["whole_host_estimate"] = cpu["value"] * phys / cpu["cores"]
    return out


def pick_cpu_baseline(threaded, pool):
    """report the better of the two CPU variants (one process with all BLAS threads,
    a pool of single-threaded processes) and name the other under ``other_variant``.  Either may be
    None (not run or incomplete).  Returns a new dict (or None)."""
    legs = [c for c in (threaded, pool) if c is not None]
    if not legs:
        return None
    best = max(legs, key=lambda c: c["value"])
    out = dict(best)
    other = pool if best is threaded else threaded
    if other is not None:
        out["other_variant"] = {"value": other["value"], "cores": other["cores"], "sample": other["sample"]}
    return out


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_census(dist, world: int, rank: int, dev):
    """Every rank's (rank, world size it saw, device index, backend is RCCL) gathered to all ranks
    with one all_gather, so the JSON line shows which collective backend really ran with how many
    ranks on which devices.  World 1: just this process."""
    import torch
    on = dist.is_initialized()
    backend = dist.get_backend() if on else None
    me = torch.tensor([rank, dist.get_world_size() if on else 1, dev.index if dev.index is not None else 0,
                       1 if backend == "nccl" else 0], dtype=torch.int64,
                      device=dev if backend == "nccl" else "cpu")
    if not on:
        rows = [me]
    else:
        rows = [torch.empty_like(me) for _ in range(world)]
        dist.all_gather(rows, me)
    return [{"rank": int(r[0]), "world_size_seen": int(r[1]), "device": int(r[2]), "rccl": bool(r[3])}
            for r in (t.cpu() for t in rows)]


def launch_ranks(n: int, script: str | None = None, argv=None) -> int:
    """torch.distributed.run-style launcher for ``bench.py --gpus N`` run directly: N child
    processes of this same command line, rank i on LOCAL_RANK i, rendezvous on 127.0.0.1.  The
    children inherit stdout, and only rank 0 prints the JSON line, so the parent relays it as is.
    If any rank fails, the rest are terminated and the first non-zero exit code is returned."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)]
                                      + list(sys.argv[1:] if argv is None else argv), env=env))
    log(f"launched {n} ranks (pids {[p.pid for p in procs]}, master 127.0.0.1:{port})")
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log(f"rank pid {p.pid} exited with {code}; stopping the other ranks")
                for q in pending:
                    q.terminate()
        time.sleep(0.2)
    return rc


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-worker":
        _cpu_worker(sys.argv[2:])
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--si-cpu-worker":
        _si_cpu_worker(sys.argv[2:])
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=19, help="timed outer iterations per instance")
    ap.add_argument("--warmup", type=int, default=1, help="untimed outer iterations per instance")
    ap.add_argument("--layout", default="sym", choices=["sym", "full", "shared"],
                    help="storage of S = Z + Z^T (shared: one Z, --batch initial points, MFMA S-pass)")
    ap.add_argument("--cycle", type=int, default=20, help="outer iterations per solve before restart")
    ap.add_argument("--dim", type=int, default=4000, help="problem dimension n")
    ap.add_argument("--batch", type=int, default=128, help="instances per GPU")
    ap.add_argument("--cpu-budget", type=float, default=60.0,
                    help="seconds allowed for the BLAS-threaded CPU baseline (0 = skip every CPU leg)")
    ap.add_argument("--cpu-pool-budget", type=float, default=150.0,
                    help="seconds allowed for each single-threaded pool process to complete the window")
    ap.add_argument("--ref-structured-dim", type=int, default=1000,
                    help="n of the reference-structured CPU variant (R) reported as an extra (0 = skip)")
    ap.add_argument("--ref-structured-budget", type=float, default=20.0)
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="also time this many single-threaded oracle processes (0 = only the BLAS-threaded one)")
    ap.add_argument("--seed0", type=int, default=20251212)
    ap.add_argument("--problem", default="nonnegpca", choices=["nonnegpca", "si", "stiefel"],
                    help="si: StableIdentification (d=5 fixture, starts cycled + perturbed), one launch per solve")
    ap.add_argument("--stiefel-p", type=int, default=50, help="p of Stiefel(n, p) for --problem stiefel")
    ap.add_argument("--si-dim", type=int, default=5,
                    help="block size d of --problem si (5: the reference fixture; else si.synthetic_problem)")
    ap.add_argument("--trs", default="tCG", choices=["tCG", "Exact_RepMat"],
                    help="subproblem solver (Exact_RepMat: manifold.dim <= 96, with the second-order test)")
    ap.add_argument("--stream-groups", type=int, default=0, choices=[0, 1, 2],
                    help="instance groups on separate streams (0 = library default)")
    ap.add_argument("--spass-kind", type=int, default=1, choices=[0, 1, 2, 3],
                    help="sym layout S-pass: 1 = automatic (rule on n alone: persistent super-tile kernel for n >= 2561, "
                         "per-tile kernel below; batch-independent bits), 0 = per-tile kernel only, 2 = super-tile kernel "
                         "always, 3 = super-tile for launches with >= 1 unit per CU if a bind-time timing preferred it")
    ap.add_argument("--persistent", type=int, default=1, choices=[0, 1, 2],
                    help="k_persist for small batches: 1 = cooperative launch (default), 2 = plain launch (A/B), 0 = off")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r4_traffic_spass_sup.json"),
                    help="per instance-pass HBM bytes of the S-pass from a committed rocprofv3 PMC summary (scripts/gate.sh pmc_spass)")
    ap.add_argument("--si-pmc-json", default=os.path.join(ROOT, "profiles", "r5_si_pmc.json"),
                    help="k_si issue-rate PMC summary (scripts/si_pmc_summary.py) for --problem si's roofline")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--dump", default="",
                    help="rank 0 writes the gathered x, y and stats of every global instance to this .npz")
    ap.add_argument("--dist-at-1", action="store_true",
                    help="with --gpus 1: still initialise a (one-rank) process group, so the collectives run")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on cuda:0 (use with --backend gloo on a 1-GPU box)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` outside torchrun: launch the N ranks here, before anything
        # touches the GPU (children are started as subprocesses, never exec'd)
        sys.exit(launch_ranks(args.gpus))

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    if world > 1 or args.dist_at_1:
        # --dist-at-1: a one-rank process group on the one GPU, so every collective call site of
        # the N-GPU path (rank census, timing all_reduce, final all_gather) runs over RCCL
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dev_idx = 0 if args.same_device else local
        torch.cuda.set_device(dev_idx)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(args.backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    if args.problem == "stiefel":
        bench_stiefel(args, world, rank, dev, dist)
        if dist.is_initialized():
            dist.destroy_process_group()
        return
    if args.problem == "si":
        bench_si(args, world, rank, dev, dist)
        if dist.is_initialized():
            dist.destroy_process_group()
        return

    import engine
    from problems import manviofun

    n, B, W, K = args.dim, args.batch, args.warmup, args.steps
    eng = engine.NonnegPCABatch(n, B, log_capacity=2048, layout=args.layout, stream_groups=args.stream_groups,
                                spass_kind=args.spass_kind, drain_logs=False, persistent=args.persistent)
    nS = 1 if args.layout == "shared" else B
    log(f"rank {rank}/{world}: generating {B} instances n={n} ({nS * eng.inst_stride * 8 / 1e9:.1f} GB S)")
    # global instance ids owned by this rank: rank, rank+world, ... (seed seed0 + id)
    gen_ids = [rank + world * i for i in range(B)]
    xg, yg = eng.generate_synthetic(args.seed0, ids=gen_ids)
    opt = {"maxiter": W + 2 * K, "tolresid": 0.0, "maxtime": math.inf, "manviofun": manviofun, **trs_options(args.trs)}
    eng.begin(xg, yg, opt, restart_every=args.cycle)
    torch.cuda.synchronize(dev)
    t0 = time.time()
    eng.run_until(W)
    torch.cuda.synchronize(dev)
    log(f"rank {rank}: warmup ({W} outer iterations) {time.time() - t0:.2f}s")
    st0 = eng.stats()
    # Small batches run as replayed hipGraphs, which per-launch HIP events would disable: time them
    # unprofiled and take the kernel timing from a second, profiled window of the same length.
    graph_mode = (args.layout == "shared") or (B * eng.inst_stride * 8 < 2e8)
    if not graph_mode:
        engine.profile_enable(eng, True)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    eng.run_until(W + K)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if dist.is_initialized():
        dist.barrier()
    st1 = eng.stats()
    if graph_mode:
        engine.profile_enable(eng, True)
        eng.run_until(W + 2 * K)
        prof = engine.profile_read(eng)
        st_p = eng.stats()
        passes_prof = float((st_p[:, engine.C["RIPTRM_STAT_PASSES"]] - st1[:, engine.C["RIPTRM_STAT_PASSES"]]).sum())
        rhs_prof = float((st_p[:, engine.C["RIPTRM_STAT_RHS"]] - st1[:, engine.C["RIPTRM_STAT_RHS"]]).sum())
    else:
        prof = engine.profile_read(eng)
    engine.profile_enable(eng, False)
    C = engine.C
    d = lambda f: float((st1[:, C[f"RIPTRM_STAT_{f}"]] - st0[:, C[f"RIPTRM_STAT_{f}"]]).sum())
    outer = d("OUTER_ITERS")
    passes, inner, tcg = d("PASSES"), d("INNER_ITERS"), d("TCG_ITERS")
    counts = torch.tensor([outer, passes, inner, tcg, prof["gemv_ms"], prof["gemv_launches"]],
                          dtype=torch.float64, device=dev)
    tmax = torch.tensor([el], dtype=torch.float64, device=dev)
    ranks_seen = rank_census(dist, world, rank, dev)
    if dist.is_initialized():
        from distributed import gather_rows
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        # final gather of per-instance results (x, y, stats) over RCCL, in global instance order
        res = eng.result()
        total = B * world
        gx = gather_rows(res.x.contiguous(), total, world, rank)
        gy = gather_rows(res.y.contiguous(), total, world, rank)
        gs = gather_rows(torch.as_tensor(res.stats, device=dev), total, world, rank)
    elif args.dump:
        res = eng.result()
        gx, gy, gs = res.x, res.y, torch.as_tensor(res.stats)
    if args.dump and rank == 0:
        # gathered per-instance results in global instance order (tests compare them bitwise)
        np.savez(args.dump, x=gx.cpu().numpy()[:, :n], y=gy.cpu().numpy()[:, :n], stats=gs.cpu().numpy(),
                 ids=np.arange(B * world), seed0=args.seed0, outer_target=W + K)
    T = float(tmax.item())
    outer_all, passes_all, inner_all, tcg_all, gemv_ms_all, gemv_n_all = [float(v) for v in counts.tolist()]

    if rank == 0:
        # algorithmic bytes of one instance-pass: the stored S (sym: upper-triangle tiles incl.
        # padding, ~4 n^2; full: 8 n^2) + the vectors in/out
        s_bytes = 8.0 * eng.inst_stride if args.layout == "sym" else 8.0 * n * n
        bytes_per_pass = s_bytes + 16.0 * n
        # rank-0 kernel timing (every rank runs the same kernel on its own batch)
        gemv_s = prof["gemv_ms"] / 1e3
        passes_r0 = float((st1[:, C["RIPTRM_STAT_PASSES"]] - st0[:, C["RIPTRM_STAT_PASSES"]]).sum())
        rhs_r0 = float((st1[:, C["RIPTRM_STAT_RHS"]] - st0[:, C["RIPTRM_STAT_RHS"]]).sum())
        if graph_mode:   # kernel timing came from the profiled second window
            passes_r0, rhs_r0 = passes_prof, rhs_prof
        achieved = (passes_r0 * bytes_per_pass / gemv_s / 1e9) if gemv_s > 0 else None
        nl = max(1, int(prof["gemv_launches"]))
        traffic = None
        cal = eng.spass_calibration() if args.layout == "sym" else {}
        spass_kernel = cal.get("kernel", "k_spass_sym")
        spass_label = ("k_spass_sym (S-pass, one workgroup per symmetric 128x128 tile)" if spass_kernel == "k_spass_sym" else
                       "k_spass_sup (S-pass, persistent: one workgroup per CU over 2x2-tile units, partial sums "
                       "written in bursts)")
        if os.path.exists(args.traffic_json) and args.layout == "sym":
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("n") == n and tj.get("kernel", "k_spass_sym") == spass_kernel:
                    # per-launch HBM bytes scaled to this run's mean instances per launch
                    traffic = tj["hbm_bytes_per_instance_pass"] * passes_r0 / nl
            except Exception as e:  # pragma: no cover
                log(f"traffic json unreadable: {e}")
        persist = eng.persistent_state()["active"] if args.layout == "sym" else False
        if persist:
            # k_persist: the whole lock-step loop in one launch per chunk, S held in LDS.  Its time
            # is per-pass latency (barrier + reductions), not bandwidth: price the passes it served
            # at the bytes the lock-step S-pass would stream, and give the per-pass latency.
            kern_s = prof["state_ms"] / 1e3
            eff = (passes_r0 * bytes_per_pass / kern_s / 1e9) if kern_s > 0 else None
            nl = max(1, int(prof["state_launches"]))
            roofline = {"bound": "hbm", "achieved": eff, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": (eff / HBM_PEAK_GBS) if eff else None, "traffic": None,
                        "bytes_definition": ("stored S per instance-pass (symmetric tiles, "
                                             f"{s_bytes / 1e6:.2f} MB at n={n}) + 16 n, as the lock-step S-pass would "
                                             "stream it; k_persist reads S from HBM once per launch and serves every "
                                             "pass from LDS, so this is an effective rate of a latency-bound loop"),
                        "kernel": ("k_persist (one launch per chunk: every 128x128 tile of S in LDS, one workgroup "
                                   "per tile, replicated state machine, one in-launch barrier per pass)"),
                        "bytes_per_launch": passes_r0 * bytes_per_pass / nl,
                        "avg_launch_us": prof["state_ms"] * 1e3 / nl,
                        "us_per_pass": (kern_s * 1e6 / passes_r0) if passes_r0 > 0 else None}
        elif args.layout == "shared":
            # dense product on the fp64 matrix cores: 2 n^2 algorithmic flops per right-hand side
            # (RIPTRM_STAT_RHS: a trial pass multiplies two, a tCG pass one)
            flops = rhs_r0 * 2.0 * n * n
            tf = flops / gemv_s / 1e12 if gemv_s > 0 else None
            roofline = {"bound": "mfma", "achieved": tf, "peak": MFMA_F64_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": (tf / MFMA_F64_PEAK_TFS) if tf else None, "traffic": None,
                        "kernel": ("k_spass_mm (shared-S multi-start S-pass, v_mfma_f64_16x16x4_f64; 128 right-hand sides x "
                                   f"{64 if ((n + 31) // 32 * 32 + 127) // 128 * MM_KZ < 256 else 128} rows per "
                                   "workgroup, 8 waves, V and S K-steps staged in LDS by global_load_lds, "
                                   f"{MM_KZ} K slices)"),
                        "flops_per_launch": flops / nl, "avg_launch_us": prof["gemv_ms"] * 1e3 / nl}
        else:
            # the same launches priced with the bytes symmetry strictly requires (one triangle incl. the
            # diagonal + the vectors): what a layout without padded diagonal / edge tiles would move
            min_bytes = 8.0 * n * (n + 1) / 2 + 16.0 * n
            ach_min = (passes_r0 * min_bytes / gemv_s / 1e9) if gemv_s > 0 else None
            roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                        "traffic": traffic,
                        "bytes_definition": ("stored S per instance-pass in the symmetric-tile layout (upper-triangle "
                                             "128x128 tiles incl. the whole diagonal tiles and the 32-column-padded "
                                             f"edge: {s_bytes / 1e6:.2f} MB at n={n}) + 16 n vector bytes")
                        if args.layout == "sym" else "8 n^2 (full S) + 16 n vector bytes per instance-pass",
                        "frac_min_bytes": (ach_min / HBM_PEAK_GBS) if ach_min else None,
                        "min_bytes_definition": "n(n+1)/2 * 8 (one triangle incl. the diagonal) + 16 n per instance-pass",
                        "kernel": spass_label if args.layout == "sym" else "k_gemv (S-pass, full matrix)",
                        "bytes_per_launch": passes_r0 * bytes_per_pass / nl,
                        "avg_launch_us": prof["gemv_ms"] * 1e3 / nl}
        # the state kernel's vector work (the Sphere projection / retraction and the tCG updates,
        # fused in k_state): per instance-step it reads x, y, cxCur, delta, eta, Heta, r and the
        # S-pass's partial sums of every element (one per super-tile / tile column), and writes
        # delta, eta, Heta, r back
        state_roofline = None
        if not graph_mode and not persist and prof["state_ms"] > 0 and args.layout == "sym":
            nt_ = -(-n // 128)
            parts = -(-nt_ // 2) if spass_kernel == "k_spass_sup" else nt_
            sbytes = passes_r0 * (11 + parts) * 8.0 * n
            sach = sbytes / (prof["state_ms"] / 1e3) / 1e9
            state_roofline = {"bound": "hbm", "achieved": sach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": sach / HBM_PEAK_GBS, "bytes_per_launch": sbytes / max(1, prof["state_launches"]),
                              "avg_launch_us": prof["state_ms"] * 1e3 / max(1, prof["state_launches"]),
                              "bytes_definition": (f"per instance-step (11 + {parts}) x 8 n bytes: x, y, cxCur, delta, eta, "
                                                   f"Heta, r read and delta, eta, Heta, r written, plus the {parts} "
                                                   "partial sums of every element the S-pass left"),
                              "kernel": "k_state (tCG step, Sphere projection / retraction, trial point, acceptance; "
                                        "runs beside the other stream group's S-pass)"}
        spass_roofline = None
        tri_lo, tri_hi = engine.C["RIPTRM_TRS_TRI_MIN"], engine.C["RIPTRM_TRS_TRI_MAX"]
        if args.trs == "Exact_RepMat" and 96 < n - 1 < tri_lo and rank == 0:
            # the eigensolver, not the S-pass, sets this line's time: price it, keep the S-pass in detail
            spass_roofline, roofline = roofline, eig_roofline(n - 1, B, dev)
        elif args.trs == "Exact_RepMat" and tri_lo <= n - 1 <= tri_hi and rank == 0:
            # the tridiagonal path's subproblem service (riptrm_tri.h) sets this line's time
            spass_roofline, roofline = roofline, tri_roofline(n - 1, dev, min(B, 64))
        cpu = None
        if args.cpu_budget > 0 and world == 1:
            positions = window_positions(W, K, args.cycle)
            log(f"CPU baseline (oracle) over positions {_pos_text(positions)} ...")
            ipo = (inner_all / outer_all) if outer_all > 0 else None
            threaded = cpu_baseline(n, positions, args.cpu_budget, args.trs, ipo)
            # the pool runs one instance per process: never more processes than the workload has
            # instances (configs[1] is ONE instance; 16 processes would time 16x its work)
            procs = min(args.cpu_procs, B)
            pool = None
            if procs > 0:
                log(f"CPU baseline, {procs} single-threaded processes ...")
                pool = cpu_baseline_pool(n, positions, args.cpu_pool_budget, procs, args.trs, ipo)
            cpu = pick_cpu_baseline(threaded, pool)
            if cpu is not None:
                cpu.update(host_cpu_info())
                cpu.update(core_rationale(cpu))
                cpu["gpu_over_cpu"] = (outer_all / T) / cpu["value"]
                if args.ref_structured_dim > 0:
                    log(f"CPU reference-structured variant (R), n={args.ref_structured_dim} ...")
                    cpu["extra_reference_structured"] = cpu_reference_structured(args.ref_structured_dim,
                                                                                 args.ref_structured_budget)
        out = {
            "metric": METRIC,
            "value": outer_all / T,
            "unit": "outer iterations/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": T / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference generator recipe src/NonnegPCA/generator.py:9-65, drawn on device)",
            "config": {"workload": (f"NonnegPCA n={n}, one Z with {B} initial points per GPU (multi-start, "
                                    f"the problem_initialpoint axis; SURVEY 8d variant)") if args.layout == "shared"
                                   else (f"NonnegPCA n={n}, batch of {B} independent instances per GPU"
                                         + (" (BASELINE configs[2]; configs[3] at 8 GPUs)" if (n, B) == (4000, 128) else
                                            " (BASELINE configs[1])" if (n, B) == (1000, 1) else ""))
                                   + ("" if args.trs == "tCG" else ", TRS_solver=Exact_RepMat + second-order test"),
                       "trs_solver": args.trs,
                       "n": n, "batch_per_gpu": B, "global_batch": B * world,
                       "outer_window": [W + 1, W + K], "restart_every": args.cycle, "layout": args.layout,
                       "parallelism": f"instance-sharded x{world}", "world_size": world,
                       "backend": dist.get_backend() if dist.is_initialized() else None, "ranks": ranks_seen},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "detail": {"inner_iterations_per_s": inner_all / T, "tcg_iterations_per_s": tcg_all / T,
                       "s_passes_per_s": passes_all / T,
                       "gemv_time_frac": None if graph_mode else (prof["gemv_ms"] / 1e3) / T,
                       "kernel_timing": ("second profiled window, outer iterations "
                                         f"{W + K + 1}..{W + 2 * K} (the timed window replays hipGraphs)")
                       if graph_mode else "HIP events inside the timed window",
                       "state_kernel_ms": prof["state_ms"], "state_launches": prof["state_launches"],
                       "gemv_launches": prof["gemv_launches"],
                       "state_kernel_roofline": state_roofline,
                       **({"spass_roofline": spass_roofline} if spass_roofline else {}),
                       **({"spass_calibration": cal} if cal.get("ms_per_launch_tile") else {}),
                       **({"exact_repmat_note": (
                           "manifold.dim > 96: the subproblems are served in batched passes between lock-step "
                           "chunks (csrc/riptrm_trs_big.hip); the pass, not the S-pass (detail.spass_roofline), sets "
                           "this line's time: up to order 149 the hand-written eigensolver (csrc/riptrm_eig.h) with the "
                           "CG in its eigen-coordinates; 150..1024 the cooperative tridiagonalisation and the subproblem "
                           "in T's coordinates (csrc/riptrm_tri.h); a subproblem at an accepted trial point reuses that "
                           "point's eigenpairs / tridiagonal form (riptrm_trs_bind_cache)"),
                           "trs_cache": dict(zip(("hits", "subproblems"), eng.trs_cache_stats()))}
                          if args.trs == "Exact_RepMat" and n - 1 > engine.C["RIPTRM_TRS_DIM_MAX"] else {})},
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def bench_stiefel(args, world, rank, dev, dist):
    """Stiefel(n, p) kernels (BASELINE configs[4] size (200, 50) x 256 per GPU):
    --steps projections and retractions of the whole batch, HIP-event timed on the stream."""
    import numpy as np
    import torch
    from stiefel import StiefelBatch
    n, p, B = args.dim, args.stiefel_p, args.batch
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed0 + rank)
    X = torch.linalg.qr(torch.randn(B, n, p, dtype=torch.float64, device=dev, generator=g))[0].contiguous()
    W = torch.randn(B, n, p, dtype=torch.float64, device=dev, generator=g)
    st = StiefelBatch(n, p)
    U = (0.1 * st.projection(X, W)).contiguous()
    res = {}
    for name, fn in (("projection", lambda: st.projection(X, W)), ("retraction", lambda: st.retraction(X, U))):
        for _ in range(max(1, args.warmup)):
            fn()
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        res[name] = e0.elapsed_time(e1) / 1e3 / args.steps
    t = torch.tensor([res["projection"], res["retraction"]], dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    tp, tr = [float(v) for v in t.tolist()]
    if rank != 0:
        return
    gbs = 3.0 * n * p * 8 * B / tp / 1e9    # read X, U; write the result
    tfs = 4.0 * n * p * p * B / tp / 1e12
    hbm_floor = 3.0 * n * p * 8 * B / (HBM_PEAK_GBS * 1e9)
    mfma_floor = 4.0 * n * p * p * B / (MFMA_F64_PEAK_TFS * 1e12)
    # k_st_retr2 (point resident in LDS) when (n, p) fits 160 KiB, else the round-1 kernel
    nr, s16 = -(-n // 16) * 16, 16 * (-(-p // 16))
    fits = (nr * s16 + s16 * s16 + (s16 // 16) * (s16 // 16 + 1) // 2 * 256) * 8 <= 160 * 1024
    retr_kernel = ("k_st_retr2" if fits and os.environ.get("RIPTRM_STIEFEL_RETR", "") != "r1" else "k_st_retr_r")
    # k_st_proj3 (X and U resident in LDS) for 49 <= p <= 64, n <= 224 (csrc/riptrm_stiefel.hip proj3_ok)
    proj_kernel = ("k_st_proj3" if -(-p // 16) == 4 and n * p % 2 == 0 and -(-n // 16) <= 14 and
                   2 * n * p + (0 if n * p >= 64 * 64 else 64 * 64) <= 160 * 1024 // 8 and
                   os.environ.get("RIPTRM_STIEFEL_PROJ", "") != "r2" else "k_st_proj")
    # more points than CUs: the persistent k_st_proj4 (same arithmetic, next point copied in during the update)
    if proj_kernel == "k_st_proj3" and B > torch.cuda.get_device_properties(dev).multi_processor_count and \
            os.environ.get("RIPTRM_STIEFEL_PROJ", "") != "p3":
        proj_kernel = "k_st_proj4"
    # HBM bytes per launch from the committed PMC passes of this exact shape (FETCH_SIZE doubled
    # per MI355X_MICROARCH.md, + WRITE_SIZE); None for any other shape
    # (profiles/r4_stiefel_pmc.json: 2048 points; bytes per point scaled to this batch)
    traffic = {}
    pmc_path = os.path.join(ROOT, "profiles", "r4_stiefel_pmc.json")
    if os.path.exists(pmc_path):
        pm = json.load(open(pmc_path))
        if (pm.get("n"), pm.get("p")) == (n, p) and pm.get("B"):
            for kname, m in pm["kernels"].items():
                if "read_bytes_corrected" in m and "write_bytes" in m:
                    traffic[kname.split("::")[-1].split("<")[0]] = (m["read_bytes_corrected"] + m["write_bytes"]) / pm["B"] * B
    # CPU baseline: the pymanopt restatement (oracle/stiefel_oracle.py, NumPy) on the host, over the
    # same points until ~2 s have passed (a bounded sample; BLAS threads as configured)
    from oracle.stiefel_oracle import Stiefel as _CpuStiefel
    M = _CpuStiefel(n, p)
    Xh, Wh, Uh = X.cpu().numpy(), W.cpu().numpy(), U.cpu().numpy()
    rates = {}
    for name, fn in (("projection", lambda b: M.projection(Xh[b], Wh[b])),
                     ("retraction", lambda b: M.retraction(Xh[b], Uh[b]))):
        cnt, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            fn(cnt % B)
            cnt += 1
        rates[name] = cnt / (time.perf_counter() - t0)
    cpu = {"value": rates["projection"], "unit": "projections/s", "cores": int(os.environ.get("OMP_NUM_THREADS", "1")),
           "kind": "port", "sample": f"oracle/stiefel_oracle.py (NumPy) projection of the first points of the batch, "
                                     f"{n}x{p}, repeated for 2 s on the host"}
    cpu_retr = rates["retraction"]
    print(json.dumps({
        "metric": f"Stiefel({n},{p}) projections/sec, batch {B}/GPU",
        "value": B * world / tp, "unit": "projections/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": tp * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (random orthonormal X, Gaussian U)",
        "config": {"workload": f"Stiefel(n={n}, p={p}) x {B} per GPU (BASELINE configs[4] size)",
                   "global_batch": B * world, "parallelism": f"instance-sharded x{world}", "world_size": world},
        # binding roof = the larger of the two floors: 24 n p bytes (read X, U; write the result)
        # at HBM peak vs 4 n p^2 flops (X^T U and X sym(.)) at the FP64-matrix peak
        "roofline": {"bound": "hbm" if hbm_floor >= mfma_floor else "mfma",
                     "achieved": gbs if hbm_floor >= mfma_floor else tfs,
                     "peak": HBM_PEAK_GBS if hbm_floor >= mfma_floor else MFMA_F64_PEAK_TFS,
                     "unit": "GB/s" if hbm_floor >= mfma_floor else "TFLOP/s",
                     "frac": max(hbm_floor, mfma_floor) / tp,
                     "hbm_floor_us": hbm_floor * 1e6, "mfma_floor_us": mfma_floor * 1e6,
                     "mfma_achieved_tflops": tfs,
                     "traffic": traffic.get(proj_kernel),
                     "kernel": f"{proj_kernel} (U - X sym(X^T U), " + ("one workgroup per CU looping over its points, the next "
                                                                      "point copied into LDS during the update)"
                                                                      if proj_kernel == "k_st_proj4" else "one workgroup per point)")},
        "cpu_baseline": cpu,
        "detail": {"retractions_per_s": B * world / tr, "retraction_ms": tr * 1e3,
                   "retraction_roofline": {"bound": "hbm", "achieved": 3.0 * n * p * 8 * B / tr / 1e9,
                                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_floor / tr,
                                           "traffic": traffic.get(retr_kernel), "kernel": retr_kernel},
                   "retraction_cpu_per_s": cpu_retr,
                   "retraction_note": "CholeskyQR2, latency-bound: two p-step factorisations per point, one point "
                                      "per CU"},
    }), flush=True)


def si_instance(d: int, starts: int = 20):
    """The StableIdentification data of the SI bench line: the reference's fixture
    (dataset/StableIdentification/1, d = 5: coordinator.py:54-90 stacking, constset.csv, starts a..t)
    or, for another d, the product's restatement of the dataset recipe (si.synthetic_problem,
    generator.py:18-134), seed 1000 + d.  Returns (X, XP, h, constset rows, [(x0, y0), ...])."""
    import numpy as np
    if d == 5:
        ds = os.path.join(ROOT, "tests", "golden", "si_1")
        X = XP = None
        for i in (1, 2, 3, 4, 5):
            Xo = np.loadtxt(os.path.join(ds, f"noisyX_{i}.csv"))
            X = Xo[:, :-1] if X is None else np.hstack((X, Xo[:, :-1]))
            XP = Xo[:, 1:] if XP is None else np.hstack((XP, Xo[:, 1:]))
        y0 = np.atleast_1d(np.loadtxt(os.path.join(ds, "initineqLagmult.csv")))
        st = [(np.stack([np.loadtxt(os.path.join(ds, f"init{c}_{p}.csv")) for c in "JRQ"]), y0)
              for p in "abcdefghijklmnopqrst"]
        return X, XP, 0.02, np.loadtxt(os.path.join(ds, "constset.csv")), st
    import si
    return si.synthetic_problem(d, 1000 + d, starts=starts)


def si_starts(B: int, ids, d: int = 5):
    """StableIdentification batch: the instance's starts (si_instance: 20) cycled; copies beyond the
    first 20 perturbed (seeded by global id) so no two solves match: J + 1e-3 skew noise, R and Q
    congruence-scaled by (I + 1e-3 sym noise), which keeps them SPD."""
    import numpy as np
    X, XP, h, constset, base = si_instance(d)
    xs, ys = [], []
    for gid in ids:
        x0, y0 = base[gid % len(base)]
        x = x0.copy()
        if gid >= len(base):
            rs = np.random.RandomState(1000 + gid)
            a = rs.randn(d, d) * 1e-3
            x[0] = x[0] + (a - a.T) / 2
            for k in (1, 2):
                e = np.eye(d) + 1e-3 * (lambda b: (b + b.T) / 2)(rs.randn(d, d))
                x[k] = e @ x[k] @ e.T
        xs.append(x)
        ys.append(y0)
    return np.stack(xs), np.stack(ys), (X, XP, h, constset)


def _si_oracle_window(gid: int, K: int, budget_s: float, trs: str, d: int = 5):
    """The SI oracle on bench start `gid` (si_starts), outer iterations 1..K or as many as the
    budget allows; returns (completed outer iterations, solver seconds) or None."""
    from oracle import riptrm_oracle as RO
    from oracle import si_oracle as SI
    xs, ys, (X, XP, h, constset) = si_starts(1, [gid], d)
    orc = RO.RIPTRMOracle(dict(maxiter=K, tolresid=0.0, maxtime=1e12, manviofun=SI.si_manvio,
                               **trs_options(trs)), deadline=time.time() + budget_s)
    try:
        orc.run(SI.SIVectorized(SI.SIData(X, XP, h, constset)), xs[0], ys[0])
    except RO.BudgetExceeded:
        pass
    heads = orc.outer_heads
    last = max(heads)
    _si_oracle_window.inner_durations = list(orc.inner_durations)
    return (last, heads[last]) if last > 0 and heads[last] > 0 else None


def _si_cpu_worker(argv):
    """One single-threaded SI oracle process (run by si_cpu_pool)."""
    gid, K, budget, trs, d = int(argv[0]), int(argv[1]), float(argv[2]), argv[3], int(argv[4])
    r = _si_oracle_window(gid, K, budget, trs, d)
    print(json.dumps({"outer": r[0] if r else 0, "secs": r[1] if r else 0.0,
                      "inner": _si_oracle_window.inner_durations}), flush=True)


def si_cpu_pool(K: int, budget_s: float, procs: int, trs: str, d: int = 5, inner_per_outer=None):
    """The StableIdentification analogue of cpu_baseline_pool: `procs` single-threaded oracle
    processes run concurrently, process i solving the GPU batch's start i (si_starts) over the
    same outer window 1..K; aggregate = mean complete per-process rate x procs.  When no process
    completes the window (Exact_RepMat at d >= 8), the rate is sampled per inner step
    (_inner_sampled, with the GPU window's inner iterations per outer iteration)."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--si-cpu-worker", str(i), str(K),
                            str(budget_s), trs, str(d)], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env,
                           text=True)
          for i in range(procs)]
    rates, inner = [], []
    for p in ps:
        out, _ = p.communicate(timeout=budget_s + 600)
        try:
            r = json.loads(out.strip().splitlines()[-1])
        except Exception:
            continue
        inner.extend(r.get("inner", []))
        if r["outer"] == K and r["secs"] > 0:
            rates.append(r["outer"] / r["secs"])
    if not rates:
        return _inner_sampled(inner, inner_per_outer, procs, procs, None, trs, None, budget_s,
                              what=(f"oracle/si_oracle.py SIVectorized, d={d}, {procs} single-threaded processes, process i "
                                    f"solving the GPU batch's start i"))
    return {"value": sum(rates) / len(rates) * procs, "unit": "outer iterations/s", "cores": int(procs),
            "kind": "port",
            "sample": (f"oracle/si_oracle.py SIVectorized, {procs} single-threaded processes, process i solving the GPU "
                       f"batch's start i (fixture starts a.. in order) over outer iterations 1..{K} within a "
                       f"{budget_s:.0f} s budget; {len(rates)}/{procs} completed, aggregate = mean complete per-process "
                       f"rate x {procs}, evaluation time excluded as RIPTRM.py:932-941")}


def tri_roofline(m: int, dev, B: int = 1, reps: int = 5):
    """The Exact_RepMat HBM service's dominant kernel from order 150 on, the cooperative tridiagonalisation
    (csrc/riptrm_tri.h k_tridiag_dist, ~m / 16 workgroups), timed live with HIP events on torch's current
    stream (the library runs on it) around riptrm_sym_tridiag on B frame-like matrices (O(1) symmetric
    part plus diagonal barrier terms up to 1e6; B = the line's batch, several matrices per cooperative
    launch): the reduction alone, as the service runs it per pass of subproblems and of trial points.
    Bound: latency.  Each matrix's m - 1 columns are one all-to-all exchange each
    (every workgroup publishes its rows' p = tau A v and polls every other's), a chain no bandwidth can
    shorten; the floor is m - 1 hand-offs at the measured single hop (MI355X_MICROARCH.md,
    handoff-1to1: ~1.0 us on an idle chip).  Its flops (4/3 m^3) at the FP64 vector peak are reported
    beside it (flops_frac)."""
    import numpy as np
    import torch
    import trs
    rs = np.random.RandomState(m)
    mats = []
    for _ in range(B):
        D = rs.randn(m, m) / np.sqrt(m)
        mats.append(D + D.T + np.diag(np.where(rs.rand(m) < 0.3, 10.0 ** rs.uniform(2, 6, m), 0.0)))
    A = torch.tensor(np.stack(mats), dtype=torch.float64, device=dev)
    for _ in range(2):
        _, _, info = trs.sym_tridiag(A)
    assert int(info.abs().sum()) == 0
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        trs.sym_tridiag(A)
        e1.record()
        torch.cuda.synchronize(dev)
        ts.append(e0.elapsed_time(e1) / 1e3)
    t = sorted(ts)[len(ts) // 2]
    hop = 1.0e-6
    ach = B * (m - 1) / t
    G = (m + 15) // 16 if m > 512 else (m + 31) // 32 if m > 256 else (m + 63) // 64
    return {"bound": "latency", "achieved": ach, "peak": B / hop, "unit": "columns/s", "frac": ach / (B / hop),
            "traffic": None, "avg_launch_us": t * 1e6,
            "kernel": (f"riptrm_tri::k_tridiag_dist on {G} cooperative workgroups per matrix: the tridiagonal reduction "
                       f"of {B} order-{m} subproblem matrices through riptrm_sym_tridiag"),
            "flops_frac": (B * 4.0 / 3.0 * m ** 3 / t) / 81.7e12,
            "why": ("latency-bound: one all-to-all exchange per tridiagonalisation column; floor = m - 1 hand-offs "
                    "at ~1.0 us (MI355X_MICROARCH.md handoff-1to1, idle chip)")}


LDS_BYTES_PER_CLK = 256       # MI355X_MICROARCH.md: LDS 64 dwords wide per clock per CU
CLOCK_HZ = 2.4e9              # max engine clock


def eig_roofline(m: int, B: int, dev, reps: int = 5):
    """The Exact_RepMat HBM service's dominant kernel, the hand-written eigensolver (csrc/riptrm_eig.h,
    manifold.dim 97..149), timed live with HIP events on the library's stream: B matrices of order m
    shaped like the frame matrices (O(1) symmetric part plus diagonal barrier terms up to 1e6),
    compact eigenpairs as the service takes them.  Bound: LDS of the CUs it occupies (one workgroup
    per matrix holds it in LDS for the tridiagonalisation, its dominant phase); algorithmic bytes =
    that phase's LDS traffic, per column with r trailing rows r^2 doubles read by the symmetric
    mat-vec and r (r + 1) read + written by the rank-2 update."""
    import ctypes

    import numpy as np
    import torch
    import trs
    rs = np.random.RandomState(m)
    mats = []
    for _ in range(B):
        D = rs.randn(m, m) / np.sqrt(m)
        D = D + D.T + np.diag(np.where(rs.rand(m) < 0.3, 10.0 ** rs.uniform(2, 6, m), 0.0))
        mats.append(D)
    A = torch.tensor(np.stack(mats), dtype=torch.float64, device=dev)
    V = A.clone()
    w = torch.empty((B, m), dtype=torch.float64, device=dev)
    info = torch.empty(B, dtype=torch.int32, device=dev)
    ctx = trs._context(A.device)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    call = lambda: ctx.check(ctx.lib.riptrm_sym_eig(ctx.h, m, B, p(V), m, m * m, p(w), m, p(info), 2), "riptrm_sym_eig")  # noqa: E731
    for _ in range(2):
        V.copy_(A)
        call()
    ts = []
    for _ in range(reps):
        V.copy_(A)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call()
        e1.record()
        torch.cuda.synchronize(dev)
        ts.append(e0.elapsed_time(e1) / 1e3)
    t = sorted(ts)[len(ts) // 2]
    per = 8.0 * sum(2 * r * r + r for r in range(1, m))
    cus = min(B, 256)
    ach = B * per / t / 1e9
    peak = cus * LDS_BYTES_PER_CLK * CLOCK_HZ / 1e9
    return {"bound": "lds", "achieved": ach, "peak": peak, "unit": "GB/s", "frac": ach / peak, "traffic": None,
            "kernel": (f"riptrm_eig (k_eig_lds: tridiagonalisation one 1024-thread workgroup per matrix, eigenvalues / "
                       f"twisted vectors over ~50 indices per workgroup, MFMA Gram-Schmidt), {B} matrices of order {m}, "
                       "compact eigenpairs"),
            "bytes_definition": ("tridiagonalisation's LDS traffic per matrix, sum over columns of (2 r^2 + r) doubles "
                                 f"(symmetric mat-vec + rank-2 update), {per / 1e6:.1f} MB at m={m}; peak = LDS of the "
                                 f"{cus} CUs one workgroup per matrix occupies ({LDS_BYTES_PER_CLK} B/clock at 2.4 GHz)"),
            "avg_launch_us": t * 1e6, "bytes_per_launch": B * per,
            "why": ("no HBM / MFMA roof: the matrices live in LDS; the tridiagonalisation's dependent column steps "
                    "(three workgroup barriers each) keep it latency-bound")}


def si_roofline(args, d, hvps, kern_s, sec, passes):
    """The SI line's roof.  k_si runs each instance's whole solve on one wave: a dependent chain of
    d x d products, LDS round trips and wave reductions, no HBM stream and no matrix-core work worth
    pricing, so its bound is the issue rate of one wave (one instruction per cycle).  achieved =
    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES from a committed rocprofv3 PMC pass of this d
    (scripts/si_pmc_summary.py -> --si-pmc-json), the fraction of each wave's lifetime in which it
    issues; peak 1.  The latency floor per instance-step is stated beside it: device time per HVP per
    instance, from the instrumented launch's section clocks."""
    issue = None
    if os.path.exists(args.si_pmc_json):
        try:
            pm = json.load(open(args.si_pmc_json))
            if pm.get("d") == d and pm.get("issue_frac") is not None:
                issue = pm
        except Exception as e:  # pragma: no cover
            log(f"si pmc json unreadable: {e}")
    us_hvp = sec["hvp"] / max(1.0, passes) * 1e6
    return {"bound": "issue", "achieved": issue["issue_frac"] if issue else None, "peak": 1.0,
            "unit": "instructions issued per wave-cycle (one wave per instance)",
            "frac": issue["issue_frac"] if issue else None, "traffic": None,
            "pmc": ({k: issue[k] for k in ("wait_frac", "wait_inst_frac", "valu_insts_per_wave_cycle", "source")}
                    if issue else None),
            "latency_floor_us_per_hvp_per_instance": us_hvp,
            "hvps_per_s_M": hvps / kern_s / 1e6,
            "kernel": "k_si (one 64-lane workgroup per instance, whole solve per launch)", "kernel_ms": kern_s * 1e3,
            "why": "latency-bound single-wave chains; HBM traffic is the problem data only (no roof applies)"}


def bench_si(args, world, rank, dev, dist):
    """StableIdentification throughput: one HIP launch runs every instance's whole solve
    (maxiter = warmup + steps); the timed launch is bracketed by barriers + syncs."""
    import numpy as np
    import torch
    import si
    B, W, K = args.batch, args.warmup, args.steps
    ids = [rank + world * i for i in range(B)]
    d = args.si_dim
    xs, ys, (X, XP, h, constset) = si_starts(B, ids, d)
    cons = si.expand_constset(constset)
    eng = si.SIBatch(d, X.shape[1], cons.shape[0], B, log_capacity=16)
    eng.load(X, XP, h, cons)
    opt = {"manviofun": si.si_manviofun, "tolresid": 0.0, "maxtime": math.inf,
           "maxiter": max(1, W), "save_inner_iteration": True, **trs_options(args.trs)}
    eng.solve(xs, ys, opt)          # warmup launch (W outer iterations), untimed
    opt["maxiter"] = K
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    eng.begin(xs, ys, opt)
    e1.record()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if dist.is_initialized():
        dist.barrier()
    kern_s = e0.elapsed_time(e1) / 1e3
    st = eng.stats()
    # section breakdown from a second, instrumented launch (device clock per section)
    eng.profile_enable(True)
    eng.begin(xs, ys, opt)
    sec = eng.profile_read()
    eng.profile_enable(False)
    secfrac = {k: (v / sec["total"] if sec["total"] > 0 else None) for k, v in sec.items() if k != "total"}
    C = si.C
    tot = lambda f: float(st[:, C[f"RIPTRM_STAT_{f}"]].sum())
    counts = torch.tensor([tot("OUTER_ITERS"), tot("INNER_ITERS"), tot("TCG_ITERS"), tot("PASSES")],
                          dtype=torch.float64, device=dev)
    tmax = torch.tensor([el], dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    outer, inner, tcg, hvps = [float(v) for v in counts.tolist()]
    T = float(tmax.item())
    if rank != 0:
        return
    tdim = d * (d - 1) // 2 + d * (d + 1)   # manifold.dim of Product(Skew(d), SPD(d), SPD(d))
    cpu = None
    if args.cpu_budget > 0 and world == 1:
        ipo = inner / outer if outer > 0 else None
        one = _si_oracle_window(0, K, args.cpu_budget, args.trs, d)
        if one is None:   # not one outer iteration within the budget: sampled per inner step
            cpu = _inner_sampled(_si_oracle_window.inner_durations, ipo, 1, 1, None, args.trs, None, args.cpu_budget,
                                 what=f"oracle/si_oracle.py SIVectorized (NumPy, closed-form Lagrangian), d={d}, start 0")
        if one is not None:
            last, secs = one
            cpu = {"value": last / secs, "unit": "outer iterations/s", "cores": 1, "kind": "port",
                   "sample": f"oracle/si_oracle.py SIVectorized (NumPy, closed-form Lagrangian), d={d}, start 0, outer "
                             f"iterations 1..{last} ({secs:.1f} s, evaluation time excluded as RIPTRM.py:932-941)"}
        procs = min(args.cpu_procs, B)
        pool = None
        if procs > 0:
            log(f"SI CPU baseline, {procs} single-threaded processes ...")
            pool = si_cpu_pool(K, args.cpu_pool_budget, procs, args.trs, d, ipo)
        cpu = pick_cpu_baseline(cpu, pool)
        if cpu is not None:
            cpu.update(host_cpu_info())
            cpu.update(core_rationale(cpu))
            cpu["gpu_over_cpu"] = (outer / T) / cpu["value"]
    print(json.dumps({
        "metric": f"outer RIPTRM iterations/sec, StableIdentification d={d} (Product(Skew,SPD,SPD)), batch {B}/GPU",
        "value": outer / T, "unit": "outer iterations/s", "n_gpus": world, "steps": K, "warmup": W,
        "ms_per_step": T / K * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64",
        "data": ("reference fixture dataset/StableIdentification/1 (noisy X, 16 constraints), starts a..t cycled + perturbed"
                 if d == 5 else f"synthetic: si.synthetic_problem(d={d}, seed {1000 + d}) (the reference's dataset recipe), "
                                "20 starts cycled + perturbed"),
        "config": {"workload": f"StableIdentification d={d} N={X.shape[1]} m={cons.shape[0]}, {B} starts per GPU, "
                               f"outer iterations 1..{K}"
                               + ("" if args.trs == "tCG" else ", TRS_solver=Exact_RepMat + second-order test"),
                   "trs_solver": args.trs,
                   "global_batch": B * world, "parallelism": f"instance-sharded x{world}", "world_size": world},
        "roofline": si_roofline(args, d, hvps, kern_s, sec, tot("PASSES")),
        # the HBM TRS service's eigensolver at this manifold.dim (the line's other half: DESIGN 7b)
        **({"service_eig_roofline": eig_roofline(tdim, B, dev)} if args.trs != "tCG" and 96 < tdim < si.C["RIPTRM_TRS_TRI_MIN"] else {}),
        "cpu_baseline": cpu,
        "detail": {"inner_iterations_per_s": inner / T, "tcg_iterations_per_s": tcg / T, "hvps_per_s": hvps / T,
                   "section_fraction": secfrac, "us_per_hvp_per_instance": sec["hvp"] / max(1.0, tot("PASSES")) * 1e6,
                   # HBM TRS service (Exact_RepMat, d >= 8): subproblems whose CG was decided on their
                   # eigenpairs, and CGs skipped by the certified bound (since the context was made)
                   "trs_cg_checked_skipped": (list(eng.trs_skip_stats()) if args.trs != "tCG" else None),
                   # subproblems served from the keyed eigendecomposition cache / served (last solve)
                   "trs_cache_hits_subproblems": (list(eng.trs_cache_stats()) if args.trs != "tCG" else None)},
    }), flush=True)


if __name__ == "__main__":
    main()
