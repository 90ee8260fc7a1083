"""bench.py's own N-rank launcher (`python bench.py --gpus N` outside torchrun): N child processes,
one per rank, with the torch.distributed.run environment; a failing rank stops the others and
its exit code is returned.  CPU only: the children here are a stub script, not the bench."""
import json
import os
import sys

import bench

STUB = """
import json, os, sys
out = sys.argv[1]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys}, f)
sys.exit(int(sys.argv[2]) if os.environ["RANK"] == sys.argv[3] else 0)
"""


def _stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return str(p)


def test_launcher_sets_rank_environment(tmp_path, monkeypatch):
    monkeypatch.delenv("MASTER_PORT", raising=False)
    rc = bench.launch_ranks(4, script=_stub(tmp_path), argv=[str(tmp_path), "0", "-1"])
    assert rc == 0
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    for r, e in enumerate(envs):
        assert e["RANK"] == str(r) and e["LOCAL_RANK"] == str(r) and e["WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1"
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_launcher_propagates_failure(tmp_path):
    rc = bench.launch_ranks(2, script=_stub(tmp_path), argv=[str(tmp_path), "7", "1"])
    assert rc == 7


def test_gpus_mismatch_with_world_size_is_refused(monkeypatch, capsys):
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--cpu-budget", "0"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def _leg(v, cores, name):
    return {"value": v, "unit": "outer iterations/s", "cores": cores, "kind": "port", "sample": name}


def test_cpu_baseline_selection_names_the_other_leg():
    """the better CPU variant is the baseline, the other is kept under
    other_variant -- also when the BLAS-threaded leg wins (the pool's number was lost)."""
    threaded, pool = _leg(5.9, 16, "threaded"), _leg(4.1, 16, "pool")
    out = bench.pick_cpu_baseline(threaded, pool)
    assert out["sample"] == "threaded" and out["other_variant"]["sample"] == "pool"
    assert out["other_variant"]["value"] == 4.1
    out = bench.pick_cpu_baseline(_leg(3.0, 16, "threaded"), _leg(7.5, 16, "pool"))
    assert out["sample"] == "pool" and out["other_variant"]["sample"] == "threaded"
    out = bench.pick_cpu_baseline(None, pool)
    assert out["sample"] == "pool" and "other_variant" not in out
    out = bench.pick_cpu_baseline(threaded, None)
    assert out["sample"] == "threaded" and "other_variant" not in out
    assert bench.pick_cpu_baseline(None, None) is None
    # the inputs are not modified
    assert "other_variant" not in threaded and "other_variant" not in pool


def test_host_cpu_info():
    info = bench.host_cpu_info()
    assert info["os_cpu_count"] == os.cpu_count()
    assert info["cpu_model"]
