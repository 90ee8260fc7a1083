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
