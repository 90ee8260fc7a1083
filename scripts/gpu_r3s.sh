# Round 3 Stiefel iteration: GPU tests, phase stamps (200,50)x256, bench at B = 256 and 2048
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stiefel.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
echo "pytest stiefel rc=$rc"; grep -E "passed|failed|FAILED" $O/t.log | tail -5
[ $rc -eq 0 ] || exit $rc
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/stamps_build.log 2>&1 || { cat $O/stamps_build.log; exit 3; }
timeout -k 10 120 /tmp/stamps 200 50 256 > $O/stamps.jsonl 2>&1 || { cat $O/stamps.jsonl; exit 4; }
cat $O/stamps.jsonl
for B in 256 2048; do
  timeout -k 10 300 python bench.py --problem stiefel --dim 200 --batch $B --steps 50 --warmup 3 > $O/bench_b$B.json 2> $O/bench_b$B.err || exit 5
  python -c "import json; d=json.load(open('$O/bench_b$B.json')); print('B=$B proj us', d['ms_per_step']*1e3, 'frac', d['roofline']['frac'], 'retr us', d['detail']['retraction_ms']*1e3, 'frac', d['detail']['retraction_roofline']['frac'])"
done
