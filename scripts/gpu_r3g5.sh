# Round 3 final gate (after the Stiefel work): smoke, full GPU suite, headline bench + rocprofv3,
# configs[1] bench, SI bench, Stiefel bench + rocprofv3, Stiefel PMC traffic passes
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3g5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 420 python bench.py > $O/bench_headline.json 2> $O/bench_headline.err || exit $?
python -c "import json; d=json.load(open('$O/bench_headline.json')); print('headline', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 240 python bench.py --dim 1000 --batch 1 > $O/bench_cfg1.json 2> $O/bench_cfg1.err || exit $?
python -c "import json; d=json.load(open('$O/bench_cfg1.json')); print('cfg1', d['value'])"
timeout -k 10 300 python bench.py --problem si --batch 256 > $O/bench_si_b256.json 2> $O/bench_si.err || exit $?
python -c "import json; d=json.load(open('$O/bench_si_b256.json')); print('si', d['value'])"
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/stamps_build.log 2>&1 || { cat $O/stamps_build.log; exit 3; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/stpmc_$c -o p -- /tmp/stamps 200 50 256 > $O/stpmc_$c.log 2>&1 || exit $?
  echo "stiefel pmc $c ok"
done
python scripts/stiefel_pmc_summary.py $(find $O/stpmc_FETCH_SIZE -name "*counter_collection.csv" | head -1) $(find $O/stpmc_WRITE_SIZE -name "*counter_collection.csv" | head -1) $O/r3_stiefel_pmc.json && cp $O/r3_stiefel_pmc.json profiles/r3_stiefel_pmc.json || exit 4
timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch 256 > $O/bench_stiefel_b256.json 2> $O/st256.err || exit $?
timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch 2048 --cpu-budget 20 > $O/bench_stiefel_b2048.json 2> $O/st2048.err || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python bench.py --problem stiefel --dim 200 --batch 256 --cpu-budget 0 > $O/bench_stiefel_rocprof.json 2> $O/st_rocprof.log || exit $?
echo "stiefel rocprof ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o head -- python bench.py --cpu-budget 0 > $O/bench_headline_rocprof.json 2> $O/head_rocprof.log || exit $?
echo "headline rocprof ok"
exit 0
