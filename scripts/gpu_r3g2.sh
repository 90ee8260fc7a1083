# Round 3 final gate, part 2: default bench (headline, with its CPU baselines), its rocprofv3
# kernel stats; configs[1] bench + stats; SI bench with the 16-process CPU pool; Stiefel stats + PMC.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3g2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python bench.py > $O/bench_headline.json 2> $O/bench_headline.err || exit $?
python -c "import json; d=json.load(open('$O/bench_headline.json')); print('headline', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o head -- python bench.py --cpu-budget 0 > $O/bench_headline_rocprof.json 2> $O/head_rocprof.log || exit $?
echo "headline rocprof ok"
timeout -k 10 240 python bench.py --dim 1000 --batch 1 > $O/bench_cfg1.json 2> $O/bench_cfg1.err || exit $?
python -c "import json; d=json.load(open('$O/bench_cfg1.json')); print('cfg1', d['value'], d['roofline'].get('us_per_pass'))"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg1 -o cfg1 -- python bench.py --dim 1000 --batch 1 --cpu-budget 0 > $O/bench_cfg1_rocprof.json 2> $O/cfg1_rocprof.log || exit $?
echo "cfg1 rocprof ok"
timeout -k 10 300 python bench.py --problem si --batch 256 > $O/bench_si_b256.json 2> $O/bench_si.err || exit $?
python -c "import json; d=json.load(open('$O/bench_si_b256.json')); print('si', d['value'], d['cpu_baseline'])"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python bench.py --problem stiefel --dim 200 --batch 256 --cpu-budget 0 > $O/bench_stiefel_rocprof.json 2> $O/st_rocprof.log || exit $?
echo "stiefel rocprof ok"
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/stamps_build.log 2>&1 || { cat $O/stamps_build.log; exit 3; }
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F64"; do
  t=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/stpmc_$t -o p -- /tmp/stamps 200 50 256 > $O/stpmc_$t.log 2>&1 || exit $?
  echo "stiefel pmc $t ok"
done
exit 0
