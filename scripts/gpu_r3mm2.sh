# Round 3: fused in0+in1 MFMA tile for the shared layout: parity, A/B (RIPTRM_MM_FUSE), rocprofv3
# kernel stats and one PMC pass (MFMA busy) of the fused build
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3mm2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "shared" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
for f in 1 0 1 0; do
  RIPTRM_MM_FUSE=$f timeout -k 10 300 python bench.py --layout shared --cpu-budget 0 > $O/bench_f$f.json 2> $O/bench_f$f.err || exit 5
  python -c "import json; d=json.load(open('$O/bench_f$f.json')); r=d['roofline']; print('fuse=$f', round(d['value'],1), 'it/s', 'mfma', round(r['achieved'],2), 'TF frac', round(r['frac'],3), 'launch us', round(r['avg_launch_us'],1), 'state ms', round(d['detail']['state_kernel_ms'],1))"
  cat $O/bench_f$f.json >> $O/ab.jsonl
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python bench.py --layout shared --cpu-budget 0 > $O/bench_rocprof.json 2> $O/rocprof.log; rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o pmc -- python bench.py --layout shared --cpu-budget 0 --warmup 1 --steps 3 > $O/bench_pmc.json 2> $O/pmc.log; rc=$?
echo "pmc rc=$rc"
exit $rc
