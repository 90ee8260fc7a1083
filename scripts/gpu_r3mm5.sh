# Round 3: shared-S MFMA S-pass, in1 tiles inside the in0 workgroups; 16 waves (default) vs 8
# (libriptrm_hip_w8.so, -DRIPTRM_MM_WAVES=8), same box; parity, rocprofv3 stats, MFMA PMC.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3mm5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "shared" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
PKG=riemannian-interior-point-trust-region-method_amd
for v in w16 w8 w16 w8; do
  if [ $v = w8 ]; then export RIPTRM_LIB=$GRAFT_REPO_ROOT/$PKG/libriptrm_hip_w8.so; else unset RIPTRM_LIB; fi
  timeout -k 10 300 python bench.py --layout shared --cpu-budget 0 > $O/bench_$v.json 2> $O/bench_$v.err || exit 5
  python -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('$v', round(d['value'],1), 'it/s', 'mfma', round(r['achieved'],2), 'TF frac', round(r['frac'],3), 'launch us', round(r['avg_launch_us'],1), 'state ms', round(d['detail']['state_kernel_ms'],1))"
  cat $O/bench_$v.json >> $O/ab.jsonl
done
unset RIPTRM_LIB
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python bench.py --layout shared --cpu-budget 0 > $O/bench_rocprof.json 2> $O/rocprof.log; rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o pmc -- python bench.py --layout shared --cpu-budget 0 --warmup 1 --steps 3 > $O/bench_pmc.json 2> $O/pmc.log; rc=$?
echo "pmc rc=$rc"
exit $rc
