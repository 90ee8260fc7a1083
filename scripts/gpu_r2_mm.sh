# Shared-layout (multi-start) MFMA S-pass: parity tests, the bench line under rocprofv3 kernel
# stats, then one PMC pass (MFMA busy cycles) over a short bench run.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2mm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "shared" > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --layout shared --cpu-budget 0 > $O/bench.json 2> $O/bench.log; rc=$?
head -c 1500 $O/bench.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python bench.py --layout shared --cpu-budget 0 > $O/bench_rocprof.json 2> $O/rocprof.log; rc=$?
echo "rocprof rc=$rc"; head -c 400 $O/bench_rocprof.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o pmc -- python bench.py --layout shared --cpu-budget 0 --warmup 1 --steps 3 > $O/bench_pmc.json 2> $O/pmc.log; rc=$?
echo "pmc rc=$rc"
exit $rc
