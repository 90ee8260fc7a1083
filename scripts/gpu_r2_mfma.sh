# MFMA S-pass (shared layout) tuning: tools/mfma_bench variants at n = 4000, 128 right-hand
# sides (FILTER selects variants by name), optionally one PMC pass (MFMA busy / instruction counts).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2m}
mkdir -p $O
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_bench.hip -o /tmp/mfma_bench > $O/build.log 2>&1 || { echo build failed; cat $O/build.log; exit 3; }
timeout -k 10 300 /tmp/mfma_bench 4000 128 ${FILTER:-glds} > $O/mfma_bench.jsonl 2>&1; rc=$?
cat $O/mfma_bench.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 /tmp/mfma_bench 1000 128 ${FILTER:-glds} > $O/mfma_bench_1000.jsonl 2>&1; rc=$?
cat $O/mfma_bench_1000.jsonl
[ $rc -eq 0 ] || exit $rc
if [ -n "${PMC:-}" ]; then
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o pmc -- /tmp/mfma_bench 4000 128 "$PMC" > $O/pmc_run.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -5 $O/pmc_run.log
fi
exit $rc
