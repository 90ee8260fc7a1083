# Shared-layout bench + kernel stats only (A/B of S-pass parameters).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2mmq}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python bench.py --layout shared --cpu-budget 0 > $O/bench_rocprof.json 2> $O/rocprof.log; rc=$?
echo "rocprof rc=$rc"; head -c 300 $O/bench_rocprof.json; echo
exit $rc
