# BASELINE configs[1]: NonnegPCA n=1000 single instance — bench line + kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfg1
export TMPDIR=/tmp
O=gpurun_out/cfg1
timeout -k 10 300 python bench.py --dim 1000 --batch 1 --steps 19 --warmup 1 --cpu-budget 20 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o cfg1 -- python bench.py --dim 1000 --batch 1 --steps 19 --warmup 1 --cpu-budget 0 > $O/prof_bench.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"
head -6 $O/prof/cfg1_kernel_stats.csv
exit $rc
