set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/exact -o exact -- python bench.py --trs Exact_RepMat \
  --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 > $O/bench_exact_rocprof.json 2> $O/exact_rocprof.log || { tail $O/exact_rocprof.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
f=$(find $O/exact -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-8
