# Round-2 profiles: rocprofv3 kernel stats of the configs[1] bench (persistent mode) and of the
# headline bench, each under its own limit.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2p}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg1 -o cfg1 -- python bench.py --dim 1000 --batch 1 --cpu-budget 0 > $O/cfg1_bench.json 2> $O/cfg1.log; rc=$?
echo "cfg1 rocprof rc=$rc"; head -c 300 $O/cfg1_bench.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o head -- python bench.py --cpu-budget 0 --warmup 5 --steps 20 > $O/head_bench.json 2> $O/head.log; rc=$?
echo "headline rocprof rc=$rc"; head -c 300 $O/head_bench.json; echo
exit $rc
