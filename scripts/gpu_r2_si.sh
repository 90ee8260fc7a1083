# Round-2 StableIdentification bench lines (tCG and Exact_RepMat, 256 starts) with their CPU baselines.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2si
mkdir -p $O
export TMPDIR=/tmp
for trs in tCG Exact_RepMat; do
  timeout -k 10 400 python bench.py --problem si --batch 256 --steps 20 --warmup 1 --cpu-budget 20 --trs $trs > $O/bench_si_$trs.json 2> $O/bench_si_$trs.err; rc=$?
  echo "bench si $trs rc=$rc"; cut -c1-600 $O/bench_si_$trs.json; tail -2 $O/bench_si_$trs.err
  [ $rc -eq 0 ] || exit $rc
done
