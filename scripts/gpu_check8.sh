set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
for g in 1 2; do
  timeout -k 10 300 python bench.py --layout shared --cpu-budget 0 --stream-groups $g > gpurun_out/bench_shared_g$g.json 2> gpurun_out/bench_shared_g$g.err; rc=$?
  echo "bench shared groups=$g rc=$rc"; cat gpurun_out/bench_shared_g$g.json
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --layout shared --cpu-budget 0 --dim 1000 --batch 64 > gpurun_out/bench_shared_n1000.json 2> gpurun_out/bench_shared_n1000.err; rc=$?
echo "bench shared n1000 rc=$rc"; cat gpurun_out/bench_shared_n1000.json
exit $rc
