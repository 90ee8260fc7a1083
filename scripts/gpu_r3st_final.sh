# Stiefel measurements on the final tree (VALU Gram tail): PMC traffic passes, bench at 256 / 2048
# points, rocprofv3 kernel stats at 256 points.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3st_final}
mkdir -p $O
export TMPDIR=/tmp
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/stamps_build.log 2>&1 || { cat $O/stamps_build.log; exit 3; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/stpmc_$c -o p -- /tmp/stamps 200 50 256 > $O/stpmc_$c.log 2>&1 || exit $?
  echo "stiefel pmc $c ok"
done
python scripts/stiefel_pmc_summary.py $(find $O/stpmc_FETCH_SIZE -name "*counter_collection.csv" | head -1) $(find $O/stpmc_WRITE_SIZE -name "*counter_collection.csv" | head -1) $O/r3_stiefel_pmc.json || exit 4
timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch 256 > $O/bench_stiefel_b256.json 2> $O/st256.err || exit $?
timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch 2048 --cpu-budget 20 > $O/bench_stiefel_b2048.json 2> $O/st2048.err || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python bench.py --problem stiefel --dim 200 --batch 256 --cpu-budget 0 > $O/bench_stiefel_rocprof.json 2> $O/st_rocprof.log || exit $?
echo "stiefel rocprof ok"
exit 0
