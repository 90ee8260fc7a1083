# Round-2 retraction kernel (k_st_retr2): Stiefel GPU tests, phase stamps, Stiefel bench, then the full gate.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2r}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stiefel.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_stiefel.log 2>&1; rc=$?
echo "pytest stiefel rc=$rc"; tail -20 $O/gpu_stiefel.log
[ $rc -eq 0 ] || exit $rc
C=riemannian-interior-point-trust-region-method_amd/csrc
for fb in ${FBS:-1 2 4}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DRIPTRM_ST_FB=$fb -DRIPTRM_ST_COMBINED=${COMB:-0} -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps$fb > $O/stamps_build.log 2>&1 || { cat $O/stamps_build.log; exit 3; }
  echo "# FB=$fb COMBINED=${COMB:-0}" >> $O/stamps.jsonl
  timeout -k 10 120 /tmp/stamps$fb 200 50 256 >> $O/stamps.jsonl 2>&1; rc=$?
  [ $rc -eq 0 ] || { cat $O/stamps.jsonl; exit $rc; }
done
cat $O/stamps.jsonl
timeout -k 10 300 python bench.py --problem stiefel --dim 200 --batch 256 --steps 50 --warmup 3 > $O/bench_stiefel.json 2> $O/bench_stiefel.err; rc=$?
echo "bench rc=$rc"; cat $O/bench_stiefel.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o st -- python bench.py --problem stiefel --dim 200 --batch 256 --steps 50 --warmup 3 > $O/bench_stiefel_prof.json 2> $O/prof.err; rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
[ "${GATE:-1}" = 1 ] || exit 0
bash scripts/gpu_gate.sh
