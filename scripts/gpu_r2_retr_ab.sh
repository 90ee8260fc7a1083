# Same-box A/B of the retraction factor variants (phase stamps), after the Stiefel GPU tests.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stiefel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_stiefel.log 2>&1; rc=$?
echo "pytest stiefel rc=$rc"; tail -3 $O/gpu_stiefel.log
[ $rc -eq 0 ] || exit $rc
C=riemannian-interior-point-trust-region-method_amd/csrc
for v in "1 1" "0 2" "1 1"; do
  set -- $v
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DRIPTRM_ST_COMBINED=$1 -DRIPTRM_ST_FB=$2 -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps_$1_$2 > $O/stamps_build.log 2>&1 || { cat $O/stamps_build.log; exit 3; }
  echo "# COMBINED=$1 FB=$2" >> $O/stamps.jsonl
  timeout -k 10 120 /tmp/stamps_$1_$2 200 50 256 >> $O/stamps.jsonl 2>&1; rc=$?
  [ $rc -eq 0 ] || { cat $O/stamps.jsonl; exit $rc; }
done
cat $O/stamps.jsonl
timeout -k 10 300 python bench.py --problem stiefel --dim 200 --batch 256 --steps 50 --warmup 3 > $O/bench_stiefel.json 2> $O/bench_stiefel.err; rc=$?
echo "bench rc=$rc"; cut -c1-300 $O/bench_stiefel.json
exit $rc
