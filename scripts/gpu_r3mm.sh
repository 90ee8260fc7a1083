# Round 3: shared-S MFMA S-pass, MM_KZ = 4 (default build) vs 8 (libriptrm_hip_kz8.so), same box
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3mm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_stiefel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/st.log 2>&1; rc=$?
echo "stiefel rc=$rc"; tail -2 $O/st.log
[ $rc -eq 0 ] || exit $rc
PKG=riemannian-interior-point-trust-region-method_amd
for v in kz4 kz8 kz4 kz8; do
  if [ $v = kz8 ]; then export RIPTRM_LIB=$GRAFT_REPO_ROOT/$PKG/libriptrm_hip_kz8.so; else unset RIPTRM_LIB; fi
  timeout -k 10 300 python bench.py --layout shared --cpu-budget 0 > $O/bench_$v.json 2> $O/bench_$v.err || exit 5
  python -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('$v', round(d['value'],1), 'it/s', 'mfma', round(r['achieved'],2), 'TF frac', round(r['frac'],3), 'launch us', round(r['avg_launch_us'],1), 'state ms', round(d['detail']['state_kernel_ms'],1))"
  cat $O/bench_$v.json >> $O/ab.jsonl
done
