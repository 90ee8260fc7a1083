# Same-box A/B: super-tile S-pass (kind 2) vs the variant with v's row entries hoisted (kind 3).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "spass or super" --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 2 3 2 3; do
  timeout -k 10 300 python bench.py --cpu-budget 0 --spass-kind $k > $O/k$k.json 2> $O/k$k.err; rc=$?
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$O/k$k.json'));print('kind $k', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
