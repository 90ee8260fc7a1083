# Round 3: k_st_proj3 with 16 waves (default) vs 8 (RIPTRM_STIEFEL_PROJ=w8): Stiefel tests, phase
# stamps of both, bench A/B on one box.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3st}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_stiefel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/st.log 2>&1; rc=$?
echo "stiefel tests rc=$rc"; tail -2 $O/st.log
[ $rc -eq 0 ] || exit $rc
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/build.log 2>&1 || { cat $O/build.log; exit 3; }
timeout -k 10 60 /tmp/stamps 200 50 256 > $O/stamps.jsonl 2>&1 || exit $?
cat $O/stamps.jsonl
for v in w16 w8 w16 w8; do
  if [ $v = w8 ]; then export RIPTRM_STIEFEL_PROJ=w8; else unset RIPTRM_STIEFEL_PROJ; fi
  timeout -k 10 120 python bench.py --problem stiefel --dim 200 --batch 256 --cpu-budget 0 > $O/b_$v.json 2> $O/b_$v.err || exit $?
  python -c "import json; d=json.load(open('$O/b_$v.json')); print('$v proj_us', round(d['ms_per_step']*1e3,2), 'retr_us', round(d['detail']['retraction_ms']*1e3,2))"
  cat $O/b_$v.json >> $O/ab.jsonl
done
