# Round 3: k_st_retr2 with the single-wave factor (default build, RIPTRM_ST_FACTOR=1) vs the 8-wave
# exchange (stamps tool built with -DRIPTRM_ST_FACTOR=0): Stiefel tests, phase stamps, bench.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3st2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_stiefel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/st.log 2>&1; rc=$?
echo "stiefel tests rc=$rc"; tail -3 $O/st.log
[ $rc -eq 0 ] || exit $rc
C=riemannian-interior-point-trust-region-method_amd/csrc
for f in 1 0; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DRIPTRM_ST_FACTOR=$f -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps$f > $O/build$f.log 2>&1 || { cat $O/build$f.log; exit 3; }
  timeout -k 10 60 /tmp/stamps$f 200 50 256 > $O/stamps_f$f.jsonl 2>&1 || exit $?
  echo "factor=$f"; grep retr2 $O/stamps_f$f.jsonl
done
timeout -k 10 120 python bench.py --problem stiefel --dim 200 --batch 256 --cpu-budget 0 > $O/b.json 2> $O/b.err || exit $?
python -c "import json; d=json.load(open('$O/b.json')); print('proj_us', round(d['ms_per_step']*1e3,2), 'retr_us', round(d['detail']['retraction_ms']*1e3,2))"
