set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5k}
mkdir -p $O
export TMPDIR=/tmp
for m in 100 199; do
  RIPTRM_EIG_STAMPS=1 timeout -k 10 120 python scripts/eig_stamps.py $m 64 >> $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
done
cat $O/stamps.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "sym_eig or above_lds or hard_case" tests/test_gpu_trs.py > $O/trs.log 2>&1 || { tail -30 $O/trs.log; exit 1; }
tail -1 $O/trs.log
