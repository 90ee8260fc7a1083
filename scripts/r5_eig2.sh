set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5l}
mkdir -p $O
export TMPDIR=/tmp
for m in 100 199; do
  RIPTRM_EIG_STAMPS=1 timeout -k 10 120 python scripts/eig_stamps.py $m 64 >> $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
done
grep -v "^\[eig" $O/stamps.txt
OUT=${OUT:-r5l} bash scripts/r5_g3.sh
