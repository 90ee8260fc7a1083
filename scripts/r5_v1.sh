# eigensolver stamps, then the Exact tests and the two Exact benches
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5u}
mkdir -p $O
export TMPDIR=/tmp
for m in 100 199; do
  RIPTRM_EIG_STAMPS=1 timeout -k 10 120 python scripts/eig_stamps.py $m 64 >> $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
done
grep "compact:" $O/stamps.txt
grep "eig stamps" $O/stamps.txt | awk 'NR==5 || NR==14'
OUT=${OUT:-r5u} bash scripts/r5_p4.sh
