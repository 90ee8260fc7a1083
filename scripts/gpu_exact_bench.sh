# Exact_RepMat benches: StableIdentification fixture (d=5, dim 40) and NonnegPCA n=97 / n=50.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/exact
export TMPDIR=/tmp
O=gpurun_out/exact
timeout -k 10 300 python -u bench.py --problem si --trs Exact_RepMat --batch 256 --warmup 1 --steps 6 --cpu-budget 15 > $O/si.json 2> $O/si.err; rc=$?; echo "si rc=$rc"; cat $O/si.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --trs Exact_RepMat --dim 97 --batch 256 --warmup 1 --steps 10 --cpu-budget 15 > $O/np97.json 2> $O/np97.err; rc=$?; echo "np97 rc=$rc"; cat $O/np97.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --trs Exact_RepMat --dim 50 --batch 1 --warmup 1 --steps 10 --cpu-budget 15 > $O/np50.json 2> $O/np50.err; rc=$?; echo "np50 rc=$rc"; cat $O/np50.json
exit $rc
