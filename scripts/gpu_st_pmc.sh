# Stiefel kernels: instruction-issue and instruction-cache PMC passes (each its own run).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-stpmc}
mkdir -p $O
export TMPDIR=/tmp
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/build.log 2>&1 || { cat $O/build.log; exit 3; }
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o p1 -- /tmp/stamps 200 50 256 > $O/p1.log 2>&1; rc=$?
echo "p1 rc=$rc"; tail -2 $O/p1.log
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_TC_INST_REQ GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- /tmp/stamps 200 50 256 > $O/p2.log 2>&1; rc=$?
echo "p2 rc=$rc"; tail -2 $O/p2.log
exit $rc
