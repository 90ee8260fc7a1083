# Stiefel kernels: MFMA busy and clock counters (one rocprofv3 --pmc pass over tools/stiefel_stamps)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3pmc
mkdir -p $O
export TMPDIR=/tmp
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/build.log 2>&1 || { cat $O/build.log; exit 3; }
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o p -- /tmp/stamps 200 50 256 > $O/pmc.log 2>&1 || exit $?
echo pmc ok
