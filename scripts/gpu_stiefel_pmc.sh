set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/stpmc
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INST_CYCLES_VMEM_RD --output-format csv -d gpurun_out/stpmc -o p1 -- python scripts/stiefel_one.py > gpurun_out/stpmc/log1.txt 2>&1; rc=$?
echo "rc=$rc"
exit $rc
