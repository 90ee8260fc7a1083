set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/stpmc2
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/stpmc2 -o p1 -- python bench.py --dim 1000 --batch 1 --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/stpmc2/log1.txt 2>&1; rc=$?
echo "rc=$rc"
exit $rc
