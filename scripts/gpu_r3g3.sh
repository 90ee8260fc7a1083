# Round 3 final gate, part 3: SI bench with the 16-process CPU pool; Stiefel stats + PMC
# (part 2 stopped at a rocprofv3 crash in process exit after the configs[1] stats were written).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3g3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --problem si --batch 256 > $O/bench_si_b256.json 2> $O/bench_si.err || exit $?
python -c "import json; d=json.load(open('$O/bench_si_b256.json')); print('si', d['value'], d['cpu_baseline'])"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python bench.py --problem stiefel --dim 200 --batch 256 --cpu-budget 0 > $O/bench_stiefel_rocprof.json 2> $O/st_rocprof.log || exit $?
echo "stiefel rocprof ok"
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/stamps_build.log 2>&1 || { cat $O/stamps_build.log; exit 3; }
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F64"; do
  t=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/stpmc_$t -o p -- /tmp/stamps 200 50 256 > $O/stpmc_$t.log 2>&1 || exit $?
  echo "stiefel pmc $t ok"
done
exit 0
