#!/bin/bash
# Stiefel round-3 A/B through RIPTRM_LIB (tools/build_stiefel_variant.sh): tests on the default build, then
# bench.py --problem stiefel per library at (200, 50) x 256 (twice) and x 2048
set -o pipefail
mkdir -p gpurun_out/r3g
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stiefel.py > gpurun_out/r3g/tests.log 2>&1 || { tail -30 gpurun_out/r3g/tests.log; exit 1; }
tail -1 gpurun_out/r3g/tests.log
for v in ${VARIANTS:-default g2 g4u r2}; do
  if [ $v = default ]; then unset RIPTRM_LIB; else export RIPTRM_LIB=$PWD/tools/bin/lib_$v.so; fi
  for B in 256 256 2048; do
    timeout -k 10 120 python bench.py --problem stiefel --dim 200 --batch $B --cpu-budget 0 > gpurun_out/r3g/b_${v}_$B.json 2> gpurun_out/r3g/b_${v}_$B.err || { tail gpurun_out/r3g/b_${v}_$B.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/r3g/b_${v}_$B.json'))
print('$v', $B, 'proj_us', round(d['ms_per_step']*1e3,2), 'retr_us', round(d['detail']['retraction_ms']*1e3,2))"
  done
done
