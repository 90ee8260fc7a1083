#!/bin/bash
# Stiefel retraction round-3 variants: phase stamps per build (tools/bin/st_stamps_*), the GPU tests, the bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stiefel.py > gpurun_out/st_tests.log 2>&1 || { tail -30 gpurun_out/st_tests.log; exit 1; }
tail -2 gpurun_out/st_tests.log
for v in ${VARIANTS:-f2}; do
  timeout -k 10 60 tools/bin/st_stamps_$v 200 50 256 > gpurun_out/st_$v.jsonl 2>&1 || exit 1
  timeout -k 10 60 tools/bin/st_stamps_$v 200 50 2048 >> gpurun_out/st_$v.jsonl 2>&1 || exit 1
  echo "== $v"; grep retr2 gpurun_out/st_$v.jsonl
done
timeout -k 10 120 python bench.py --problem stiefel --dim 200 --batch 256 --cpu-budget 0 > gpurun_out/st_b256.json 2> gpurun_out/st_b256.err || exit 1
timeout -k 10 120 python bench.py --problem stiefel --dim 200 --batch 2048 --cpu-budget 0 > gpurun_out/st_b2048.json 2> gpurun_out/st_b2048.err || exit 1
python -c "
import json
for f in ('gpurun_out/st_b256.json','gpurun_out/st_b2048.json'):
    d=json.load(open(f)); print(f, 'proj_us', round(d['ms_per_step']*1e3,2), 'retr_us', round(d['detail']['retraction_ms']*1e3,2))"
