#!/bin/bash
# StableIdentification Exact_RepMat on the HBM path (d >= 8): bench lines at d = 8 (64 starts) and d = 16 (16 starts)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-si_exact}; mkdir -p $O
timeout -k 10 300 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 > $O/si8_exact.json 2> $O/si8.err || { tail $O/si8.err; exit 1; }
timeout -k 10 170 python bench.py --problem si --si-dim 16 --trs Exact_RepMat --batch 16 --steps 1 --warmup 1 --cpu-budget 0 > $O/si16_exact.json 2> $O/si16.err || { tail $O/si16.err; exit 1; }
for f in si8_exact si16_exact; do
  python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'])"
done
