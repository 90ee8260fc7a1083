#!/bin/bash
# StableIdentification Exact_RepMat on the HBM path (d >= 8): the bench line at d = 8 (64 starts).
# (d = 16 with 16 starts did not finish two outer iterations within 170 s: each inner iteration
# there builds 392 x 392 matrices and runs rocSOLVER on them twice.)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-si_exact}; mkdir -p $O
timeout -k 10 300 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 > $O/si8_exact.json 2> $O/si8.err || { tail $O/si8.err; exit 1; }
for f in si8_exact; do
  python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'])"
done
