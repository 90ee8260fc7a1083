#!/bin/bash
# Same-box A/B of a knob on the SI Exact_RepMat HBM path (d = 8, 64 starts): default vs $VAR=$ALT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-ab_si_exact}; mkdir -p $O
for r in 1 2; do
  for v in default alt; do
    if [ $v = alt ]; then export ${VAR}=${ALT}; else unset ${VAR}; fi
    timeout -k 10 300 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 > $O/si8_${v}_$r.json 2> $O/si8_${v}_$r.err || { tail $O/si8_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/si8_${v}_$r.json')); print('si8 $v run $r', round(d['value'], 2), round(d['ms_per_step'], 1))"
  done
done
