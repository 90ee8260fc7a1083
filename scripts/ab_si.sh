#!/bin/bash
# Same-box A/B of the SI bench: the in-tree library against tools/bin/lib_$1.so (RIPTRM_LIB), alternated
set -o pipefail
O=gpurun_out/${OUT:-ab_si}; mkdir -p $O
alt=tools/bin/lib_$1.so
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export RIPTRM_LIB=$alt; else unset RIPTRM_LIB; fi
    timeout -k 10 300 python bench.py --problem si --batch ${SI_B:-256} --cpu-budget 0 > $O/si_${v}_$r.json 2> $O/si_${v}_$r.err || exit 1
    python -c "import json,sys; d=json.load(open('$O/si_${v}_$r.json')); print('$v', $r, d['value'])"
  done
done
