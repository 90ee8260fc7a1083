#!/bin/bash
# Same-box A/B of a Stiefel knob: bench.py --problem stiefel alternating the default and $VAR=$ALT.
#   OUT=r4p5 VAR=RIPTRM_STIEFEL_PROJ ALT=p3 B="256 2048" bash scripts/ab_stiefel.sh
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-ab_stiefel}; mkdir -p $O
for b in ${B:-256}; do
  for r in 1 2; do
    for v in default alt; do
      if [ $v = alt ]; then export ${VAR}=${ALT}; else unset ${VAR}; fi
      timeout -k 10 300 python bench.py --problem stiefel --dim ${DIM:-200} --batch $b --cpu-budget 0 > $O/st_${b}_${v}_$r.json 2> $O/st_${b}_${v}_$r.err || { tail $O/st_${b}_${v}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/st_${b}_${v}_$r.json')); dd=d['detail']; print('B=$b $v run $r proj_us', round(d['ms_per_step'] * 1e3, 2), 'frac', d['roofline']['frac'], 'kernel', d['roofline'].get('kernel'), 'retr_us', round(dd['retraction_ms'] * 1e3, 2))"
    done
  done
done
