set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r4st}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stiefel.py -x -q --timeout 200 > $O/stiefel_tests.log 2>&1 || { tail -30 $O/stiefel_tests.log; exit 1; }
tail -2 $O/stiefel_tests.log
for B in 256 2048; do
  timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch $B --cpu-budget 0 > $O/st_p4_b$B.json 2> $O/st_p4_b$B.err
  RIPTRM_STIEFEL_PROJ=p3 timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch $B --cpu-budget 0 > $O/st_p3_b$B.json 2> $O/st_p3_b$B.err
  python -c "
import json
for v in ('p4','p3'):
    d=json.load(open('$O/st_%s_b$B.json' % v)); print(v, $B, 'proj us', round(d['ms_per_step']*1e3,2), 'frac', round(d['roofline']['frac'],3))"
done
for B in 256 2048; do
  RIPTRM_STIEFEL_PROJ=nt timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch $B --cpu-budget 0 > $O/st_nt_b$B.json 2> $O/st_nt_b$B.err
  python -c "
import json
d=json.load(open('$O/st_nt_b$B.json')); print('no-tail', $B, 'proj us', round(d['ms_per_step']*1e3,2), 'frac', round(d['roofline']['frac'],3))"
done
