set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 400 python -u scripts/debug_flip.py 73 20 20 > $O/debug_flip_73.jsonl 2> $O/debug_flip.err || { tail $O/debug_flip.err; exit 1; }
tail -12 $O/debug_flip_73.jsonl | cut -c1-600
for e in d j dj; do
  RIPTRM_BIG_EIG=$e timeout -k 10 300 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 > $O/exact_eig_$e.json 2> $O/exact_eig_$e.err || { tail $O/exact_eig_$e.err; exit 1; }
  python -c "import json; d=json.load(open('$O/exact_eig_$e.json')); print('$e', d['value'], d['ms_per_step'])"
done
