set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 400 python -u scripts/debug_flip.py 73 20 20 > $O/debug_flip_73.jsonl 2> $O/debug_flip.err || { tail $O/debug_flip.err; exit 1; }
tail -12 $O/debug_flip_73.jsonl | cut -c1-600
for e in d j dj; do
  RIPTRM_BIG_EIG=$e timeout -k 10 300 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 > $O/exact_eig_$e.json 2> $O/exact_eig_$e.err || { tail $O/exact_eig_$e.err; exit 1; }
  python -c "import json; d=json.load(open('$O/exact_eig_$e.json')); print('$e', d['value'], d['ms_per_step'])"
done
for cfg in "--batch 128" "--batch 128 --stream-groups 2" "--batch 256" "--batch 256 --stream-groups 2"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 python bench.py --layout shared --cpu-budget 0 $cfg > $O/shared_$tag.json 2> $O/shared_$tag.err || { tail $O/shared_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/shared_$tag.json')); print('shared $cfg', round(d['value'],1), 'frac', d['roofline']['frac'], 'state_ms', d['detail']['state_kernel_ms'], 'timing', d['detail']['kernel_timing'][:30])"
done
