export TMPDIR=/tmp
for k in 1 2 3; do
for v in 0 1; do
  echo "== NO_TRIPLES=$v"
  EDSBWT_NO_TRIPLES=$v timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step']['deep'])" || exit 1
done; done
