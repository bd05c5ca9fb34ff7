#!/bin/bash
# A/B of engine tuning knobs on C3 (one bench line per setting; tuning aid)
export TMPDIR=/tmp
run() { echo "== $*"; env "$@" timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); k=d['kernel_ms_per_step']; print(d['value'], d['ms_per_step'], 'deep', k['deep'], 'step', k['step'], 'link_sort', k['link_sort'], 'ovf', d['engine']['deep_overflow'])"; }
for spec in "$@"; do run $spec || exit 1; done
echo EXIT $?
