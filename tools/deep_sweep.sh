#!/bin/bash
# Deep-cutover / register-list sweep on C3 (tuning aid; prints one bench line per setting)
export TMPDIR=/tmp
run() { echo "== $*"; env "$@" timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step']['deep'], d['kernel_ms_per_step']['step'], d['engine']['deep_from_depth'], d['engine']['deep_overflow'])"; }
run EDSBWT_DEEP_K=8 &&
run EDSBWT_LOCATE_SAMPLES=0 &&
run EDSBWT_DEEP_K=4 &&
run EDSBWT_DEEP_SHARE=0.3 &&
run EDSBWT_DEEP_SHARE=0.2 &&
run EDSBWT_DEEP_SHARE=0.3 EDSBWT_DEEP_ITEMS=4 &&
run EDSBWT_DEEP_SHARE=0.7 &&
run EDSBWT_DEEP_K=4 EDSBWT_DEEP_SHARE=0.3
echo EXIT $?
