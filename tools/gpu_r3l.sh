#!/bin/bash
# k_deep_wave (one wavefront per wide list): parity tests that reach the wide lists, the C2 and C3
# device legs (A/B against the lane-per-pattern k_deep_wide), the C3 lane-utilisation trace, and
# the C5 level-step TCC pass (tools/gpu_r3k.sh).
export TMPDIR=/tmp
TAG=${1:-r3l}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "deep_overflow or deferred or random_eds or c2_production or rank16 or larger_eds or long_patterns or kmer_start or c5_style or grouped" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
w() { python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])"; }
for spec in "X=1" "EDSBWT_DEEP_WAVE=0"; do
  echo "== c2 $spec" >> gpurun_out/${TAG}_ab.txt
  env $spec timeout -k 10 200 python bench.py --config c2 --no-cpu --no-e2e --steps 10 --warmup 2 2>/dev/null | w >> gpurun_out/${TAG}_ab.txt || exit 1
  echo "== c3 $spec" >> gpurun_out/${TAG}_ab.txt
  env $spec timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 10 --warmup 2 2>/dev/null | w >> gpurun_out/${TAG}_ab.txt || exit 1
done
bash tools/gpu_r3k.sh ${TAG}
