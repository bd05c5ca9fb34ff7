#!/bin/bash
# k_deep_refill (lane-refill walk for the packed direct start): parity tests that take the direct
# start, then the C3 and C2 device legs A/B against k_deep_fast (EDSBWT_DEEP_REFILL=0).
export TMPDIR=/tmp
TAG=${1:-r3n}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${TESTS:-direct or pair or single_row or deferred or production or many_chunks or kmer_start or grouped or smoke or console}" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
w() { python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])"; }
for spec in ${SPECS:-X=1 EDSBWT_DEEP_REFILL=0 X=2}; do
  echo "== c3 $spec" >> gpurun_out/${TAG}_ab.txt
  env $spec timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 20 --warmup 3 2>/dev/null | w >> gpurun_out/${TAG}_ab.txt || exit 1
  echo "== c2 $spec" >> gpurun_out/${TAG}_ab.txt
  env $spec timeout -k 10 200 python bench.py --config c2 --no-cpu --no-e2e --steps 20 --warmup 3 2>/dev/null | w >> gpurun_out/${TAG}_ab.txt || exit 1
done
B="python3 bench.py --no-cpu --no-e2e --steps 5 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o c3 --output-format csv -- $B > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.log
rm -f gpurun_out/${TAG}_prof/*kernel_trace.csv
cat gpurun_out/${TAG}_ab.txt
