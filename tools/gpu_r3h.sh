#!/bin/bash
# rk16 (all-symbol 16-B rank entries): parity tests, then C5 whole-batch timing with and without.
export TMPDIR=/tmp
TAG=${1:-r3h}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "rank16 or random_eds or grouped or c5_style or kmer_start or deep_overflow" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --config c5 --no-cpu --no-e2e --steps 2 --warmup 1 > gpurun_out/${TAG}_c5_rk16.json 2> gpurun_out/${TAG}_c5_rk16.log &&
EDSBWT_NO_RANK16=1 timeout -k 10 300 python bench.py --config c5 --no-cpu --no-e2e --steps 2 --warmup 1 > gpurun_out/${TAG}_c5_occ.json 2> gpurun_out/${TAG}_c5_occ.log
echo EXIT $?
