#!/bin/bash
# Round-3 re-entry check: the whole GPU suite at HEAD, then the default bench line (C3) and C2.
export TMPDIR=/tmp
TAG=${1:-r3z}
mkdir -p gpurun_out
bash tools/gpu_full.sh ${TAG} || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.log || exit 1
timeout -k 10 300 python bench.py --config c2 --no-cpu > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.log || exit 1
head -c 600 gpurun_out/${TAG}_bench_c3.json
