#!/bin/bash
# Round-3 close: the whole GPU suite, smoke, the default bench line (C3) and the C5 / C2 lines at HEAD.
export TMPDIR=/tmp
TAG=${1:-r3final}
mkdir -p gpurun_out
bash tools/gpu_full.sh ${TAG} || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.log || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.log || exit 1
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.log
echo EXIT $?
