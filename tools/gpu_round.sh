#!/bin/bash
# One GPU-box pass: parity tests, default bench line, gather calibration, and the
# rocprofv3 kernel-trace + separate FETCH_SIZE / WRITE_SIZE passes behind profiles/.
# Usage (from the repo root, on the box): bash tools/gpu_round.sh <tag>
export TMPDIR=/tmp
TAG=${1:-run}
B="python3 bench.py --no-cpu --steps 3 --warmup 1"
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --dist-backend gloo --patterns 2000000 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.log &&
timeout -k 10 120 tools/_build/calib_gather 16 100 1024 > gpurun_out/calib.json 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_fetch -o calib --output-format csv -- tools/_build/calib_gather 100 > gpurun_out/calib_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- $B > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.log &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o pmc --output-format csv -- $B > gpurun_out/${TAG}_fetch.json 2> gpurun_out/${TAG}_fetch.log &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o pmc --output-format csv -- $B > gpurun_out/${TAG}_write.json 2> gpurun_out/${TAG}_write.log
echo EXIT $?
