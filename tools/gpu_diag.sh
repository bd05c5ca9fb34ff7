#!/bin/bash
# Diagnostics pass: PCIe shapes, an end-to-end run with the chunk timeline, a kernel +
# copy trace, the device-resident kernel trace, and the C2 line.   bash tools/gpu_diag.sh <tag>
export TMPDIR=/tmp
TAG=${1:-dg}
mkdir -p gpurun_out
timeout -k 10 120 tools/_build/pcie_bw > gpurun_out/${TAG}_pcie.json 2>&1 &&
EDSBWT_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu --no-device --steps 2 --warmup 1 > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/${TAG}_ct -o ct --output-format csv -- python3 bench.py --no-cpu --no-device --steps 2 --warmup 1 > gpurun_out/${TAG}_ct.json 2> gpurun_out/${TAG}_ct.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_kt.json 2> gpurun_out/${TAG}_kt.log &&
timeout -k 10 300 python -u bench.py --config c2 --no-cpu > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.log
echo EXIT $?
