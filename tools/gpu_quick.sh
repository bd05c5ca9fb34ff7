export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log &&
timeout -k 10 300 python bench.py --no-cpu --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log
echo EXIT $?
