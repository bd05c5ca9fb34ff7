# round-5 GPU pass ak: parity of the counter-free deep builds (per-call EDSBWT_NO_COUNTERS, k_deep's
# build without counters), then interleaved C3 lines: counter-free timed steps (default) against
# --timed-counters, and a kernel trace of the default line
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "wide_kmer or k_deep_builds or packed_direct or search_device" > gpurun_out/r5ak_tests.log 2>&1 || { tail -30 gpurun_out/r5ak_tests.log; exit 1; }
tail -2 gpurun_out/r5ak_tests.log
for k in 1 2 3; do
  for opt in "" "--timed-counters"; do
    timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 $opt > gpurun_out/r5ak_line.json 2>> gpurun_out/r5ak_err.log || exit 2
    cp gpurun_out/r5ak_line.json gpurun_out/r5ak_line_${k}${opt:+_tc}.json
    python3 -c "import json;d=json.load(open('gpurun_out/r5ak_line.json'));r=d['roofline'];print('$k', '${opt:-default}', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'], r['kernel'], r['frac'], r['lines_per_launch'], r['counters'])" | tee -a gpurun_out/r5ak_summary.txt
  done
done
bash tools/gpu.sh r5ak trace:c3 || exit 3
