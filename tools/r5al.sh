# round-5 GPU pass al: the counter-free k_deep builds (6 waves: 80 VGPRs + 56 B scratch; 5 waves) exact,
# then interleaved C3 lines with EDSBWT_DEEPQ_WAVES=6 / 5 (both counter-free in the timed steps)
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "k_deep_builds" > gpurun_out/r5al_tests.log 2>&1 || { tail -30 gpurun_out/r5al_tests.log; exit 1; }
tail -2 gpurun_out/r5al_tests.log
for k in 1 2 3; do
  for spec in "EDSBWT_DEEPQ_WAVES=6" "EDSBWT_DEEPQ_WAVES=5"; do
    env $spec timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 > gpurun_out/r5al_line.json 2>> gpurun_out/r5al_err.log || exit 2
    python3 -c "import json;d=json.load(open('gpurun_out/r5al_line.json'));print('$k', '$spec', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" | tee -a gpurun_out/r5al_summary.txt
  done
done
