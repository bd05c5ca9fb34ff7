# round-5 GPU pass ab: k_deep's 8-wave build — parity of every k_deep build, then interleaved C3 A/B of
# k_deep at 5, 6 and 8 waves per SIMD (20 timed steps per line, device-resident leg only)
export TMPDIR=/tmp
bash tools/gpu.sh r5ab "test:k_deep_builds or wide_kmer" || exit 1
for k in 1 2 3; do
  for w in 6 8 5; do
    EDSBWT_DEEPQ_WAVES=$w timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 > gpurun_out/r5ab_line.json 2>> gpurun_out/r5ab_err.log || exit 2
    python3 -c "import json;d=json.load(open('gpurun_out/r5ab_line.json'));print('$k', 'waves $w', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" | tee -a gpurun_out/r5ab_summary.txt
  done
done
