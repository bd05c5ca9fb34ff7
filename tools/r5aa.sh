# round-5 GPU pass aa: interleaved C3 A/B, 20 timed steps per line, device-resident leg only:
# the current build vs the previous one (libedsbwt_ab0.so), each with k_deep at 5 and 6 waves per SIMD
export TMPDIR=/tmp
mkdir -p gpurun_out
python3 bench.py --no-cpu --no-e2e --config c3 --steps 3 --warmup 1 > /dev/null 2> gpurun_out/r5aa_warm.log || exit 1
for k in 1 2 3; do
  for spec in "EDSBWT_TRACE=0" "EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so" "EDSBWT_DEEPQ_WAVES=6" "EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so EDSBWT_DEEPQ_WAVES=6"; do
    env $spec timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 > gpurun_out/r5aa_line.json 2>> gpurun_out/r5aa_err.log || exit 2
    python3 -c "import json;d=json.load(open('gpurun_out/r5aa_line.json'));print('$k', '$spec', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" | tee -a gpurun_out/r5aa_summary.txt
  done
done
