# round-5 GPU pass ai: the deep kernels without the record-offset tile sums (one register and an
# atomic path fewer) — parity on the direct-start / locate tests, then interleaved C3 A/B against the
# previous build (libedsbwt_ab0.so), 20 timed steps per line
export TMPDIR=/tmp
bash tools/gpu.sh r5ai "test:wide_kmer or packed_direct or c3_production or deferred or readme or random_eds or k_deep_builds or count_only_counts" || exit 1
for k in 1 2 3; do
  for spec in "EDSBWT_TRACE=0" "EDSBWT_LIB=eds-bwt_amd/_build/libedsbwt_ab0.so"; do
    env $spec timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 > gpurun_out/r5ai_line.json 2>> gpurun_out/r5ai_err.log || exit 2
    python3 -c "import json;d=json.load(open('gpurun_out/r5ai_line.json'));print('$k', '$spec', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" | tee -a gpurun_out/r5ai_summary.txt
  done
done
