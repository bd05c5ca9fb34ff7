# round-5 GPU pass aj: k_deep_direct with and without its per-lane work counters on the tile-free
# build (interleaved C3 lines, 20 timed steps each)
export TMPDIR=/tmp
for k in 1 2 3; do
  for spec in "EDSBWT_DEEP_STATS=0" "EDSBWT_DEEP_STATS=1"; do
    env $spec timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 > gpurun_out/r5aj_line.json 2>> gpurun_out/r5aj_err.log || exit 2
    python3 -c "import json;d=json.load(open('gpurun_out/r5aj_line.json'));print('$k', '$spec', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" | tee -a gpurun_out/r5aj_summary.txt
  done
done
