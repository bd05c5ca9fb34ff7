# round-5 GPU pass ad: k_deep_direct at 8 / 7 / 6 waves per SIMD on the final tree (32-bit indices,
# k_deep at 6 waves): interleaved C3 lines, 20 timed steps each, device-resident leg only
export TMPDIR=/tmp
for k in 1 2 3; do
  for w in 8 7 6; do
    EDSBWT_DIRECT_WAVES=$w timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 > gpurun_out/r5ad_line.json 2>> gpurun_out/r5ad_err.log || exit 2
    python3 -c "import json;d=json.load(open('gpurun_out/r5ad_line.json'));print('$k', 'direct waves $w', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" | tee -a gpurun_out/r5ad_summary.txt
  done
done
