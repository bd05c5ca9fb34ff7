# round-5 GPU pass ar: 64-B wide D-mer entries with the first link's segment ranks — parity, then
# interleaved C3 lines with EDSBWT_KT1_LINK=1 / 0 and a kernel trace
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "wide_kmer or packed_direct or readme or random_eds or single_row or search_device or k_deep_builds or many_tiles or c3" > gpurun_out/r5ar_t.log 2>&1 || { tail -30 gpurun_out/r5ar_t.log; exit 1; }
tail -2 gpurun_out/r5ar_t.log
for k in 1 2 3; do
  for spec in "EDSBWT_KT1_LINK=1" "EDSBWT_KT1_LINK=0"; do
    env $spec timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 > gpurun_out/r5ar_line.json 2>> gpurun_out/r5ar_err.log || exit 2
    cp gpurun_out/r5ar_line.json gpurun_out/r5ar_line_${k}_${spec: -1}.json
    python3 -c "import json;d=json.load(open('gpurun_out/r5ar_line.json'));print('$k', '$spec', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'], d['config']['index_device_bytes'])" | tee -a gpurun_out/r5ar_summary.txt
  done
done
bash tools/gpu.sh r5ar trace:c3 || exit 3
