# round-5 GPU pass aq: the look-back record offsets in k_locate_pp — parity (many chunks, the A/B
# fallbacks of _compare, the C3-shaped tests), then interleaved C3 lines with and without it
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "lookback" > gpurun_out/r5aq_t1.log 2>&1 || { tail -30 gpurun_out/r5aq_t1.log; exit 1; }
tail -2 gpurun_out/r5aq_t1.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "readme or random_eds or wide_kmer or packed_direct or single_row or search_device or c3" > gpurun_out/r5aq_t2.log 2>&1 || { tail -30 gpurun_out/r5aq_t2.log; exit 1; }
tail -2 gpurun_out/r5aq_t2.log
for k in 1 2 3; do
  for spec in "EDSBWT_LOC_LOOKBACK=1" "EDSBWT_LOC_LOOKBACK=0"; do
    env $spec timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --config c3 --steps 20 --warmup 3 > gpurun_out/r5aq_line.json 2>> gpurun_out/r5aq_err.log || exit 2
    cp gpurun_out/r5aq_line.json gpurun_out/r5aq_line_${k}_${spec: -1}.json
    python3 -c "import json;d=json.load(open('gpurun_out/r5aq_line.json'));print('$k', '$spec', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" | tee -a gpurun_out/r5aq_summary.txt
  done
done
bash tools/gpu.sh r5aq trace:c3 || exit 3
