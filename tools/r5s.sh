# round-5 GPU pass s: the whole GPU suite + smoke on the final tree, then the C5 located line with
# batches sized at 40 B per record, a C2 line (whole-chunk packing by default), the split direct walk A/B
export TMPDIR=/tmp
bash tools/gpu.sh r5s suite || exit 1
bash tools/gpu.sh r5s quick:c5:2 quick:c2:20 ab:c3:EDSBWT_DIRECT_SPLIT=0:EDSBWT_DIRECT_SPLIT=1:EDSBWT_DIRECT_SPLIT=0 || exit 2
python3 - <<'PY'
import json
d = json.load(open('gpurun_out/r5s_quick_c5.json'))
l = d.get('located', {})
print({k: l.get(k) for k in ('chunks', 'records_per_step', 'seconds_per_step', 'records_per_sec', 'records_equal_counts')}, d.get('ms_per_step'))
d = json.load(open('gpurun_out/r5s_quick_c2.json'))
print(d['ms_per_step'], d['e2e']['ms_wall_median'])
PY
# k_deep_direct's load kinds on C3 (the clock build): how many patterns the wide entry's text
# window finishes, and how many go on to per-row text entries, segment rows and rank steps
EDSBWT_LIB=$PWD/eds-bwt_amd/_build/libedsbwt_clk.so EDSBWT_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 2 --warmup 1 --config c3 > gpurun_out/r5s_clk_c3.json 2> gpurun_out/r5s_clk_c3.log || exit 3
grep -a "k_deep_direct loads\|deep from depth\|k_deep lane-steps" gpurun_out/r5s_clk_c3.log | tail -4
