# round-5 GPU pass o: k_locate_lists (records straight from the level walk's lists) — locate parity, the
# C5 located step's trace — and the C2 end-to-end A/B (byte counts, streamed packing)
export TMPDIR=/tmp
bash tools/gpu.sh r5o "test:level_table or c5_style or grouped_search or random_eds or device_ids or legacy or split_locate or locate_sample_rates or readme or larger_eds or shard_first or search_lines_pipeline" || exit 1
bash tools/gpu.sh r5o trloc:c5 > gpurun_out/r5o_trloc.out 2>&1 || { tail -30 gpurun_out/r5o_trloc.out; exit 2; }
python3 - <<'PY'
import json
line = [l for l in open('gpurun_out/r5o_trloc_c5.json') if l.startswith('{')][-1]
d = json.loads(line)
l = d.get('located', {})
print({k: l.get(k) for k in ('chunks', 'records_per_step', 'seconds_per_step', 'records_per_sec', 'records_equal_counts', 'setup_s')}, d.get('ms_per_step'))
print(d['device_resident'].get('kernel_ms_per_step'))
PY
bash tools/gpu.sh r5o ab:c2:EDSBWT_SMALL_COUNTS=1:EDSBWT_SMALL_COUNTS=2:EDSBWT_PACK_STREAMED=0 || exit 3
