# round-5 GPU pass p: k_locate_lists at 4 intervals per lane (parity, C5 located trace with every kernel
# class timed), the C2 end-to-end timeline, and a fresh C3 PMC profile + bench line
export TMPDIR=/tmp
bash tools/gpu.sh r5p "test:level_table or c5_style or grouped_search or random_eds or device_ids or legacy or split_locate or readme" || exit 1
EDSBWT_BENCH_PROFILE=full bash tools/gpu.sh r5p trloc:c5 > gpurun_out/r5p_trloc.out 2>&1 || { tail -30 gpurun_out/r5p_trloc.out; exit 2; }
python3 - <<'PY'
import json
line = [l for l in open('gpurun_out/r5p_trloc_c5.json') if l.startswith('{')][-1]
d = json.loads(line)
l = d.get('located', {})
print({k: l.get(k) for k in ('chunks', 'records_per_step', 'seconds_per_step', 'records_per_sec', 'records_equal_counts', 'setup_s')}, d.get('ms_per_step'))
print(d['device_resident'].get('kernel_ms_per_step'))
PY
bash tools/gpu.sh r5p e2etrace:c2 prof:c3 bench:c3 || exit 3
