# round-5 GPU pass q: k_locate_lists with 4 strided slots (parity + the C5 located step), then the
# 8-rank gloo rehearsal of C4 on this one card with every rank's tables sized for its HBM share
export TMPDIR=/tmp
bash tools/gpu.sh r5q "test:level_table or c5_style or grouped_search or random_eds or device_ids or legacy or readme" || exit 1
bash tools/gpu.sh r5q trloc:c5 > gpurun_out/r5q_trloc.out 2>&1 || { tail -30 gpurun_out/r5q_trloc.out; exit 2; }
python3 - <<'PY'
import json
line = [l for l in open('gpurun_out/r5q_trloc_c5.json') if l.startswith('{')][-1]
d = json.loads(line)
l = d.get('located', {})
print({k: l.get(k) for k in ('chunks', 'records_per_step', 'seconds_per_step', 'records_per_sec', 'records_equal_counts', 'setup_s')}, d.get('ms_per_step'))
print(d['device_resident'].get('kernel_ms_per_step'))
PY
bash tools/gpu.sh r5q rehearse:8:c4 || exit 3
