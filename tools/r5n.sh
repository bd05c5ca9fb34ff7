# round-5 GPU pass n: the C5 production parity test (progress lines keep the run visibly alive), the C5
# located step's trace with the LDS-staged k_locate, the C2 PMC profile and a full C2 bench line
export TMPDIR=/tmp
bash tools/gpu.sh r5n "test:c5_production" || exit 1
bash tools/gpu.sh r5n trloc:c5 > gpurun_out/r5n_trloc.out 2>&1 || { tail -30 gpurun_out/r5n_trloc.out; exit 2; }
python3 - <<'PY'
import json
line = [l for l in open('gpurun_out/r5n_trloc_c5.json') if l.startswith('{')][-1]
d = json.loads(line)
l = d.get('located', {})
print({k: l.get(k) for k in ('chunks', 'records_per_step', 'seconds_per_step', 'records_per_sec', 'records_equal_counts', 'setup_s')}, d.get('ms_per_step'))
print(d['device_resident'].get('kernel_ms_per_step'))
PY
bash tools/gpu.sh r5n prof:c2 bench:c2 || exit 3
