# round-5 GPU pass i: kernel trace of C5 with the located leg (where its 3.8 s go)
export TMPDIR=/tmp
bash tools/gpu.sh r5i trloc:c5 || exit 1
python3 - <<'PY'
import json
line = [l for l in open('gpurun_out/r5i_trloc_c5.json') if l.startswith('{')][-1]
d = json.loads(line)
l = d.get('located', {})
print({k: l.get(k) for k in ('records', 'seconds', 'records_per_sec', 'chunks')})
PY
