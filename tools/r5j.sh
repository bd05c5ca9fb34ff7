# round-5 GPU pass j: parity of the fused tiles / located long-list paths, C3 tile A/B, then the C5 located trace
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "random_eds or wide_kmer or packed_direct or single_row or deferred or locate or level_table or c5_style or search_lines or readme or larger_eds or grouped or counts_paths" > gpurun_out/r5j_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5j_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu.sh r5j ab:c3:EDSBWT_TILE_FUSE=1:EDSBWT_TILE_FUSE=0:EDSBWT_TILE_FUSE=1 || exit 2
bash tools/gpu.sh r5j trloc:c5 || exit 3
python3 - <<'PY'
import json
line = [l for l in open('gpurun_out/r5j_trloc_c5.json') if l.startswith('{')][-1]
d = json.loads(line)
l = d.get('located', {})
print({k: l.get(k) for k in ('records', 'seconds', 'records_per_sec', 'chunks', 'records_equal_counts')}, d.get('ms_per_step'))
PY
