# round-5 GPU pass l: the id-map search parity, the C5 located step in suffix-ordered batches (kernel
# trace), then the C5 production parity test under the native fault trace (r5k: a host fault there)
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "device_ids or level_table or grouped_search or split_locate" > gpurun_out/r5l_tests.log 2>&1 || { tail -30 gpurun_out/r5l_tests.log; exit 1; }
tail -2 gpurun_out/r5l_tests.log
bash tools/gpu.sh r5l trloc:c5 > gpurun_out/r5l_trloc.out 2>&1 || { tail -30 gpurun_out/r5l_trloc.out; exit 2; }
python3 - <<'PY'
import json
line = [l for l in open('gpurun_out/r5l_trloc_c5.json') if l.startswith('{')][-1]
d = json.loads(line)
l = d.get('located', {})
print({k: l.get(k) for k in ('chunks', 'records_per_step', 'seconds_per_step', 'records_per_sec', 'records_equal_counts', 'setup_s')}, d.get('ms_per_step'))
print(d['device_resident'].get('kernel_ms_per_step'))
PY
EDSBWT_SEGV_TRACE=1 timeout -k 10 900 python -u -m pytest tests/test_production_gpu.py -x -v -k c5_production --timeout 800 --timeout-method thread > gpurun_out/r5l_c5prod.log 2>&1; rc=$?
grep -a "\[edsbwt\]\|libedsbwt\|PASSED\|FAILED\|passed\|failed" gpurun_out/r5l_c5prod.log | tail -40
exit $rc
