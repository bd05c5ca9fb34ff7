# round-5 GPU pass m: LDS-staged k_locate + compact level-table finisher archive: locate parity
# (every locate mode), the C5 production parity test, then the C5 located step's kernel trace
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "device_ids or level_table or grouped_search or split_locate or locate_sample_rates or c5_style or random_eds or readme or larger_eds or deferred or many_chunks or legacy or shard_first" > gpurun_out/r5m_tests.log 2>&1 || { tail -40 gpurun_out/r5m_tests.log; exit 1; }
tail -2 gpurun_out/r5m_tests.log
timeout -k 10 900 python -u -m pytest tests/test_production_gpu.py -x -v -k c5_production --timeout 800 --timeout-method thread > gpurun_out/r5m_c5prod.log 2>&1 || { grep -a "\[edsbwt\]\|libedsbwt\|Error\|error" gpurun_out/r5m_c5prod.log | tail -40; exit 2; }
tail -2 gpurun_out/r5m_c5prod.log
bash tools/gpu.sh r5m trloc:c5 > gpurun_out/r5m_trloc.out 2>&1 || { tail -30 gpurun_out/r5m_trloc.out; exit 3; }
python3 - <<'PY'
import json
line = [l for l in open('gpurun_out/r5m_trloc_c5.json') if l.startswith('{')][-1]
d = json.loads(line)
l = d.get('located', {})
print({k: l.get(k) for k in ('chunks', 'records_per_step', 'seconds_per_step', 'records_per_sec', 'records_equal_counts', 'setup_s')}, d.get('ms_per_step'))
print(d['device_resident'].get('kernel_ms_per_step'))
PY
