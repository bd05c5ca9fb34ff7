# round-5 GPU pass u: C5 located batches at 30 / 40 B per record, C2 chunking A/B, the N > 1 exchange
# path over RCCL with one rank (bench.py --dist-self), and the direct-start parity tests (segtab3 off)
export TMPDIR=/tmp
bash tools/gpu.sh r5u "test:wide_kmer or packed_direct" || exit 1
EDSBWT_LOCATED_BPR=30 bash tools/gpu.sh r5u30 quick:c5:2 || exit 2
bash tools/gpu.sh r5u ab:c2:EDSBWT_CHUNK_SINGLE_MB=24:EDSBWT_CHUNK_SINGLE_MB=8:EDSBWT_CHUNK_SINGLE_MB=4 rccl:c3 || exit 3
python3 - <<'PY'
import json
d = json.load(open('gpurun_out/r5u30_quick_c5.json'))
l = d.get('located', {})
print({k: l.get(k) for k in ('chunks', 'records_per_step', 'seconds_per_step', 'records_per_sec', 'records_equal_counts')}, d.get('ms_per_step'))
PY
