#!/bin/bash
# Wide k-mer table + input-order direct start: parity tests that take the direct start, the
# random-gather rate against table size (address translation: the wide table is 34 GB at C3),
# and the C3 / C2 device legs.
export TMPDIR=/tmp
TAG=${1:-r3t}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${TESTS:-wide_kmer or packed_direct or pair or single_row or deferred or production or kmer_start or smoke}" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 180 tools/_build/calib_gather --tlb 1024 4096 16384 34816 65536 > gpurun_out/${TAG}_calib_tlb.json 2>&1 || exit 1
cat gpurun_out/${TAG}_calib_tlb.json
bash tools/gpu_ab3.sh ${TAG} c3 20 X=1 EDSBWT_KT1_WIDE=0 EDSBWT_KT1_WIDE=0,EDSBWT_DIRECT_SORT_BITS=0 || exit 1
bash tools/gpu_ab3.sh ${TAG}c2 c2 20 X=1 EDSBWT_KT1_WIDE=0
