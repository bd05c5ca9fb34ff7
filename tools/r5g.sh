# round-5 GPU pass g: grouped k-mer table build (tests, C3 open peak), deep-kernel occupancy A/B
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "grouped or kmer_start_table or level_table or k_deep_builds or wide_kmer or packed_direct or prepare" > gpurun_out/r5g_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5g_tests.log
[ $rc -eq 0 ] || exit 1
EDSBWT_TRACE=1 timeout -k 10 600 python bench.py --no-cpu --no-e2e --no-located --steps 10 --warmup 2 --config c3 > gpurun_out/r5g_c3.json 2> gpurun_out/r5g_c3.log || exit 2
grep "index open\|k-mer start table\|level start table" gpurun_out/r5g_c3.log | head -5; rm -f gpurun_out/r5g_c3.log
head -c 700 gpurun_out/r5g_c3.json; echo
bash tools/gpu.sh r5g ab:c3:EDSBWT_DIRECT_WAVES=8:EDSBWT_DIRECT_WAVES=7:EDSBWT_DIRECT_WAVES=6 ab:c3:EDSBWT_DEEPQ_WAVES=1:EDSBWT_DEEPQ_WAVES=5 || exit 3
