# round-5 GPU pass: new parity tests, the CLI at C3 with/without edsbwt_prepare, k_deep clocks, k_deep pair-step A/B
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "k_deep_builds or cli_gpus or readme_kat or cli_ or abi or prepare or pair_blocks or random_eds" > gpurun_out/r5f_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5f_tests.log
[ $rc -eq 0 ] || exit 1
EDSBWT_CLI_NO_PREPARE=1 timeout -k 10 400 python tools/cli_timing.py --config c3 --runs 2 --check 16 > gpurun_out/r5f_cli_noprep.json 2> gpurun_out/r5f_cli_noprep.err || exit 2
EDSBWT_TRACE=2 timeout -k 10 300 python tools/cli_timing.py --config c3 --runs 2 --check 512 --log gpurun_out/r5f_cli_trace.log > gpurun_out/r5f_cli.json 2> gpurun_out/r5f_cli.err || exit 3
head -c 600 gpurun_out/r5f_cli_noprep.json; echo; head -c 900 gpurun_out/r5f_cli.json; echo
EDSBWT_LIB=$PWD/eds-bwt_amd/_build/libedsbwt_clk.so EDSBWT_TRACE=1 timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-located --steps 2 --warmup 1 --config c3 > gpurun_out/r5f_clk.json 2> gpurun_out/r5f_clk.log || exit 4
grep "lane-steps\|lane utilisation\|queued for k_deep" gpurun_out/r5f_clk.log | tail -6 > gpurun_out/r5f_clk_tail.txt; cat gpurun_out/r5f_clk_tail.txt; rm -f gpurun_out/r5f_clk.log
bash tools/gpu.sh r5f ab:c3:EDSBWT_DEEPQ_PAIRS=1:EDSBWT_DEEPQ_PAIRS=0:EDSBWT_DEEPQ_PAIRS=1 || exit 5
