# round-5 GPU pass k: the whole GPU suite + smoke on the merged tree (HBM share, persistent host
# workers), then the 8-rank gloo rehearsal of C4 on this one card at the production config
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5k_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5k_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5k_smoke.log 2>&1 || { tail -20 gpurun_out/r5k_smoke.log; exit 2; }
tail -2 gpurun_out/r5k_smoke.log
bash tools/gpu.sh r5k rehearse:8:c4 || exit 3
