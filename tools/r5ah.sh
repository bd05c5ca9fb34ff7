# round-5 GPU pass ah: every k_deep build against the oracle on the final tree, repeated (plain, then the
# device-invariant build with poisoned allocations)
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/kdeep_stress.py --reps 10 --out gpurun_out/r5ah_kdeep_stress_plain.json > gpurun_out/r5ah_plain.log 2>&1 || { tail -20 gpurun_out/r5ah_plain.log; exit 1; }
tail -1 gpurun_out/r5ah_plain.log
EDSBWT_LIB=$PWD/eds-bwt_amd/_build/libedsbwt_dbg.so EDSBWT_POISON=1 timeout -k 10 900 python3 -u tools/kdeep_stress.py --reps 4 --out gpurun_out/r5ah_kdeep_stress_dbg_poison.json > gpurun_out/r5ah_dbg.log 2>&1 || { tail -20 gpurun_out/r5ah_dbg.log; exit 2; }
tail -1 gpurun_out/r5ah_dbg.log
