# round-5 GPU pass ae: host timeline of the C3 device-resident search (EDSBWT_TRACE=2: every launch's
# host time inside a search) — the per-step fixed cost beside the kernels
export TMPDIR=/tmp
bash tools/gpu.sh r5ae hostmarks:c3 || exit 1
