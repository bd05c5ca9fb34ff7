# round-5 GPU pass ac: the final tree — the whole GPU suite + smoke, then full bench lines (CPU
# baseline included) for C3 (the default config), C2 and C5 (the located step)
export TMPDIR=/tmp
bash tools/gpu.sh r5ac suite || exit 1
bash tools/gpu.sh r5ac bench:c3 bench:c2 || exit 2
bash tools/gpu.sh r5ac bench:c5:2:1 || exit 3
