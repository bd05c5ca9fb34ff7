# round-5 GPU pass an: the whole GPU suite + smoke() on the tree with the counter-free timed steps,
# then the C4 and C5 bench lines
export TMPDIR=/tmp
bash tools/gpu.sh r5an suite bench:c4 bench:c5:3:1
