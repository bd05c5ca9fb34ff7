# round-5 GPU pass as (final tree): the whole GPU suite + smoke(), the C3 / C2 / C4 / C5 bench lines,
# and the C3 profile (kernel trace + PMC passes)
export TMPDIR=/tmp
bash tools/gpu.sh r5as suite bench:c3 bench:c2 prof:c3 bench:c4 bench:c5:3:1
