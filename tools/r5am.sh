# round-5 GPU pass am: C3 and C2 bench lines on the counter-free timed steps, and the C3 profile
# (kernel trace + PMC passes -> profiles/traffic_c3.json's per-launch DRAM bytes)
export TMPDIR=/tmp
bash tools/gpu.sh r5am bench:c3 bench:c2 prof:c3
