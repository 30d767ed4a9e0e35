#!/bin/bash
# the 30 m crowded swarm: k_qhull per-job stats and the builds handed to k_qhull_big
set -e
mkdir -p gpurun_out
LQRO_HOT=0 timeout -k 10 240 python -u scripts/qhull_prof.py 30 > gpurun_out/r3i_qprof_30_plain.txt 2>&1
