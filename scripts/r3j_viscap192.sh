#!/bin/bash
# the 30 m crowded swarm with k_qhull's visible cap at 192 (profile build
# liblqro_qprof192.so): hull phase, per-job stats, builds left to k_qhull_big
set -e
mkdir -p gpurun_out
LQRO_LIB=liblqro_qprof192.so LQRO_HOT=0 timeout -k 10 200 python -u scripts/qhull_prof.py 30 > gpurun_out/r3j_qprof192_30_plain.txt 2>&1
LQRO_LIB=liblqro_qprof.so LQRO_HOT=0 timeout -k 10 200 python -u scripts/qhull_prof.py 30 > gpurun_out/r3j_qprof128_30_plain.txt 2>&1
