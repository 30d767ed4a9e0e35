#!/bin/bash
# k_qhull phase profiles of the crowded C3-sized swarms (Qhull order)
set -e
mkdir -p gpurun_out
for b in 30 22; do
  timeout -k 10 240 python -u scripts/qhull_prof.py $b > gpurun_out/r3h_qprof_$b.txt 2>&1
done
