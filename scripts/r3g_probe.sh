set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 180 python scripts/qhull_prof.py > $O/r3g_qprof.txt 2>&1
timeout -k 10 180 python scripts/qhull_prof.py 22 > $O/r3g_qprof22.txt 2>&1
echo done
