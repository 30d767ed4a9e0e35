set -e
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
LQRO_LIB=liblqro_qp.so timeout -k 10 300 python -u scripts/qhull_prof.py > $O/qprof_c3.txt 2>&1
echo done
