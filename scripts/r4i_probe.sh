set -e
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
LQRO_LIB=liblqro_qpn.so timeout -k 10 300 python -u scripts/qhull_prof.py > $O/qprof_nopf.txt 2>&1
echo done
