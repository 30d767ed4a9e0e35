set -e
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
LQRO_LIB=liblqro_qp.so timeout -k 10 300 python -u scripts/qhull_prof.py > $O/qprof_c3.txt 2>&1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
echo done
