# the Qhull-order GPU tests, an optional LQRO_QHULL_LONGPROF split (QLONG=1,
# liblqro_qlong.so) and an A/B of the C3 step against variant libraries (AB=...):
#   TAG=rX AB="liblqro_base.so" bash scripts/qhull_ab.sh   (GPU box, repo root)
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_qhull_c3.py tests/test_gpu_qhull_shards.py tests/test_gpu_hull_caps.py} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
if [ -n "$QLONG" ]; then
LQRO_LIB=liblqro_qlong.so timeout -k 10 200 python3 scripts/qhull_long.py 4 > $O/qlong.txt 2>&1
cat $O/qlong.txt
fi
bash scripts/ab_lib.sh ${TAG:-r6t} ${AB:-liblqro_r6base.so}
