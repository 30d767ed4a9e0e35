set -e
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_qhull_order.py tests/test_gpu_qhull_shards.py "tests/test_gpu_configs.py::test_c5_qhull_order_largest_hulls" tests/test_gpu_parity.py tests/test_gpu_hull_caps.py tests/test_gpu_lp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u scripts/c3_step.py 4 > $O/c3_step.log 2>&1
tail -2 $O/c3_step.log | cut -c1-120
timeout -k 10 400 python -u scripts/crowded.py --qhull 30 22 > $O/crowded.log 2>&1
tail -8 $O/crowded.log
echo done
