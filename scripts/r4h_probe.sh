set -e
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_qhull_order.py tests/test_gpu_qhull_shards.py "tests/test_gpu_configs.py::test_c5_qhull_order_largest_hulls" "tests/test_gpu_parity.py::test_dense_swarm_inside_hull" "tests/test_gpu_parity.py::test_qhull_order_per_agent_gains" tests/test_gpu_hull_caps.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LQRO_QSIDE=0 timeout -k 10 300 python -u scripts/c3_step.py 4 > $O/c3_step_noqside.log 2>&1
timeout -k 10 300 python -u scripts/c3_step.py 4 > $O/c3_step.log 2>&1
tail -2 $O/c3_step_noqside.log | cut -c1-120
tail -2 $O/c3_step.log | cut -c1-120
LQRO_LIB=liblqro_qp.so timeout -k 10 300 python -u scripts/qhull_prof.py > $O/qprof_c3.txt 2>&1
echo done
