set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_qhull_shards.py tests/test_gpu_0_multirank.py > $O/r3v_tests.log 2>&1
echo done
