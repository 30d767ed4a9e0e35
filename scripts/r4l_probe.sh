set -e
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dyn.py tests/test_gpu_synth.py tests/test_cpp_consumer.py tests/test_cpp_sharded.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
