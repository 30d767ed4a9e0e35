set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_qhull_order.py > $O/r3v_tests.log 2>&1
timeout -k 10 180 python scripts/qhull_prof.py > $O/r3v_qprof.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs > $O/r3v_bench_q.json 2> $O/r3v_bench_q.err
echo done
