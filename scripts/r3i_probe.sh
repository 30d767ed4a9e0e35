set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_qhull_order.py tests/test_cpp_sharded.py tests/test_gpu_dyn.py > $O/r3i_tests.log 2>&1
timeout -k 10 180 python scripts/qhull_prof.py > $O/r3i_qprof.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs --hull-rule qhull > $O/r3i_bench_q.json 2> $O/r3i_bench_q.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r3i_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-roofline-probe > $O/r3i_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r3i_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-roofline-probe > $O/r3i_write.log 2>&1
echo done
