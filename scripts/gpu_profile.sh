# Round profile: GPU tests, the bench line, rocprofv3 kernel trace/stats of the
# same bench command, and FETCH_SIZE / WRITE_SIZE passes (separate runs).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/prof_write.log 2>&1
timeout -k 10 200 python -u scripts/dyn_bench.py > gpurun_out/dyn_bench.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dyn -o run -- python3 scripts/dyn_bench.py > gpurun_out/prof_dyn.log 2>&1
echo done
