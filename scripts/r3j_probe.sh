set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $O/r3j_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r3j_smoke.log 2>&1
timeout -k 10 180 python scripts/qhull_prof.py > $O/r3j_qprof.txt 2>&1
timeout -k 10 180 python scripts/qhull_prof.py 22 > $O/r3j_qprof22.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs > $O/r3j_bench_q.json 2> $O/r3j_bench_q.err
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs --hull-rule canonical > $O/r3j_bench_c.json 2> $O/r3j_bench_c.err
echo done
