#!/bin/bash
# LP latency rewrite + early LP: the GPU suite, k_lp4's time on the C3 hardest rows (new vs old
# LP), C3 steps with the early LP on and off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4e
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lp.py \
  > gpurun_out/r4e/tests_lp.log 2>&1 || { tail -30 gpurun_out/r4e/tests_lp.log; exit 1; }
tail -2 gpurun_out/r4e/tests_lp.log
for L in liblqro.so liblqro_oldlp.so; do
  LQRO_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e/prof_$L -o run -- \
    python3 scripts/lp_rows_time.py > gpurun_out/r4e/lp_$L.log 2>&1 || { tail -20 gpurun_out/r4e/lp_$L.log; exit 1; }
  tail -1 gpurun_out/r4e/lp_$L.log
  f=$(find gpurun_out/r4e/prof_$L -name '*kernel_stats.csv' | head -1)
  grep -E "k_lp" "$f"
done
LQRO_EARLY_LP=0 timeout -k 10 200 python3 scripts/c3_step.py 4 > gpurun_out/r4e/c3_step_noearly.log 2>&1 && tail -2 gpurun_out/r4e/c3_step_noearly.log
timeout -k 10 200 python3 scripts/c3_step.py 4 > gpurun_out/r4e/c3_step.log 2>&1 && tail -2 gpurun_out/r4e/c3_step.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs > gpurun_out/r4e/bench.json 2> gpurun_out/r4e/bench.err || { tail -20 gpurun_out/r4e/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4e/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'ms', d['ms_per_step'], 'host_cpp', d.get('host_cpp'))"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r4e/tests.log 2>&1; rc=$?; tail -5 gpurun_out/r4e/tests.log; exit $rc
