# round 4: the GPU suite, smoke, the round profile (bench line, kernel trace, PMC traffic, SQ counters)
set -e
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -3 $O/smoke.log
timeout -k 10 900 bash scripts/gpu_profile.sh r4f > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -2 $O/profile.log
echo done
