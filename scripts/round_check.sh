# the whole GPU suite, smoke, the C3 A/B against a base library and k_dynw's
# kernel trace (GPU box, repo root): bash scripts/round_check.sh TAG [base.so]
set -e
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -n "$2" ]; then bash scripts/ab_lib.sh $T "$2"; fi
bash scripts/dyn_ab.sh ${T}_dyn
