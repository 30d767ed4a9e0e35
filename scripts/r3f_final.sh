set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $O/r3f_gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r3f_smoke.log 2>&1
bash scripts/gpu_profile.sh r3f > $O/r3f_profile.log 2>&1
echo done
