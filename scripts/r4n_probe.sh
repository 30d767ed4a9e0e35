set -e
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 300 python -u scripts/c4_step.py 3 > $O/c4.log 2>&1; tail -1 $O/c4.log | cut -c1-160
timeout -k 10 300 python -u scripts/c3_step.py 4 > $O/c3.log 2>&1; tail -1 $O/c3.log | cut -c1-160
echo done
