# k_dynw after inlining its device functions (no call frames): parity, time,
# kernel trace and HBM traffic (GPU box, repo root): bash scripts/r4w_dyn.sh TAG
set -e
T=$1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dyn.py > $O/${T}_dyn_tests.txt 2>&1
tail -1 $O/${T}_dyn_tests.txt
timeout -k 10 200 python3 scripts/dyn_bench.py > $O/${T}_dyn_bench.txt 2>&1
cp $O/dyn_bench.json $O/${T}_dyn_bench.json
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- $B > $O/${T}_kt.log 2>&1
python3 scripts/kernel_breakdown.py $O/${T}_kt $O/${T}_kernel_breakdown.json > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${T}_pf -o run -- $B > $O/${T}_pf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${T}_pw -o run -- $B > $O/${T}_pw.log 2>&1
python3 scripts/pmc_traffic.py $O/${T}_pf $O/${T}_pw $O/${T}_pmc_traffic.json > /dev/null
echo dyn done
