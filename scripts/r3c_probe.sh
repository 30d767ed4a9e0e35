set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs --hull-rule qhull > $O/r3c_bench_q.json 2> $O/r3c_bench_q.err
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs --hull-rule canonical > $O/r3c_bench_c.json 2> $O/r3c_bench_c.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r3c_kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-roofline-probe --hull-rule qhull > $O/r3c_kt.log 2>&1
python3 scripts/kernel_breakdown.py $O/r3c_kt $O/r3c_kernel_breakdown.json > /dev/null
echo done
