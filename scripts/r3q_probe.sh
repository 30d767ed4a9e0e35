set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r3q_smoke.log 2>&1
timeout -k 10 900 python bench.py > $O/r3q_bench.json 2> $O/r3q_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r3q_kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs > $O/r3q_kt.log 2>&1
python3 scripts/kernel_breakdown.py $O/r3q_kt $O/r3q_kernel_breakdown.json > /dev/null
python3 -c "import glob,shutil;shutil.copy(glob.glob('$O/r3q_kt/**/*kernel_stats.csv',recursive=True)[0],'$O/r3q_kernel_stats.csv')"
echo done
