# Round profile (run on the GPU box from the repo root):
#   bash scripts/gpu_profile.sh TAG
# FETCH_SIZE / WRITE_SIZE passes, the bench line, a rocprofv3 kernel
# trace/stats of the same bench command and two SQ counter passes (each its own run),
# summarised into gpurun_out/TAG_*.  Every step has its own time limit; the
# first failure ends the script.
set -e
TAG=${1:-rX}
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
# the profiled command runs C3 only (--no-configs): C4 / C5 steps can take the
# plain schedule, whose full-grid k_pair launches would otherwise be averaged
# with the C3 roofline probe's (same grid)
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs"
# the traffic passes first: their summary (stamped with this liblqro.so) goes
# into profiles/ so that the bench line below cites it as roofline.traffic
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- $B > $O/prof_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- $B > $O/prof_write.log 2>&1
python3 scripts/pmc_traffic.py $O/prof_fetch $O/prof_write $O/${TAG}_pmc_traffic.json > /dev/null
cp $O/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_traffic.json
# k_qhull's own traffic: with LQRO_QSIDE=0 the side builds run as k_qhull
# launches (not inside k_qside, whose count mixes the builds with its rows)
LQRO_QSIDE=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch_q -o run -- $B > $O/prof_fetch_q.log 2>&1
LQRO_QSIDE=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write_q -o run -- $B > $O/prof_write_q.log 2>&1
python3 scripts/pmc_traffic.py $O/prof_fetch_q $O/prof_write_q $O/${TAG}_pmc_traffic_qhull.json > /dev/null
cp $O/${TAG}_pmc_traffic_qhull.json profiles/${TAG}_pmc_traffic_qhull.json
timeout -k 10 300 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- $B > $O/prof_kt.log 2>&1
python3 scripts/kernel_breakdown.py $O/prof_kt $O/${TAG}_kernel_breakdown.json > /dev/null
python3 -c "import glob,shutil;shutil.copy(glob.glob('$O/prof_kt/**/*kernel_stats.csv',recursive=True)[0],'$O/${TAG}_kernel_stats.csv')"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/prof_sq1 -o run -- $B > $O/prof_sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $O/prof_sq2 -o run -- $B > $O/prof_sq2.log 2>&1
KMS=$(python3 -c "import json;d=json.load(open('$O/${TAG}_kernel_breakdown.json'));print(max((r for r in d if r['kernel'].startswith('k_pair<16')), key=lambda r: r['workgroups'])['avg_ms'])")
python3 scripts/pmc_sq.py $O/${TAG}_pmc_sq.json $O/prof_sq1 $O/prof_sq2 --kernel-ms $KMS > /dev/null
echo profile $TAG done
