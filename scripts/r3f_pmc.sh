set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
export LQRO_LIB=liblqro.so
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM --output-format csv -d $O/r3f_sq1 -o run -- python3 scripts/qhull_prof.py > $O/r3f_sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $O/r3f_sq2 -o run -- python3 scripts/qhull_prof.py > $O/r3f_sq2.log 2>&1
echo done
