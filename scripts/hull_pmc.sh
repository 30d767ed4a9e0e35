# SQ counter passes over one C3 step, reported for k_hull
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/hpmc
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/hpmc/p1 -o run -- python scripts/pair_only.py 1 > gpurun_out/hpmc/p1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/hpmc/p2 -o run -- python scripts/pair_only.py 1 > gpurun_out/hpmc/p2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_INT32 SQ_INST_LEVEL_VMEM --output-format csv -d gpurun_out/hpmc/p3 -o run -- python scripts/pair_only.py 1 > gpurun_out/hpmc/p3.log 2>&1
echo done
