set -e
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 300 python -u scripts/c3_step.py 4 > $O/c3_step.log 2>&1
LQRO_LIB=liblqro_qp.so timeout -k 10 300 python -u scripts/qhull_prof.py > $O/qprof_c3.txt 2>&1
cd /tmp
LQRO_LIB=liblqro_g.so timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --output-format csv -d $GRAFT_REPO_ROOT/$O/pcs -o pcs -- python3 $GRAFT_REPO_ROOT/scripts/c3_step.py 3 > $GRAFT_REPO_ROOT/$O/pcs.log 2>&1
echo done
