set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python scripts/qhull_prof.py > gpurun_out/r3m_qprof.txt 2>&1
bash scripts/qhull_pmc.sh r3m_qpmc > gpurun_out/r3m_qpmc.txt 2>&1
echo done
