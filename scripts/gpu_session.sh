set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/mlp1; export TMPDIR=/tmp
rm -rf gpurun_out/mlp1/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mlp1/prof -o m -- python3 scripts/prof_mlp_once.py > gpurun_out/mlp1/prof.log 2>&1 || { tail gpurun_out/mlp1/prof.log; exit 1; }
grep done gpurun_out/mlp1/prof.log; cut -d, -f1-4 gpurun_out/mlp1/prof/m_kernel_stats.csv | cut -c1-120
