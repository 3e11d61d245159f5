set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/final6; export TMPDIR=/tmp
rm -rf gpurun_out/final6/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final6/prof -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/final6/b.log 2>&1 || exit 1
tail -1 gpurun_out/final6/b.log | cut -c1-120
