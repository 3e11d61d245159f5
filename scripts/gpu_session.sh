set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/mlp; export TMPDIR=/tmp
for nc in 1 2 1 2; do
GSD_MLP_NC=$nc timeout -k 10 300 python3 scripts/prof_deform_mlp.py --iters 30 > gpurun_out/mlp/m.log 2>&1 || { tail -20 gpurun_out/mlp/m.log; exit 1; }
echo "NC=$nc"; grep "bfloat16.*fwd+bwd" gpurun_out/mlp/m.log | cut -c1-70
done
GSD_MLP_NC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py > gpurun_out/mlp/t.log 2>&1; rc=$?; tail -1 gpurun_out/mlp/t.log; exit $rc
