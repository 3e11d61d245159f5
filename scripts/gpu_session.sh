set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/mlp; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py tests/test_gpu_train.py -k "mlp or relu or offset" > gpurun_out/mlp/t.log 2>&1; rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/mlp/t.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 scripts/prof_deform_mlp.py --iters 20 > gpurun_out/mlp/m.log 2>&1 || { tail -20 gpurun_out/mlp/m.log; exit 1; }
grep "P=" gpurun_out/mlp/m.log
