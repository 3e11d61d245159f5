set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/mlp; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mlp.py > gpurun_out/mlp/t.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/mlp/t.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 scripts/prof_deform_mlp.py > gpurun_out/mlp/mlp.log 2>&1 || { tail -20 gpurun_out/mlp/mlp.log; exit 1; }
grep -v amdgpu.ids gpurun_out/mlp/mlp.log
