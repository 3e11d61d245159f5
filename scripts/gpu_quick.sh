#!/bin/bash
# Quick GPU check of a kernel change: the rasterizer parity tests, then per-kernel times of
# prof_render.py (cfg 4, 30 fwd+bwd passes).  TESTS overrides the test selection.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q -m gpu -p no:cacheprovider \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/prof_render.py --iters 30 --timing > gpurun_out/quick.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/quick.log; exit $rc
