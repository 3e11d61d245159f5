set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python scripts/prof_densify.py --steps 3 > gpurun_out/dens.log 2>&1 && \
timeout -k 10 400 python bench.py --config 5 --steps 300 --warmup 5 > gpurun_out/b5.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dens.log | cut -c1-160 | tail -20; tail -c 2500 gpurun_out/b5.log; exit $rc
