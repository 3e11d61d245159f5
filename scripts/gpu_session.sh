set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PROF_OPS2=1 timeout -k 10 300 python scripts/prof_densify.py --steps 2 > gpurun_out/dens2.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/dens2.log | cut -c1-150 | grep -A28 "(2nd)" | head -28; exit $rc
