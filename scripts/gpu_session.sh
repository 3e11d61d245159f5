set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/mlp; export TMPDIR=/tmp
for v in build build_sp build build_sp; do
GSD_HIP_LIB=$GRAFT_REPO_ROOT/gaussian-splatting_deformable_amd/$v/libgsd_hip.so timeout -k 10 300 python3 scripts/prof_deform_mlp.py --iters 30 > gpurun_out/mlp/m.log 2>&1 || { tail -20 gpurun_out/mlp/m.log; exit 1; }
echo "$v"; grep "bfloat16.*fwd+bwd" gpurun_out/mlp/m.log | cut -c1-70
done
