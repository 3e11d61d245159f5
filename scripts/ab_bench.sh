#!/bin/bash
# A/B: bench.py against libgsd_hip.so built from the working tree and from .ab/<name>/ source snapshots
# (e.g. `git archive <rev> gaussian-splatting_deformable_amd/csrc include | tar -x -C .ab/base`).
# Only the native library differs between the runs; the Python side is the working tree's.  The snapshots are older
# sources than the tree, so their build ids differ from it: GSD_SKIP_BUILD_ID=1 lifts _native's provenance check.
# RENDER=1: per-kernel times of scripts/prof_render.py (rasterizer fwd+bwd only) instead of bench.py.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
run() {  # name, csrc dir
  local name="$1" src="$2" out="/tmp/gsdab_$1"; mkdir -p "$out"
  make -s -C "$src" OUT="$out" -j16 > "$out/build.log" 2>&1 || { echo "build $name failed"; tail "$out/build.log"; exit 1; }
  if [ -n "$RENDER" ]; then
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB="$out/libgsd_hip.so" timeout -k 10 300 python scripts/prof_render.py --iters ${ITERS:-30} --timing \
        > gpurun_out/ab_$name.log 2>&1
    local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$name.log
    [ $rc -ne 0 ] && exit $rc
    return 0
  fi
  GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB="$out/libgsd_hip.so" timeout -k 10 600 python bench.py --cpu-baseline off ${BENCH_ARGS} > gpurun_out/ab_$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_$name.log; exit $rc; }
  tail -1 gpurun_out/ab_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('views/s', d['value'], 'ms/step', d['ms_per_step'], 'fwd_bwd', d['fwd_bwd_ms_per_view']); print({k: v for k, v in d['kernels_ms'].items()})"
}
for rep in 1 2; do
  run cur gaussian-splatting_deformable_amd/csrc
  for d in .ab/*/; do n=$(basename "$d"); run "$n" "$d/gaussian-splatting_deformable_amd/csrc"; done
done
exit 0
