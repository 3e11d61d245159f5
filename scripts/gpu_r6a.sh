#!/bin/bash
# Round 6, first pass: the counter list; the changed GPU tests (needle chain vs the oracle fed with the HIP's own
# render gradients, the measured bar of the fused offset-network step, P = 0 network heads); the issue-slot breakdown
# of the render kernels at cfg4 (SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY, plus instruction mixes);
# the bench step's own PMC passes (traffic of every kernel in kernels_ms); the one-rank RCCL step against N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6a}; O="gpurun_out/$OUT"; mkdir -p "$O"
timeout -k 10 90 rocprofv3 -L > "$O/counters.txt" 2>&1; echo "counter list rc=$? lines=$(wc -l < "$O/counters.txt")"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
      "tests/test_gpu_parity.py::test_anisotropic_gaussians_forward_and_backward" \
      "tests/test_gpu_train.py::test_step_in_backward_with_offset_network" \
      "tests/test_gpu_mlp.py::test_empty_point_set_gives_empty_heads" > "$O/tests.log" 2>&1 \
      || { tail -40 "$O/tests.log"; exit 1; }
  tail -3 "$O/tests.log"
fi
pick() { for c in "$@"; do grep -qw "$c" "$O/counters.txt" && printf '%s ' "$c"; done; }
S1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
S2="$(pick SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC)GRBM_GUI_ACTIVE"
S3="$(pick SQ_INSTS_VMEM SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES)GRBM_GUI_ACTIVE"
echo "S2=$S2"; echo "S3=$S3"
PMC_OUT="$O/stall_cfg4" KREGEX=render PROF_ARGS="--config 4 --iters 3" PMC_PASSES="$S1;$S2;$S3" bash scripts/gpu_pmc.sh || exit 1
# the bench step's kernels (bench.py itself after --, no wrapper): traffic and VALU / stall figures per kernel
B1="FETCH_SIZE GRBM_GUI_ACTIVE"
B2="WRITE_SIZE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
PMC_OUT="$O/bench_pmc" PROF_SCRIPT=bench.py PROF_ARGS="--gpus 1 --steps 10 --warmup 3 --cpu-baseline off" \
    PMC_PASSES="$B1;$B2" bash scripts/gpu_pmc.sh || exit 1
# the one-rank RCCL step (the N > 1 path) against the N = 1 step, A/B/A/B on this box
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 10 --cpu-baseline off > "$O/bench_n1_$rep.log" 2>&1 \
      || { tail -20 "$O/bench_n1_$rep.log"; exit 1; }
  tail -1 "$O/bench_n1_$rep.log" | cut -c1-300
  GSD_DP_ONE_RANK=1 MASTER_ADDR=127.0.0.1 timeout -k 10 300 python bench.py --steps 40 --warmup 10 --cpu-baseline off \
      > "$O/bench_dp1_$rep.log" 2>&1 || { tail -20 "$O/bench_dp1_$rep.log"; exit 1; }
  tail -1 "$O/bench_dp1_$rep.log" | cut -c1-300
done
echo all-done
