set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
rm -rf gpurun_out/pmc gpurun_out/pmc_render; PMC_PASSES="FETCH_SIZE;WRITE_SIZE;$P3" KREGEX="gsd" PROF_ARGS="--iters 3" bash scripts/gpu_pmc.sh || exit 1
python scripts/pmc_traffic.py gpurun_out/pmc gpurun_out/pmc_traffic_render.json > /dev/null || exit 1
mv gpurun_out/pmc gpurun_out/pmc_render
python - <<'PY'
import json
d = json.load(open("gpurun_out/pmc_traffic_render.json"))
for k, v in sorted(d.items()):
    if isinstance(v, dict):
        print(k, v["hbm_bytes"], v.get("valu", {}).get("frac"), v.get("valu", {}).get("lds_issue_wait_frac"))
PY
