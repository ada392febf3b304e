# MAPPO tests, same-box epoch A/B of library builds (args: lib dirs under mini-marl_amd/) and the gradient passes'
# traffic (tools/pmc_mappo.sh) of the in-tree build
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mappo.py > gpurun_out/tm.log 2>&1
rc=$?
tail -2 gpurun_out/tm.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_mappo.sh "$@" || exit 1
timeout -k 10 600 bash tools/pmc_mappo.sh gpurun_out/pm_check > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/pm_check/pmc_mappo.json"))
tot = 0.0
for k, v in d["kernels"].items():
    tot += v["traffic_bytes"]
    if "grad" in k:
        print(k[:50], round(v["fetch_bytes"] / 1e6, 1), round(v["write_bytes"] / 1e6, 1))
print("all mappo kernels, bytes per dispatch summed:", round(tot / 1e9, 3), "GB")
PY
