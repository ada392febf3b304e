# MAPPO: gpu tests, epoch timing at cfg3, kernel stats of one episode
mkdir -p gpurun_out/mappo
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mappo.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/mappo/t.log 2>&1
rc=$?; tail -3 gpurun_out/mappo/t.log; grep "^E  \|FAILED" gpurun_out/mappo/t.log | head -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mb_mappo.py --episodes 2 > gpurun_out/mappo/mb.json 2> gpurun_out/mappo/mb.err || { tail -5 gpurun_out/mappo/mb.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/mappo/mb.json')); print({k: d[k] for k in ('rollout_ms_per_step','compute_ms','train_ms','train_ms_per_epoch')})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mappo/st -- python3 tools/mb_mappo.py --episodes 1 --epochs 4 > gpurun_out/mappo/st.log 2>&1 || { tail -5 gpurun_out/mappo/st.log; exit 1; }
python3 profiles/summarize.py gpurun_out/mappo/st | grep -i "mappo\|mgr" | head -12
