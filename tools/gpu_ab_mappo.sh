# same-box A/B of MAPPO epoch time across library builds (lib dirs as arguments)
mkdir -p gpurun_out/abm
for d in "$@"; do
  MB_LIB=mini-marl_amd/$d/libminimarl.so timeout -k 10 300 python -u tools/mb_mappo.py --episodes 2 > gpurun_out/abm/$d.json 2> gpurun_out/abm/err.log || { tail -5 gpurun_out/abm/err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abm/$d.json').read().strip().split('\n')[-1]); print('$d', {k: d[k] for k in ('rollout_ms_per_step','train_ms_per_epoch')})"
done
