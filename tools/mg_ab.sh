# Time tools/mb_mappo.py (5 epochs) for each lib/var_*.so given: mg_ab.sh base nog ...
set -e
for n in "$@"; do
  echo -n "$n "
  MM_LIB=mini-marl_amd/lib/var_$n.so timeout -k 10 120 python3 tools/mb_mappo.py --episodes 1 --epochs 5 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['train_ms_per_epoch'],3), d['train_info']['critic_grad_norm'])"
done
