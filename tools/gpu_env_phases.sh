# env step phase split (MM_ENV_DBG: stop after phase k) at 4096 x 8, with and without the obs_cur copy
mkdir -p gpurun_out
for d in 0 1 2 3 4 5 0; do MM_ENV_DBG=$d timeout -k 10 60 python tools/mb_env.py > gpurun_out/env_$d.log 2>&1 || { tail -5 gpurun_out/env_$d.log; exit 1; }; echo "dbg=$d $(tail -1 gpurun_out/env_$d.log)"; done
MB_CUR=0 timeout -k 10 60 python tools/mb_env.py | tail -1
