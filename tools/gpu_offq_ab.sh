timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_offq.py > gpurun_out/to.log 2>&1; tail -1 gpurun_out/to.log
for d in lib lib_r6b lib lib_r6b; do MB_LIB=mini-marl_amd/$d/libminimarl.so timeout -k 10 120 python3 tools/mb_offq.py 8 qmix 2>/dev/null | tail -1 | cut -c90-200; done
