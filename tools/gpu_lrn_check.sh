# learner tests + B=4096 update kernel stats of the in-tree build
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_learner.py tests/test_gpu_headline.py -k "learner" > gpurun_out/tl.log 2>&1
rc=$?; tail -1 gpurun_out/tl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/mb_learner_big.py | tail -1
bash tools/prof_lrn_big.sh | grep -E "loss_reduce|outer_batch|tmv|mixer_gi|mixer_fwd"
