set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -m gpu -k "cfg5_benched" -q --timeout 200 > gpurun_out/cfg5.log 2>&1; tail -2 gpurun_out/cfg5.log
timeout -k 10 200 bash tools/gpu_quick_bench.sh --steps 20 --warmup 5 || exit 1
timeout -k 10 300 bash tools/pmc_fwd_sq.sh > gpurun_out/pmc_fwd_sq.log 2>&1; tail -40 gpurun_out/pmc_fwd_sq.log
