bash tools/gpu_all.sh 700 && bash tools/gpu_quick_bench.sh --steps 20
