set -o pipefail
mkdir -p gpurun_out/fused3
for m in 0; do
MM_ROLL_MODE=$m timeout -k 10 120 python -u tools/roll_trace.py > gpurun_out/fused3/trace$m.txt 2>&1 &&
MM_ROLL_MODE=$m timeout -k 10 120 python -u tools/roll_probe.py > gpurun_out/fused3/probe$m.json 2>&1 || exit 1
head -11 gpurun_out/fused3/trace$m.txt; cat gpurun_out/fused3/probe$m.json
done
