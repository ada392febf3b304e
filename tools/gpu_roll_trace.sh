set -o pipefail
mkdir -p gpurun_out/rtrace
timeout -k 10 120 python -u tools/roll_trace.py > gpurun_out/rtrace/trace.txt 2>&1; rc=$?
cat gpurun_out/rtrace/trace.txt; exit $rc
