set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u bench.py > gpurun_out/final/bench_default.log 2> gpurun_out/final/bench_default.err
rc=$?; grep '^{"metric"' gpurun_out/final/bench_default.log | tail -1 > gpurun_out/final/bench_default.json; exit $rc
