# kernel stats of the B=32 learner update at the bench's PER shape (E=4096, capacity 65536)
export TMPDIR=/tmp
mkdir -p gpurun_out/plrn
MB_E=4096 MB_CAP=65536 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/plrn/stats -- python3 tools/mb_learner.py > gpurun_out/plrn/log.txt 2>&1
rc=$?
tail -1 gpurun_out/plrn/log.txt
python3 profiles/summarize.py gpurun_out/plrn/stats > gpurun_out/plrn/kernel_stats.txt
head -40 gpurun_out/plrn/kernel_stats.txt
exit $rc
