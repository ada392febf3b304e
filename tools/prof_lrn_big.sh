# kernel stats of the B=4096 QMIX learner update (tools/mb_learner_big.py) under rocprofv3
export TMPDIR=/tmp
mkdir -p gpurun_out/plrnb
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/plrnb/stats -- python3 tools/mb_learner_big.py > gpurun_out/plrnb/log.txt 2>&1
rc=$?
tail -1 gpurun_out/plrnb/log.txt
python3 profiles/summarize.py gpurun_out/plrnb/stats > gpurun_out/plrnb/kernel_stats.txt
head -30 gpurun_out/plrnb/kernel_stats.txt
exit $rc
