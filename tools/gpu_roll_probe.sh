set -o pipefail
O=gpurun_out/rprobe
mkdir -p $O
timeout -k 10 120 python -u tools/roll_probe.py > $O/base.json 2>&1 &&
for k in 1 2 4 7; do MM_LIB=$PWD/probe/libmm_$k.so timeout -k 10 120 python -u tools/roll_probe.py > $O/p$k.json 2>&1 || exit 1; done
cat $O/*.json
