# Kernel-level profile of the offpolicy QMix update (tools/mb_offq.py) at N = 2 and N = 8
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_offq
rm -rf $O && mkdir -p $O
for n in 2 8; do
  timeout -k 5 180 rocprofv3 --output-format csv --kernel-trace --stats -d $O/n$n -- python3 tools/mb_offq.py $n qmix > $O/n$n.log 2>&1
done
