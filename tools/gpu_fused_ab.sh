# A/B of the fused one-launch rollout step vs the two-launch step (headline bench, short), plus a kernel trace
set -o pipefail
O=gpurun_out/fab
mkdir -p $O
B="python -u bench.py --steps 20 --repeats 10 --learner-steps 5 --learner-big-steps 0 --train-episodes 1 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline"
timeout -k 10 300 $B > $O/fused1.json 2> $O/fused1.err &&
MM_FUSED_STEP=0 timeout -k 10 300 $B > $O/two1.json 2> $O/two1.err &&
timeout -k 10 300 $B > $O/fused2.json 2> $O/fused2.err &&
MM_FUSED_STEP=0 timeout -k 10 300 $B > $O/two2.json 2> $O/two2.err &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py --steps 20 --repeats 3 --learner-steps 5 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline > $O/prof.log 2>&1
for f in $O/*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['ms_per_step_min'], d['roofline']['kernel_us'], d['train_loop'] and d['train_loop'].get('ms_per_episode'))"; done
