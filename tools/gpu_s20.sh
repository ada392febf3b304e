# The driver-style short region (--steps 20), twice, with the bench's 10-region median.
set -o pipefail
mkdir -p gpurun_out/s20
B="python -u bench.py --steps 20 --repeats 10 --learner-steps 5 --learner-big-steps 0 --train-episodes 1 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/s20/a.json 2> gpurun_out/s20/a.err && timeout -k 10 300 $B > gpurun_out/s20/b.json 2> gpurun_out/s20/b.err
for f in gpurun_out/s20/a.json gpurun_out/s20/b.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['ms_per_step_min'], d['ms_per_step_max'], d['roofline']['kernel_us'])"; done
