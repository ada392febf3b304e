# rocprofv3 kernel stats of one python command: prof_kernels.sh <outdir> <top> <python args...>
set -e
export TMPDIR=/tmp
OUT=gpurun_out/$1; TOP=$2; shift 2
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 "$@" > $OUT/run.log 2>&1
tail -2 $OUT/run.log
python3 tools/kstats.py $(find $OUT -name '*kernel_stats.csv') $TOP
