# PMC passes on the env step kernel (tools/mb_env.py), one rocprofv3 run per counter group
export TMPDIR=/tmp
O=gpurun_out/pmc_env
mkdir -p $O
timeout -s KILL 60 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/p1 -- python3 tools/mb_env.py > $O/p1.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --output-format csv --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU -d $O/p2 -- python3 tools/mb_env.py > $O/p2.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --output-format csv --kernel-trace --stats -d $O/kt -- python3 tools/mb_env.py > $O/kt.log 2>&1 || exit 1
python3 tools/pmc_sum.py $O env_step
