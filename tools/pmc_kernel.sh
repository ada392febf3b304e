# Three PMC passes (one rocprofv3 run each) + kernel trace for one command; summary filtered by kernel.
# usage: bash tools/pmc_kernel.sh <outdir> <kernel-substring> <python script + args...>
export TMPDIR=/tmp
O=$1; K=$2; shift 2
mkdir -p $O
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/p1 -- python3 "$@" > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM -d $O/p2 -- python3 "$@" > $O/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/p3 -- python3 "$@" > $O/p3.log 2>&1 || exit 1
python3 tools/pmc_sum.py $O "$K"
