# PMC passes (separate runs, counters within the per-block limits) + kernel stats of the fused rollout step
# (tools/mb_rollout.py, in-tree library only)
set -e
export TMPDIR=/tmp
O=gpurun_out/pmc_rs
rm -rf $O && mkdir -p $O
timeout -k 10 120 python3 tools/mb_rollout.py > $O/mb.log 2>&1
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/p1 -- python3 tools/mb_rollout.py > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM -d $O/p2 -- python3 tools/mb_rollout.py > $O/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/p3 -- python3 tools/mb_rollout.py > $O/p3.log 2>&1
python3 tools/pmc_sum.py $O "_h3_kernel" > $O/summary.txt
cat $O/mb.log | grep "{"
cat $O/summary.txt
