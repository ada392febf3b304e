# SQ counters of the fp16x3 agent forward (tools/mb_fwd.py): LDS busy / conflicts vs MFMA busy
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_h3
rm -rf $O && mkdir -p $O
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS -d $O/p1 -- python3 tools/mb_fwd.py > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES -d $O/p2 -- python3 tools/mb_fwd.py > $O/p2.log 2>&1
