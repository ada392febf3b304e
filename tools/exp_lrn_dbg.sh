# per-kernel times of the B=32 learner update under the REC debug knobs (MM_REC_DBG)
for d in 0 1 2 4 7; do
  echo "== MM_REC_DBG=$d"
  MM_REC_DBG=$d bash tools/prof_kernels.sh prof_dbg$d 5 tools/mb_learner.py 2>&1 | grep -E "seq|ms_per|avg_us" | head -6
done
