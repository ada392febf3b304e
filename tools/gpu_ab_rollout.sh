# fused-step A/B over experiment library builds in exp/ (MM_LIB), then the in-tree library
mkdir -p gpurun_out
for f in exp/*.so; do
  MM_LIB=$PWD/$f MB_UNFUSED=0 timeout -k 10 120 python3 tools/mb_rollout.py || exit 1
done
timeout -k 10 120 python3 tools/mb_rollout.py
