# same-box A/B of chunk-kernel builds: "lib_dir[:hold]" arguments (hold = hidden states in the [N][H][E] layout)
mkdir -p gpurun_out/ab
: > gpurun_out/ab/res.jsonl
for v in "$@"; do
  d=${v%%:*}; h=0; [ "$d" != "$v" ] && h=${v##*:}
  MB_LIB=mini-marl_amd/$d/libminimarl.so MB_HOLD=$h timeout -k 10 240 python -u tools/mb_chunk.py chunk >> gpurun_out/ab/res.jsonl 2> gpurun_out/ab/err.log || { tail -5 gpurun_out/ab/err.log; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab/res.jsonl')][-1]; c=d['chunk']; print('$v', round(c['chunk_kernel_10steps_us'],1), round(c['region20_phase0_ms_per_step']['median']*1e3,2), round(c['region20_phase5_ms_per_step']['median']*1e3,2), c['state_sha1'])"
done
