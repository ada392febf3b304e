#!/bin/bash
# same-box timing of library builds (args: build dirs under mini-marl_amd/, e.g. lib lib_abl1): tools/mb_chunk_abl.py
mkdir -p gpurun_out/abl
: > gpurun_out/abl/res.jsonl
for d in "$@"; do
  MB_LIB=mini-marl_amd/$d/libminimarl.so timeout -k 10 120 python -u tools/mb_chunk_abl.py >> gpurun_out/abl/res.jsonl 2> gpurun_out/abl/err.log || { tail -5 gpurun_out/abl/err.log; exit 1; }
  tail -1 gpurun_out/abl/res.jsonl
done
