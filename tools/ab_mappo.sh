#!/bin/bash
# A/B of two builds of libminimarl.so (ab/old.so, ab/new.so) on the MAPPO phases, interleaved
mkdir -p gpurun_out
cp mini-marl_amd/lib/libminimarl.so ab/cur.so
for r in 1 2; do
  for v in old new; do
    cp ab/$v.so mini-marl_amd/lib/libminimarl.so
    echo -n "$v " ; timeout -k 10 200 python3 tools/mb_mappo.py --episodes 2 --epochs 2 | tail -1 || exit 1
  done
done
cp ab/cur.so mini-marl_amd/lib/libminimarl.so
