#!/bin/bash
set -o pipefail
OUT=gpurun_out/r05_dbg2
mkdir -p $OUT
timeout -k 10 120 python3 tools/dbg_stem2.py > $OUT/stem2.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/stem2.txt | tail -12; exit $rc
