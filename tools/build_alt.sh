#!/bin/bash
# Build an A/B variant of libgmz.so on the CPU host: tools/build_alt.sh NAME "-DMACRO=V ..."
#   -> datou-gomoku-muzero_amd/_alt/libgmz_NAME.so (objects in _alt/o_NAME, gpurun-ignored; the .so travels).
# Select it at run time with GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_NAME.so.
set -e
NAME=$1
DEFS=$2
cd "$(dirname "$0")/../datou-gomoku-muzero_amd/csrc"
make -s -j8 OBJDIR=../_alt/o_$NAME OUT=../_alt/libgmz_$NAME.so EXTRA="$DEFS"
echo "built _alt/libgmz_$NAME.so ($DEFS)"
