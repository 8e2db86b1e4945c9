#!/bin/bash
# round 5, the exact final tree: the whole GPU test suite + smoke()
set -o pipefail
bash tools/gpu.sh tests r05_final10 && bash tools/gpu.sh smoke r05_final10
