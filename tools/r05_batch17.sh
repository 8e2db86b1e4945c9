#!/bin/bash
# round 5, after the 2-step BatchNorm elementwise grids: the whole GPU test suite + smoke() on the final code, then the driver's default bench line.
set -o pipefail
bash tools/gpu.sh tests r05_final5 && bash tools/gpu.sh smoke r05_final5 && bash tools/gpu.sh bench r05_final5
