#!/bin/bash
# round 5, after the paired BatchNorm apply pass: the whole GPU test suite + smoke() on the final code, then the driver's default bench line.
set -o pipefail
bash tools/gpu.sh tests r05_final6 && bash tools/gpu.sh smoke r05_final6 && bash tools/gpu.sh bench r05_final6
