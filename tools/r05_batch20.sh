#!/bin/bash
# round 5, final build (backward apply pairing off): the whole GPU test suite + smoke() on the final code, then the driver's default bench line.
set -o pipefail
bash tools/gpu.sh tests r05_final7 && bash tools/gpu.sh smoke r05_final7 && bash tools/gpu.sh bench r05_final7
