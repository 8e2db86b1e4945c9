#!/bin/bash
# round 5 final: the whole GPU test suite (one pytest process), then smoke().
set -o pipefail
bash tools/gpu.sh tests r05_final && bash tools/gpu.sh smoke r05_final
