#!/bin/bash
# round 5: the whole GPU test suite + smoke() on the final code, then the tree kernel's PMC bytes (headline + g8192).
set -o pipefail
bash tools/gpu.sh tests r05_final && bash tools/gpu.sh smoke r05_final && bash tools/r05_pmc_tree.sh r05_final/pmc_tree
