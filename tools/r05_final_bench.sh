#!/bin/bash
# round 5 final: the driver's default bench line, the self-play step's rocprofv3 kernel stats, the tower PMC passes.
set -o pipefail
bash tools/gpu.sh bench r05_final && bash tools/gpu.sh trace r05_final && bash tools/gpu.sh pmc r05_final
