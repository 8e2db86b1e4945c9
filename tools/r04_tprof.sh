#!/bin/bash
# trainer step kernel trace (graph-replayed) -> gpurun_out/tprof/ + summary json
set -o pipefail
bash tools/trainer_profile.sh --per > gpurun_out/tprof_run.txt 2>&1 || { tail -20 gpurun_out/tprof_run.txt; exit 1; }
python3 tools/trainer_trace_summary.py gpurun_out/tprof/trace/run_kernel_trace.csv gpurun_out/tprof/bench.json gpurun_out/r04_trainer_trace.json 400
python3 -c "
import json; d=json.load(open('gpurun_out/r04_trainer_trace.json')); print(d['source']); print('launches/step', d['launches_per_step'])
for n,v in list(d['kernels'].items())[:40]: print('%7.3f ms %6.1f x %6.2f us  %s' % (v['ms_per_step'], v['launches_per_step'], v['mean_us'], n[:100]))
"
