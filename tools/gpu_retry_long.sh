#!/bin/bash
# usage: gpu_retry.sh OUTFILE TIMEOUT CMD ; retries only when no box/slot was available (nothing ran)
out=$1; to=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" $out && ! grep -q "status=ok\|status=fail\|rc=[0-9]" $out; then
    echo "attempt $i: transient, waiting" >> $out.retries; sleep 150; continue
  fi
  break
done
echo "done rc=$rc" >> $out
