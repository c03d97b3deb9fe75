#!/bin/bash
# retry a gpurun call while the pool has no box (nothing ran, nothing charged); stop on any
# other outcome.  usage: gpurun_retry.sh OUTFILE TIMEOUT 'cmd'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  if grep -q "no free box\|slot(s) on this pod are busy\|backing off\|stopped responding while being prepared" $OUT && ! grep -q "status=ok" $OUT; then
    sleep 150; continue
  fi
  break
done
