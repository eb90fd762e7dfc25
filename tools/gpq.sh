#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports no free slot (exit 3: nothing ran,
# nothing charged); any other outcome ends it.  usage: tools/gpq.sh <out file> <timeout s> '<command>'
out=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
