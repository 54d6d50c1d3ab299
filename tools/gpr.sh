#!/bin/bash
# run one gpurun command; retry only when no box/slot was available (exit 3 / transient), never after a GPU run
out=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout 1500 /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|GPU slot(s) on this pod are busy\|backing off\|taken away" $out && ! grep -q "status=ok\|status=fail" $out; then
    sleep 120; continue
  fi
  exit $rc
done
exit $rc
