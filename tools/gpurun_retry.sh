#!/bin/bash
# retry gpurun while the pool has no free box (exit 3 / transient); stops at the first real run
LOG=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $LOG.try 2>&1; rc=$?
  if grep -q "status=transient" $LOG.try; then echo "try $i transient" >> $LOG; sleep 200; continue; fi
  cat $LOG.try >> $LOG; echo "rc=$rc" >> $LOG; exit $rc
done
echo "gave up" >> $LOG
