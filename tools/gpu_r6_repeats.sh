#!/bin/bash
# round 6: the default bench line repeated on one box (run-to-run spread of the headline,
# the parity sub-object and the CPU baseline)
mkdir -p gpurun_out
rm -f gpurun_out/r6_repeats.jsonl
for i in 1 2; do
  timeout -k 10 420 python -u bench.py > gpurun_out/r6_repeat_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r6_repeat_$i.log >> gpurun_out/r6_repeats.jsonl
done
