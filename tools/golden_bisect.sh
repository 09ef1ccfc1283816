#!/bin/bash
# golden-run (ResNet-50 batch 128, 60 steps) under several env settings (one "VAR=value" per
# argument); stops at the first run that ends other than pass (0) / assertion failure (1)
i=0
for a in "$@"; do
  i=$((i+1))
  env $a timeout -k 10 200 python -u -m pytest tests/test_gpu_e2e.py -k batch128 -q -s \
    --timeout 180 --timeout-method thread > gpurun_out/g_$i.log 2>&1
  rc=$?
  echo "$i $a rc=$rc $(grep -h 'max |d|' gpurun_out/g_$i.log)" >> gpurun_out/g_sum.log
  [ $rc -le 1 ] || exit $rc
done
