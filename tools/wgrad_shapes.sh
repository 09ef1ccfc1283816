#!/bin/bash
# usage (GPU box): tools/wgrad_shapes.sh [variant ...] — the ResNet-50 CIFAR weight-gradient
# shapes of one step (batch 512 x 2 views) through tools/wgrad_probe.py (kernel + split reduce)
set -e
for shp in "1024 128 16 128 3 1 1" "1024 256 8 256 3 1 1" "1024 512 4 512 3 1 1" \
           "1024 128 32 128 3 2 1" "1024 1024 8 256 1 1 0" "1024 256 8 1024 1 1 0" \
           "1024 512 16 128 1 1 0" "1024 128 16 512 1 1 0" "1024 256 32 64 1 1 0" \
           "1024 2048 4 512 1 1 0" "1024 512 4 2048 1 1 0"; do
  echo "== $shp"
  if [ $# -eq 0 ]; then timeout -k 5 120 python tools/wgrad_probe.py $shp -1 10
  else for v in "$@"; do timeout -k 5 120 python tools/wgrad_probe.py $shp $v 10; done; fi
done
