set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp; export TMPDIR=/tmp
mkdir -p $R/gpurun_out/api17
timeout -k 10 300 rocprofv3 --hip-trace --stats -f csv -d $R/gpurun_out/api17 -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-graph > $R/gpurun_out/api17/bench.log 2>&1
find $R/gpurun_out/api17 -name '*trace.csv' -size +20M -delete
ls -la $R/gpurun_out/api17 >> $R/gpurun_out/api17/bench.log
