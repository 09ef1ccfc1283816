set -o pipefail
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/prof_lag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d $out -o run -- python3 $root/bench.py --no-graph --steps 6 --warmup 3 > $out/bench.json
rc=$?
python3 $root/tools/launch_lag.py $out 4 > $out/lag.txt 2>&1
python3 $root/tools/idle_summary.py $out/run_kernel_trace.csv 4 > $out/idle.txt 2>&1
find $out -name '*.csv' -size +30M -delete
exit $rc
