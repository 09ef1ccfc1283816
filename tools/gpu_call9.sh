set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/t9.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t9.log
tools/envab.sh 2 "SIMCLR_FUSED_BWD1X1=0" "SIMCLR_FUSED_BWD1X1=1" > gpurun_out/ab9.txt 2>&1 || exit 1
PROF_STEPS=5 timeout -k 10 300 tools/prof.sh r3dual -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 3 --no-graph > gpurun_out/prof9.txt 2>&1
