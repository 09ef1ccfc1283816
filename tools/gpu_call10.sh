set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread > gpurun_out/t10.log 2>&1 || { echo "tests failed" >> gpurun_out/t10.log; exit 1; }
tools/envab.sh 2 "SIMCLR_FUSED_BWD1X1=0" "SIMCLR_FUSED_BWD1X1=1" > gpurun_out/ab10.txt 2>&1 || exit 1
tools/envab.sh 2 "SIMCLR_BWD1X1_BPS=128" "SIMCLR_BWD1X1_BPS=256" >> gpurun_out/ab10.txt 2>&1 || exit 1
