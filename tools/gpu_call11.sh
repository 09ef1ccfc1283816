set -o pipefail
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/convbench11.txt 2>&1
tools/envab.sh 2 "SIMCLR_SKIP_WGRAD=0" "SIMCLR_SKIP_WGRAD=1" > gpurun_out/ab11.txt 2>&1
