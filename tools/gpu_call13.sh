set -o pipefail
tools/envab.sh 2 "SIMCLR_WGRAD_TARGET_PCT=60" "SIMCLR_WGRAD_TARGET_PCT=45" > gpurun_out/ab13.txt 2>&1 || exit 1
tools/envab.sh 2 "SIMCLR_WGRAD_TARGET_PCT=60" "SIMCLR_WGRAD_TARGET_PCT=80" >> gpurun_out/ab13.txt 2>&1 || exit 1
tools/envab.sh 2 "SIMCLR_BNB_MAX_CIN=128" "SIMCLR_BNB_MAX_CIN=64" >> gpurun_out/ab13.txt 2>&1 || exit 1
