set -o pipefail
timeout -k 10 200 python -u tools/host_profile.py > gpurun_out/hostprof16.txt 2>&1
timeout -k 10 200 python -u tools/issue_cost.py > gpurun_out/issue16.txt 2>&1
timeout -k 10 300 tools/runidle.sh r3 --no-graph > gpurun_out/idle16.log 2>&1
