set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/t15.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t15.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke15.log 2>&1; echo "smoke rc=$?" >> gpurun_out/smoke15.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/b15.log 2>&1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/b15b.log 2>&1
