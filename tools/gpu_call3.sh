timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fused.py tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1 || { echo "tests failed"; exit 1; }
tools/envab.sh 2 "SIMCLR_WGRAD_INKERNEL_REDUCE=0" "SIMCLR_WGRAD_INKERNEL_REDUCE=1" > gpurun_out/ab3.txt 2>&1 || exit 1
BACKENDS=torch tools/e2e_diag.sh 30 > gpurun_out/e2e_diag_torch.txt 2>&1
