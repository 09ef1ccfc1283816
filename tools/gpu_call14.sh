set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fused.py -q -k "wgrad or prologue or bn_backward" --timeout 200 --timeout-method thread > gpurun_out/t14.log 2>&1; echo "rc=$?" >> gpurun_out/t14.log
for sh in "1024 256 8 256 3 1 1" "1024 128 16 128 3 1 1" "1024 512 4 512 3 1 1" "1024 1024 8 256 1 1 0" "1024 256 8 1024 1 1 0"; do
  echo "== $sh" >> gpurun_out/wprobe14.txt
  timeout -k 10 100 python -u tools/wgrad_probe.py $sh -1 20 >> gpurun_out/wprobe14.txt 2>&1
done
