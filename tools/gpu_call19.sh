set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fused.py -q -k "wgrad or prologue" --timeout 200 --timeout-method thread > gpurun_out/t19.log 2>&1; echo "rc=$?" >> gpurun_out/t19.log
for sh in "1024 256 8 256 3 1 1" "1024 128 16 128 3 1 1" "1024 512 4 512 3 1 1" "1024 1024 8 256 1 1 0" "1024 256 8 1024 1 1 0" "1024 512 16 128 1 1 0"; do
  echo "== $sh" >> gpurun_out/wprobe19.txt
  for v in 0 5 6 9 19 20 21 22; do timeout -k 10 60 python -u tools/wgrad_probe.py $sh $v 20 >> gpurun_out/wprobe19.txt 2>&1; done
done
