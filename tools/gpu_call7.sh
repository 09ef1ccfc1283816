set -o pipefail
export MIOPEN_FIND_MODE=FAST
timeout -k 10 200 python -u -m pytest tests/test_gpu_dual.py -q --timeout 120 --timeout-method thread > gpurun_out/t7.log 2>&1; echo "dual rc=$?" >> gpurun_out/t7.log
D="data.synthetic=true data.synthetic_size=50000 data.synthetic_colour=false data.synthetic_noise=90 experiment.base_cnn=resnet18"
timeout -k 10 150 python -u main.py $D runtime.backend=torch runtime.precision=fp32 experiment.batches=512 parameter.epochs=30 parameter.warmup_epochs=2 runtime.max_steps=20 runtime.log_every=2 hydra.run.dir=/tmp/m7 > gpurun_out/main_torch7.log 2>&1
timeout -k 10 100 python -u tools/torch_step_probe.py resnet18 512 6 > gpurun_out/tprobe7.txt 2>&1
