#!/bin/bash
# Root-cause run for profiles/r3_e2e_probe_diag.md: SimCLR-pretrain ResNet-18 (the reference's
# default backbone) on the texture-only, noise-90 synthetic set with the HIP path (bf16) and the
# torch path (fp32) for the same epochs, then tools/probe_diag.py on both run directories
# (random-init encoder included).  Usage (GPU box, repo root): tools/e2e_diag.sh EPOCHS
set -o pipefail
E=${1:-20}; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/e2e_diag
rm -rf "$out"; mkdir -p "$out"
DATA="data.synthetic=true data.synthetic_size=50000 data.synthetic_colour=false data.synthetic_noise=90 experiment.base_cnn=resnet18 $*"
for be in ${BACKENDS:-hip torch}; do
  run=${TMPDIR:-/tmp}/simclr_diag_$be
  rm -rf "$run"; mkdir -p "$run/run"
  timeout -k 10 120 python - <<PY || exit $?
import torch, sys
sys.path.insert(0, "$root")
from simclr_amd.models import ContrastiveModel
torch.manual_seed(7)
m = ContrastiveModel("resnet18")
torch.save({"module." + k: v for k, v in m.state_dict().items()}, "$run/run/epoch=0-cifar10.pt")
PY
  prec=bf16; [ $be = torch ] && prec=fp32
  # (the torch path's MIOpen convolutions keep the default find mode: ~45 s of solver search on
  # the first step, then 85 ms/step; MIOPEN_FIND_MODE=FAST from an empty find-db picks solvers
  # that run 1.26 s/step — profiles/r3_optimization_log.md)
  echo "pretrain $be $E epochs"
  timeout -k 10 1200 python main.py $DATA runtime.backend=$be runtime.precision=$prec \
    experiment.batches=512 parameter.epochs=$E parameter.warmup_epochs=2 \
    experiment.save_model_epoch=$E runtime.log_every=25 hydra.run.dir=$run/run \
    > "$out/pretrain_$be.log" 2>&1 || exit $?
  tail -2 "$out/pretrain_$be.log"; cp "$run/run/metrics.jsonl" "$out/metrics_$be.jsonl"
  echo "probe diag $be"
  timeout -k 10 900 python tools/probe_diag.py "$run/run" $DATA runtime.backend=$be \
    runtime.precision=$prec experiment.batches=512 parameter.epochs=30 \
    hydra.run.dir=$out/diag_$be > "$out/diag_$be.log" 2>&1 || exit $?
  grep -v "^\[" "$out/diag_$be.log" | grep "cifar10.pt" || true
done
