#!/bin/bash
# End-to-end accuracy proxy on ONE GPU (no CIFAR on the box): SimCLR-pretrain ResNet-50
# (CIFAR stem) on the class-structured synthetic 32x32 set, then linear-probe and centroid-probe
# the encoder features with eval.py, next to the same probes of the random-init encoder.
# Usage (GPU box, repo root): tools/e2e_probe.sh EPOCHS [extra overrides...]
set -o pipefail
E=${1:-20}; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/e2e          # logs + results (small)
run=${TMPDIR:-/tmp}/simclr_e2e    # checkpoints (112 MB each) stay off gpurun_out
rm -rf "$out" "$run"; mkdir -p "$out" "$run/run"
COMMON="data.synthetic=true data.synthetic_size=50000 experiment.base_cnn=resnet50 model.cifar_stem=true $*"
# the random-init encoder, in the reference checkpoint format, next to the trained one
timeout -k 10 120 python - <<PY || exit $?
import torch, sys
sys.path.insert(0, "$root")
from simclr_amd.models import ContrastiveModel
torch.manual_seed(7)
m = ContrastiveModel("resnet50", cifar_stem=True)
torch.save({"module." + k: v for k, v in m.state_dict().items()}, "$run/run/epoch=0-cifar10.pt")
PY
echo "pretrain $E epochs"
timeout -k 10 900 python main.py $COMMON experiment.batches=512 parameter.epochs=$E \
  parameter.warmup_epochs=2 experiment.save_model_epoch=$E hydra.run.dir=$run/run \
  > "$out/pretrain.log" 2>&1 || exit $?
tail -3 "$out/pretrain.log"; cp "$run/run/metrics.jsonl" "$out/" 2>/dev/null
echo "linear probe"
timeout -k 10 600 python eval.py $COMMON experiment.batches=512 experiment.target_dir=$run/run \
  parameter.classifier=linear parameter.epochs=30 hydra.run.dir=$out/ev_linear \
  > "$out/eval_linear.log" 2>&1 || exit $?
echo "centroid probe"
timeout -k 10 600 python eval.py $COMMON experiment.batches=512 experiment.target_dir=$run/run \
  parameter.classifier=centroid hydra.run.dir=$out/ev_centroid > "$out/eval_centroid.log" 2>&1 || exit $?
python - <<PY
import json
for kind in ("linear", "centroid"):
    r = json.load(open("$out/ev_%s/results.json" % kind))
    for ck, v in sorted(r.items()):
        acc = v.get("highest_val_acc", v.get("val_acc"))
        print(f"{kind:9s} {ck:22s} val top-1 {acc}")
PY
