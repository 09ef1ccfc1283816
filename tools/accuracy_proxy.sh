#!/bin/bash
# Mid-difficulty accuracy proxy (no CIFAR on the box): SimCLR-pretrain the
# same encoder from the same seed on the HIP bf16 path and on the stock fp32 torch path
# (runtime.backend=torch runtime.precision=fp32) on the synthetic TEXTURE set
# (data/datasets.py synthetic_texture_dataset), then run eval.py's linear and centroid probes on
# both — each encoder through both evaluation backends — next to the random-init encoder (epoch=0, same weights in
# both run dirs).  Per-epoch losses: metrics.jsonl of each run.
# Usage (GPU box, repo root): tools/accuracy_proxy.sh EPOCHS NOISE SIZE [extra overrides...]
set -o pipefail
E=${1:-20}; NOISE=${2:-40}; N=${3:-10000}; shift 3
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${PROXY_TAG:-proxy}
out=$root/gpurun_out/$tag
run=${TMPDIR:-/tmp}/simclr_$tag
rm -rf "$out" "$run"; mkdir -p "$out" "$run/hip" "$run/torch"
COMMON="data.synthetic=true data.synthetic_kind=texture data.synthetic_size=$N data.synthetic_noise=$NOISE experiment.batches=${BATCH:-256} $*"
timeout -k 10 120 python - <<PY || exit $?
import torch, sys
sys.path.insert(0, "$root")
from simclr_amd.config import compose, task_config, CONF_DIR
from simclr_amd.models import ContrastiveModel
from simclr_amd.utils.misc import seed_everything
cfg = task_config(compose(str(CONF_DIR), "config", "$COMMON".split()))
seed_everything(cfg["parameter"]["seed"])  # the seed main.py builds its model under
m = ContrastiveModel(cfg["experiment"]["base_cnn"], d=cfg["parameter"]["d"],
                     cifar_stem=cfg.get("model", {}).get("cifar_stem"))
sd = {"module." + k: v for k, v in m.state_dict().items()}
for d in ("hip", "torch"):
    torch.save(sd, "$run/%s/epoch=0-cifar10.pt" % d)
PY
for path in hip torch; do
  extra=""
  [ $path = torch ] && extra="runtime.backend=torch runtime.precision=fp32"
  echo "pretrain $path $E epochs"
  timeout -k 10 900 python main.py $COMMON $extra parameter.epochs=$E parameter.warmup_epochs=2 \
    experiment.save_model_epoch=$E hydra.run.dir=$run/$path > "$out/pretrain_$path.log" 2>&1 || exit $?
  tail -2 "$out/pretrain_$path.log"; cp "$run/$path/metrics.jsonl" "$out/metrics_$path.jsonl"
done
# every pretrained encoder through BOTH evaluation paths (HIP bf16 features and stock fp32
# features), so a difference between the pretraining paths is not confused with one between
# the feature extractors
for path in hip torch; do
  for ev in hip torch; do
    eextra=""
    [ $ev = torch ] && eextra="runtime.backend=torch runtime.precision=fp32"
    for kind in linear centroid; do
      timeout -k 10 600 python eval.py $COMMON $eextra experiment.target_dir=$run/$path \
        parameter.classifier=$kind parameter.epochs=${PROBE_EPOCHS:-30} \
        hydra.run.dir=$out/ev_${path}_${ev}_$kind > "$out/eval_${path}_${ev}_$kind.log" 2>&1 || exit $?
    done
  done
done
python - <<PY
import json
rows = []
for path in ("hip", "torch"):
    for ev in ("hip", "torch"):
        for kind in ("linear", "centroid"):
            r = json.load(open("$out/ev_%s_%s_%s/results.json" % (path, ev, kind)))
            for ck, v in sorted(r.items()):
                acc = v.get("highest_val_acc", v.get("val_acc"))
                rows.append((path, ev, kind, ck, acc))
                print(f"pretrain {path:6s} eval {ev:6s} {kind:9s} {ck:22s} val top-1 {acc}")
json.dump(rows, open("$out/summary.json", "w"))
for path in ("hip", "torch"):
    ls = [json.loads(l) for l in open("$out/metrics_%s.jsonl" % path)]
    print(path, "loss per epoch:", " ".join("%.3f" % l["loss"] for l in ls))
PY
