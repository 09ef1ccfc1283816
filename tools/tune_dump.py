"""Print the autotuned igemm variants of prologue launches (--all: every igemm launch) after two
ResNet-50 steps."""
import sys, torch
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simclr_amd.config import compose, task_config, CONF_DIR
from simclr_amd.data.datasets import synthetic_dataset
from simclr_amd.data.loader import ContrastiveLoader
from simclr_amd.parallel import state as pstate
from simclr_amd.train.pretrain import Trainer
from simclr_amd.ops import tuning, _ext
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
st = pstate.get(); st.device = dev
cfg = task_config(compose(str(CONF_DIR), "config", ["experiment.base_cnn=resnet50", "model.cifar_stem=true", "experiment.batches=512", "data.synthetic=true", "parameter.epochs=10"]))
tr = Trainer(cfg, st, 50000)
loader = ContrastiveLoader(synthetic_dataset(8192, 10), 512, dev, seed=7)
it = iter(loader)
for _ in range(2): tr.step(next(it)[0])
torch.cuda.synchronize()
ops = _ext.ops()
for k, v in tuning.table().items():
    if k[0] == "igemm" and (k[7] or k[3] or "--all" in sys.argv):
        print("bnb" if k[7] else "pro" if k[3] else "dual" if k[8] else "-", "M=%d N=%d K=%d" % (k[1][0]*k[1][4]*k[1][5], k[1][14], k[1][6]*k[1][7]*k[1][3]), "epi", k[4], "->", v, "glds" if ops.igemm_variant_glds(v) else "nt", ops.igemm_variant_bm(v))
    elif k[0] == "wgrad" and "--all" in sys.argv:
        g = k[1]
        print("wgrad", "M=%d N=%d K=%d" % (g[0] * g[4] * g[5], g[14], g[6] * g[7] * g[3]),
              "pro" if k[3] else "-", "dpro" if k[4] else "-", "->", v,
              "splits", ops.wgrad_splits(list(g), v))
