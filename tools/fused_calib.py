import sys, pytest
sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
from _fused_compare import run_three, summary, violations
class MP:
    def __init__(self): self.undo=[]
    def setattr(self, obj, name, val):
        self.undo.append((obj, name, getattr(obj, name))); setattr(obj, name, val)
    def close(self):
        for o,n,v in reversed(self.undo): setattr(o,n,v)
        self.undo=[]
for loss in ("energy", "projection"):
    pass
for loss in ("projection",):
    for mut in (None, ("dgrad", "layer3.1", 1), ("fwd", "layer3.1", 1), ("fwd", "layer3.0", 2), ("dgrad", "layer2.2", 0)):
        mp = MP()
        mt = run_three("resnet50", True, 32, mp, block_out=True, mutate=mut, loss=loss)
        mp.close()
        print("CALIB", loss, mut, summary(mt, top=8), flush=True)
        small = sorted(mt["param"].items(), key=lambda kv: kv[1][0])
