"""Epoch boundary under a slow rank-0 save: rank 0 alone logs and writes the
checkpoint + resume file at each epoch end, which can take seconds for ResNet-50 with optimizer
state.  No other rank may start the next epoch's first step (whose BatchNorm exchange would wait
on rank 0 with the IPC path's 2 s spin bound, csrc/bn.hip) before rank 0 is done: pretrain()
barriers after the rank-0 work.  2 gloo ranks on CPU, rank 0's save slowed to 3 s.
Reference: the per-epoch save of /root/reference/main.py:124-131."""
import json
import os
import socket
import time

import pytest
import torch.multiprocessing as mp

SAVE_DELAY_S = 3.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    os.chdir(out_dir)
    import simclr_amd.train.pretrain as P
    from simclr_amd.config import CONF_DIR, compose, task_config
    from simclr_amd.runtime.dist import cleanup

    events = []
    orig_save = P.save_reference_checkpoint

    def slow_save(*a, **kw):
        time.sleep(SAVE_DELAY_S)
        orig_save(*a, **kw)
        events.append(("save_done", time.time()))

    orig_step = P.Trainer.step

    def step(self, x):
        events.append(("step", time.time()))
        return orig_step(self, x)

    P.save_reference_checkpoint = slow_save
    P.Trainer.step = step
    cfg = task_config(compose(str(CONF_DIR), "config", [
        "data.synthetic=true", "data.synthetic_size=32", "experiment.batches=8",
        "experiment.base_cnn=resnet18", "parameter.epochs=2", "parameter.warmup_epochs=1",
        "experiment.save_model_epoch=1", "parameter.use_cuda=false",
        "runtime.save_resume=false"]))
    try:
        P.pretrain(cfg)
    finally:
        cleanup()
    with open(os.path.join(out_dir, f"events{rank}.json"), "w") as f:
        json.dump(events, f)


@pytest.mark.timeout(600)
def test_no_rank_starts_next_epoch_during_rank0_save(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    ev0 = json.loads((tmp_path / "events0.json").read_text())
    ev1 = json.loads((tmp_path / "events1.json").read_text())
    saves = [t for k, t in ev0 if k == "save_done"]
    steps1 = [t for k, t in ev1 if k == "step"]
    # 32 images / (8 per rank x 2 ranks): 2 steps per epoch, 2 epochs
    assert len(saves) == 2 and len(steps1) == 4, (ev0, ev1)
    assert steps1[2] >= saves[0], "rank 1 began epoch 2 while rank 0 was still saving epoch 1"
