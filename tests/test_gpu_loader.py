"""The device-resident loader never synchronises the stream, including at an epoch rollover
(SURVEY §2.2 "Data sharding"; reference ``DistributedSampler.set_epoch``,
/root/reference/main.py:102,169): the shard order is uploaded from pinned memory with a
non-blocking copy, so the host keeps issuing while earlier steps still run."""
import pytest
import torch

from simclr_amd.data.datasets import synthetic_dataset
from simclr_amd.data.loader import ContrastiveLoader, shard_indices


@pytest.mark.gpu
def test_epoch_rollover_has_no_device_sync():
    dev = torch.device("cuda", 0)
    ds = synthetic_dataset(640, 10, seed=0)
    ld = ContrastiveLoader(ds, 64, dev, rank=1, world=2, seed=7)  # 5 steps per epoch
    got = []
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")  # any synchronising call in the loop raises
    try:
        for ep in (1, 2, 3):
            ld.set_epoch(ep)
            for x, y in ld:
                got.append((x, y))
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert len(got) == 15
    # the uploaded order is DistributedSampler's (labels of the yielded batches match)
    want = torch.from_numpy(ds.labels[shard_indices(640, 3, 1, 2)[:320]])
    have = torch.cat([y for _, y in got[10:]]).cpu()
    assert torch.equal(have, want)
