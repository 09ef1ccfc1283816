"""Resume restores the random generators (torch host / device, NumPy) saved with the optimizer
state, so the draws after a resume continue the interrupted run's sequence (an extension: the
reference saves weights only, /root/reference/main.py:129-131).  Also: the attribution knobs
that drop gradients are refused by the training entry points."""
import numpy as np
import pytest
import torch

from simclr_amd.models.contrastive import ContrastiveModel
from simclr_amd.utils.checkpoint import load_resume, save_resume


def test_resume_restores_rng(tmp_path):
    m = ContrastiveModel("resnet18")
    torch.manual_seed(5)
    np.random.seed(5)
    torch.rand(3)
    np.random.rand(2)
    path = str(tmp_path / "resume-1.pt")
    save_resume(path, m, None, epoch=1, step=10)
    want_t, want_n = torch.rand(4), np.random.rand(4)
    torch.manual_seed(123)
    np.random.seed(123)
    blob = load_resume(path, m)
    assert blob["epoch"] == 1 and blob["step"] == 10
    assert torch.equal(torch.rand(4), want_t)
    assert np.array_equal(np.random.rand(4), want_n)


@pytest.mark.parametrize("knob", ["SIMCLR_SKIP_WGRAD", "SIMCLR_EXPERIMENT_SKIP_BNRED"])
def test_training_refuses_attribution_knobs(monkeypatch, knob):
    from simclr_amd.train.pretrain import pretrain
    from simclr_amd.train.supervised import supervised
    monkeypatch.setenv(knob, "1")
    for fn in (pretrain, supervised):
        with pytest.raises(RuntimeError, match=knob):
            fn({})
