"""Checkpoint schema and interchange with the reference's format."""
import copy

import torch
import torch.nn as nn

from distributed_pytorch_example_amd.models import SimpleNet
from distributed_pytorch_example_amd.optim import Adam
from distributed_pytorch_example_amd.utils.checkpoint import load_checkpoint, save_checkpoint

REF_GROUP_KEYS = {"lr", "betas", "eps", "weight_decay", "amsgrad", "maximize", "foreach", "capturable", "differentiable",
                  "fused", "decoupled_weight_decay", "params"}


def _reference_simplenet():
    """The reference's SimpleNet built from plain torch.nn (same structure, train.py:32-50)."""
    class Ref(nn.Module):
        def __init__(self):
            super().__init__()
            self.flatten = nn.Flatten()
            self.layers = nn.Sequential(nn.Linear(784, 256), nn.ReLU(), nn.Dropout(0.2), nn.Linear(256, 256), nn.ReLU(),
                                        nn.Dropout(0.2), nn.Linear(256, 10))

        def forward(self, x):
            return self.layers(self.flatten(x))
    return Ref()


def _train_a_bit(model, opt, steps=3):
    for _ in range(steps):
        x, y = torch.randn(16, 784), torch.randint(0, 10, (16,))
        opt.zero_grad()
        nn.functional.cross_entropy(model(x), y).backward()
        opt.step()


def test_schema_and_weights_only_load(tmp_path):
    m = SimpleNet()
    opt = Adam(m.parameters(), lr=1e-3)
    _train_a_bit(m, opt)
    p = tmp_path / "latest_model.pt"
    save_checkpoint(m, opt, 4, 1.25, str(p))
    ck = torch.load(p, weights_only=True)
    assert list(ck.keys()) == ["epoch", "model_state_dict", "optimizer_state_dict", "loss"]
    assert ck["epoch"] == 4 and ck["loss"] == 1.25
    assert list(ck["model_state_dict"].keys()) == [f"layers.{i}.{k}" for i in (0, 3, 6) for k in ("weight", "bias")]
    assert set(ck["optimizer_state_dict"]["param_groups"][0].keys()) == REF_GROUP_KEYS
    st = ck["optimizer_state_dict"]["state"][0]
    assert set(st.keys()) == {"step", "exp_avg", "exp_avg_sq"} and st["step"].dim() == 0


def test_reference_checkpoint_loads_into_ours(tmp_path):
    ref = _reference_simplenet()
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    _train_a_bit(ref, ropt)
    p = tmp_path / "ref.pt"
    torch.save({"epoch": 2, "model_state_dict": ref.state_dict(), "optimizer_state_dict": ropt.state_dict(), "loss": 0.5}, p)
    ours = SimpleNet()
    oopt = Adam(ours.parameters(), lr=1e-3)
    assert load_checkpoint(ours, oopt, str(p), torch.device("cpu")) == 2
    for (n, a), (_, b) in zip(ours.state_dict().items(), ref.state_dict().items()):
        assert torch.equal(a, b), n
    # identical subsequent updates
    torch.manual_seed(0)
    _train_a_bit(ours, oopt, 2)
    torch.manual_seed(0)
    _train_a_bit(ref, ropt, 2)
    ours.eval(); ref.eval()
    x = torch.randn(4, 784)
    assert torch.allclose(ours(x), ref(x), atol=1e-6)


def test_our_checkpoint_loads_into_reference(tmp_path):
    ours = SimpleNet()
    oopt = Adam(ours.parameters(), lr=1e-3)
    _train_a_bit(ours, oopt)
    p = tmp_path / "ours.pt"
    save_checkpoint(ours, oopt, 7, 0.1, str(p))
    ck = torch.load(p, map_location="cpu", weights_only=True)
    ref = _reference_simplenet()
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    ref.load_state_dict(ck["model_state_dict"])
    ropt.load_state_dict(ck["optimizer_state_dict"])
    assert ck["epoch"] == 7


def test_async_save(tmp_path):
    from distributed_pytorch_example_amd.utils.checkpoint import wait_pending

    m = SimpleNet()
    opt = Adam(m.parameters())
    save_checkpoint(m, opt, 1, 0.0, str(tmp_path / "a.pt"), async_save=True)
    wait_pending()
    assert torch.load(tmp_path / "a.pt", weights_only=True)["epoch"] == 1
