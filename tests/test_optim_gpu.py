"""Fused optimizers vs torch.optim on the GPU: mid-run load_state_dict, SGD maximize +
weight decay, resuming from a stock torch.optim.SGD state (ADVICE r1 findings)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _params(seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return [torch.randn(257, 33, device=dev, generator=g).requires_grad_(True),
            torch.randn(1000, device=dev, generator=g).requires_grad_(True)]


def _set_grads(ps, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    for p in ps:
        p.grad = torch.randn(p.shape, device=dev, generator=g)


def test_adam_load_state_dict_mid_run(C):
    from distributed_pytorch_example_amd.optim import Adam

    ours_p, ref_p, other_p = _params(0), _params(0), _params(1)
    ours = Adam(ours_p, lr=1e-2)
    ref = torch.optim.Adam(ref_p, lr=1e-2)
    other = torch.optim.Adam(other_p, lr=1e-2)
    for s in range(3):  # ours has stepped (device table + step counters built) ...
        _set_grads(ours_p, s); ours.step()
        _set_grads(other_p, 10 + s); other.step()
    sd = copy.deepcopy(other.state_dict())  # ... then loads a DIFFERENT run's state
    ours.load_state_dict(sd)
    ref.load_state_dict(copy.deepcopy(sd))
    with torch.no_grad():
        for a, b, c in zip(ours_p, ref_p, other_p):
            a.copy_(c); b.copy_(c)
    for s in range(3):
        _set_grads(ours_p, 20 + s); ours.step()
        _set_grads(ref_p, 20 + s); ref.step()
    torch.cuda.synchronize()
    for a, b in zip(ours_p, ref_p):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
    for st_o, st_r in zip(ours.state_dict()["state"].values(), ref.state_dict()["state"].values()):
        assert float(st_o["step"]) == float(st_r["step"]) == 6.0
        assert torch.allclose(st_o["exp_avg"], st_r["exp_avg"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("nesterov", [False, True])
def test_sgd_maximize_weight_decay(C, nesterov):
    from distributed_pytorch_example_amd.optim import SGD

    ours_p, ref_p = _params(2), _params(2)
    kw = dict(lr=0.05, momentum=0.9, weight_decay=1e-2, maximize=True, nesterov=nesterov)
    ours, ref = SGD(ours_p, **kw), torch.optim.SGD(ref_p, **kw)
    for s in range(4):
        _set_grads(ours_p, s); ours.step()
        _set_grads(ref_p, s); ref.step()
    torch.cuda.synchronize()
    for a, b in zip(ours_p, ref_p):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
    for a, b in zip(ours.state_dict()["state"].values(), ref.state_dict()["state"].values()):
        assert torch.allclose(a["momentum_buffer"], b["momentum_buffer"], rtol=1e-5, atol=1e-6)


def test_sgd_resume_from_stock_torch_state(C):
    """A stock torch.optim.SGD state has momentum buffers but no 'step': the first fused step after
    loading must use the loaded buffer (torch semantics), not restart momentum."""
    from distributed_pytorch_example_amd.optim import SGD

    ref_p, ours_p = _params(3), _params(3)
    ref = torch.optim.SGD(ref_p, lr=0.05, momentum=0.9)
    for s in range(2):
        _set_grads(ref_p, s); ref.step()
    sd = copy.deepcopy(ref.state_dict())
    assert "step" not in next(iter(sd["state"].values()))
    with torch.no_grad():
        for a, b in zip(ours_p, ref_p):
            a.copy_(b)
    ours = SGD(ours_p, lr=0.05, momentum=0.9)
    ours.load_state_dict(sd)
    _set_grads(ours_p, 7); ours.step()
    _set_grads(ref_p, 7); ref.step()
    torch.cuda.synchronize()
    for a, b in zip(ours_p, ref_p):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
