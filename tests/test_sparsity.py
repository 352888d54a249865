"""ASP 2:4 structured sparsity (reference tests: apex/contrib/sparsity/test)."""
import pytest
import torch

from tests.conftest import devices


@pytest.mark.parametrize("pattern", ["m4n2_1d", "m4n2_2d_best", "m4n2_2d_greedy"])
def test_masks_are_2_of_4(pattern):
    from beforeholiday_amd.contrib.sparsity import create_mask
    torch.manual_seed(0)
    w = torch.randn(32, 64)
    m = create_mask(w, pattern)
    assert m.shape == w.shape
    groups = m.view(32, 16, 4).sum(-1)
    if pattern == "m4n2_2d_greedy":  # greedy may leave a row short; never over budget
        assert (groups <= 2).all() and groups.float().mean() > 1.5
    else:
        assert (groups == 2).all()
    if pattern == "m4n2_1d":  # keeps the 2 largest magnitudes of each group
        top = w.abs().view(32, 16, 4).topk(2, -1).indices
        kept = torch.zeros(32, 16, 4).scatter_(-1, top, 1.0)
        assert torch.equal(kept.view(32, 64), m)
    if "2d" in pattern:
        cols = m.view(8, 4, 16, 4).permute(0, 2, 1, 3).sum(2)  # per 4x4 block, column sums
        assert (cols <= 2).all()


@pytest.mark.parametrize("device", devices())
def test_asp_workflow(device):
    from beforeholiday_amd.contrib.sparsity import ASP
    ASP._reset()
    torch.manual_seed(1)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 16),
                                torch.nn.Linear(16, 3)).to(device)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    ASP.init_model_for_pruning(model, "m4n2_1d", verbosity=0, allow_recompute_mask=True, allow_permutation=False)
    ASP.init_optimizer_for_pruning(opt)
    ASP.compute_sparse_masks()
    assert ASP.is_sparsity_enabled()
    w0 = model[0].weight.detach()
    assert float((w0 == 0).float().mean()) == pytest.approx(0.5)
    x = torch.randn(8, 32, device=device)
    model(x).sum().backward()
    opt.step()
    assert torch.equal(model[0].weight == 0, w0 == 0)  # pruned entries stay pruned
    assert not (model[3].weight == 0).all()  # [3, 16] not eligible (rows % 8)
    ASP.restore_pruned_weights()
    assert not ASP.is_sparsity_enabled()
    ASP._reset()
