"""CPU tests: the oracle against the reference's golden vectors and against autograd."""
import itertools

import numpy as np
import pytest
import torch

from oracle import listmle as LM
from oracle import sampler as S

STRATS = ["thresh", "info", "pure", "masked"]


def _case(golden, ci):
    h, w, L, R = [int(v) for v in golden[f"c{ci}_shape"]]
    mask = np.unpackbits(golden[f"c{ci}_mask"])[: h * w].reshape(h, w).astype(bool)
    gt = golden[f"c{ci}_codes"].astype(np.float32) / np.float32(255)
    return h, w, L, R, mask, gt


def _within_list_canonical(out):
    o = np.asarray(out, np.float64)
    res = []
    for lst in o:
        k = np.lexsort((lst[:, 0], -lst[:, 1]))
        res.append(lst[k])
    return np.array(res)


@pytest.mark.parametrize("ci", range(4))
@pytest.mark.parametrize("strategy", STRATS)
def test_sampler_oracle_matches_reference_golden(golden, ci, strategy):
    """Replaying the reference's recorded np.random draws reproduces its output up to the order
    of EQUAL keys (tie order is machine-dependent in the reference: unstable numpy sort)."""
    h, w, L, R, mask, gt = _case(golden, ci)
    draws = golden[f"c{ci}_{strategy}_draws"]
    ref = golden[f"c{ci}_{strategy}_out"]
    out, used = S.sample_masked_point_batch(strategy, mask.astype(np.float32), gt, R, L, draws)
    assert used.size == draws.size == S.n_candidates(R, strategy) * L
    assert out.shape == ref.shape and out.dtype == np.float32
    # same lists, same list scores in the same order
    a, b = _within_list_canonical(out), _within_list_canonical(ref)
    sa = S.score_candidates(out, strategy, gt)
    sb = S.score_candidates(ref, strategy, gt)
    np.testing.assert_array_equal(sa, sb)
    np.testing.assert_array_equal(S.canonical_lists(out), S.canonical_lists(ref))
    # lists at different positions differ only by a permutation among equal scores
    for i in range(len(a)):
        if not np.array_equal(a[i], b[i]):
            same = np.where(sb == sa[i])[0]
            assert any(np.array_equal(a[i], b[j]) for j in same)
    # every list is sorted by depth, descending; indices are valid masked pixels
    assert np.all(np.diff(out[:, :, 1], axis=1) <= 0)
    flat = out[:, :, 0].astype(np.int64)
    assert np.all(mask.reshape(-1)[flat])
    np.testing.assert_array_equal(out[:, :, 1], gt.reshape(-1)[flat])


def test_sampler_oracle_live_rng_matches_recorded_stream(golden):
    """With draws=None the oracle consumes np.random in the reference's order."""
    h, w, L, R, mask, gt = _case(golden, 1)
    np.random.seed(1000 * 1 + len("info"))
    _, used = S.sample_masked_point_batch("info", mask.astype(np.float32), gt, R, L, None)
    np.testing.assert_array_equal(used, golden["c1_info_draws"])


def test_depth_relation_known_answers(golden):
    np.testing.assert_array_equal(S.get_depth_relation32(golden["rel_d1"], golden["rel_d2"]),
                                  golden["rel_out"])


@pytest.mark.parametrize("n", list(range(1, 40)) + [64, 100, 128, 129, 200, 500])
def test_pairwise_sum_matches_numpy(n):
    rng = np.random.default_rng(n)
    for _ in range(20):
        x = (rng.standard_normal(n) * rng.uniform(0, 100, n)).astype(np.float32)
        assert S.pairwise_sum32(x) == x.sum()


def test_info_expected_list_is_float32_linspace():
    gt = np.array([[0.2, 0.9], [0.5, 0.3]], np.float32)
    e = S.info_expected_list(gt, 5)
    assert e.dtype == np.float32 and e.shape == (5,) and e[-1] == np.float32(0.9)


# ----------------------------------------------------------------------------- ListMLE oracle
def _torch_listmle(s, lab):
    """Direct autograd restatement of the tfr formula on tie-free labels."""
    s = torch.tensor(s, dtype=torch.float64, requires_grad=True)
    lab_t = torch.tensor(lab, dtype=torch.float64)
    valid = lab_t >= 0
    sv = torch.where(valid, s, torch.full_like(s, np.log(1e-10)))
    score = torch.where(valid, lab_t, lab_t.clamp(min=0).min(dim=1, keepdim=True).values - 1e-6)
    order = torch.argsort(score, dim=1, descending=True)
    t = torch.gather(sv, 1, order)
    m = t.max(dim=1, keepdim=True).values
    C = torch.flip(torch.cumsum(torch.flip(torch.exp(t - m), [1]), 1), [1])
    nll = (torch.log(C) - (t - m)).sum(1)
    nll.sum().backward()
    return nll.detach().numpy(), s.grad.numpy()


@pytest.mark.parametrize("L", [2, 3, 5, 17, 64, 130])
def test_listmle_closed_form_gradient(L):
    rng = np.random.default_rng(L)
    N = 40
    s = rng.standard_normal((N, L)) * 3
    lab = rng.permutation(N * L).reshape(N, L).astype(np.float64) / (N * L)  # tie-free
    lab[0, 0] = -1.0  # one invalid element
    nll, g = LM.listmle_fwd_bwd(s, lab)
    nll_t, g_t = _torch_listmle(s, lab)
    np.testing.assert_allclose(nll, nll_t, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(g, g_t, rtol=1e-10, atol=1e-12)


def test_listmle_ties_loss_is_one_of_the_permutation_losses():
    """tfr shuffles tied labels randomly; the deterministic order picks one of those losses."""
    rng = np.random.default_rng(0)
    s = rng.standard_normal((1, 5))
    lab = np.array([[0.5, 0.2, 0.5, 0.9, 0.2]])
    nll, _ = LM.listmle_fwd_bwd(s, lab)
    cands = set()
    for perm in itertools.permutations(range(5)):
        p = np.array(perm)
        keys = lab[0][p]
        if np.all(np.diff(keys) <= 0):  # a descending order of labels = one tie resolution
            t = s[0][p]
            m = t.max()
            e = np.exp(t - m)
            C = np.cumsum(e[::-1])[::-1]
            cands.add(round(float((np.log(C) - (t - m)).sum()), 10))
    assert round(float(nll[0]), 10) in cands


def test_hourglass_loss_gather_and_scatter():
    rng = np.random.default_rng(1)
    B, H, W, R, L = 2, 6, 7, 4, 3
    pred = rng.standard_normal((B, H, W, 1))
    idx = rng.integers(0, H * W, (B, R, L))
    idx[0, 0, 1] = idx[0, 1, 2]  # duplicate pixel across lists
    lab = rng.permutation(B * R * L).reshape(B, R, L) / (B * R * L)
    y = np.stack([idx.astype(np.float32), lab.astype(np.float32)], -1)
    loss, dpred = LM.hourglass_nll(y, pred, B, L)
    # finite differences on a few pixels
    eps = 1e-6
    for b, p in [(0, idx[0, 0, 1]), (1, idx[1, 2, 0]), (0, 5)]:
        pp = pred.copy().reshape(B, -1)
        pp[b, p] += eps
        lp, _ = LM.hourglass_nll(y, pp.reshape(pred.shape), B, L)
        pp[b, p] -= 2 * eps
        lm, _ = LM.hourglass_nll(y, pp.reshape(pred.shape), B, L)
        assert abs((lp - lm) / (2 * eps) - dpred.reshape(B, -1)[b, p]) < 1e-7


def test_redweb_oracle_counts_match_survey():
    """142.54 GFLOP per 448x448 image per train step, 53,120
    encoder-BN parameters, ~8.65 M trainable in total."""
    from oracle import redweb as OR
    assert abs(OR.conv_flops_per_image(448, 448) / 1e9 - 142.54) < 0.01
    spec = OR.param_specs()
    enc_bn = sum(int(np.prod(s)) for n, s, k in spec
                 if k == "trainable" and not n.startswith(("ffl", "aol")))
    assert enc_bn == 53120
    assert sum(int(np.prod(s)) for n, s, k in spec if k == "trainable") == 8647299


def test_redweb_oracle_shapes_small():
    from oracle import redweb as OR
    torch.manual_seed(0)
    P = {n: torch.randn(s, dtype=torch.float64) * 0.05 for n, s, _ in OR.param_specs()}
    taps = {}
    with torch.no_grad():
        out = OR.forward(P, torch.rand(1, 64, 64, 3, dtype=torch.float64), taps=taps)
    assert out.shape == (1, 64, 64, 1)
    assert taps["conv2_block3_out"].shape == (1, 256, 16, 16)
    assert taps["conv5_block3_out"].shape == (1, 2048, 2, 2)
    assert taps["ffl2"].shape == (1, 64, 32, 32)
