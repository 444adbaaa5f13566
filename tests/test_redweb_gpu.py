"""GPU parity of the whole ff_redweb (ResNet-50 + ReDWeb decoder) training step against the fp64
CPU oracle (oracle/redweb.py), same seeded Keras-default weights and inputs on both sides.
Criteria as tests/test_model_gpu.py: activations / loss within 1e-3 relative; gradients as close
to the fp64 truth as the fp32 restatement of the same graph is."""
import numpy as np
import pytest
import torch

from oracle import listmle as LM
from oracle import redweb as OR
from pldepth_amd import kernels as K
from pldepth_amd.models.redweb_ff import RedWebFF, preprocess_input

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("fixed_schedules")]
TOL = 1e-3


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def make_rankings(rng, B, H, W, R, L):
    idx = rng.integers(0, H * W, (B, R, L))
    lab = rng.permutation(B * R * L).reshape(B, R, L) / (B * R * L)
    lab = -np.sort(-lab, axis=-1)
    return np.ascontiguousarray(np.stack([idx.astype(np.float32), lab.astype(np.float32)], -1))


STRUCTURAL_ZERO = {"aol/conv0/bias", "aol/conv1/bias", "aol/conv2/bias"}


@pytest.fixture(scope="module")
def step_results(cuda, fixed_schedules):
    B, H, R, L = 2, 128, 16, 5
    eng = RedWebFF((H, H, 3), B, seed=0)
    rng = np.random.default_rng(1)
    x01 = rng.random((B, H, H, 3)).astype(np.float32)
    x = preprocess_input(x01)
    weights = eng.get_weights()
    eng.act["input"].copy_(torch.from_numpy(x))
    pred = eng.forward(training=True)
    y = make_rankings(rng, B, H, H, R, L)
    loss, dpred, _ = K.listmle_fwd_bwd(pred, torch.from_numpy(y).to(cuda), B, R, L)
    eng.backward(dpred)
    torch.cuda.synchronize()
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    x64 = torch.tensor(x, dtype=torch.float64)
    taps = {}
    with torch.no_grad():
        pred_ref = OR.forward(P, x64, taps=taps, preprocessed=True)
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred_ref.numpy(), B, L)
    grads_ref, _ = OR.train_step_grads(P, x64, torch.tensor(dpred_ref), preprocessed=True)
    P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in weights.items()}
    grads_32, _ = OR.train_step_grads(P32, torch.tensor(x), torch.tensor(dpred_ref).float(),
                                      preprocessed=True)
    return dict(eng=eng, pred=pred, pred_ref=pred_ref, taps=taps, loss=loss.item(),
                loss_ref=loss_ref, grads_ref=grads_ref, grads_32=grads_32, dpred=dpred,
                dpred_ref=dpred_ref, weights=weights, x01=x01)


def test_parameter_names_match_oracle(step_results):
    eng = step_results["eng"]
    spec = {n: (s, k) for n, s, k in OR.param_specs()}
    mine = {}
    for store, kind in ((eng.params, "trainable"), (eng.frozen, "frozen"), (eng.stats, "stat")):
        for n, s, _ in store.specs:
            mine[n] = (tuple(s), kind)
    assert mine == spec
    assert eng.count_trainable() == 8647299
    assert abs(eng.conv_flops_per_image() - OR.conv_flops_per_image(eng.H, eng.W)) < 1.0


def test_preprocess_matches_oracle(step_results):
    x01 = step_results["x01"]
    ref = OR.caffe_preprocess(torch.tensor(x01, dtype=torch.float64)).numpy()
    np.testing.assert_allclose(preprocess_input(x01), ref, rtol=0, atol=1e-4)


def test_forward_activations(step_results):
    r = step_results
    eng, taps = r["eng"], r["taps"]
    for name in ["conv1_relu", "pool1_pool", "conv2_block1_out", "conv3_block4_out",
                 "conv4_block3_out", "conv5_block3_out", "ffl0", "ffl1"]:
        mine = eng.act[name if not name.startswith("ffl") else name + "/out"]
        e = rel(mine, taps[name].permute(0, 2, 3, 1))
        assert e < TOL, (name, e)
    assert rel(r["pred"], r["pred_ref"]) < TOL


def test_loss_and_dpred(step_results):
    r = step_results
    assert abs(r["loss"] - r["loss_ref"]) / abs(r["loss_ref"]) < TOL
    assert rel(r["dpred"], torch.tensor(r["dpred_ref"])) < TOL


def test_trainable_gradients(step_results):
    r = step_results
    eng, g64, g32 = r["eng"], r["grads_ref"], r["grads_32"]
    assert set(g64) == set(eng.params.names())
    keys = [k for k in g64 if k not in STRUCTURAL_ZERO]
    flat = lambda g: torch.cat([g[k].detach().double().cpu().flatten() for k in keys])
    a, b, c = flat({k: eng.grads[k] for k in keys}), flat(g64), flat(g32)
    err_gpu = float((a - b).norm() / b.norm())
    err_32 = float((c - b).norm() / b.norm())
    cos_gpu = float(a @ b / (a.norm() * b.norm()))
    print(f"GRAD global rel-L2: hip {err_gpu:.3e}  fp32-oracle {err_32:.3e}  cos {cos_gpu:.6f}")
    assert err_gpu <= 2.0 * err_32 + TOL
    assert cos_gpu > 0.995
    worst32 = max(rel(g32[k], g64[k]) for k in keys)
    for k in keys:
        assert rel(eng.grads[k], g64[k]) <= max(TOL, 2.0 * worst32), k
    scale = float(b.abs().max())
    for k in STRUCTURAL_ZERO:
        assert float(eng.grads[k].abs().max()) <= 1e-3 * scale + 1e-6, k


def test_inference_mode_uses_moving_statistics(step_results):
    eng = step_results["eng"]
    w = eng.get_weights()
    pred = eng.forward(training=False).clone()
    torch.cuda.synchronize()
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in w.items()}
    x64 = eng.act["input"].double().cpu()
    saved = OR.bn_train
    OR_mm = {}

    def bn_infer(x, gamma, beta, eps):
        name = OR_mm[(id(gamma))]
        mm = P[name + "/moving_mean"].view(1, -1, 1, 1)
        mv = P[name + "/moving_variance"].view(1, -1, 1, 1)
        return (x - mm) / torch.sqrt(mv + eps) * gamma.view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)

    for n in P:
        if n.endswith("/gamma"):
            OR_mm[id(P[n])] = n[:-len("/gamma")]
    OR.bn_train = bn_infer
    try:
        with torch.no_grad():
            ref = OR.forward(P, x64, preprocessed=True)
    finally:
        OR.bn_train = saved
    assert rel(pred, ref) < TOL


def test_trainer_step_runs_graph_captured(cuda):
    """One graph-captured ReplicaTrainer step on ff_redweb (GPU sampler -> fwd -> ListMLE ->
    bwd -> Adam) changes the trainable parameters and only them."""
    from pldepth_amd.trainer import ReplicaTrainer
    B, H = 2, 64
    tr = ReplicaTrainer((H, H, 3), B, 5, 20, 1, seed=0, model="ff_redweb")
    rng = np.random.default_rng(0)
    x = preprocess_input(rng.random((B, H, H, 3)).astype(np.float32))
    gt = rng.random((B, H, H)).astype(np.float32)
    tr.set_batch(torch.from_numpy(x), torch.from_numpy(gt), torch.ones(B, H, H))
    eng = tr.engine
    p0 = eng.params.buf.clone()
    f0 = eng.frozen.buf.clone()
    tr.step_eager(0.01)
    tr.capture()
    tr.step(0.01)
    tr.synchronize()
    assert np.isfinite(tr.loss_value())
    assert not torch.equal(p0, eng.params.buf)
    assert torch.equal(f0, eng.frozen.buf)
