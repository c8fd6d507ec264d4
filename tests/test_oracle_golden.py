"""CPU: the oracle (oracle/) pinned against the reference's own outputs (tests/golden/)."""
import hashlib

import numpy as np
import pytest

import oracle
from oracle import ppo_ref as R


def _cases(g):
    names = sorted({k.split("/")[0] for k in g.files})
    for n in names:
        yield n, {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith(n + "/")}


def test_gae_c_oracle_bit_exact(golden):
    g = golden("gae.npz")
    n = 0
    for name, c in _cases(g):
        boot = None if "no_boot" in c else c["bootstrap"]
        a, r = oracle.gae_c(c["values"], c["rewards"], c["dones"], c["timeouts"], c["last_values"], boot,
                            float(c["gamma"]), float(c["lam"]))
        assert np.array_equal(a.view(np.uint32), c["adv"].view(np.uint32)), name
        assert np.array_equal(r.view(np.uint32), c["ret"].view(np.uint32)), name
        n += 1
    assert n == 11


def test_gae_numpy_oracle_bit_exact(golden):
    for name, c in _cases(golden("gae.npz")):
        boot = None if "no_boot" in c else c["bootstrap"]
        a, r = R.gae_numpy(c["values"], c["rewards"], c["dones"], c["timeouts"], c["last_values"], boot,
                           float(c["gamma"]), float(c["lam"]))
        assert np.array_equal(a.view(np.uint32), c["adv"].view(np.uint32)), name


def test_gae_constants_follow_numpy_weak_scalars():
    # c2 = f32(gamma*lambda in double), not f32(gamma)*f32(lambda) (SURVEY.md §7 hard part c)
    assert np.float32(0.98 * 0.8) != np.float32(0.98) * np.float32(0.8)


def test_sampler_oracle_bit_exact(golden):
    s = golden("sampler.npz")
    for ep in range(4):
        assert np.array_equal(oracle.sampler_stream(256, 20, 42 + ep), s[f"n256_p20_e{ep}"])
    assert np.array_equal(oracle.sampler_stream(7, 2, 42), s["n7_p2_e0"])
    assert np.array_equal(oracle.sampler_stream(1, 5, 42), s["n1_p5_e0"])
    big = oracle.sampler_stream(131072, 2, 42)
    assert np.array_equal(big[:4096], s["n131072_p2_e0/head"])
    assert hashlib.sha256(big.tobytes()).digest() == bytes(s["n131072_p2_e0/sha256"])


@pytest.mark.parametrize("tag", ["cartpole", "lunar_ent"])
def test_ppo_numpy_oracle_vs_reference_step(golden, tag):
    z = golden("ppo_step.npz")
    D, H1, H2, A, B = (int(x) for x in z[f"{tag}/dims"])
    clip, cvf, vf, ent, lr = (float(x) for x in z[f"{tag}/hparams"])
    dims = (D, H1, H2, A)
    loss, met, g = R.ppo_loss_and_grads(z[f"{tag}/params0"], dims, z[f"{tag}/obs"], z[f"{tag}/actions"],
                                        z[f"{tag}/old_logprobs"], z[f"{tag}/old_values"], z[f"{tag}/advantages"],
                                        z[f"{tag}/returns"], clip=clip, clip_vf=cvf, vf_coef=vf, ent_coef=ent)
    assert abs(loss - float(z[f"{tag}/loss"])) < 1e-6
    np.testing.assert_allclose(g, z[f"{tag}/grads_raw"], atol=1e-6, rtol=0)
    gc, total = R.clip_grad_norm(g, dims, 0.5)
    assert abs(total - float(z[f"{tag}/total_norm"])) < 1e-6
    np.testing.assert_allclose(gc, z[f"{tag}/grads_clipped"], atol=1e-6, rtol=0)
    p1, _, _ = R.adam_step(z[f"{tag}/params0"], gc, np.zeros_like(gc), np.zeros_like(gc), 1, lr)
    np.testing.assert_allclose(p1, z[f"{tag}/params1"], atol=1e-6, rtol=0)
    ref = dict(zip([str(x) for x in z[f"{tag}/metric_names"]], z[f"{tag}/metric_values"]))
    for k, v in ref.items():
        assert abs(met[k] - v) < 1e-5, k


def test_masked_categorical_known_answers():
    # tests/test_masked_categorical.py of the reference: uniform over 3 valid -> log 3
    logits = np.zeros((1, 5), np.float32)
    valid = np.array([True, True, True, False, False])
    z = np.where(valid, logits, -np.inf)
    ln = R.log_softmax(z)
    p = np.exp(ln)
    H = -(p * np.where(valid, np.log(p + 1e-8), 0)).sum()
    assert abs(H - np.log(3)) < 1e-5
    assert abs(ln[0, 0] + np.log(3)) < 1e-6


@pytest.mark.parametrize("tag", ["pong", "breakout"])
def test_cnn_oracle_vs_reference_step(golden, tag):
    """oracle/cnn_ref.py (torch-CPU restatement) against the reference's CNNActorCritic +
    losses_for_batch + clip_grad_norm_ + Adam on the same deterministic case."""
    from oracle import cnn_case as K, cnn_ref as C
    z = golden("cnn_step.npz")
    valid, clip, ent, lr, B, pseed, bseed = {"pong": ([0, 3, 4], 0.2, 0.01, 3e-4, 48, 1, 3),
                                             "breakout": ([0, 1, 3, 4], 0.1, 0.01, 3e-4, 40, 2, 5)}[tag]
    shapes = C.cnn_param_shapes()
    p0 = K.cnn_params(pseed)
    loss, met, g, logits, values = C.loss_and_grads(p0, shapes, *K.cnn_batch(bseed, B, valid), valid=valid, clip=clip,
                                                    clip_vf=0.2, vf_coef=0.5, ent_coef=ent)
    assert abs(loss - float(z[f"{tag}/loss"])) < 1e-5 * max(1.0, abs(loss))
    fin = np.isfinite(z[f"{tag}/logits"])
    assert np.array_equal(fin, np.isfinite(logits))
    import torch
    ln = (torch.as_tensor(logits) - torch.logsumexp(torch.as_tensor(logits), -1, keepdim=True)).numpy()
    np.testing.assert_allclose(ln[fin], z[f"{tag}/logits"][fin], atol=1e-5, rtol=0)   # Categorical.logits
    np.testing.assert_allclose(values, z[f"{tag}/values"], atol=1e-5, rtol=0)
    norms, o = [], 0
    for _, s in shapes:
        k = int(np.prod(s))
        norms.append(np.linalg.norm(g[o:o + k].astype(np.float64)))
        o += k
    np.testing.assert_allclose(norms, z[f"{tag}/tensor_norms"], rtol=1e-4, atol=1e-7)
    sel = z[f"{tag}/sel"]
    gmax = np.abs(g).max()
    np.testing.assert_allclose(g[sel], z[f"{tag}/grads_sel"], atol=1e-5 * gmax, rtol=0)
    P = p0.size
    p1, _, _, _, total = C.clip_and_adam(p0, g, shapes, np.zeros(P, np.float32), np.zeros(P, np.float32), 1, lr)
    # torch-CPU clip_grad_norm_ accumulates the 1.6M-element mlp.0.weight norm in fp32 (~3e-5
    # relative off the exact norm of its own per-tensor norms, which match ours to 1e-7 above)
    assert abs(total - float(z[f"{tag}/total_norm"])) < 1e-4 * total
    np.testing.assert_allclose(p1[sel], z[f"{tag}/params1_sel"], atol=2e-6, rtol=0)
    ref = dict(zip([str(x) for x in z[f"{tag}/metric_names"]], z[f"{tag}/metric_values"]))
    for k, v in met.items():
        if k in ref:
            assert abs(v - ref[k]) < 1e-4 * max(1.0, abs(v)), k


def test_atari_oracle_known_answers():
    """OpenCV RGB2GRAY known answers and box-filter invariants of oracle/atari_ref.py."""
    from oracle import atari_ref as A
    px = np.array([[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0]], np.uint8)
    assert A.gray(px).tolist() == [76, 150, 29, 255, 0]
    for n_out, n_in in ((84, 210), (84, 160)):
        starts, w, sc = A.area_tables(n_out, n_in)
        for ws in w:
            assert abs(sum(float(x) for x in ws) - sc) < 1e-6 and len(ws) <= 4
    const = np.full((2, 2, 210, 160, 3), 200, np.uint8)
    g = A.gray(const[0, 0, :1, :1])[0, 0]
    assert (A.preprocess(const) == g).all()          # a flat image stays flat
    fr = A.render(42, [0, 1], 5)
    assert fr.shape == (2, 2, 210, 160, 3) and fr.std() > 50
    out = A.preprocess(fr)
    assert out.shape == (2, 84, 84) and out.dtype == np.uint8
    env = A.AtariEnvTwin(3, episode_len=4)
    assert (env.stack[:, :3] == 0).all()
    for _ in range(5):
        r, d, _ = env.step()
        assert r.min() >= -1 and r.max() < 1


@pytest.mark.parametrize("case", ["normal", "offset", "skewed", "constant", "single"])
def test_rollout_adv_norm_oracle_vs_reference(golden, case):
    """oracle/ppo_ref.py normalize_advantages_rollout and its written-out model (numpy_f32_sum: the
    steps gs_normalize_advantages takes on the device) against the reference's own
    _normalize_advantages outputs (adv_norm.npz), bit for bit."""
    from oracle.ppo_ref import normalize_advantages_model, normalize_advantages_rollout
    z = golden("adv_norm.npz")
    a, want = z[f"{case}/in"], z[f"{case}/out"]
    for f in (normalize_advantages_rollout, normalize_advantages_model):
        assert np.array_equal(f(a).view(np.uint32), want.view(np.uint32)), f.__name__


def test_numpy_f32_sum_model_matches_numpy():
    """The device's summation model (numpy's float32 pairwise sums over 8192-element buffer chunks)
    equals np.add.reduce bit for bit, at sizes around every boundary of the model (8, 128, the
    chunk) and at the C2 / C3 rollout sizes, on data with a large common offset (where the order of
    the additions shows in the result)."""
    from oracle.ppo_ref import numpy_f32_sum
    rng = np.random.default_rng(0)
    for n in (1, 7, 8, 9, 127, 128, 129, 136, 143, 255, 257, 1000, 8191, 8192, 8193, 20001, 131072, 2 ** 21 + 5):
        a = (rng.standard_normal(n) * 3.0 + 100.0).astype(np.float32)
        assert numpy_f32_sum(a) == np.add.reduce(a), n


def test_adv_norm_model_above_2_24_matches_numpy():
    """Above 2^24 elements the count is not a float32: numpy divides the float32 sums by it in
    float64 (_mean / _var: float32 / np.intp), and so must the model the device kernel follows
    (gs_gae.hip np_div_count) — bit for bit against normalize_advantages_rollout."""
    from oracle.ppo_ref import normalize_advantages_model, normalize_advantages_rollout
    a = (np.random.default_rng(5).standard_normal((4097, 4096)) * 1.5 + 4.0).astype(np.float32)
    assert a.size > 2 ** 24
    assert np.array_equal(normalize_advantages_model(a).view(np.uint32), normalize_advantages_rollout(a).view(np.uint32))


@pytest.mark.parametrize("tag", ["cartpole", "lunar_ent"])
def test_activation_stats_oracle_vs_reference(golden, tag):
    """oracle/ppo_ref.py activation_stats against the reference's forward-hook values recorded on
    the same batch (ppo_step.npz activation_names / values: utils/models.py:121-147 on backbone.0 /
    backbone.2): mean / std within 1e-6 relative, dead fractions exact."""
    from oracle import ppo_ref as R
    z = golden("ppo_step.npz")
    D, H1, H2, A, B = (int(x) for x in z[f"{tag}/dims"])
    got = R.activation_stats(z[f"{tag}/params0"], (D, H1, H2, A), z[f"{tag}/obs"])
    ref = dict(zip([str(x) for x in z[f"{tag}/activation_names"]], z[f"{tag}/activation_values"]))
    for li, layer in enumerate(("backbone.0", "backbone.2")):
        for ki, k in enumerate(("mean", "std", "dead_pct", "dead_max")):
            want = ref[f"opt/activations/{layer}/{k}"]
            if ki >= 2:
                assert got[4 * li + ki] == want, (layer, k)
            else:
                np.testing.assert_allclose(got[4 * li + ki], want, rtol=1e-6, atol=1e-9, err_msg=f"{layer}/{k}")
