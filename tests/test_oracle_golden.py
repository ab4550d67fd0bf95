"""Pin the CPU oracle against golden vectors made by importing the reference itself
(tests/golden/make_ref_vectors.py) and against the .h5 weight fixtures."""
import random

import numpy as np
import pytest

from conftest import load_weights
from oracle import buffer as obuf
from oracle import env as oenv
from cacto_amd.confs import load_conf


def _tree(cap, idx, vals):
    st, mt = obuf.SumSegmentTree(cap), obuf.MinSegmentTree(cap)
    for i, v in zip(idx, vals):
        st[int(i)] = float(v)
        mt[int(i)] = float(v)
    return st, mt


@pytest.mark.parametrize("cap", [16, 65536])
def test_segment_tree_bit_exact(ref_vectors, cap):
    g = {k[len("st%d_" % cap):]: v for k, v in ref_vectors.items() if k.startswith("st%d_" % cap)}
    st, mt = _tree(cap, g["idx"], g["vals"])
    assert st.sum() == g["total"][0] and mt.min() == g["total"][1]
    assert [st.find_prefixsum_idx(float(p)) for p in g["ps"]] == list(g["found"])
    assert [st.sum(0, int(e)) for e in g["ends"]] == list(g["prefix"])
    assert [st.sum(int(a), int(b)) for a, b in g["ranges"]] == list(g["rsum"])
    assert [mt.min(int(a), int(b)) for a, b in g["ranges"]] == list(g["rmin"])


def test_per_stratified_sampling_bit_exact(ref_vectors):
    leaves = ref_vectors["per_leaves"]
    per = obuf.PrioritizedReplayBuffer(65536, 3, 0.6, 0.6, 1e-2, 0.95, 64)
    for i, v in enumerate(leaves):
        per.it_sum[i] = float(v)
    per.next_idx = len(leaves)
    assert per.it_sum.sum(0, len(leaves) - 1) == ref_vectors["per_ptotal"][0]
    idx = per.sample_proportional(list(ref_vectors["per_u"]))
    np.testing.assert_array_equal(idx, ref_vectors["per_idx"])


def test_replay_buffer_add_wrap_gather(ref_vectors):
    rb = obuf.ReplayBuffer(64, 5)
    rows = ref_vectors["rb_adds"]
    off = 0
    for L in ref_vectors["rb_eplens"]:
        rb.add_rows(rows[off:off + L])
        off += L
    np.testing.assert_array_equal(rb.storage, ref_vectors["rb_storage"])
    assert [rb.next_idx, rb.full] == list(ref_vectors["rb_next_full"])
    s, r, sn, dvdx, d, term = rb.gather(ref_vectors["rb_sidx"])
    for name, got in zip(["s", "r", "sn", "dvdx", "d", "term"], [s, r, sn, dvdx, d, term]):
        np.testing.assert_array_equal(got, ref_vectors["rb_sample_" + name])
        assert got.dtype == ref_vectors["rb_sample_" + name].dtype


@pytest.mark.parametrize("system", ["single_integrator", "double_integrator"])
def test_reset_bit_exact(ref_vectors, system):
    conf = load_conf(system)
    env = oenv.make_env(conf)
    rng = random.Random(0)
    got = np.asarray([env.reset(rng) for _ in range(200)])
    np.testing.assert_array_equal(got, ref_vectors[system[:1] + "i_reset"])


def test_si_env_bit_exact(ref_vectors):
    conf = load_conf("single_integrator")
    env = oenv.make_env(conf)
    S, A, W = ref_vectors["si_S"], ref_vectors["si_A"], ref_vectors["si_W"]
    np.testing.assert_array_equal([env.reward(w, s, a) for w, s, a in zip(W, S, A)],
                                  ref_vectors["si_reward"])
    np.testing.assert_array_equal([env.reward(w, s) for w, s in zip(W, S)],
                                  ref_vectors["si_reward_noa"])
    np.testing.assert_array_equal([env.simulate(s, a) for s, a in zip(S, A)], ref_vectors["si_sim"])
    np.testing.assert_array_equal([env.simulate(s, a) for s, a in
                                   zip(S.astype(np.float32), A.astype(np.float32))],
                                  ref_vectors["si_sim32"])
    np.testing.assert_array_equal([env.derivative(s, a) for s, a in zip(S, A)], ref_vectors["si_der"])
    np.testing.assert_array_equal([env.get_end_effector_position(s) for s in S], ref_vectors["si_ee"])


def test_di_reward_bit_exact(ref_vectors):
    conf = load_conf("double_integrator")
    env = oenv.make_env(conf)
    S, A, W = ref_vectors["di_S"], ref_vectors["di_A"], ref_vectors["si_W"]
    np.testing.assert_array_equal([env.reward(w, s, a) for w, s, a in zip(W, S, A)],
                                  ref_vectors["di_reward"])
    np.testing.assert_array_equal([env.reward(w, s) for w, s in zip(W, S.astype(np.float32))],
                                  ref_vectors["di_reward32"])


@pytest.mark.parametrize("system,tag", [("car", "car"), ("car_park", "cp")])
def test_car_envs_bit_exact(ref_vectors, system, tag):
    """Car / CarPark against the reference classes (environment.py:364-652) imported with a TF
    scalar stub that keeps TF's operand casting (tests/golden/make_ref_vectors.py)."""
    conf = load_conf(system)
    env = oenv.make_env(conf)
    S, A, W = ref_vectors[tag + "_S"], ref_vectors[tag + "_A"], ref_vectors[tag + "_W"]
    S32, A32 = S.astype(np.float32), A.astype(np.float32)
    np.testing.assert_array_equal([env.simulate(s, a) for s, a in zip(S, A)], ref_vectors[tag + "_sim"])
    np.testing.assert_array_equal([env.simulate(s, a) for s, a in zip(S32, A32)], ref_vectors[tag + "_sim32"])
    np.testing.assert_array_equal([env.derivative(s, a) for s, a in zip(S, A)], ref_vectors[tag + "_der"])
    np.testing.assert_array_equal([env.get_end_effector_position(s) for s in S], ref_vectors[tag + "_ee"])
    # CarPark.obs_cost_fun's `term**(-1/2)` runs through numpy's SIMD (SVML) pow on AVX-512 hosts, which
    # is not correctly rounded and differs between numpy builds (1.26 vs 2.x here): few-ulp agreement.
    # With a float32 state it also rotates the check points with numpy's float32 np.cos/np.sin (SIMD,
    # build-dependent): float32-level agreement there. Under the generating numpy (1.26) both are
    # bit-exact (checked when the vectors were made).
    if tag == "car":
        cmp64 = cmp32 = np.testing.assert_array_equal
    else:
        cmp64 = lambda a, b: np.testing.assert_allclose(a, b, rtol=1e-13, atol=1e-16)
        cmp32 = lambda a, b: np.testing.assert_allclose(a, b, rtol=1e-7, atol=1e-12)
    cmp64([env.reward(w, s, a) for w, s, a in zip(W, S, A)], ref_vectors[tag + "_reward"])
    cmp32([env.reward(w, s) for w, s in zip(W, S32)], ref_vectors[tag + "_reward32"])
    if tag == "cp":   # the obstacle term is exercised
        assert np.ptp(ref_vectors[tag + "_reward"]) > 1e-3


def test_rl_solve_bit_exact(ref_vectors):
    p, t, sn, d, term = obuf.rl_solve(ref_vectors["rls_states"], ref_vectors["rls_cost"], 25)
    np.testing.assert_array_equal(p, ref_vectors["rls_partial"])
    np.testing.assert_array_equal(t, ref_vectors["rls_total"])
    np.testing.assert_array_equal(sn, ref_vectors["rls_snext"])
    np.testing.assert_array_equal(d, ref_vectors["rls_done"])
    np.testing.assert_array_equal(term, ref_vectors["rls_term"])


def test_weight_fixtures_shapes_and_identities():
    """Layer shapes match SURVEY §8 and target_critic_0 == critic_0 (RL.py:99)."""
    w = load_weights("di_seed0_0")
    assert [a.shape for a in w["actor"]] == [(5, 256), (256,), (256, 256), (256,), (256, 2), (2,)]
    assert sum(a.size for a in w["actor"]) == 67842
    assert sum(a.size for a in w["critic"]) == 29505
    for a, b in zip(w["critic"], w["target"]):
        np.testing.assert_array_equal(a, b)
    # Keras init: zero actor biases (glorot kernels), SIREN kernels within sqrt(6/fan_in)
    for b in w["actor"][1::2]:
        assert not b.any()
    for k, fan_in in zip(w["critic"][0:8:2], [5, 64, 64, 128]):
        assert np.abs(k).max() <= np.sqrt(6.0 / fan_in) + 1e-6


@pytest.mark.parametrize("system", ["single_integrator", "double_integrator"])
def test_product_env_reset_bit_exact(ref_vectors, system):
    """cacto_amd.environment.Env.reset itself (host CPython `random`, environment.py:46-55) against
    the reference's own draws after random.seed(0). reset touches only self.conf, so it runs here
    without the device handle the rest of Env needs."""
    import types
    from cacto_amd.environment import Env
    conf = load_conf(system)
    env = types.SimpleNamespace(conf=conf)
    random.seed(0)
    got = np.asarray([Env.reset(env) for _ in range(200)])
    np.testing.assert_array_equal(got, ref_vectors[system[:1] + "i_reset"])
