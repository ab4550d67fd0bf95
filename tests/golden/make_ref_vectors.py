"""Generate golden vectors by importing the reference's own Python modules from /root/reference.

Run in THIS container (the reference is not on the GPU box) with the numpy-1.x interpreter, so the
reference's numpy-1.24 scalar-promotion semantics hold:

    /opt/conda/bin/python3.9 -B tests/golden/make_ref_vectors.py

TensorFlow, Pinocchio and CasADi are absent, so small stub modules (written below, into a temp dir)
stand in for the few names the imported modules touch at import time:
  * `tensorflow`: convert_to_tensor -> np.asarray (only used by the buffer's sample path),
    keras.losses placeholder;
  * `pinocchio` / `pinocchio.casadi` / `robot_utils` (DI conf only): a RobotWrapper whose model is
    the double-integrator of urdf/double_integrator.urdf (two prismatic joints X, Y; EE at (q0,q1,0)).
Only functions whose arithmetic is plain Python/numpy are recorded (segment trees, ring buffer,
Env.reset, SI/DI rewards, SI simulate/derivative, RL_Solve). Output: tests/golden/ref_vectors.npz.
"""
import json
import os
import random
import sys

sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference tree
import tempfile
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_vectors.npz")


def install_stubs():
    tf = types.ModuleType("tensorflow")
    tf.float32 = np.float32
    tf.float64 = np.float64
    tf.convert_to_tensor = lambda x, dtype=None: np.asarray(x, dtype=dtype)
    tf.is_tensor = lambda x: False
    keras = types.ModuleType("tensorflow.keras")
    losses = types.SimpleNamespace(MeanSquaredError=lambda *a, **k: None,
                                   Reduction=types.SimpleNamespace(NONE=None))
    keras.losses = losses
    keras.layers = types.SimpleNamespace()
    keras.regularizers = types.SimpleNamespace()
    tf.keras = keras
    tf.function = lambda f: f

    class TFScalar:
        """Eager TF scalar: the other operand is converted to THIS tensor's dtype (no numpy
        promotion), as tf.convert_to_tensor(x, dtype=y.dtype) does in TF binary ops."""

        def __init__(self, v, dt):
            self.dt = dt
            self.v = dt(v)

        def _o(self, x):
            return self.dt(x.v if isinstance(x, TFScalar) else x)

        def __mul__(self, x): return TFScalar(self.v * self._o(x), self.dt)
        __rmul__ = __mul__
        def __add__(self, x): return TFScalar(self.v + self._o(x), self.dt)
        def __radd__(self, x): return TFScalar(self._o(x) + self.v, self.dt)
        def __truediv__(self, x): return TFScalar(self.v / self._o(x), self.dt)
        def __float__(self): return float(self.v)

    def _trig(fn):
        def f(x):
            dt = np.float32 if isinstance(x, np.float32) else np.float64
            return TFScalar(fn(float(x)), dt)   # libm cos/sin, rounded to the tensor dtype
        return f
    import math as _m
    tf.cos, tf.sin = _trig(_m.cos), _trig(_m.sin)
    sys.modules["tensorflow"] = tf
    sys.modules["tensorflow.keras"] = keras

    class Placement:
        def __init__(self, t):
            self.translation = t

    class Model:
        nq = nv = 2
        effortLimit = np.array([100.0, 100.0])

        def getFrameId(self, name):
            assert name == "EE"
            return 0

        def createData(self):
            return None

    class Robot:
        nq = nv = na = 2

        def __init__(self):
            self.model = Model()

        @staticmethod
        def BuildFromURDF(path, pkgs=None):
            assert path.endswith("double_integrator.urdf"), path
            return Robot()

        def framePlacement(self, q, frame, recompute=True):
            t = np.zeros(3)
            t[0], t[1] = q[0], q[1]
            return Placement(t)

    pin = types.ModuleType("pinocchio")
    cpin = types.ModuleType("pinocchio.casadi")
    cpin.Model = lambda m: m
    pin.casadi = cpin
    sys.modules["pinocchio"] = pin
    sys.modules["pinocchio.casadi"] = cpin
    ru = types.ModuleType("robot_utils")
    ru.RobotWrapper = Robot
    ru.RobotSimulator = lambda *a, **k: None
    sys.modules["robot_utils"] = ru


def main():
    install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)   # robot confs resolve URDFs relative to cwd (conf_double_integrator.py:158)
    import segment_tree
    import replay_buffer
    import environment
    import conf_single_integrator as csi
    import conf_double_integrator as cdi
    import RL
    import conf_car as ccar
    import conf_car_park as ccp
    os.chdir(cwd)

    out = {}
    rng = np.random.RandomState(1234)

    # ---- segment trees (segment_tree.py) ----
    for cap in (16, 65536):
        st = segment_tree.SumSegmentTree(cap)
        mt = segment_tree.MinSegmentTree(cap)
        n = 11 if cap == 16 else 5000
        idx = rng.choice(cap, size=n, replace=False) if cap > 16 else np.arange(n)
        vals = rng.uniform(0.01, 3.0, size=n) ** 0.6
        for i, v in zip(idx, vals):
            st[int(i)] = float(v)
            mt[int(i)] = float(v)
        total = st.sum()
        # prefix sums incl. exact node-boundary values and the top end
        ps = list(rng.uniform(0, total, size=400 if cap > 16 else 40))
        ps += [0.0, total, total + 5e-6, st._value[2], st._value[4]]
        found = [st.find_prefixsum_idx(float(p)) for p in ps]
        ends = list(range(2, min(cap, 4096), 7 if cap > 16 else 1)) + [cap]
        prefix = [st.sum(0, e) for e in ends]
        ranges = [(int(a), int(b)) for a, b in rng.randint(0, cap, size=(60, 2)) if a < b - 1]
        rsum = [st.sum(a, b) for a, b in ranges]
        rmin = [mt.min(a, b) for a, b in ranges]
        k = "st%d_" % cap
        out[k + "idx"] = np.asarray(idx, dtype=np.int64)
        out[k + "vals"] = np.asarray(vals)
        out[k + "ps"] = np.asarray(ps)
        out[k + "found"] = np.asarray(found, dtype=np.int64)
        out[k + "ends"] = np.asarray(ends, dtype=np.int64)
        out[k + "prefix"] = np.asarray(prefix)
        out[k + "ranges"] = np.asarray(ranges, dtype=np.int64)
        out[k + "rsum"] = np.asarray(rsum)
        out[k + "rmin"] = np.asarray(rmin)
        out[k + "total"] = np.asarray([total, mt.min()])

    # ---- stratified proportional sampling on the reference tree (replay_buffer.py:139-157) ----
    cap = 65536
    st = segment_tree.SumSegmentTree(cap)
    max_idx = 3000
    leaves = rng.uniform(0.05, 2.0, size=max_idx) ** 0.6
    for i, v in enumerate(leaves):
        st[i] = float(v)
    B = 64
    pyrng = random.Random(7)
    u = [pyrng.random() for _ in range(B)]
    p_total = st.sum(0, max_idx - 1)
    seg = p_total / B
    per_idx = [st.find_prefixsum_idx(uu * seg + i * seg) for i, uu in enumerate(u)]
    out["per_leaves"] = leaves
    out["per_u"] = np.asarray(u)
    out["per_idx"] = np.asarray(per_idx, dtype=np.int64)
    out["per_ptotal"] = np.asarray([p_total, st.sum()])

    # ---- ReplayBuffer add/wrap/sample (replay_buffer.py:9-83) ----
    conf = types.SimpleNamespace(REPLAY_SIZE=64, nb_state=5, BATCH_SIZE=16)
    rb = replay_buffer.ReplayBuffer(conf)
    ep_lens = [20, 30, 25, 17]
    adds = []
    for L in ep_lens:
        ep = [rng.normal(size=(L, 5)), rng.normal(size=L), rng.normal(size=(L, 5)),
              rng.normal(size=(L, 5)), (rng.uniform(size=L) < .3).astype(float),
              np.eye(1, L, L - 1)[0]]
        adds.append(ep)
        rb.add(*[[e] for e in ep])
    np.random.seed(99)
    sample = rb.sample()
    np.random.seed(99)
    sidx = np.random.randint(0, 64 if rb.full else rb.next_idx, size=16)
    out["rb_storage"] = rb.storage_mat.copy()
    out["rb_next_full"] = np.asarray([rb.next_idx, rb.full])
    out["rb_eplens"] = np.asarray(ep_lens)
    out["rb_adds"] = np.concatenate([np.concatenate([e[0], e[1][:, None], e[2], e[3], e[4][:, None],
                                                     e[5][:, None]], axis=1) for e in adds])
    out["rb_sidx"] = sidx
    for name, arr in zip(["s", "r", "sn", "dvdx", "d", "term", "w"], sample[:7]):
        out["rb_sample_" + name] = np.asarray(arr)

    # ---- Env.reset with random.seed(0) (environment.py:46-55) ----
    for tag, c, cls in (("si", csi, environment.SingleIntegrator),
                        ("di", cdi, environment.DoubleIntegrator)):
        env = cls(c)
        random.seed(0)
        out[tag + "_reset"] = np.asarray([env.reset() for _ in range(200)])

    # ---- rewards / dynamics ----
    si = environment.SingleIntegrator(csi)
    di = environment.DoubleIntegrator(cdi)
    n = 300
    S = np.column_stack([rng.uniform(-16, 16, size=(n, 2)), rng.uniform(0, 5, size=n)])
    S[:20, :2] = rng.uniform(-8, -6, size=(20, 2))       # near the target (peak term active)
    S[20:40, :2] = np.array([-2.0, 0.0]) + rng.normal(scale=.5, size=(20, 2))  # inside ellipse 1
    A = rng.uniform(-7, 7, size=(n, 2))
    W = np.where(rng.uniform(size=(n, 1)) < .5, csi.cost_weights_running, csi.cost_weights_terminal)
    out["si_S"], out["si_A"], out["si_W"] = S, A, W
    out["si_reward"] = np.asarray([si.reward(w, s, a) for w, s, a in zip(W, S, A)])
    out["si_reward_noa"] = np.asarray([si.reward(w, s) for w, s in zip(W, S)])
    out["si_sim"] = np.asarray([si.simulate(s, a) for s, a in zip(S, A)])
    S32, A32 = S.astype(np.float32), A.astype(np.float32)
    out["si_sim32"] = np.asarray([si.simulate(s, a) for s, a in zip(S32, A32)])
    out["si_der"] = np.asarray([si.derivative(s, a) for s, a in zip(S, A)])
    out["si_ee"] = np.asarray([si.get_end_effector_position(s) for s in S])
    SD = np.column_stack([S[:, :2], rng.uniform(-6, 6, size=(n, 2)), S[:, 2]])
    AD = rng.uniform(-2.5, 2.5, size=(n, 2))
    out["di_S"], out["di_A"] = SD, AD
    out["di_reward"] = np.asarray([di.reward(w, s, a) for w, s, a in zip(W, SD, AD)])
    out["di_reward32"] = np.asarray([di.reward(w, s) for w, s in zip(W, SD.astype(np.float32))])

    # ---- car / car_park (environment.py:364-652) ----
    car, cpk = environment.Car(ccar), environment.CarPark(ccp)
    n = 200
    for tag, env, c in (("car", car, ccar), ("cp", cpk, ccp)):
        lo, hi = np.asarray(c.x_init_min, float), np.asarray(c.x_init_max, float)
        S = lo + (hi - lo) * rng.uniform(size=(n, 6))
        S[:, 3] = rng.uniform(-5, 5, size=n)
        S[:, 4] = rng.uniform(-0.5, 0.5, size=n)
        if tag == "cp":
            S[:, 1] = rng.uniform(-1.0, 7.5, size=n)   # reach the boxes' edges
        A = rng.uniform(-1, 1, size=(n, 2)) * c.u_max
        Wc = np.where(rng.uniform(size=(n, 1)) < .5, c.cost_weights_running, c.cost_weights_terminal)
        S32, A32 = S.astype(np.float32), A.astype(np.float32)
        out[tag + "_S"], out[tag + "_A"], out[tag + "_W"] = S, A, Wc
        out[tag + "_sim"] = np.asarray([env.simulate(s, a) for s, a in zip(S, A)])
        out[tag + "_sim32"] = np.asarray([env.simulate(s, a) for s, a in zip(S32, A32)])
        out[tag + "_der"] = np.asarray([env.derivative(s, a) for s, a in zip(S, A)])
        out[tag + "_ee"] = np.asarray([env.get_end_effector_position(s) for s in S])
        out[tag + "_reward"] = np.asarray([env.reward(w, s, a) for w, s, a in zip(Wc, S, A)])
        out[tag + "_reward32"] = np.asarray([env.reward(w, s) for w, s in zip(Wc, S32)])

    # ---- RL_Solve n-step targets (RL.py:145-189) ----
    rl = RL.RL_AC(si, None, csi, 0)
    T = 37
    rl.NSTEPS_SH = T
    states = rng.normal(size=(T + 1, 3))
    cost = rng.uniform(0, 2, size=T + 1)
    res = rl.RL_Solve(np.zeros((T, 2)), states, cost)
    out["rls_states"], out["rls_cost"] = states, cost
    out["rls_partial"], out["rls_total"], out["rls_snext"] = res[1], res[2], res[3]
    out["rls_done"], out["rls_term"] = res[4], res[6]

    np.savez_compressed(OUT, **out)
    meta = {"numpy": np.__version__, "python": sys.version.split()[0], "keys": sorted(out)}
    with open(OUT.replace(".npz", ".json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", OUT, len(out), "arrays")


if __name__ == "__main__":
    main()
