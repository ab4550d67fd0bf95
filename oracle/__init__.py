"""CPU ORACLE — test infrastructure only.

A float64 numpy restatement of the reference's hot path (nadimkanazi/cacto @ /root/reference),
used ONLY by `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg, as the
checker / CPU baseline. The product path (`cacto_amd`) never imports it.

Each function cites the reference file:line it restates. Where the reference computes in float32
(TF ops, `tf.convert_to_tensor(..., tf.float32)`) the oracle says so and rounds at the same points.

Pinning:
  * segment tree / PER indices   — bit-exact against golden vectors produced by importing the
                                   reference's `segment_tree.py` (tests/golden/make_ref_vectors.py);
  * replay buffer add/wrap/gather — golden vectors from the reference `ReplayBuffer` under a TF
                                   stub module (same script);
  * SI / car / car_park env       — golden vectors from the reference env classes under TF and
                                   Pinocchio stubs (same script);
  * DI / manipulator dynamics     — Pinocchio is absent: pinned analytically (DI: M = I, nle = 0;
                                   manipulator: independent sympy Lagrangian, tests/test_oracle_*)
                                   and by the DI final-policy known-answer test against the figure
                                   `PolicyEvaluationSingleInit_6_51000.png`;
  * actor / critic / Sobolev / Adam — TF/Keras/tf_siren are absent: restated from the formulas,
                                   checked by finite differences and pinned by the .h5 weight
                                   fixtures (tests/golden/weights). Keras-Adam numerics beyond the
                                   formula are "parity unpinned" (DESIGN.md).
"""
