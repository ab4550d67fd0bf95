"""Convert the reference's Keras-2.11 .h5 checkpoints into small .npz weight fixtures.

Run with the interpreter that has h5py (this container: /opt/conda/bin/python3.9):

    /opt/conda/bin/python3.9 -B tests/golden/make_h5_fixtures.py

Only the tensors are read (h5py datasets; nothing is executed from the files). The layer order
is the Keras `trainable_variables` order the reference's optimizers iterate over
(NeuralNetwork.py:51-63 actor, :95-108 sine critic): kernel, bias per layer; kernels are [in, out].
Sources: `Results Double Integrator/Results set test/NNs/N_try_{0,6}` (seed 0, w_S=0.01) and
`Results Single Integrator/Results set test/NNs/N_try_{0,5}` (seeds 0 and 10).
"""
import os
import sys

sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference tree

import h5py
import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "weights")

ACTOR_LAYERS = ["dense", "dense_1", "dense_2"]
CRITIC_LAYERS = ["sinusodial_representation_dense", "sinusodial_representation_dense_1",
                 "sinusodial_representation_dense_2", "sinusodial_representation_dense_3", "dense_3"]


def read(path):
    """Return the list [kernel0, bias0, kernel1, bias1, ...] in model layer order."""
    with h5py.File(path, "r") as f:
        names = [n.decode() if isinstance(n, bytes) else str(n) for n in f.attrs["layer_names"]]
        out = []
        for n in names:
            g = f[n]
            if n not in g:
                continue  # input / activation layers carry no weights
            sub = g[n]
            out.append(np.asarray(sub["kernel:0"], dtype=np.float32))
            out.append(np.asarray(sub["bias:0"], dtype=np.float32))
        return out


def save(tag, files):
    os.makedirs(OUT, exist_ok=True)
    arrays = {}
    for key, path in files.items():
        for i, a in enumerate(read(path)):
            arrays["%s_%d" % (key, i)] = a
    np.savez_compressed(os.path.join(OUT, tag + ".npz"), **arrays)
    print(tag, {k: v.shape for k, v in arrays.items()})


def main():
    di = os.path.join(REF, "Results Double Integrator/Results set test/NNs/N_try_6")
    si = os.path.join(REF, "Results Single Integrator/Results set test/NNs")
    save("di_seed0_0", {"actor": os.path.join(di, "actor_0.h5"),
                        "critic": os.path.join(di, "critic_0.h5"),
                        "target": os.path.join(di, "target_critic_0.h5")})
    save("di_seed0_final", {"actor": os.path.join(di, "actor_final.h5"),
                            "critic": os.path.join(di, "critic_final.h5"),
                            "target": os.path.join(di, "target_critic_final.h5")})
    save("si_seed0_0", {"actor": os.path.join(si, "N_try_0/actor_0.h5"),
                        "critic": os.path.join(si, "N_try_0/critic_0.h5"),
                        "target": os.path.join(si, "N_try_0/target_critic_0.h5")})
    save("si_seed10_0", {"actor": os.path.join(si, "N_try_5/actor_0.h5"),
                         "critic": os.path.join(si, "N_try_5/critic_0.h5")})
    return 0


if __name__ == "__main__":
    sys.exit(main())
