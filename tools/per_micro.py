"""PER kernels alone (no concurrent chains): sample + priority update at B on a full 2^16-row tree,
timed per call with HIP events on the library's stream. Prints one line per phase (us per call).

    python tools/per_micro.py [B] [iters]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cacto_amd import _lib as L
from cacto_amd.system import dptr, stream

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cap = 1 << 16
rng = np.random.default_rng(0)
leaves = rng.uniform(0.01, 2.0, size=cap) ** 0.6
st, mt = np.zeros(2 * cap), np.full(2 * cap, np.inf)
st[cap:], mt[cap:] = leaves, leaves
lo = cap // 2
while lo >= 1:
    k = np.arange(lo, 2 * lo)
    st[k] = st[2 * k] + st[2 * k + 1]
    mt[k] = np.minimum(mt[2 * k], mt[2 * k + 1])
    lo //= 2
sd, md = torch.as_tensor(st, device="cuda"), torch.as_tensor(mt, device="cuda")
cnt = torch.zeros(cap, dtype=torch.float64, device="cuda")
maxp = torch.ones(1, dtype=torch.float64, device="cuda")
U = torch.as_tensor(rng.uniform(size=(iters, B)), device="cuda")
y = torch.as_tensor(rng.normal(size=B).astype(np.float32), device="cuda")
V = torch.as_tensor(rng.normal(size=B).astype(np.float32), device="cuda")
idx = torch.empty(B, dtype=torch.int32, device="cuda")
w = torch.empty(B, dtype=torch.float32, device="cuda")
s = stream()


def sample(i):
    L.lib().call("cacto_per_sample", dptr(sd), dptr(md), cap, cap, 0.6, dptr(U[i]), B, dptr(idx), dptr(w), dptr(cnt), s)


def update():
    L.lib().call("cacto_per_update", dptr(sd), dptr(md), cap, dptr(idx), dptr(y), dptr(V), dptr(cnt), 0.95, 1e-2, 0.6,
                 dptr(maxp), B, s)


def timed(fn, name):
    for i in range(5):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    print("%-20s B=%d: %.1f us per call" % (name, B, e0.elapsed_time(e1) * 1e3 / iters), flush=True)


timed(lambda i: sample(i), "sample")
timed(lambda i: update(), "update")
timed(lambda i: (sample(i), update()), "sample+update")
