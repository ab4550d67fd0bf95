"""Phase stamps of the multi-workgroup PER sampler (diagnostic build, s_memtime of thread 0 of each
workgroup): staging + batch scalars, LDS descent, tail (global levels + leaf), IS weight. Standalone,
B = 4096 on a full 2^16 tree; prints the mean ticks per phase over the workgroups of the last call.

    python -c "from cacto_amd import build; build.build_variant('libcacto_diag', ['CACTO_STAMPS'])"
    CACTO_HIP_LIB=cacto_amd/libcacto_diag.so [CACTO_PER_TOP=4096] python tools/per_stamps.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cacto_amd import _lib as L  # noqa: E402
from cacto_amd.system import dptr, stream  # noqa: E402

B, cap = 4096, 1 << 16
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
idx = torch.empty(B, dtype=torch.int32, device="cuda")
w = torch.empty(B, dtype=torch.float32, device="cuda")
acc = np.zeros(4)
sub = np.zeros(3)
n = 0
for it in range(50):
    u = torch.as_tensor(rng.uniform(size=B), device="cuda")
    L.lib().call("cacto_per_sample", dptr(sd), dptr(md), cap, cap, 0.6, dptr(u), B, dptr(idx), dptr(w), None, stream())
    torch.cuda.synchronize()
    if it < 10:
        continue
    buf = (ctypes.c_ulonglong * (64 * 8))()
    L.lib().call("cacto_debug_per_stamps", buf)
    s = np.array(buf[:], dtype=np.int64).reshape(64, 8)[: B // 256]
    acc += np.diff(s[:, :5], axis=1).mean(axis=0)
    sub += (s[:, [5, 6, 7]] - s[:, [0]]).mean(axis=0)
    tot = s[:, 4].max() - s[:, 0].min()
    n += 1
print("per workgroup (mean ticks): stage+scalars %.0f, LDS descent %.0f, tail %.0f, IS weight %.0f" % tuple(acc / n))
print("thread 0 from start: walk done %.0f, staged top in LDS %.0f, segment formed %.0f" % tuple(sub / n))
