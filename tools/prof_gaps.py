"""Gaps between consecutive learner kernels of a rocpd kernel trace (the timed update loop):
median kernel duration and median idle gap before each kernel kind, over the last N dispatches.

    python tools/prof_gaps.py gpurun_out/prof_r03/t128/run_results.db [N]
"""
import re
import sqlite3
import statistics
import sys

db = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
rows = sqlite3.connect(db).cursor().execute("select name, start, end from kernels order by start").fetchall()
learn = [r for r in rows if re.search(r"k_chain_pair|k_wgrad|k_critic_grad|k_actor_grad|k_adam|k_per_", r[0])][-N:]


def kind(n):
    m = re.match(r"(?:void )?(?:cacto::)?([\w]+)", n)
    return m.group(1) if m else n[:40]


dur, gap = {}, {}
for i, (n, s, e) in enumerate(learn):
    dur.setdefault(kind(n), []).append(e - s)
    if i:
        gap.setdefault(kind(learn[i - 1][0]) + " -> " + kind(n), []).append(s - learn[i - 1][2])
for k, v in sorted(dur.items()):
    print("kernel %-28s n=%5d median %.2f us" % (k, len(v), statistics.median(v) / 1e3))
for k, v in sorted(gap.items()):
    print("gap    %-44s n=%5d median %.2f us" % (k, len(v), statistics.median(v) / 1e3))
