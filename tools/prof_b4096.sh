# kernel trace of the DI update loop at B = 128 and manipulator B = 64 (paired single-stream pipeline)
set -e
export TMPDIR=/tmp
D=gpurun_out/prof_b4096
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o run -- python3 bench.py --steps 5 --warmup 2 --update-steps 500 --batches 4096 --extra-systems= --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0 > $D/b.json 2> $D/b.err
python3 tools/prof_summary.py stats $D/t/run_results.db > $D/stats.csv
python3 - <<'PY'
import sqlite3
cur = sqlite3.connect("gpurun_out/prof_b4096/t/run_results.db").cursor()
rows = cur.execute("select name, start, end from kernels order by start").fetchall()
# gaps between consecutive update kernels in the timed loop (last 300 dispatches of the chain/fused pair)
sel = [r for r in rows if "k_wgrad" in r[0]][-600:]
import statistics
d = {}
for i in range(1, len(sel)):
    key = ("pair" if "pair" in sel[i-1][0] else "fused") + "->" + ("pair" if "pair" in sel[i][0] else "fused")
    d.setdefault(key, []).append(sel[i][1] - sel[i-1][2])
for k, v in d.items():
    print("gap", k, "median ns", statistics.median(v))
PY
