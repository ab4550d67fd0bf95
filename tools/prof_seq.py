"""Kernel sequence of a rocpd database: python tools/prof_seq.py DB [start] [count]."""
import re
import sqlite3
import sys

db = sys.argv[1]
start = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else 50
rows = sqlite3.connect(db).cursor().execute("select name, duration from kernels order by start").fetchall()
for k, (n, d) in enumerate(rows[start:start + count], start):
    m = re.match(r"(?:void )?(?:cacto::)?([\w:<>\-]+?)\(", n)
    print(k, m.group(1) if m else n[:60], round(d / 1000, 2))
