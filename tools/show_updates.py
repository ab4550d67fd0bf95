"""Print the critic-updates/s entries of bench.py JSON lines: python tools/show_updates.py FILE..."""
import json
import sys

for fn in sys.argv[1:]:
    d = json.loads(open(fn).read().strip().splitlines()[-1])

    def walk(o, p=""):
        if isinstance(o, dict):
            for k, v in o.items():
                walk(v, p + "." + k)
        elif isinstance(o, (int, float)) and "critic_updates" in p and p.endswith(".value"):
            print(fn, p, round(o, 1))
    walk(d)
