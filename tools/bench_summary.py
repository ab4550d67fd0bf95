"""Print the headline figures of a bench.py JSON line: python tools/bench_summary.py FILE"""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("DI rollout %.1f M env-steps/s  k_rollout %.3f ms  frac %.3f" % (d["value"] / 1e6, r["kernel_ms"], r["frac"]))
if d.get("long_region"):
    lr = d["long_region"]
    print("  long region: %d batches, %.2f s, median %.1f M/s, spread %.3f" % (lr["batches"], lr["seconds"],
                                                                             lr["median"] / 1e6, lr["spread"]))
for k, v in d["critic_updates"].items():
    print("  DI %s: %.0f updates/s (%.1f us) mfma %.3f" % (k, v["value"], v["ms_per_update"] * 1e3, v["mfma_frac"]))
for s, e in (d.get("extra_systems") or {}).items():
    print("%s rollout %.1f M/s frac %.3f ddp %.2f ms; " % (s, e["env_steps_per_s"] / 1e6, e["rollout_mfma_frac"],
                                                           e["ddp_labels"]["ms_per_call"]) +
          ", ".join("%s %.0f/s (mfma %.3f)" % (k, v["value"], v["mfma_frac"]) for k, v in e["critic_updates"].items()))
if d.get("config0"):
    print("config0", json.dumps(d["config0"].get("gpu")), d["config0"].get("speedup_vs_cpu"))
