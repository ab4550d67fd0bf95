"""Per-kernel register / scratch / LDS / occupancy table of one csrc/*.hip file, from the
compiler's kernel-resource-usage remarks (gfx950). Diagnostic only.
    python tools/resource_usage.py rollout_kernels.hip [name-filter]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cacto_amd.build import CSRC, FLAGS, hipcc  # noqa: E402


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "rollout_kernels.hip"
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    defines = ["-D" + d for d in sys.argv[3:]]
    cmd = [hipcc()] + FLAGS + defines + ["-c", os.path.join(CSRC, src), "-o", "/tmp/_ru.o",
                                         "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"LDS Size \[bytes/block\]|SGPRs): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1).split(" ")[0], m.group(2)
        if k == "Function":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    names = subprocess.run(["c++filt"], input="\n".join(r_["name"] for r_ in rows), capture_output=True,
                           text=True).stdout.splitlines()
    print("%-60s %5s %5s %7s %4s %7s" % ("kernel", "VGPR", "AGPR", "scratch", "occ", "LDS"))
    for r_, n in zip(rows, names):
        n = re.sub(r"\(.*", "", n).replace("cacto::", "")
        if filt and filt not in n:
            continue
        print("%-60s %5s %5s %7s %4s %7s" % (n[:60], r_.get("VGPRs"), r_.get("AGPRs"), r_.get("ScratchSize"),
                                              r_.get("Occupancy"), r_.get("LDS")))


if __name__ == "__main__":
    main()
