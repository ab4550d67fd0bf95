"""Build libcacto_hip.so in-tree for gfx950 (hipcc; no cmake, no JIT cache).

    python -m cacto_amd.build          # or __graft_entry__.build()
"""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_obj")
LIB = os.path.join(HERE, "libcacto_hip.so")
ARCH = os.environ.get("CACTO_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=" + ARCH,
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
SOURCES = ["core.hip", "env_kernels.hip", "net_kernels.hip", "rollout_kernels.hip", "ddp_kernels.hip", "learn_kernels.hip", "replay_kernels.hip"]


def hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _deps_mtime():
    newest = 0.0
    for root in (CSRC, os.path.join(HERE, "..", "include")):
        for f in os.listdir(root):
            newest = max(newest, os.path.getmtime(os.path.join(root, f)))
    return newest


def _compile(src):
    obj = os.path.join(OBJ, src.replace(".hip", ".o"))
    cmd = [hipcc()] + FLAGS + ["-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed on %s:\n%s" % (src, r.stderr[-6000:]))
    return obj


def build_variant(name, defines):
    """A diagnostic build (e.g. in-kernel timestamps) into cacto_amd/<name>.so."""
    out = os.path.join(HERE, name + ".so")
    objs = []
    os.makedirs(OBJ, exist_ok=True)
    for src in SOURCES:
        obj = os.path.join(OBJ, name + "_" + src.replace(".hip", ".o"))
        cmd = [hipcc()] + FLAGS + ["-D" + d for d in defines] + ["-c", os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-4000:])
        objs.append(obj)
    r = subprocess.run([hipcc(), "--offload-arch=" + ARCH, "-shared", "-o", out] + objs, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-4000:])
    return out


def build(force=False, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _deps_mtime():
        if verbose:
            print("libcacto_hip.so up to date")
        return LIB
    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 4)) as ex:
        objs = list(ex.map(_compile, SOURCES))
    cmd = [hipcc(), "--offload-arch=" + ARCH, "-shared", "-o", LIB + ".tmp"] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stderr[-6000:])
    os.replace(LIB + ".tmp", LIB)
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
