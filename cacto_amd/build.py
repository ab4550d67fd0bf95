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


def build_variant(name, defines, force=True, verbose=False):
    """Another build of the library with extra defines into cacto_amd/<name>.so: diagnostic builds
    (in-kernel timestamps) and the sine-elu critic build (VARIANTS)."""
    out = os.path.join(HERE, name + ".so")
    if not force and os.path.exists(out) and os.path.getmtime(out) >= _deps_mtime():
        return out
    os.makedirs(OBJ, exist_ok=True)

    def one(src):
        obj = os.path.join(OBJ, name + "_" + src.replace(".hip", ".o"))
        cmd = [hipcc()] + FLAGS + ["-D" + d for d in defines] + ["-c", os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-4000:])
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 4)) as ex:
        objs = list(ex.map(one, SOURCES))
    r = subprocess.run([hipcc(), "--offload-arch=" + ARCH, "-shared", "-o", out + ".tmp"] + objs, capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-4000:])
    os.replace(out + ".tmp", out)
    if verbose:
        print("built", out)
    return out


# library variants built beside libcacto_hip.so: critic_type 'sine-elu' (NeuralNetwork.py:80-93) has
# its elu layers compiled in only here, so the default (sine) build's chain kernels carry no branch
VARIANTS = {"libcacto_hip_sine_elu": ["CACTO_CRITIC_ELU"]}


def build(force=False, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _deps_mtime():
        if verbose:
            print("libcacto_hip.so up to date")
        build_variants(verbose=verbose)
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
    build_variants(verbose=verbose)
    return LIB


def build_variants(force=False, verbose=True):
    for name, defines in VARIANTS.items():
        build_variant(name, defines, force=force, verbose=verbose)


if __name__ == "__main__":
    build(force="--force" in sys.argv)
