"""Build libxpgnn.so for gfx950 in-tree:  python -m bikg_graph_explainability_public_amd.build"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "xpgnn.hip")
OUT = os.path.join(HERE, "libxpgnn.so")
ARCH = os.environ.get("XPG_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"),
              shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def build(force=False, verbose=True):
    deps = [SRC, os.path.join(HERE, "csrc", "khop.hip"), os.path.join(HERE, "csrc", "host_rng.h"),
            os.path.join(HERE, "csrc", "plan_host.h"),
            os.path.join(os.path.dirname(HERE), "include", "xpgnn.h")]
    if not force and os.path.exists(OUT) and \
            all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    # -fno-slp-vectorize: SLP pairs independent per-row/column chains into packed fp32 ops and
    # keeps both halves live (the grid surrogate kernels spill; no kernel here gains from it)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fno-slp-vectorize", "-fPIC",
           "-shared", "-Wall", "-o", OUT + ".tmp", SRC]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
