"""Build libdreamer_hip.so for gfx950 in-tree (``python -m dreamer_amd.build``).

hipcc cross-compiles without a GPU, so this runs in the build container and
the resulting .so travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libdreamer_hip.so")
SOURCES = ["scan.hip", "dream.hip", "bptt.hip", "gemm.hip", "conv.hip", "conv_bf16.hip", "conv_split.hip", "conv_glds.hip", "wmconv.hip", "gru.hip", "ops.hip", "engine.hip", "wm.hip", "act.hip"]
ARCH = os.environ.get("DREAMER_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
    "-ffp-contract=off",            # parity: no fma contraction in elementwise code
    "-fno-gpu-rdc", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
]


def _compile(src):
    obj = os.path.join(OBJ, src.replace(".hip", ".o"))
    srcp = os.path.join(CSRC, src)
    deps = [srcp] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "dreamer_hip.h"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(p) for p in deps):
        return obj
    cmd = [HIPCC, *CFLAGS, "-c", srcp, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(o) for o in objs):
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
