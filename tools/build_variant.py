"""Build a variant of libdreamer_hip.so with extra compiler flags for kernel
A/B runs: python tools/build_variant.py NAME -DKNOB=1 ...  ->
tools/variants/libdreamer_hip_NAME.so, loaded when DREAMER_LIB_VARIANT=NAME."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dreamer_amd import build as B  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    obj = os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants", f"_build_{name}")
    os.makedirs(obj, exist_ok=True)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants", f"libdreamer_hip_{name}.so")

    def comp(src):
        o = os.path.join(obj, src.replace(".hip", ".o"))
        r = subprocess.run([B.HIPCC, *B.CFLAGS, *flags, "-c", os.path.join(B.CSRC, src), "-o", o],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return o

    with ThreadPoolExecutor(max_workers=len(B.SOURCES)) as ex:
        objs = list(ex.map(comp, B.SOURCES))
    r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr)
    print("built", out)


if __name__ == "__main__":
    main()
