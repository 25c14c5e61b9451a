"""Build tools/kbench/kbench (links dreamer_amd/_build/*.o except engine)."""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from dreamer_amd import build as B  # noqa: E402

B.build(verbose=False)
# gemm / gru are rebuilt with phase timestamps (-DDR_PHASE_TIMING)
objs = [o for o in glob.glob(os.path.join(ROOT, "dreamer_amd", "_build", "*.o"))
        if os.path.basename(o) not in ("gemm.o", "gru.o")]
for src in ("gemm", "gru"):
    o = os.path.join(HERE, src + "_ts.o")
    extra = os.environ.get("KB_DEFS", "").split()
    r = subprocess.run([B.HIPCC, *B.CFLAGS, "-DDR_PHASE_TIMING", *extra, "-c", os.path.join(B.CSRC, src + ".hip"), "-o", o],
                       capture_output=True, text=True)
    if r.returncode:
        print(r.stdout, r.stderr)
        sys.exit(1)
    objs.append(o)
obj = os.path.join(HERE, "kbench.o")
for cmd in ([B.HIPCC, *B.CFLAGS, "-c", os.path.join(HERE, "kbench.hip"), "-o", obj],
            [B.HIPCC, f"--offload-arch={B.ARCH}", obj, *objs, "-o", os.path.join(HERE, os.environ.get("KB_OUT", "kbench"))]):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        print(r.stdout, r.stderr)
        sys.exit(1)
print("built", os.path.join(HERE, "kbench"))
