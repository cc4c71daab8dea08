"""Build liblbsim.so in-tree for gfx950 (hipcc).  `python -m marllb_amd.build [--force]`.

One translation unit (csrc/lbsim_api.hip includes the kernels).  -ffp-contract=off is part of
the numerical contract: no FMA contraction, so integer state and every
observation column are bit-reproducible against oracle/.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "lbsim_api.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in sorted(os.listdir(os.path.join(HERE, "csrc")))]
DEPS.append(os.path.join(ROOT, "include", "lbsim.h"))
OUT = os.path.join(HERE, "liblbsim.so")
ARCH = os.environ.get("LBSIM_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-Wall",
         f"--offload-arch={ARCH}"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build_library(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return OUT
    cmd = [hipcc(), *FLAGS, "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
