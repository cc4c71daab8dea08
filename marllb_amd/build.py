"""Build liblbsim.so in-tree for gfx950 (hipcc).  `python -m marllb_amd.build [--force]`.

Several translation units (csrc/*.hip, see csrc/lbsim_internal.h) compiled in parallel to objects
under build/, then linked into marllb_amd/liblbsim.so.  -ffp-contract=off is part of the
numerical contract: no FMA contraction, so integer state and every observation
column are bit-reproducible against oracle/.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJDIR = os.path.join(ROOT, "build", "lbsim")
DEPS = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))]
DEPS.append(os.path.join(ROOT, "include", "lbsim.h"))
OUT = os.path.join(HERE, "liblbsim.so")
ARCH = os.environ.get("LBSIM_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-Wall", f"--offload-arch={ARCH}"]
# (source, extra defines, object name)
UNITS = [
    ("lbsim_api.hip", [], "api.o"),
    ("lbsim_dyn.hip", ["-DLBSIM_DYN_MODE=0"], "dyn_step.o"),
    ("lbsim_dyn.hip", ["-DLBSIM_DYN_MODE=1"], "dyn_reset.o"),
    ("lbsim_dyn.hip", ["-DLBSIM_DYN_MODE=2"], "dyn_step_nr.o"),
    ("lbsim_obs.hip", [], "obs.o"),
    ("lbsim_pol.hip", [], "pol.o"),
    ("lbsim_step.hip", [], "step.o"),
]


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


def _compile(unit, verbose: bool) -> str:
    src, defs, out = unit
    cmd = [hipcc(), *FLAGS, *defs, "-c", "-o", out + ".tmp", os.path.join(CSRC, src)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_library(force: bool = False, verbose: bool = False, jobs: int = 0,
                  variant: str | None = None, defines: tuple = (), only: tuple = ()) -> str:
    """Build liblbsim.so, or with `variant` an A/B build with extra `defines` into
    marllb_amd/exp/liblbsim_<variant>.so (loaded through LBSIM_LIBRARY, see _lib.py).  `only`
    (object names, e.g. "dyn_step.o"): compile just those units (a variant's own, or the main
    build's when no variant is named) and link the main build's objects for the rest."""
    out, objdir = OUT, OBJDIR
    if variant:
        out = os.path.join(HERE, "exp", f"liblbsim_{variant}.so")
        objdir = os.path.join(ROOT, "build", f"lbsim_{variant}")
    elif not force and not only and up_to_date():
        return OUT
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    jobs = jobs or min(len(UNITS), os.cpu_count() or 1, 16)
    units = [(src, [*defs, *defines], os.path.join(objdir, obj)) for src, defs, obj in UNITS
             if not only or obj in only]
    with ThreadPoolExecutor(jobs) as ex:
        built = dict(zip([u[2] for u in units], ex.map(lambda u: _compile(u, verbose), units)))
    objs = [built.get(os.path.join(objdir, obj), os.path.join(OBJDIR, obj)) for _, _, obj in UNITS]
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    variant = args[args.index("--variant") + 1] if "--variant" in args else None
    defines = tuple(a for a in args if a.startswith("-D"))
    only = tuple(args[args.index("--only") + 1].split(",")) if "--only" in args else ()
    print(build_library(force="--force" in args, verbose=True, variant=variant, defines=defines,
                        only=only))
