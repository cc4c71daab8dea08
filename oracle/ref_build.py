"""Compile the reference's own C reservoir twin into oracle/_ref/ (gitignored, travels as a .so).

The header is compiled where it lies under /root/reference; only our 20-line driver
(oracle/ref_driver.c) is in this repo.  Runs only where /root/reference exists (build container).
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REF_HEADER = ("/root/reference/simulation-mode/problem-01-reservoir-sampling/src/reservoir.h")
OUT_DIR = os.path.join(HERE, "_ref")
OUT = os.path.join(OUT_DIR, "libref_reservoir.so")


def build_reference(header: str = REF_HEADER) -> str:
    if not os.path.exists(header):
        raise FileNotFoundError(header)
    os.makedirs(OUT_DIR, exist_ok=True)
    src = os.path.join(HERE, "ref_driver.c")
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(src),
                                                             os.path.getmtime(header)):
        return OUT
    subprocess.run(["gcc", "-O2", "-std=gnu99", "-fPIC", "-shared",
                    f'-DREF_RESERVOIR_H="{header}"', "-o", OUT, src, "-lm"], check=True)
    return OUT


if __name__ == "__main__":
    print(build_reference())
