#!/usr/bin/env python3
"""VGPR / SGPR / spill / scratch / LDS of the kernels in a built object's gfx950 code object
(from the AMDGPU metadata notes), for checking register allocation after a change.

    python tools/kernel_resources.py build/lbsim/step.o [name-regex]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(obj: str, tmp: str) -> str:
    fat = os.path.join(tmp, "fatbin.bin")
    co = os.path.join(tmp, "gfx950.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def kernels(co: str):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                           text=True, check=True).stdout
    out, cur = [], None
    for line in notes.splitlines():
        if re.match(r"\s+- \.agpr_count", line):
            cur = {}
            out.append(cur)
        m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"private_segment_fixed_size|group_segment_fixed_size):\s+(\S+)", line)
        if m and cur is not None and m.group(1) not in cur:
            cur[m.group(1)] = m.group(2)
    return out


def main():
    obj = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    with tempfile.TemporaryDirectory() as tmp:
        for k in kernels(code_object(obj, tmp)):
            name = subprocess.run(["c++filt", k.get("name", "?")], capture_output=True,
                                  text=True).stdout.strip()
            name = name.replace("(anonymous namespace)::", "").replace("lbk::", "")
            name = re.sub(r"\(.*", "", name).replace("void ", "")
            if pat and not pat.search(name):
                continue
            print(f"{name:70s} vgpr {k.get('vgpr_count'):>4} spill {k.get('vgpr_spill_count'):>4} "
                  f"sgpr_spill {k.get('sgpr_spill_count', '0'):>4} scratch "
                  f"{k.get('private_segment_fixed_size'):>4} lds {k.get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
