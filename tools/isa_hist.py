"""Opcode histogram of one kernel's loops in a gfx950 assembly listing (hipcc --save-temps .s).

    python tools/isa_hist.py <listing.s> <mangled kernel name> [--out DIR]

Writes DIR/<short>.s (the kernel's listing), DIR/<short>_loops.txt: for every natural loop (a
block labelled "Inner Loop Header" and the back-edge branch to it) its basic blocks, each with its
instruction count by class (VALU, SALU, LDS, VMEM load/store, SMEM, branch, DPP, f64, waitcnt),
and an opcode histogram of the whole loop body.  Blocks are listed in layout order with their
execution condition as the compiler wrote it (`s_cbranch_execz` skips, so a block behind one runs
only when some lane takes it).  Used for DESIGN.md §5's dynamics accounting.
"""
import collections
import os
import re
import sys


def classify(op: str, line: str) -> str:
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic")):
        return "vmem_store"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if "_dpp" in op or " quad_perm:" in line or " row_" in line:
            return "valu_dpp"
        if "f64" in op:
            return "valu_f64"
        if op.startswith(("v_mad_u64", "v_mad_i64")):
            return "valu_mad64"
        return "valu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "."
    os.makedirs(out, exist_ok=True)
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(lines)) if ".end_amdhsa_kernel" in lines[i])
    body = lines[start:end + 1]
    short = re.sub(r"[^A-Za-z0-9_]", "_", name)[-60:]
    open(os.path.join(out, short + ".s"), "w").write("\n".join(body) + "\n")

    # basic blocks: label lines ".LBBx_y:" and "; %bb.N:" comments start blocks; the compiler
    # annotates loop membership ("in Loop: Header=BBx_y Depth=d", the header "Inner Loop Header"),
    # on the label line or the comment line after it
    blocks, cur = [], None
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", l) or re.match(r"^; (%bb\.\d+):", l)
        if m:
            cur = {"label": m.group(1), "line": i, "ins": [], "note": l}
            blocks.append(cur)
            continue
        s = l.strip()
        if cur is None or not s:
            continue
        if s.startswith(";"):
            if not cur["ins"]:
                cur["note"] += " " + s
            continue
        if s.startswith("."):
            continue
        op = s.split()[0]
        cur["ins"].append((op, s))
    rep = []
    for k, b in enumerate(blocks):
        if "Loop Header" not in b["note"] or "Header=" in b["note"]:
            continue
        hdr = b["label"].lstrip(".")[1:]  # ".LBB68_103" -> "BB68_103"
        members = [j for j, bb in enumerate(blocks) if j == k or f"Header={hdr} " in bb["note"] + " "]
        hist = collections.Counter()
        cls_tot = collections.Counter()
        rep.append(f"=== loop {b['label']}: {len(members)} blocks, listing lines "
                   f"{blocks[members[0]]['line']}..{blocks[members[-1]]['line']}")
        for j in members:
            bb = blocks[j]
            cls = collections.Counter(classify(o, s) for o, s in bb["ins"])
            cls_tot.update(cls)
            hist.update(o for o, _ in bb["ins"])
            gate = ""
            for o, s in blocks[j - 1]["ins"] if j > 0 else []:
                if o.startswith("s_cbranch"):
                    gate = f"  [after {o} -> {s.split()[-1]}]"
            rep.append(f"  {bb['label']:<12} {len(bb['ins']):4d} ins  " +
                       " ".join(f"{c}={n}" for c, n in sorted(cls.items())) + gate)
        rep.append("  total: " + " ".join(f"{c}={n}" for c, n in sorted(cls_tot.items())) +
                   f"  ({sum(cls_tot.values())} instructions)")
        rep.append("  opcodes: " + ", ".join(f"{o} {n}" for o, n in hist.most_common()))
        rep.append("")
    txt = "\n".join(rep)
    open(os.path.join(out, short + "_loops.txt"), "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
