"""Print the compressed instruction sequence of a kernel's innermost loop from a hipcc --save-temps .s file.

    python tools/asm_loop.py <file.s> <kernel-name-substring> [max_chars]

M = MFMA, R = ds_read, W = ds_write, D = buffer/global load to LDS, G = global/buffer load to VGPRs, SCR = scratch,
|B| = s_barrier, w(...) = s_waitcnt, v = other VALU, . = runs of SALU. Used to check that hipcc kept the intended
MFMA / LDS / DMA interleave and did not spill or insert full waits inside the loop.
"""
import re
import sys


def main(path, name, width=1200):
    s = open(path).read()
    starts = [m.start() for m in re.finditer(r"^(_Z\S*%s\S*):" % re.escape(name), s, re.M)]
    if not starts:
        sys.exit(f"no kernel matching {name}")
    a = starts[0]
    b = s.index(".Lfunc_end", a)
    body = s[a:b].split("\n")
    print(body[0])
    heads = [i for i, l in enumerate(body) if "Loop Header" in l]
    labels = [i for i, l in enumerate(body) if re.match(r"^\.LBB\S*:", l)]
    for h in heads:
        # every basic block of the loop (hipcc rotates loops, so the header is not necessarily first): the header's
        # own block plus each block labelled "in Loop: Header=<this header>", in file order
        mh = re.match(r"^\.L(BB\S*):", body[h])
        if mh is None:
            continue
        hid = mh.group(1)
        blocks = []
        for j, li in enumerate(labels):
            if li == h or ("Header=%s " % hid) in body[li] + " ":
                end = labels[j + 1] if j + 1 < len(labels) else len(body)
                blocks.append((li, end))
        seq = []
        for a_, b_ in blocks:
            for l in body[a_:b_]:
                seq.append(_code(l))
        seq = [x for x in seq if x]
        out = re.sub(r"(\. )+", ". ", " ".join(seq))
        n = sum(b_ - a_ for a_, b_ in blocks)
        print(f"loop at line {h} ({n} lines, {len(blocks)} blocks, {seq.count('M')} MFMA, {seq.count('v')} VALU, "
              f"{seq.count('R')} ds_read): {out[:width]}\n")


def _code(l):
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        return None
    op = t.split()[0]
    if op.startswith("v_mfma"):
        return "M"
    if op.startswith("ds_read"):
        return "R"
    if op.startswith("ds_write"):
        return "W"
    if op.startswith(("buffer_load", "global_load")) and " lds" in t:
        return "D"
    if op.startswith(("buffer_load", "global_load")):
        return "G"
    if op.startswith("scratch"):
        return "SCR"
    if op == "s_barrier":
        return "|B|"
    if op == "s_waitcnt":
        return "w(" + t.split(None, 1)[1] + ")"
    if op.startswith("v_"):
        return "v"
    if op.startswith("s_"):
        return "."
    return op

if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1200)
