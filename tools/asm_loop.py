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
    for h in heads:
        end = next((i for i in range(h + 1, len(body)) if "s_cbranch" in body[i] and ".LBB" in body[i] and
                    body[i].split()[-1] + ":" == body[h].split()[0]), None)
        if end is None:
            end = next(i for i in range(h + 1, len(body)) if "s_cbranch" in body[i])
        seq = []
        for l in body[h:end + 1]:
            t = l.strip()
            if not t or t.startswith(";") or t.startswith("."):
                continue
            op = t.split()[0]
            if op.startswith("v_mfma"):
                op = "M"
            elif op.startswith("ds_read"):
                op = "R"
            elif op.startswith("ds_write"):
                op = "W"
            elif op.startswith(("buffer_load", "global_load")) and " lds" in t:
                op = "D"
            elif op.startswith(("buffer_load", "global_load")):
                op = "G"
            elif op.startswith("scratch"):
                op = "SCR"
            elif op == "s_barrier":
                op = "|B|"
            elif op == "s_waitcnt":
                op = "w(" + t.split(None, 1)[1] + ")"
            elif op.startswith("v_"):
                op = "v"
            elif op.startswith("s_"):
                op = "."
            seq.append(op)
        out = re.sub(r"(\. )+", ". ", " ".join(seq))
        print(f"loop at line {h} ({end - h} lines): {out[:width]}\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1200)
