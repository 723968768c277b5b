"""Wait-state lint for the inline-asm MFMAs of a kernel (hipcc pads nothing inside `asm` and only one state after it).

For every `v_mfma_*` between `;;#ASMSTART` / `;;#ASMEND` in a hipcc `--save-temps` .s file it checks, in program order
inside the basic block:
  * before: no VALU / v_accvgpr instruction writing one of the MFMA's source registers (A, B, C) within the 2 issue
    states in front of it (VALU write -> MFMA read);
  * after: no instruction other than an MFMA that accumulates into exactly the same registers reads or writes the
    MFMA's destination within 16 states after it (MFMA result -> reader / writer), s_nop N counting N + 1 states.
It prints each violation with its line and exits 1 if any; the counts are conservative (an intervening MFMA counts
as one state although it holds the issue for 8+ cycles).

    python tools/check_mfma_asm_hazards.py /tmp/asm/flash_attn-hip-amdgcn-amd-amdhsa-gfx950.s attn_bwd_dq_w4
"""
import re
import sys

REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            k, lo, hi = m.group(3), int(m.group(4)), int(m.group(5))
            out.update((k, i) for i in range(lo, hi + 1))
    return out


def parse(line):
    line = line.split(";")[0].strip()
    if not line or line.endswith(":") or line.startswith("."):
        return None
    op, _, rest = line.partition(" ")
    ops = [o.strip() for o in rest.split(",")] if rest else []
    return op, ops


def states(op, ops):
    if op == "s_nop":
        return int(ops[0], 0) + 1
    return 1


def main(path, name):
    text = open(path).read().split("\n")
    starts = [i for i, l in enumerate(text) if re.match(r"^(_Z\S*%s\S*):" % re.escape(name), l)]
    bad = 0
    for s in starts:
        e = next(i for i in range(s, len(text)) if text[i].startswith(".Lfunc_end"))
        body = []
        in_asm = False
        for i in range(s, e):
            l = text[i]
            if ";;#ASMSTART" in l:
                in_asm = True
                continue
            if ";;#ASMEND" in l:
                in_asm = False
                continue
            if re.match(r"^\.LBB|^\S+:", l):
                body.append(("LABEL", i, None, None))
                continue
            p = parse(l)
            if p:
                body.append((p[0], i, p[1], in_asm))
        for k, (op, ln, ops, asm) in enumerate(body):
            if not (asm and op and op.startswith("v_mfma")):
                continue
            dst = regs(ops[0])
            srcs = regs(",".join(ops[1:]))
            # before: VALU writes of the sources within 2 states
            st = 0
            for j in range(k - 1, -1, -1):
                op2, ln2, ops2, asm2 = body[j]
                if op2 == "LABEL":
                    break
                if (op2.startswith("v_") and not op2.startswith("v_mfma")) and ops2 and regs(ops2[0]) & srcs:
                    print(f"{path}:{ln + 1}: VALU write {text[ln2].strip()} -> asm MFMA source read ({st} states)")
                    bad += 1
                st += states(op2, ops2)
                if st >= 2:
                    break
            # after: readers / writers of dst within 16 states
            st = 0
            for j in range(k + 1, len(body)):
                op2, ln2, ops2, asm2 = body[j]
                if op2 == "LABEL":
                    break
                if op2.startswith("v_mfma") and ops2 and regs(ops2[0]) == dst and regs(ops2[-1]) == dst:
                    break  # the next MFMA of the same accumulation chain: interlocked
                if ops2 and (regs(",".join(ops2)) & dst):
                    print(f"{path}:{ln + 1}: asm MFMA result -> {text[ln2].strip()} after {st} states")
                    bad += 1
                    break
                st += states(op2, ops2)
                if st >= 16:
                    break
    print(f"{bad} violation(s) in kernels matching {name}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
