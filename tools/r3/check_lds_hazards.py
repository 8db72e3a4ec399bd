"""Static check of hipcc output: no instruction may read a VGPR that an LDS read (ds_read*) has not yet delivered.

LDS reads complete in issue order and decrement lgkmcnt; ``s_waitcnt lgkmcnt(N)`` retires all but the N youngest.
Inline-asm reads hand their destination registers to the compiler as if already written, so a use hoisted above
its wait reads stale data. This walks each kernel's straight-line code (labels reset nothing: the check is
checked within each basic block; block boundaries reset it) and reports every use of a register that is still the
destination of an outstanding LDS read. Usage: check_lds_hazards.py <file.s> [kernel-substring ...]"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def op_is_branch(s):
    return s.startswith("s_cbranch") or s.startswith("s_branch") or s.startswith("s_setpc")


def check(lines, name):
    pend = []  # [(dest regs)] oldest first
    bad = 0
    for ln, line in lines:
        s = line.split(";")[0].strip()
        if s.endswith(":") or op_is_branch(s):
            pend = []  # basic-block boundary: the compiler orders waits across blocks itself
            continue
        if not s or s.startswith("."):
            continue
        op, _, rest = s.partition(" ")
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", rest)
            if m:
                keep = int(m.group(1))
                pend = pend[len(pend) - keep:] if keep < len(pend) else pend
            continue
        if op.startswith("s_"):
            continue
        args = [a.strip() for a in rest.split(",")]
        if op.startswith("ds_read") or op.startswith("ds_bpermute"):
            srcs = regs(",".join(args[1:]))
            hit = srcs & set().union(*pend) if pend else set()
            if hit:
                bad += 1
                print(f"{name}:{ln}: {s}   <- address reg(s) {sorted(hit)} not yet delivered")
            pend.append(regs(args[0]))
            continue
        if op.startswith("ds_"):
            continue
        if not pend:
            continue
        live = set().union(*pend)
        # sources: everything but the first operand (dest) -- MFMA / VALU / VMEM alike
        srcs = regs(",".join(args[1:]))
        hit = srcs & live
        if hit:
            bad += 1
            print(f"{name}:{ln}: {s}   <- reg(s) {sorted(hit)} still in flight from an LDS read")
        # a write to an in-flight destination is a WAW hazard as well
        dst = regs(args[0]) if args else set()
        if dst & live and not op.startswith("v_mfma"):
            bad += 1
            print(f"{name}:{ln}: {s}   <- overwrites reg(s) {sorted(dst & live)} of an outstanding LDS read")
    return bad


def main():
    path = sys.argv[1]
    subs = sys.argv[2:]
    text = open(path).read().splitlines()
    total = 0
    cur, body = None, []
    for i, line in enumerate(text, 1):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            if cur and (not subs or any(x in cur for x in subs)):
                total += check(body, cur[:60])
            cur, body = m.group(1), []
            continue
        if cur:
            body.append((i, line))
            if "s_endpgm" in line:
                if not subs or any(x in cur for x in subs):
                    total += check(body, cur[:60])
                cur, body = None, []
    print(f"hazards: {total}")
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
