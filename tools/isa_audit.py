"""ISA audit for kernels that issue inline-asm vector loads (the compiler neither counts nor waits for them): along
the text of each kernel, model the in-order vector-memory queue (every buffer / global load and store joins it; an
`s_waitcnt vmcnt(k)` retires all but the k youngest) and report any instruction other than a load that reads or
writes a VGPR an outstanding inline-asm load (between ;;#ASMSTART / ;;#ASMEND) still has to write -- the compiler
waits for its own loads itself.  Straight-line model: branches are followed in text order,
which is what the unrolled K loops of these kernels are.

usage: isa_audit.py file.s [kernel-substring ...]   (exit 1 on a finding)"""
import re
import sys


def _regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def audit(asm_text, kernel):
    """Findings (line, instruction, registers) for one kernel's symbol in an assembly listing."""
    i = asm_text.index(kernel + ":")
    body = [ln.strip() for ln in asm_text[i:asm_text.index(".Lfunc_end", i)].split("\n")]
    queue, found, in_asm = [], [], False
    for n, ln in enumerate(body):
        if ln.startswith(";;#ASMSTART"):
            in_asm = True
        elif ln.startswith(";;#ASMEND"):
            in_asm = False
        if not ln or ln.startswith((";", ".")):
            continue
        op = ln.split()[0]
        ops = [t.strip(",") for t in ln.split()[1:]]
        if op.startswith("s_waitcnt"):
            m = re.search(r"vmcnt\((\d+)\)", ln)
            if m:
                del queue[:max(0, len(queue) - int(m.group(1)))]
            continue
        pending = set().union(*(r for _, r in queue)) if queue else set()
        used = set().union(*(_regs(t) for t in ops)) if ops else set()
        is_load = op.startswith(("buffer_load", "global_load"))
        if used & pending and not is_load:
            found.append((n, ln, sorted(used & pending)))
        if is_load:   # only inline-asm loads are untracked by the compiler; its own loads it waits for itself
            queue.append((n, _regs(ops[0]) if in_asm and " lds" not in ln else set()))
        elif op.startswith(("buffer_store", "global_store", "global_atomic", "buffer_atomic")):
            queue.append((n, set()))
    return found


def kernels(asm_text, pattern):
    return sorted(set(re.findall(r"^(_Z\w*" + pattern + r"\w*):", asm_text, re.M)))


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    bad = 0
    for pat in sys.argv[2:] or [""]:
        for k in kernels(text, pat):
            f = audit(text, k)
            bad += len(f)
            print(f"{k}: {len(f)} findings" + "".join(f"\n  {n}: {ln} {r}" for n, ln, r in f[:5]))
    sys.exit(1 if bad else 0)
