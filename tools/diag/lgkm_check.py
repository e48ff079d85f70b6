"""Static check of hand-counted LDS waits in a kernel's ISA (the asm reads of vb_attn_bwd_kv128.hip).

Walks the kernel's instructions in text order and models the LDS counter: every ds_read* pushes its
destination registers, every `s_waitcnt lgkmcnt(N)` retires the oldest reads until N remain (LDS
returns in order). Any other instruction that names a register of a read still in flight -- as a
source or a destination -- is reported. Text order follows the fall-through path, which for the
kv128 kernel covers every transition the loop makes (prologue -> tile 0 -> steady tiles -> drain).

Usage: python tools/diag/lgkm_check.py <file.s> <kernel symbol>
  (hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S ... -o file.s)
"""
import re
import sys

REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.update(f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add(f"{m.group(4)}{m.group(5)}")
    return out


def check(path, name):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    pending = []   # [(line, set of regs)]
    errors = 0
    n_reads = n_waits = 0
    for ln in range(start + 1, end):
        raw = lines[ln].split(";")[0].strip()
        if not raw or raw.startswith(".") or raw.endswith(":"):
            continue
        op, _, rest = raw.partition(" ")
        if op.startswith("s_waitcnt"):
            m = re.search(r"lgkmcnt\((\d+)\)", rest)
            if m:
                n_waits += 1
                keep = int(m.group(1))
                while len(pending) > keep:
                    pending.pop(0)
            continue
        if op.startswith("ds_read"):
            dst, _, src = rest.partition(",")
            used = regs(src)
            for pl, pr in pending:
                if used & pr:
                    print(f"line {ln + 1}: address of {raw!r} from read at line {pl + 1} still in flight")
                    errors += 1
            pending.append((ln, regs(dst)))
            n_reads += 1
            continue
        if op.startswith("ds_"):
            # compiler-visible LDS op: it also counts; the compiler waits for its own results
            pending.append((ln, set()))
            continue
        if op.startswith("s_") and not op.startswith("s_load"):
            continue
        if op.startswith("s_load"):
            pending = pending  # SMEM also counts in lgkm but returns out of order; the compiler
            continue           # waits lgkmcnt(0) for it, which this model handles when it appears
        used = regs(rest)
        for pl, pr in pending:
            hit = used & pr
            if hit:
                print(f"line {ln + 1}: {raw!r} uses {sorted(hit)[:4]} loaded at line {pl + 1}, not yet waited for")
                errors += 1
    print(f"{name}: {n_reads} LDS reads, {n_waits} lgkmcnt waits, {errors} violations")
    return errors


if __name__ == "__main__":
    sys.exit(1 if check(sys.argv[1], sys.argv[2]) else 0)
