"""Static check of hand-counted LDS waits in a kernel's ISA (the asm reads of vb_attn_bwd_kv.hip).

Models the LDS counter over the kernel's control-flow graph: every ds_read* pushes its destination
registers, every `s_waitcnt lgkmcnt(N)` retires the oldest reads until N remain (LDS returns in
order). Any other instruction that names a register of a read still in flight -- as a source or a
destination -- is reported. The walk follows every branch (`s_branch`, `s_cbranch_*`, fall-through)
and visits each (block, in-flight state) pair once, so loops and the uniform branches hipcc emits
for scalar selects are covered.

Usage: python tools/diag/lgkm_check.py <file.s> <kernel symbol>
  (hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S ... -o file.s)
"""
import re
import sys

REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")
LABEL = re.compile(r"^(\.?[A-Za-z_$][\w.$]*):")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.update(f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add(f"{m.group(4)}{m.group(5)}")
    return frozenset(out)


def blocks_of(lines, start, end):
    """[(label, [(line_no, op, rest)], successors)] in text order."""
    blocks, cur, label = [], [], "entry"
    for ln in range(start + 1, end):
        raw = lines[ln].split(";")[0].rstrip()
        m = LABEL.match(raw.strip())
        if m and not raw.startswith("\t"):
            blocks.append([label, cur])
            label, cur = m.group(1), []
            continue
        s = raw.strip()
        if not s or s.startswith("."):
            continue
        op, _, rest = s.partition(" ")
        cur.append((ln, op, rest.strip()))
        if op.startswith("s_cbranch") or op == "s_branch" or op == "s_endpgm":
            blocks.append([label, cur])    # a branch ends the block (hipcc marks the next one
            label, cur = f"anon{ln}", []   # only with a "; %bb.N:" comment)
    blocks.append([label, cur])
    index = {b[0]: i for i, b in enumerate(blocks)}
    out = []
    for i, (label, ins) in enumerate(blocks):
        succ = []
        last = ins[-1] if ins else None
        nxt = i + 1 if i + 1 < len(blocks) else None
        if last and last[1] == "s_branch":
            succ = [index[last[2]]]
        elif last and last[1].startswith("s_cbranch"):
            succ = [index[last[2]]] + ([nxt] if nxt is not None else [])
        elif last and last[1] in ("s_endpgm", "s_setpc_b64"):
            succ = []
        elif nxt is not None:
            succ = [nxt]
        out.append((label, ins, succ))
    return out


def check(path, name, verbose=True):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks = blocks_of(lines, start, end)
    bad = {}
    n_reads = sum(1 for _, ins, _ in blocks for _, op, _ in ins if op.startswith("ds_read"))
    n_waits = sum(1 for _, ins, _ in blocks for _, op, r in ins if op == "s_waitcnt" and "lgkmcnt" in r)
    seen = set()
    work = [(0, ())]
    while work:
        bi, state = work.pop()
        if (bi, state) in seen:
            continue
        seen.add((bi, state))
        pending = list(state)
        _, ins, succ = blocks[bi]
        for ln, op, rest in ins:
            if op == "s_waitcnt":
                m = re.search(r"lgkmcnt\((\d+)\)", rest)
                if m:
                    keep = int(m.group(1))
                    while len(pending) > keep:
                        pending.pop(0)
                continue
            if op.startswith("ds_read"):
                dst, _, src = rest.partition(",")
                used = regs(src)
                for pl, pr in pending:
                    if used & pr:
                        bad.setdefault(ln, f"line {ln + 1}: address of {op} {rest!r} from read at line {pl + 1} in flight")
                pending.append((ln, regs(dst)))
                del pending[:-15]   # the 4-bit counter: the 16th outstanding read waits for the oldest
                continue
            if op.startswith("ds_"):
                pending.append((ln, frozenset()))   # compiler-visible LDS op: counts, hipcc waits for it
                del pending[:-15]
                continue
            if op.startswith("s_"):
                continue
            used = regs(rest)
            for pl, pr in pending:
                hit = used & pr
                if hit:
                    bad.setdefault(ln, f"line {ln + 1}: {op} {rest!r} uses {sorted(hit)[:4]} loaded at line {pl + 1}, not yet waited for")
        for s in succ:
            work.append((s, tuple(pending)))
    if verbose:
        for ln in sorted(bad)[:20]:
            print(bad[ln])
        print(f"{name}: {n_reads} LDS reads, {n_waits} lgkmcnt waits, {len(blocks)} blocks, "
              f"{len(seen)} block states, {len(bad)} violations")
    return len(bad)


if __name__ == "__main__":
    sys.exit(1 if check(sys.argv[1], sys.argv[2]) else 0)
