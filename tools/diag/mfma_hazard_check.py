"""Static check of the VALU <-> MFMA register hazards of inline-asm MFMAs (vb_attn_bwd_kv.hip).

hipcc pads the wait states a VALU write needs before an MFMA reads the same register (2 on gfx950)
only for the MFMAs it generates; an MFMA written in inline asm is invisible to that pass. This tool
walks the kernel's control-flow graph (tools/diag/lgkm_check.py's block parser) and, for every
v_mfma, looks back over the instructions issued just before it (each instruction is one wait state,
`s_nop N` is N+1) on every path; a VALU instruction (v_*, other than an MFMA) that writes one of the
MFMA's source registers within WAIT_STATES is reported. It also reports a VALU that reads or writes
a register an MFMA wrote fewer than XDL_WAIT wait states before it on any path into it, across
branches and loop back-edges (the MFMA-result hazard, likewise padded by hipcc only for its own
MFMAs). VALU destinations are operand 0, plus operand 1 for the swap forms (v_permlane*_swap,
v_swap_b32), which write both.

Usage: python tools/diag/mfma_hazard_check.py <file.s> <kernel symbol>
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lgkm_check import blocks_of, regs  # noqa: E402

WAIT_STATES = 2
XDL_WAIT = 19


def operands(rest):
    out, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def wait_states(item):
    """wait states one issued instruction covers (s_nop N: N + 1)"""
    return (int(item[2]) + 1) if item[1] == "s_nop" and item[2].isdigit() else 1


def xdl_cost(item):
    """as wait_states, but an MFMA's own issue holds its wave for >= 8 cycles"""
    return 8 if item[1].startswith("v_mfma") else wait_states(item)


def valu_dst(op, rest):
    """VGPRs a VALU instruction writes"""
    if not rest:
        return frozenset()
    ops = operands(rest)
    dst = regs(ops[0])
    if ("swap" in op) and len(ops) > 1:   # v_permlane16/32_swap, v_swap_b32: both operands
        dst = dst | regs(ops[1])
    return dst


def check(path, name, verbose=True):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks = blocks_of(lines, start, end)
    preds = {i: [] for i in range(len(blocks))}
    for i, (_, _, succ) in enumerate(blocks):
        for s in succ:
            preds[s].append(i)

    def tail(bi, need, seen, cost=wait_states):
        """instructions (line, op, rest) of the paths into block bi, newest first, covering `need`
        wait states (each instruction priced by `cost`); one list per path. A block already on the
        path ends it (a loop is walked once around)."""
        if need <= 0 or bi in seen:
            return [[]]
        seen = seen | {bi}
        ins = blocks[bi][1]
        acc, w = [], 0
        for item in reversed(ins):
            acc.append(item)
            w += cost(item)
            if w >= need:
                return [acc]
        paths = []
        for p in preds[bi] or [None]:
            if p is None:
                paths.append(acc)
            else:
                for t in tail(p, need - w, seen, cost):
                    paths.append(acc + t)
        return paths

    bad = {}
    n_mfma = 0
    for bi, (_, ins, _) in enumerate(blocks):
        for k, (ln, op, rest) in enumerate(ins):
            if not op.startswith("v_mfma"):
                continue
            n_mfma += 1
            ops = operands(rest)
            srcs = frozenset().union(*(regs(o) for o in ops[1:4]))
            before = list(reversed(ins[:k]))
            paths = []
            w = 0
            acc = []
            for item in before:
                acc.append(item)
                w += (int(item[2]) + 1) if item[1] == "s_nop" and item[2].isdigit() else 1
                if w >= WAIT_STATES:
                    break
            if w >= WAIT_STATES:
                paths = [acc]
            else:
                paths = [acc + t for p in (preds[bi] or []) for t in tail(p, WAIT_STATES - w, frozenset())] or [acc]
            for path in paths:
                ws = 0
                for pl, pop, prest in path:
                    if ws >= WAIT_STATES:
                        break
                    if pop.startswith("v_") and not pop.startswith("v_mfma"):
                        dst = valu_dst(pop, prest)
                        if dst & srcs:
                            bad.setdefault(ln, f"line {ln + 1}: {op} reads {sorted(dst & srcs)[:4]} written by "
                                               f"{pop} at line {pl + 1}, {ws} wait states before")
                    ws += (int(prest) + 1) if pop == "s_nop" and prest.isdigit() else 1
    # MFMA write -> VALU access: the VALU must come >= XDL_WAIT wait states after an asm MFMA that
    # writes a register it reads or writes (19 covers the 16-pass case). An MFMA's own issue holds
    # its wave for >= 8 cycles (the microbenchmark's issue hold), so each one counts 8 here.
    # The look-back walks every control-flow path into the VALU (tail()), so an MFMA before a
    # branch or at the end of the previous loop iteration is seen as well.
    for bi, (_, ins, _) in enumerate(blocks):
        for k, (ln, op, rest) in enumerate(ins):
            if not op.startswith("v_") or op.startswith("v_mfma"):
                continue
            used = regs(rest)
            acc, w = [], 0
            for item in reversed(ins[:k]):
                acc.append(item)
                w += xdl_cost(item)
                if w >= XDL_WAIT:
                    break
            if w >= XDL_WAIT:
                paths = [acc]
            else:
                paths = [acc + t for p in (preds[bi] or []) for t in tail(p, XDL_WAIT - w, frozenset(), xdl_cost)] or [acc]
            for path in paths:
                ws = 0
                for pl, pop, prest in path:
                    if ws >= XDL_WAIT:
                        break
                    if pop.startswith("v_mfma"):
                        dst = regs(operands(prest)[0])
                        if dst & used:
                            bad.setdefault(ln, f"line {ln + 1}: {op} touches {sorted(dst & used)[:4]} written by the "
                                               f"MFMA at line {pl + 1}, {ws} wait states before")
                    ws += xdl_cost((pl, pop, prest))
    if verbose:
        for ln in sorted(bad)[:20]:
            print(bad[ln])
        print(f"{name}: {n_mfma} MFMAs, {len(bad)} hazards (VALU->MFMA and MFMA->VALU)")
    return len(bad)


if __name__ == "__main__":
    sys.exit(1 if check(sys.argv[1], sys.argv[2]) else 0)
