"""Static check of SGPR spills into VGPR lanes in a kernel's ISA (round-4
verdict item 3b: the 3-wave dual build faults with a corrupted pointer, and
its SGPRs spill into lanes of v163-v167).

For one function of a `--save-temps` .s file it builds the control-flow graph
and runs a reaching-definitions analysis over every spill slot (VGPR, lane):
  * clobbers: any instruction other than v_writelane/v_readlane that writes
    (or reads) a spill VGPR, and any call whose callee's VGPR count reaches
    the spill VGPRs (they are caller-saved);
  * undefined restores: a v_readlane of a slot that some path from the entry
    reaches without a v_writelane to it;
  * torn restores: a multi-dword SGPR tuple restored from consecutive lanes
    (s[k], s[k+1] from lanes L, L+1 - a 64-bit pointer) whose lanes were not
    written together by one spill on every path (the low dword of one value
    with the high dword of another);
  * the memory instructions whose address operands come straight from such a
    restore are listed with each finding.
  python tools/spill_lanes.py <file.s> <function symbol> [--callee-vgprs sym=N ...]"""
import argparse
import collections
import json
import re
import sys

INSN = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*(?:;.*)?$")
LABEL = re.compile(r"^(\.?[A-Za-z_][\w.$]*):")
SREG = re.compile(r"^s(\d+)$")
VREG_ANY = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def parse(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    body = []
    for l in lines[start + 1:]:
        if l.startswith("\t.size\t" + sym) or l.startswith(".Lfunc_end"):
            break
        m = LABEL.match(l)
        if m:
            body.append(("label", m.group(1)))
            continue
        m = INSN.match(l)
        if m and not m.group(1).startswith("."):
            ops = [o.strip() for o in (m.group(2) or "").split(",")] if m.group(2) else []
            body.append(("insn", m.group(1), ops, l.strip()))
    return body


def blocks(body):
    """Basic blocks: (label, [insn]), successors by label."""
    bl, cur, name, k = [], [], "entry", 0
    for it in body:
        if it[0] == "label":
            bl.append((name, cur))
            name, cur = it[1], []
            continue
        cur.append(it)
        op = it[1]
        if op == "s_branch" or op.startswith("s_cbranch") or op in ("s_endpgm", "s_setpc_b64"):
            bl.append((name, cur))
            k += 1
            name, cur = "%s.ft%d" % (name, k), []
    bl.append((name, cur))
    bl = [b for b in bl if b[1] or b[0] == "entry"]
    succ = {}
    for i, (n, ins) in enumerate(bl):
        s = []
        last = ins[-1] if ins else None
        nxt = bl[i + 1][0] if i + 1 < len(bl) else None
        if last is None:
            s = [nxt] if nxt else []
        elif last[1] == "s_branch":
            s = [last[2][0]]
        elif last[1].startswith("s_cbranch"):
            s = [last[2][0]] + ([nxt] if nxt else [])
        elif last[1] in ("s_endpgm", "s_setpc_b64"):
            s = []
        else:
            s = [nxt] if nxt else []
        succ[n] = [x for x in s if x]
    return bl, succ


def lane_op(it):
    """v_writelane/v_readlane with an immediate lane (the spill form)."""
    return it[1] in ("v_writelane_b32", "v_readlane_b32") and len(it[2]) == 3 and it[2][2].isdigit()


def sreg(op):
    m = SREG.match(op)
    return int(m.group(1)) if m else None


def vregs(op):
    out = set()
    for a, b, c in VREG_ANY.findall(op):
        if a:
            out.add(int(a))
        else:
            out.update(range(int(b), int(c) + 1))
    return out


def analyze(path, sym, callee_vgprs):
    body = parse(path, sym)
    bl, succ = blocks(body)
    names = [b[0] for b in bl]
    # spill VGPRs: targets of v_writelane
    spill_v = set()
    for n, ins in bl:
        for i, it in enumerate(ins):
            if it[1] == "v_writelane_b32" and lane_op(it):
                v = vregs(it[2][0])
                spill_v |= v
    # spill pairs: the writelane of s[k+1] into lane L+1 that follows the
    # writelane of s[k] into lane L of the same VGPR in the same block, with no
    # other write to either lane between them (the two halves of one tuple)
    partner_hi, partner_lo = {}, {}
    for n, ins in bl:
        open_lo = {}  # (vgpr, lane) -> (idx, sgpr) of the last writelane there
        for i, it in enumerate(ins):
            if it[1] != "v_writelane_b32" or not lane_op(it):
                continue
            v = min(vregs(it[2][0]))
            sg = sreg(it[2][1])
            lane = int(it[2][2])
            lo = open_lo.get((v, lane - 1))
            if lo is not None and sg is not None and lo[1] is not None and sg == lo[1] + 1:
                partner_hi[(n, lo[0])] = (n, i)
                partner_lo[(n, i)] = (n, lo[0])
            open_lo[(v, lane)] = (i, sg)
    findings = collections.defaultdict(list)
    # clobbers: other instructions naming a spill VGPR; calls into callees that reach them
    for n, ins in bl:
        for i, it in enumerate(ins):
            if lane_op(it) and (vregs(it[2][0] if it[1] == "v_writelane_b32" else it[2][1]) & spill_v):
                continue
            touched = set()
            for o in it[2]:
                touched |= vregs(o) & spill_v
            if touched:
                findings["clobber"].append({"block": n, "insn": it[3], "vgprs": sorted(touched)})
            if it[1] == "s_swappc_b64":
                for cs, cnt in callee_vgprs.items():
                    if cnt > min(spill_v):
                        findings["clobber"].append({"block": n, "insn": it[3], "callee": cs, "callee_vgprs": cnt})
    # reaching definitions over slots: state = {slot: frozenset(def ids)}; None def = undefined
    UNDEF = ("undef",)
    all_slots = set()
    for n, ins in bl:
        for it in ins:
            if lane_op(it):
                vop = it[2][0] if it[1] == "v_writelane_b32" else it[2][1]
                if vregs(vop) & spill_v:
                    all_slots.add((min(vregs(vop)), int(it[2][2])))

    def transfer(n, state, visit=None):
        st = dict(state)
        for i, it in enumerate(BL[n]):
            if not lane_op(it):
                continue
            if it[1] == "v_writelane_b32":
                slot = (min(vregs(it[2][0])), int(it[2][2]))
                if slot in all_slots:
                    st[slot] = frozenset([(n, i)])
            elif visit is not None and (min(vregs(it[2][1])), int(it[2][2])) in all_slots:
                visit(n, i, it, st)
        return st
    BL = dict(bl)
    entry = {s: frozenset([UNDEF]) for s in all_slots}
    IN = {n: None for n in names}
    IN[names[0]] = entry
    OUT = {}
    work = collections.deque([names[0]])
    preds = collections.defaultdict(list)
    for n, ss in succ.items():
        for s in ss:
            preds[s].append(n)
    while work:
        n = work.popleft()
        out = transfer(n, IN[n])
        if OUT.get(n) == out:
            continue
        OUT[n] = out
        for s in succ.get(n, []):
            if s not in IN:
                continue
            ins_ = [OUT[p] for p in preds[s] if p in OUT]
            merged = {}
            for sl in all_slots:
                u = frozenset()
                for o in ins_:
                    u |= o.get(sl, frozenset())
                merged[sl] = u
            if IN[s] != merged:
                IN[s] = merged
                work.append(s)
    # visit restores with the reaching definitions
    restores = []

    def visit(n, i, it, st):
        slot = (min(vregs(it[2][1])), int(it[2][2]))
        restores.append((n, i, sreg(it[2][0]), slot, st.get(slot, frozenset())))
    for n in names:
        if IN[n] is not None:
            transfer(n, IN[n], visit)
    n_restore = len(restores)
    for n, i, s, slot, defs in restores:
        if UNDEF in defs:
            findings["undefined_restore"].append({"block": n, "insn": BL[n][i][3]})
    # torn tuple restores: consecutive readlanes into consecutive SGPRs from consecutive lanes
    by_block = collections.defaultdict(list)
    for r in restores:
        by_block[r[0]].append(r)
    n_pairs = 0
    for n, rs in by_block.items():
        rs.sort(key=lambda r: r[1])
        for a, b in zip(rs, rs[1:]):
            if a[2] is None or b[2] is None or b[2] != a[2] + 1 or b[3][0] != a[3][0] or b[3][1] != a[3][1] + 1:
                continue
            if b[1] - a[1] > 4:
                continue
            n_pairs += 1
            # every def reaching the low lane has its partner reaching the high lane, and back
            lo_ok = all(d == UNDEF or partner_hi.get(d) in b[4] for d in a[4])
            hi_ok = all(d == UNDEF or partner_lo.get(d) in a[4] for d in b[4])
            if not (lo_ok and hi_ok):
                findings["torn_restore"].append({"block": n, "lo": BL[n][a[1]][3], "hi": BL[n][b[1]][3],
                                                 "lo_defs": sorted(BL[d[0]][d[1]][3] + " @" + d[0] for d in a[4] if d != UNDEF),
                                                 "hi_defs": sorted(BL[d[0]][d[1]][3] + " @" + d[0] for d in b[4] if d != UNDEF)})
    return {"function": sym, "blocks": len(bl), "spill_vgprs": sorted(spill_v), "slots": len(all_slots),
            "spills": sum(1 for n, ins in bl for it in ins if it[1] == "v_writelane_b32"),
            "restores": n_restore, "tuple_restores_checked": n_pairs,
            "findings": {k: v for k, v in findings.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("--callee-vgprs", nargs="*", default=[])
    a = ap.parse_args()
    cv = {}
    for x in a.callee_vgprs:
        k, v = x.split("=")
        cv[k] = int(v)
    rep = analyze(a.asm, a.symbol, cv)
    json.dump(rep, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
