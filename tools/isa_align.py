"""Static checks of one kernel's ISA for the remaining candidates behind the
3-wave dual build's fault (round-5 verdict item 7):

  * VGPR/AGPR tuple alignment: gfx90a and later (gfx950 included) require
    every 64-bit-or-wider register tuple operand to start at an even register
    (the machine verifier's "Subtarget requires even aligned vector
    registers"). Lists every instruction with a tuple v[a:b] / a[a:b], b > a,
    whose a is odd, scratch spill reloads (scratch_load_dwordx*) separately.
  * LDS addresses from restored SGPRs: every ds_* instruction whose address
    VGPR is defined, within its basic block, by a v_mov_b32 (or a VALU op)
    reading an SGPR that a v_readlane in the same block restored from a spill
    lane; those are listed with the restore (tools/spill_lanes.py checks that
    the restores themselves read the lanes their spills wrote).

Builds nothing: give it the .s of a --save-temps build.
  python tools/isa_align.py <file.s> <function symbol> [--json out.json]"""
import argparse
import json
import re
import sys

INSN = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*(?:;.*)?$")
LABEL = re.compile(r"^(\.?[A-Za-z_][\w.$]*):")
TUPLE = re.compile(r"\b([va])\[(\d+):(\d+)\]")
VREG = re.compile(r"^v(\d+)$")
SREG = re.compile(r"\bs(\d+)\b")


def body_of(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    out = []
    for l in lines[start + 1:]:
        if l.startswith("\t.size\t" + sym) or l.startswith(".Lfunc_end"):
            break
        if LABEL.match(l):
            out.append(("label", l.split(":")[0]))
            continue
        m = INSN.match(l)
        if m and not m.group(1).startswith("."):
            ops = [o.strip() for o in (m.group(2) or "").split(",")] if m.group(2) else []
            out.append(("insn", m.group(1), ops, l.strip()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("sym")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    body = body_of(a.asm, a.sym)
    insns = [b for b in body if b[0] == "insn"]
    tuples = 0
    odd = []
    odd_scratch = []
    for _, op, ops, text in insns:
        for m in TUPLE.finditer(" ".join(ops)):
            lo, hi = int(m.group(2)), int(m.group(3))
            if hi <= lo:
                continue
            tuples += 1
            if lo % 2:
                (odd_scratch if op.startswith("scratch_") else odd).append(text)
    # LDS addresses built from restored SGPRs, within basic blocks
    lds_total = 0
    lds_from_restore = []
    restored = {}  # sgpr -> the v_readlane that restored it (this block)
    vdef = {}      # vgpr -> (defining text, sgprs it read)
    for it in body:
        if it[0] == "label":
            restored.clear()
            vdef.clear()
            continue
        _, op, ops, text = it
        if op == "v_readlane_b32" and ops:
            s = SREG.match(ops[0])
            if s:
                restored[int(s.group(1))] = text
            continue
        if op.startswith("ds_") and len(ops) >= 2:
            lds_total += 1
            addr = ops[1] if op.startswith(("ds_read", "ds_load")) else ops[0]
            m = VREG.match(addr)
            if m and int(m.group(1)) in vdef:
                dtext, sregs = vdef[int(m.group(1))]
                src = [restored[s] for s in sregs if s in restored]
                if src:
                    lds_from_restore.append({"ds": text, "address_def": dtext, "restore": src})
        if op.startswith("v_") and ops:
            m = VREG.match(ops[0])
            if m:
                sregs = [int(x) for o in ops[1:] for x in SREG.findall(o)]
                vdef[int(m.group(1))] = (text, sregs)
        # an SGPR overwritten by anything else is no longer the restored value
        if op.startswith("s_") and ops:
            s = SREG.match(ops[0])
            if s:
                restored.pop(int(s.group(1)), None)
        if op == "s_branch" or op.startswith("s_cbranch") or op.startswith("s_swappc") or op == "s_setpc_b64":
            restored.clear()
            vdef.clear()
    res = {"function": a.sym, "instructions": len(insns), "vector_tuples": tuples,
           "odd_aligned_tuples": len(odd), "odd_aligned_scratch_tuples": len(odd_scratch),
           "odd_examples": (odd + odd_scratch)[:20], "ds_instructions": lds_total,
           "ds_addresses_from_restored_sgprs": len(lds_from_restore), "ds_from_restore_examples": lds_from_restore[:20]}
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
