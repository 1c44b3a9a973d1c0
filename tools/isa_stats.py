"""Per-function register and scratch statistics of one HIP source (gfx950):
python tools/isa_stats.py waffle_con_amd/csrc/engine_wave.hip [-DFOO ...]
Builds with --save-temps into /tmp/isa_stats and prints, per function of the
device assembly: its own VGPR/SGPR counts, private segment bytes, scratch
instructions, SGPR-spill lane moves and lines."""
import os
import re
import subprocess
import sys


def main():
    src = os.path.abspath(sys.argv[1])
    extra = sys.argv[2:]
    out = "/tmp/isa_stats"
    os.makedirs(out, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-w",
                    "--save-temps", "-c", "-o", os.path.join(out, "x.o"), src] + extra, cwd=out, check=True)
    base = os.path.splitext(os.path.basename(src))[0]
    asm = open(os.path.join(out, base + "-hip-amdgcn-amd-amdhsa-gfx950.s")).read().splitlines()
    funcs, cur = {}, None
    for ln in asm:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            cur = m.group(1)
            funcs[cur] = {"lines": 0, "scratch": 0, "readlane": 0, "writelane": 0}
            continue
        if cur is None:
            continue
        if ln.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", ln):
            cur = None
            continue
        f = funcs[cur]
        f["lines"] += 1
        if "scratch_" in ln:
            f["scratch"] += 1
        if "v_readlane" in ln:
            f["readlane"] += 1
        if "v_writelane" in ln:
            f["writelane"] += 1
    sets = {}
    for ln in asm:
        m = re.match(r"\s*\.set\s+\.?L?(_Z\w+)\.(num_vgpr|num_sgpr|private_seg_size),\s*(.*)", ln)
        if m:
            v = m.group(3)
            num = re.match(r"(?:max\()?(\d+)", v)
            sets.setdefault(m.group(1), {})[m.group(2)] = num.group(1) if num else v
    for name, f in funcs.items():
        if "wfa_ed" in name or "dwfa" in name:
            continue
        s = sets.get(name, {})
        print("%-70s vgpr %4s sgpr %4s priv %4s | lines %6d scratch %4d readlane %5d writelane %4d" % (
            name[:70], s.get("num_vgpr", "?"), s.get("num_sgpr", "?"), s.get("private_seg_size", "?"),
            f["lines"], f["scratch"], f["readlane"], f["writelane"]))


if __name__ == "__main__":
    main()
