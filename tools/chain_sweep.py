"""Kernel time of the bench workload vs the chain run-ahead length (WC_CHAIN),
one child process per length; results must be identical across lengths.
Diagnostic only. Usage: python tools/chain_sweep.py 16 24 32 default"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, json, sys
sys.path.insert(0, %r)
import waffle_con_amd as w
from waffle_con_amd.cdwfa_config import CdwfaConfig
from bench import gen_loci
loci = gen_loci(range(1000), 10000, 100, 0.005)
batch = w.ResidentBatch(loci)
cfg = CdwfaConfig(min_count=25)
ks = []
for s in range(3):
    res, st = batch.consensus(cfg, return_errors=True)
    ks.append(st["kernel_ms"])
h = hashlib.sha256(repr(res).encode()).hexdigest()[:16]
print(json.dumps({"kernel_ms": ks, "hash": h, "updates": st["updates"], "compares": st["compares"]}))
""" % ROOT


def main():
    out = {}
    for k in sys.argv[1:]:
        env = dict(os.environ)
        if k != "default":
            env["WC_CHAIN"] = k
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
        out[k] = json.loads(line) if line.startswith("{") else line
        print(k, out[k], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
