"""Static instruction mix of the kernels in a hipcc device-assembly file (--cuda-device-only -S).

Usage: python scripts/isa_mix.py fs.s [kernel-substring ...]
Prints, per kernel, the count of each instruction class (VALU / packed fp32 VALU / DPP / SALU /
LDS / VMEM / MFMA) and register use, so a VALU diet can be checked before a GPU run.
"""
import re
import sys
from collections import Counter


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and not line.startswith(".L"):
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur and re.match(r"^\s*\.Lfunc_end", line):
            yield cur, body
            cur, body = None, []
            continue
        if cur:
            body.append(line)
    if cur:
        yield cur, body


def classify(op, line):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_pk_") and op.endswith("_f32"):
        return "valu_pk32"
    if op.startswith("v_"):
        return "valu_dpp" if ("row_" in line or "quad_perm" in line or "wave_" in line) else "valu"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, body in kernels(path):
        if subs and not any(s in name for s in subs):
            continue
        c, ops = Counter(), Counter()
        for line in body:
            t = line.strip()
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            op = t.split()[0]
            c[classify(op, t)] += 1
            ops[op] += 1
        meta = {}
        for line in body:
            m = re.search(r"; (NumVgprs|NumAgprs|Occupancy|ScratchSize|NumSgprs): (\d+)", line)
            if m:
                meta[m.group(1)] = int(m.group(2))
        print(name[:90], dict(c), meta)
        if len(subs) and "-v" in sys.argv:
            print("   ", ops.most_common(40))


if __name__ == "__main__":
    main()
