#!/usr/bin/env python3
"""Static instruction mix per kernel of a hipcc -S listing (gfx950): counts
by opcode class, to account the non-FMA VALU of a kernel.
usage: tools/isa_mix.py FILE.s [kernel-substring] [--top N]"""
import collections
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names), capture_output=True,
                             text=True).stdout.splitlines()
        return dict(zip(names, out))
    except OSError:
        return {n: n for n in names}


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    funcs, cur, meta, last = collections.OrderedDict(), None, collections.defaultdict(dict), None
    for line in open(path):
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", line)
        if m:
            cur = last = m.group(1)
            funcs[cur] = collections.Counter()
            continue
        mm = re.match(r"^; (NumVgprs|TotalNumSgprs|ScratchSize|Occupancy): (\d+)", line)
        if mm and last:
            meta[last][mm.group(1)] = int(mm.group(2))
        if cur is None:
            continue
        if line.startswith(".Lfunc_end") or line.startswith("\t.size"):
            cur = None if line.startswith("\t.size") else cur
            continue
        t = line.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        op = t.split()[0]
        funcs[cur][op] += 1
    dm = demangle(list(funcs))
    for f, c in funcs.items():
        name = dm.get(f, f)
        if sub and sub not in name:
            continue
        tot = sum(c.values())
        cls = collections.Counter()
        for op, n in c.items():
            if op.startswith("v_fma_f64"):
                cls["v_fma_f64"] += n
            elif op.startswith("v_mfma"):
                cls["mfma"] += n
            elif op.startswith("v_"):
                cls["valu_other"] += n
            elif op.startswith("s_waitcnt"):
                cls["s_waitcnt"] += n
            elif op.startswith(("s_load", "s_buffer_load")):
                cls["smem"] += n
            elif op.startswith("s_"):
                cls["salu/branch"] += n
            elif op.startswith("ds_"):
                cls["lds"] += n
            elif op.startswith(("buffer_load", "global_load", "flat_load")):
                cls["vmem_load"] += n
            elif op.startswith(("buffer_store", "global_store", "flat_store")):
                cls["vmem_store"] += n
            else:
                cls["other"] += n
        print("=" * 100)
        print(name[:200])
        print("  %s" % " ".join("%s=%s" % kv for kv in meta[f].items()))
        print("  total %d  " % tot + "  ".join("%s %d" % kv for kv in cls.most_common()))
        vo = [(op, n) for op, n in c.most_common() if op.startswith("v_") and not op.startswith("v_fma_f64")]
        print("  non-FMA VALU:", ", ".join("%s %d" % kv for kv in vo[:top]))


if __name__ == "__main__":
    main()
