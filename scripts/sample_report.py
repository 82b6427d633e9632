#!/usr/bin/env python3
"""Fold a bench/sampler.hpp sample file into a flat profile (measurement only).

    python scripts/sample_report.py <exe> <samples> [--top 40] [--lines]

Each sample is a module and an instruction address relative to its load base; llvm-symbolizer resolves it with its
inlined frames.  Printed: the share of samples per module, per innermost function (inlining included), per source
line with --lines, and per inline chain."""
import argparse
import collections
import os
import subprocess

# clang writes DWARF 5, which an older binutils addr2line cannot read: LLVM's symbolizer, where ROCm ships it
SYM = next((p for p in ("/opt/rocm/lib/llvm/bin/llvm-symbolizer",) if os.path.exists(p)), "llvm-symbolizer")


def symbolize(obj, addrs):
    """{addr: [(function, file:line), ...innermost first]} for hex addresses of one module."""
    r = subprocess.run([SYM, f"--obj={obj}", "--output-style=GNU", "-a", "-i", "-f", "-C"] + ["0x" + x for x in addrs],
                       capture_output=True, text=True)
    info, cur = {}, None
    ls = r.stdout.splitlines()
    i = 0
    while i < len(ls):
        l = ls[i].strip()
        if l.startswith("0x") and all(ch in "0123456789abcdefx" for ch in l):
            cur = format(int(l, 16), "x")
            info[cur] = []
            i += 1
            continue
        if cur is not None:
            info[cur].append((l, ls[i + 1].strip() if i + 1 < len(ls) else "?"))
        i += 2
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("exe")
    ap.add_argument("samples")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--lines", action="store_true")
    ap.add_argument("--depth", type=int, default=3)
    a = ap.parse_args()
    rows = [l.rstrip("\n").split("\t") for l in open(a.samples) if l.strip()]
    by_mod = collections.defaultdict(set)
    for mod, x in rows:
        by_mod[mod].add(x)
    info = {}
    for mod, xs in by_mod.items():
        obj = a.exe if mod == "exe" else mod
        if mod == "?" or not os.path.exists(obj):
            continue
        for x, fr in symbolize(obj, sorted(xs)).items():
            info[(mod, x)] = fr
    cnt = collections.Counter((m, x) for m, x in rows)
    total = sum(cnt.values())
    inner, line, chain, mods = collections.Counter(), collections.Counter(), collections.Counter(), collections.Counter()
    short = lambda f: f.split("(")[0].split("::")[-1][:48]
    for key, c in cnt.items():
        mods[os.path.basename(key[0])] += c
        fr = info.get(key) or [("?", "?")]
        inner[short(fr[0][0])] += c
        line[fr[0][1].split("/")[-1]] += c
        chain[" <- ".join(short(f[0]) for f in fr[: a.depth])] += c
    print(f"{total} samples")
    for title, ctr in (("module", mods), ("innermost function", inner), ("source line", line if a.lines else None),
                       (f"inline chain (inner <- outer, {a.depth} levels)", chain)):
        if ctr is None:
            continue
        print(f"\n== {title} ==")
        for k, c in ctr.most_common(a.top):
            print(f"{100 * c / total:6.2f}%  {k}")


if __name__ == "__main__":
    main()
