"""Resolve compile-time variant switches of the product kernels to their default values
(development tool: the round-6 hygiene pass that moved the ablation / experiment variants out of
mageslam_amd/csrc; the removed variants stay buildable from the revision recorded in
tools/patches/README.md with tools/abl.py's name@REV form or by applying the patches there).

  python tools/unifdef_variants.py FILE NAME=VALUE [NAME=VALUE ...]

Handles, for the given names only: the `#ifndef NAME / #define NAME v / #endif` default blocks
(removed), `#if NAME`, `#if !NAME`, `#if NAME == k`, `#if NAME != k`, `#if NAME < k` (the
selected branch kept, with #elif-free nesting), and leaves every other directive alone.
"""
import re
import sys


def evaluate(expr, values):
    e = expr.strip()
    for n, v in values.items():
        e = re.sub(rf"\b{n}\b", str(v), e)
    if re.search(r"[A-Za-z_]", e):
        return None
    return bool(eval(e.replace("!", " not ").replace(" not =", "!=").replace("&&", " and ").replace("||", " or ")))


def process(lines, values):
    out = []
    stack = []  # per #if: (mode, taking) mode 'resolved' / 'kept'
    i = 0
    names = "|".join(values)
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(rf"#ifndef\s+({names})\b", s)
        if m and i + 2 < len(lines) and re.match(rf"#define\s+{m.group(1)}\b", lines[i + 1].strip()):
            # default block: skip to its #endif (comment lines inside are dropped too)
            j = i + 1
            while not lines[j].strip().startswith("#endif"):
                j += 1
            i = j + 1
            continue
        if s.startswith("#if"):
            cond = s[3:].strip() if s.startswith("#if ") else None
            val = evaluate(cond, values) if cond is not None and re.search(rf"\b({names})\b", cond) else None
            active = all(t for _, t in stack)
            if val is None:
                stack.append(("kept", True))
                if active:
                    out.append(ln)
            else:
                stack.append(("resolved", val))
            i += 1
            continue
        if s.startswith("#else") and stack:
            mode, t = stack[-1]
            if mode == "resolved":
                stack[-1] = (mode, not t)
            elif all(tt for _, tt in stack[:-1]):
                out.append(ln)
            i += 1
            continue
        if s.startswith("#elif") and stack and stack[-1][0] == "resolved":
            raise SystemExit(f"#elif after a resolved #if at line {i + 1}")
        if s.startswith("#endif") and stack:
            mode, _ = stack.pop()
            if mode == "kept" and all(t for _, t in stack):
                out.append(ln)
            i += 1
            continue
        if all(t for _, t in stack):
            out.append(ln)
        i += 1
    return out


if __name__ == "__main__":
    path = sys.argv[1]
    values = dict(a.split("=", 1) for a in sys.argv[2:])
    with open(path) as f:
        lines = f.read().split("\n")
    res = process(lines, values)
    with open(path, "w") as f:
        f.write("\n".join(res))
