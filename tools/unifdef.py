#!/usr/bin/env python3
"""Partial preprocessor: resolve the conditionals that test a given set of
macros, keep every other directive as it is (unifdef's job; unifdef is not in
the image).  Used once to strip the measured-and-dropped experiment variants
out of the product kernels; kept for the record.

usage: tools/unifdef.py FILE [-DNAME=VALUE | -UNAME] ...   (rewrites FILE)

-DNAME=VALUE: NAME is defined with that value; an `#ifndef NAME` default block
is dropped.  -UNAME: NAME is undefined (0 inside #if).  A conditional whose
expression mentions any other identifier is kept verbatim (its branches are
still processed)."""
import re
import sys

TOK = re.compile(r"\s*(defined\s*\(\s*\w+\s*\)|defined\s+\w+|\w+|==|!=|&&|\|\||<=|>=|[()!&|<>+\-*/])")


def evaluate(expr, known):
    """Value of a #if expression, or None when it names an unknown macro."""
    expr = re.sub(r"//.*$", "", expr)
    expr = re.sub(r"/\*.*?\*/", "", expr).strip()
    out, pos = [], 0
    while pos < len(expr):
        m = TOK.match(expr, pos)
        if not m:
            return None
        t = m.group(1)
        pos = m.end()
        if t.startswith("defined"):
            name = re.sub(r"defined|[()\s]", "", t)
            if name not in known:
                return None
            out.append("1" if known[name] is not None else "0")
        elif re.fullmatch(r"\d+", t):
            out.append(t)
        elif re.fullmatch(r"\w+", t):
            if t not in known:
                return None
            out.append(str(known[t]) if known[t] is not None else "0")
        else:
            out.append({"&&": " and ", "||": " or ", "!": " not "}.get(t, t))
    return bool(eval(" ".join(out)))  # noqa: S307 -- integers and operators only


def process(lines, known):
    out = []
    # frame: [resolved?, current branch state (True / False / None), any branch taken]
    stack = []

    def live():
        return all(f[1] is not False for f in stack)

    for line in lines:
        s = line.strip()
        m = re.match(r"#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)", s)
        if not m:
            if live():
                out.append(line)
            continue
        d, rest = m.group(1), m.group(2)
        if d in ("ifdef", "ifndef"):
            name = re.sub(r"//.*$", "", rest).strip()
            if name in known:
                v = known[name] is not None
                stack.append([True, v if d == "ifdef" else not v, True])
                stack[-1][2] = stack[-1][1]
            else:
                if live():
                    out.append(line)
                stack.append([False, None, False])
        elif d == "if":
            v = evaluate(rest, known)
            if v is None:
                if live():
                    out.append(line)
                stack.append([False, None, False])
            else:
                stack.append([True, v, v])
        elif d == "elif":
            f = stack[-1]
            if not f[0]:
                if live_outer(stack):
                    out.append(line)
                continue
            v = evaluate(rest, known)
            if v is None:
                raise SystemExit(f"unresolvable #elif in a resolved chain: {s}")
            f[1] = (not f[2]) and v
            f[2] = f[2] or v
        elif d == "else":
            f = stack[-1]
            if not f[0]:
                if live_outer(stack):
                    out.append(line)
                continue
            f[1] = not f[2]
            f[2] = True
        else:  # endif
            f = stack.pop()
            if not f[0] and live():
                out.append(line)
    if stack:
        raise SystemExit("unbalanced conditionals")
    return out


def live_outer(stack):
    return all(f[1] is not False for f in stack[:-1])


def main():
    path, known = sys.argv[1], {}
    for a in sys.argv[2:]:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            known[k] = int(v or "1")
        elif a.startswith("-U"):
            known[a[2:]] = None
    lines = open(path).read().splitlines(keepends=True)
    open(path, "w").write("".join(process(lines, known)))


if __name__ == "__main__":
    main()
