"""A stand-in for `go vet`'s composite-literal check over go/src (no Go
toolchain in this image): every struct literal of a type declared in
go/src/** must use keyed fields when the struct has more than one field, and
every key must be a declared field. A positional literal of a multi-field
struct is what broke `BACKEND_TYPE=gpu` in round 5
(go/src/gpu/cache_impl.go: `&call{request, limits, now, done}` after `call`
grew to six fields): `go build` rejects a count mismatch, and a reordering of
same-typed fields would compile and silently swap them.

    python tests/go_lint.py            # lint go/src, exit 1 on findings
"""
import os
import re
import sys

IDENT = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")


def strip(src):
    """Comments and string / rune literals blanked (same length, newlines
    kept), so braces and commas inside them do not count."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            out.append(" " * (j - i))
            i = j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append(re.sub(r"[^\n]", " ", src[i:j]))
            i = j
        elif c in "\"'`":
            j = i + 1
            while j < n and src[j] != c:
                if c != "`" and src[j] == "\\":
                    j += 1
                j += 1
            j = min(j + 1, n)
            out.append(c + re.sub(r"[^\n]", " ", src[i + 1:j - 1]) + c)
            i = j
        else:
            out.append(c)
            i += 1
    return "".join(out)


def match_brace(s, i):
    """Index of the brace closing the one at s[i]."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] in "({[":
            depth += 1
        elif s[j] in ")}]":
            depth -= 1
            if depth == 0:
                return j
    raise ValueError("unbalanced braces")


def split_top(s):
    """s split at its top-level commas."""
    parts, depth, cur = [], 0, []
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    parts.append("".join(cur))
    return [p.strip() for p in parts if p.strip()]


def top_colon(s):
    depth = 0
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        elif ch == ":" and depth == 0:
            return True
    return False


def struct_fields(src):
    """{type name: [field names]} of the struct types declared in src."""
    s = strip(src)
    out = {}
    for m in re.finditer(r"\btype\s+([A-Za-z_]\w*)\s+struct\s*\{", s):
        body = s[m.end():match_brace(s, m.end() - 1)]
        names = []
        for line in re.split(r"[;\n]", body):
            line = line.strip()
            if not line:
                continue
            head = re.match(r"([A-Za-z_]\w*(?:\s*,\s*[A-Za-z_]\w*)*)\s+\S", line)
            if head:
                names.extend(x.strip() for x in head.group(1).split(","))
            else:  # an embedded field: its type's name
                names.append(line.lstrip("*").split(".")[-1])
        out[m.group(1)] = names
    return out


def lint_source(src, types, qualified=None, path="<src>"):
    """Findings for the struct literals in src of the types in `types`
    (unqualified: this package) and `qualified` ({pkg: types}: other packages
    of go/src)."""
    s = strip(src)
    findings = []
    pat = re.compile(r"(?<![\w.])(?:([A-Za-z_]\w*)\.)?([A-Za-z_]\w*)\{")
    for m in pat.finditer(s):
        pkg, name = m.group(1), m.group(2)
        fields = (qualified or {}).get(pkg, {}).get(name) if pkg else types.get(name)
        if fields is None:
            continue
        before = s[:m.start()].rstrip()
        if before.endswith("]") or before.endswith("]*"):
            continue  # an element type: []T{...}, map[K]T{...}
        if re.search(r"\b(type|struct)\s*$", before):
            continue
        end = match_brace(s, m.end() - 1)
        elems = split_top(s[m.end():end])
        line = s.count("\n", 0, m.start()) + 1
        where = "%s:%d: %s{...}" % (path, line, (pkg + "." if pkg else "") + name)
        keyed = [top_colon(e) for e in elems]
        if any(keyed) and not all(keyed):
            findings.append("%s: mixed keyed and positional elements" % where)
        elif all(keyed):
            for e in elems:
                k = e.split(":", 1)[0].strip()
                if k not in fields:
                    findings.append("%s: unknown field %r (declared: %s)" % (where, k, ", ".join(fields)))
        elif elems:
            if len(fields) > 1:
                findings.append("%s: positional literal of a %d-field struct (%d values): use keyed fields"
                                % (where, len(fields), len(elems)))
            if len(elems) != len(fields):
                findings.append("%s: %d values for %d fields" % (where, len(elems), len(fields)))
    return findings


def lint_tree(root):
    """Lint every package directory under root (go/src)."""
    pkgs = {}
    for d, _, files in os.walk(root):
        gos = sorted(f for f in files if f.endswith(".go"))
        if gos:
            srcs = {os.path.join(d, f): open(os.path.join(d, f)).read() for f in gos}
            types = {}
            for src in srcs.values():
                types.update(struct_fields(src))
            pkgs[os.path.basename(d)] = (srcs, types)
    qualified = {p: t for p, (_, t) in pkgs.items()}
    findings = []
    for p, (srcs, types) in pkgs.items():
        for path, src in srcs.items():
            findings += lint_source(src, types, qualified, os.path.relpath(path, os.path.dirname(os.path.dirname(root))))
    return findings, {p: sorted(t) for p, (_, t) in pkgs.items()}


if __name__ == "__main__":
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "go", "src")
    f, _ = lint_tree(root)
    print("\n".join(f) or "go_lint: no findings")
    sys.exit(1 if f else 0)
