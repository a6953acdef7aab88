"""Dependency-free lint gate (the reference gates on pylint, /root/reference/.pylintrc:9 fail-under=10).

pylint/ruff are configured in `.pylintrc` / `ruff.toml` for environments that have them; this
image has neither, so the same core rules are enforced here with the standard library's `ast`
and `tokenize`, and `tests/test_lint.py` fails the suite on any finding:

  E999 syntax error                     F401 unused import (outside __init__ re-exports)
  E722 bare ``except:``                 B006 mutable default argument
  E711 comparison to None with ==/!=    F541 f-string without placeholders
  E501 line longer than 120             W291 trailing whitespace / W191 tab indentation
  D100 missing module docstring (package modules)
  F811 duplicate top-level def/class    B018 useless expression statement

A line ending in ``# noqa`` (optionally ``# noqa: CODE``) is exempt, as with flake8/ruff.

Usage: ``python tools/lint.py [paths...]`` -> prints findings, exit 1 if any.
"""
from __future__ import annotations

import ast
import io
import os
import re
import sys
import tokenize

MAX_LINE = 120
DEFAULT_PATHS = ("torchkafka_amd", "torchkafka", "bench.py", "__graft_entry__.py", "setup.py", "tools",
                 "tests", "examples", "benchmarks")
SKIP_DIRS = {"__pycache__", "build", ".hypothesis", "bin", "gpurun_out"}
_NOQA = re.compile(r"#\s*noqa(?::\s*([A-Z0-9, ]+))?\s*$")


def _iter_files(paths):
    for p in paths:
        if os.path.isfile(p) and p.endswith(".py"):
            yield p
        elif os.path.isdir(p):
            for root, dirs, files in os.walk(p):
                dirs[:] = sorted(d for d in dirs if d not in SKIP_DIRS)
                for f in sorted(files):
                    if f.endswith(".py"):
                        yield os.path.join(root, f)


class _Names(ast.NodeVisitor):
    """Every identifier read anywhere in the module (names, attribute roots, string annotations)."""

    def __init__(self):
        self.used = set()

    def visit_Name(self, node):
        self.used.add(node.id)

    def visit_Attribute(self, node):
        root = node
        while isinstance(root, ast.Attribute):
            root = root.value
        if isinstance(root, ast.Name):
            self.used.add(root.id)
        self.generic_visit(node)

    def visit_Constant(self, node):
        # names inside string annotations / __all__ entries
        if isinstance(node.value, str) and node.value.replace(".", "").replace("_", "").isalnum():
            self.used.add(node.value.split(".")[0])


def _noqa(lines, lineno, code):
    if not 1 <= lineno <= len(lines):
        return False
    m = _NOQA.search(lines[lineno - 1])
    if not m:
        return False
    return m.group(1) is None or code in {c.strip() for c in m.group(1).split(",")}


def lint_source(path: str, src: str) -> list:
    out = []
    lines = src.splitlines()

    def add(lineno, code, msg):
        if not _noqa(lines, lineno, code):
            out.append((path, lineno, code, msg))

    try:
        tree = ast.parse(src, filename=path)
    except SyntaxError as e:
        return [(path, e.lineno or 0, "E999", f"syntax error: {e.msg}")]

    base = os.path.basename(path)
    is_init = base == "__init__.py"
    in_pkg = path.replace(os.sep, "/").split("/")[0] in ("torchkafka_amd", "torchkafka")

    # ---- physical lines
    for i, line in enumerate(lines, 1):
        if len(line) > MAX_LINE:
            add(i, "E501", f"line too long ({len(line)} > {MAX_LINE})")
        if line.rstrip() != line:
            add(i, "W291", "trailing whitespace")
        if line.startswith("\t"):
            add(i, "W191", "indentation contains tabs")

    # f-strings without placeholders: tokenizer view (ast merges JoinedStr parts)
    try:
        for tok in tokenize.generate_tokens(io.StringIO(src).readline):
            if tok.type == tokenize.STRING:
                s = tok.string
                prefix = s[: len(s) - len(s.lstrip("rRbBuUfF"))].lower()
                if "f" in prefix and "{" not in s:
                    add(tok.start[0], "F541", "f-string without any placeholders")
    except tokenize.TokenError:
        pass

    if in_pkg and not is_init and ast.get_docstring(tree) is None and src.strip():
        add(1, "D100", "missing module docstring")

    # ---- imports
    names = _Names()
    names.visit(tree)
    exported = set()
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            if isinstance(node.value, (ast.List, ast.Tuple)):
                exported |= {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
    if not is_init:
        for node in ast.walk(tree):
            if isinstance(node, (ast.Import, ast.ImportFrom)):
                if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                    continue
                for a in node.names:
                    if a.name == "*":
                        continue
                    bound = a.asname or a.name.split(".")[0]
                    if bound not in names.used and bound not in exported:
                        add(node.lineno, "F401", f"'{a.name}' imported but unused")

    # ---- statements
    top_defs = {}
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            if node.name in top_defs and not node.decorator_list:
                add(node.lineno, "F811", f"redefinition of '{node.name}' from line {top_defs[node.name]}")
            top_defs[node.name] = node.lineno
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            add(node.lineno, "E722", "bare 'except:'")
        elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
            for d in list(node.args.defaults) + [d for d in node.args.kw_defaults if d is not None]:
                if isinstance(d, (ast.List, ast.Dict, ast.Set)) or (
                        isinstance(d, ast.Call) and isinstance(d.func, ast.Name)
                        and d.func.id in ("list", "dict", "set")):
                    add(d.lineno, "B006", "mutable default argument")
        elif isinstance(node, ast.Compare):
            for op, right in zip(node.ops, node.comparators):
                if isinstance(op, (ast.Eq, ast.NotEq)) and isinstance(right, ast.Constant) and right.value is None:
                    add(node.lineno, "E711", "comparison to None (use 'is' / 'is not')")
        elif isinstance(node, ast.Expr):
            v = node.value
            if isinstance(v, (ast.Name, ast.Compare, ast.BinOp)) or (
                    isinstance(v, ast.Attribute) and not isinstance(v.ctx, ast.Store)):
                add(node.lineno, "B018", "useless expression statement")
    return out


def lint_paths(paths=DEFAULT_PATHS) -> list:
    findings = []
    for f in _iter_files(paths):
        with open(f, encoding="utf-8") as fh:
            findings += lint_source(os.path.relpath(f), fh.read())
    return findings


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    findings = lint_paths(argv or DEFAULT_PATHS)
    for path, line, code, msg in findings:
        print(f"{path}:{line}: {code} {msg}")
    print(f"{len(findings)} finding(s)", file=sys.stderr)
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main())
