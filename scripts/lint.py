#!/usr/bin/env python3
"""Static checks for the Python tree (the reference's ``go vet`` + golangci-lint
role, ``Makefile:30-45``, ``.golangci.yml:8-19``), with no third-party linter
needed (none is installed in the build image; ``pyproject.toml`` also configures
ruff / mypy for environments that have them).

Checks (``# noqa`` on a line silences it):
  F401  imported name never used (``__init__`` re-exports and ``__all__`` excepted)
  F811  a function / class defined twice in the same scope
  B006  mutable default argument ([], {}, set())
  F541  f-string without placeholders
  E501  line longer than 110 characters
  W291  trailing whitespace
  E722  bare ``except:``
  E999  syntax error

Usage: python scripts/lint.py [paths...]   (default: the package, tests,
scripts, bench.py, __graft_entry__.py); exit 1 when anything is reported.
"""
from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_LINE = 110
DEFAULT = ["loqa_hub_amd", "tests", "scripts", "bench.py", "__graft_entry__.py"]


def _files(paths):
    for p in paths:
        p = os.path.join(ROOT, p) if not os.path.isabs(p) else p
        if os.path.isfile(p) and p.endswith(".py"):
            yield p
        for d, dirs, fs in os.walk(p):
            # scripts/exp: one-off measurement scratch (kept for the record)
            dirs[:] = [x for x in dirs if x not in ("__pycache__", "build", ".git", "exp")]
            for f in sorted(fs):
                if f.endswith(".py"):
                    yield os.path.join(d, f)


class _Names(ast.NodeVisitor):
    def __init__(self):
        self.used: set[str] = set()

    def visit_Name(self, n):
        self.used.add(n.id)

    def visit_Attribute(self, n):
        root = n
        while isinstance(root, ast.Attribute):
            root = root.value
        if isinstance(root, ast.Name):
            self.used.add(root.id)
        self.generic_visit(n)


def _string_names(tree) -> set[str]:
    """Names mentioned in string annotations / __all__ (kept as used)."""
    out = set()
    for n in ast.walk(tree):
        if isinstance(n, ast.Constant) and isinstance(n.value, str) and len(n.value) < 200:
            for tok in n.value.replace("[", " ").replace("]", " ").replace(",", " ").replace(
                    "|", " ").replace(".", " ").split():
                if tok.isidentifier():
                    out.add(tok)
    return out


def check_file(path: str) -> list[str]:
    rel = os.path.relpath(path, ROOT)
    src = open(path, encoding="utf-8").read()
    lines = src.splitlines()
    out = []

    def report(line: int, code: str, msg: str) -> None:
        if 0 < line <= len(lines) and "noqa" in lines[line - 1]:
            return
        out.append(f"{rel}:{line}: {code} {msg}")
    try:
        tree = ast.parse(src, rel)
    except SyntaxError as e:
        return [f"{rel}:{e.lineno}: E999 {e.msg}"]
    for i, ln in enumerate(lines, 1):
        if len(ln) > MAX_LINE:
            report(i, "E501", f"line too long ({len(ln)} > {MAX_LINE})")
        if ln != ln.rstrip():
            report(i, "W291", "trailing whitespace")
    # unused imports (module scope)
    if not rel.endswith("__init__.py"):
        names = _Names()
        names.visit(tree)
        used = names.used | _string_names(tree)
        for node in tree.body:
            if isinstance(node, (ast.Import, ast.ImportFrom)):
                if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                    continue
                for a in node.names:
                    nm = (a.asname or a.name).split(".")[0]
                    if nm != "*" and nm not in used:
                        report(node.lineno, "F401", f"'{a.name}' imported but unused")
    specs = {id(n.format_spec) for n in ast.walk(tree)
             if isinstance(n, ast.FormattedValue) and n.format_spec is not None}
    for node in ast.walk(tree):
        # redefinitions in one scope
        body = getattr(node, "body", None)
        if isinstance(body, list):
            seen: dict[str, int] = {}
            for st in body:
                if isinstance(st, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
                    decos = [ast.unparse(d) for d in getattr(st, "decorator_list", [])]
                    if any("overload" in d or ".setter" in d or ".deleter" in d for d in decos):
                        continue
                    if st.name in seen:
                        report(st.lineno, "F811", f"redefinition of '{st.name}' from line {seen[st.name]}")
                    seen[st.name] = st.lineno
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            for d in node.args.defaults + node.args.kw_defaults:
                if isinstance(d, (ast.List, ast.Dict, ast.Set)):
                    report(d.lineno, "B006", "mutable default argument")
        if isinstance(node, ast.JoinedStr) and id(node) not in specs and \
                not any(isinstance(v, ast.FormattedValue) for v in node.values):
            report(node.lineno, "F541", "f-string without placeholders")
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            report(node.lineno, "E722", "bare 'except:'")
    return out


def main(argv=None) -> int:
    paths = (argv if argv is not None else sys.argv[1:]) or DEFAULT
    problems = []
    n = 0
    for f in _files(paths):
        n += 1
        problems += check_file(f)
    for p in problems:
        print(p)
    print(f"lint: {n} files, {len(problems)} problems", file=sys.stderr)
    return 1 if problems else 0


if __name__ == "__main__":
    sys.exit(main())
