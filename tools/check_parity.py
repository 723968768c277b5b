#!/usr/bin/env python3
"""Check PARITY.md's test column against the tree: every cited test file / example / tool / profile must exist, and
every cited test name (`test_foo`, `test_foo_*`, `file.py::test_foo`, parametrised `test_foo[2,3]`) must be defined
by a test function in tests/. A row citing nothing (an em dash) is only allowed for the non-goal / not-built IDs.

    python tools/check_parity.py [PARITY.md]    -> exit 0 when every citation resolves, else prints the misses"""
from __future__ import annotations

import fnmatch
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# rows whose test cell may be empty: SURVEY §7.5 non-goals and components that are documented as not built
NO_TEST_OK = {"C22", "C30", "C31", "C40", "C47", "C56", "C59", "N11", "N12", "N16", "N17"}


def _test_names():
    names = set()
    for d in ("tests",):
        for dirpath, _, files in os.walk(os.path.join(ROOT, d)):
            for f in files:
                if f.endswith(".py"):
                    with open(os.path.join(dirpath, f), encoding="utf-8") as fh:
                        names.update(re.findall(r"^\s*def (test_\w+)\s*\(", fh.read(), re.M))
    return names


def _rows(text):
    for line in text.splitlines():
        if not line.startswith("| ") or line.startswith("|---") or line.startswith("| ID ") or line.startswith("| Subsystem "):
            continue
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        yield cells[0], cells[-1]


def check(path):
    text = open(path, encoding="utf-8").read()
    names = _test_names()
    problems = []
    for rid, cell in _rows(text):
        if cell in ("—", "-", ""):
            if rid not in NO_TEST_OK:
                problems.append(f"{rid}: no test cited")
            continue
        for ref in re.findall(r"`([^`]+)`", cell):
            ref = ref.split(" ")[0]
            file_part, _, test_part = ref.partition("::")
            if re.search(r"\.(py|md|json|jsonl|csv|yaml|sh)$", file_part) or "/" in file_part:
                if re.match(r"^(tests|tools|examples|profiles)/", file_part):
                    hits = [p for p in _glob(file_part)]
                    if not hits:
                        problems.append(f"{rid}: missing file {file_part}")
                if test_part:
                    _check_name(rid, test_part, names, problems)
                continue
            if ref.startswith("test_"):
                _check_name(rid, ref, names, problems)
    return problems


def _glob(rel):
    import glob

    return glob.glob(os.path.join(ROOT, rel.rstrip("*") + ("*" if rel.endswith("*") else "")))


def _check_name(rid, ref, names, problems):
    base = re.sub(r"\[.*$", "", ref)
    if "*" in base:
        if not any(fnmatch.fnmatch(n, base) for n in names):
            problems.append(f"{rid}: no test matches {ref}")
    elif base not in names:
        problems.append(f"{rid}: no test named {ref}")


def main(argv):
    path = argv[1] if len(argv) > 1 else os.path.join(ROOT, "PARITY.md")
    problems = check(path)
    for p in problems:
        print(p)
    print(f"{len(problems)} unresolved citation(s)")
    return 1 if problems else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
