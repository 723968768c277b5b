"""PARITY.md's test column resolves: every cited test file, example, tool and profile exists and every cited test
name is defined in tests/ (tools/check_parity.py)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parity_md_citations_resolve():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_parity.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
