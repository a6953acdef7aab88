"""Lint gate (the reference ships `.pylintrc` with fail-under=10 and a pylint `dev` extra,
/root/reference/.pylintrc:9, /root/reference/setup.py:11-15).

tools/lint.py enforces the core rules with the standard library; pylint and ruff run as well
when this environment has them (it does not, so those two checks are skipped here)."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import lint  # noqa: E402


def test_repository_is_lint_clean():
    cwd = os.getcwd()
    os.chdir(ROOT)
    try:
        findings = lint.lint_paths()
    finally:
        os.chdir(cwd)
    assert not findings, "\n".join(f"{p}:{n}: {c} {m}" for p, n, c, m in findings)


@pytest.mark.parametrize("src,code", [
    ("import os\n", "F401"),
    ('"""d"""\ntry:\n    pass\nexcept:\n    pass\n', "E722"),
    ('"""d"""\ndef f(a=[]):\n    return a\n', "B006"),
    ('"""d"""\nx = 1\nif x == None:\n    pass\n', "E711"),
    ('"""d"""\nx = f"abc"\n', "F541"),
    ('"""d"""\nx = 1 \n', "W291"),
    ('"""d"""\nx = "' + "a" * 130 + '"\n', "E501"),
    ('"""d"""\ndef f():\n    pass\ndef f():\n    pass\n', "F811"),
    ('"""d"""\nx = 1\nx == 2\n', "B018"),
    ("x = (\n", "E999"),
])
def test_lint_catches(src, code):
    codes = [c for _, _, c, _ in lint.lint_source("torchkafka_amd/mod.py", src)]
    assert code in codes, codes


def test_noqa_exempts():
    assert not lint.lint_source("tests/x.py", "import os  # noqa: F401\n")


@pytest.mark.skipif(importlib.util.find_spec("ruff") is None, reason="ruff not installed in this image")
def test_ruff_clean():
    subprocess.run([sys.executable, "-m", "ruff", "check", "."], cwd=ROOT, check=True)


@pytest.mark.skipif(importlib.util.find_spec("pylint") is None, reason="pylint not installed in this image")
def test_pylint_fail_under():
    subprocess.run([sys.executable, "-m", "pylint", "--rcfile", ".pylintrc", "torchkafka_amd"], cwd=ROOT, check=True)
