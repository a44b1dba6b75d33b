"""The library's environment switches: every `getenv("ZH_…")` /
`env_int("ZH_…")` site in zarr-java_amd/csrc is a switch listed in DESIGN.md's switch table,
there are fewer than 15 of them, and each one is set to a non-default value by some GPU test
(so no non-default path is product code without coverage)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zarr-java_amd", "csrc")


def csrc_switches():
    names = set()
    for p in glob.glob(os.path.join(CSRC, "*")):
        if not p.endswith((".cpp", ".hip", ".h")):
            continue
        text = open(p, encoding="utf-8").read()
        names |= set(re.findall(r'(?:getenv|env_int)\(\s*"(ZH_[A-Z0-9_]+)"', text))
    return names


def design_table():
    text = open(os.path.join(ROOT, "DESIGN.md"), encoding="utf-8").read()
    sec = text.split("### Tuning switches", 1)[1].split("\n## ", 1)[0]
    return set(re.findall(r"^\| `(ZH_[A-Z0-9_]+)`", sec, flags=re.M))


def test_every_switch_is_in_design_table_and_few():
    got = csrc_switches()
    table = design_table()
    assert got, "no switch found: the scan is broken"
    assert got <= table, f"switches missing from DESIGN.md's table: {sorted(got - table)}"
    assert table <= got, f"DESIGN.md lists switches the library no longer reads: {sorted(table - got)}"
    assert len(got) < 15, sorted(got)


def test_every_switch_has_a_gpu_test_setting_it():
    tests = ""
    for p in glob.glob(os.path.join(ROOT, "tests", "*.py")):
        t = open(p, encoding="utf-8").read()
        if "pytest.mark.gpu" in t:
            tests += t
    missing = []
    for name in sorted(csrc_switches()):
        if not re.search(rf'setenv\(\s*"{name}"|"{name}":\s*|{name}=', tests):
            missing.append(name)
    assert not missing, f"switches no GPU test sets: {missing}"
