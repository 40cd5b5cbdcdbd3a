"""The library's environment switches: the variables the sources read with
getenv and the ones the switch table documents are the same set, at most 18 of them
(round 5's verdict: the knob count had regrown to 26 while the table said ten)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gaplac_amd", "csrc")


def read_switches():
    found = set()
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".h")):
            with open(os.path.join(CSRC, name)) as f:
                found |= set(re.findall(r'getenv\("(GAPLAC_[A-Z0-9_]+)"\)', f.read()))
    return found


def documented_switches():
    with open(os.path.join(ROOT, "DESIGN.md")) as f:
        text = f.read()
    sec = text[text.index("### 4.1 Switches"):text.index("## 5. Oracle and parity")]
    table = [ln for ln in sec.splitlines() if ln.startswith("| `GAPLAC_")]
    return {re.match(r"\| `(GAPLAC_[A-Z0-9_]+)`", ln).group(1) for ln in table}


def test_switch_table_matches_sources():
    src, doc = read_switches(), documented_switches()
    assert src == doc, {"read but not documented": sorted(src - doc), "documented but not read": sorted(doc - src)}


def test_switch_count_bounded():
    assert len(read_switches()) <= 18, sorted(read_switches())
