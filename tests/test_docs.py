"""DESIGN.md's measured numbers are generated from the committed profiles
(tools/design_numbers.py): the block between its markers must be current."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_design_numbers_block_is_current():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "design_numbers.py")], check=True,
                         capture_output=True, text=True).stdout
    with open(os.path.join(ROOT, "DESIGN.md")) as f:
        doc = f.read()
    a = doc.index("<!-- numbers:begin -->") + len("<!-- numbers:begin -->")
    b = doc.index("<!-- numbers:end -->")
    assert doc[a:b].strip() == out.strip(), "run: python tools/design_numbers.py --write"
