"""Every script path a lab / GPU shell script under tools/ names (tools/<...>.py|.sh) exists in the tree."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tool_scripts_reference_existing_files():
    missing = []
    for sh in glob.glob(os.path.join(ROOT, "tools", "**", "*.sh"), recursive=True):
        with open(sh) as f:
            text = f.read()
        for ref in set(re.findall(r"tools/[A-Za-z0-9_/]+\.(?:py|sh)", text)):
            if not os.path.exists(os.path.join(ROOT, ref)):
                missing.append(f"{os.path.relpath(sh, ROOT)} -> {ref}")
    assert not missing, missing
