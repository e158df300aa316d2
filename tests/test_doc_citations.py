"""Evidence the docs cite is in the tree: every repository path quoted in backticks in README.md, docs/*.md and
profiles/*.md exists, and none points into the scratch directory gpurun_out/ (kept out of history; the numbers
quoted from it are copied under profiles/)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIRS = ("profiles", "tools", "docs", "configs", "csrc", "tests", "homebrewnlp_mtf_amd")


def _docs():
    return [os.path.join(ROOT, "README.md")] + glob.glob(os.path.join(ROOT, "docs", "*.md")) + \
        glob.glob(os.path.join(ROOT, "profiles", "*.md"))


def _braces(ref):
    """a{b,c}d -> [abd, acd] (one level)"""
    m = re.search(r"\{([^{}]*)\}", ref)
    if not m:
        return [ref]
    return [ref[:m.start()] + alt + ref[m.end():] for alt in m.group(1).split(",")]


def test_cited_paths_exist():
    missing = []
    for doc in _docs():
        with open(doc) as f:
            text = f.read()
        for ref in set(re.findall(r"`((?:%s)/[A-Za-z0-9_./*{},-]+)" % "|".join(DIRS), text)):
            ref = ref.rstrip(".:,")
            for alt in _braces(ref):
                # a `*` cites a family of files: at least one must exist
                if not glob.glob(os.path.join(ROOT, alt)):
                    missing.append(f"{os.path.relpath(doc, ROOT)} -> {alt}")
    assert not missing, missing


def test_no_citation_of_scratch_outputs():
    bad = []
    for doc in _docs():
        with open(doc) as f:
            for n, line in enumerate(f, 1):
                if "gpurun_out/" in line:
                    bad.append(f"{os.path.relpath(doc, ROOT)}:{n}")
    assert not bad, bad
