"""The C ABI library loads (no GPU needed) and exports every symbol include/gmz.h declares."""
import os
import re

from conftest import REPO


def test_library_exports_every_header_symbol():
    import datou_gomoku_muzero_amd._lib as L
    import datou_gomoku_muzero_amd.network  # noqa: F401  (registers the gmz_net_* signatures)
    lib = L.load()
    hdr = open(os.path.join(REPO, "include", "gmz.h")).read()
    names = re.findall(r"^\s*(?:int|const char \*)\s*(gmz_\w+)\(", hdr, re.M)
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.gmz_abi_version() == 9


def test_product_package_never_imports_oracle():
    """Only tests/, smoke() and bench.py's cpu_baseline may touch oracle/ (the checker)."""
    pkg = os.path.join(REPO, "datou-gomoku-muzero_amd")
    bad = re.compile(r"\bimport oracle\b|from oracle\b|gmz_oracle|\bnetref\b|\bimport hashnet\b")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                assert not bad.search(open(os.path.join(root, f)).read()), f
