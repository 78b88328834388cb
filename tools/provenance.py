"""Provenance of measured profiles: a hash of the product sources a measurement depends on.

The GPU box receives the tree without .git, so profiles cannot carry a usable git head at measurement time.
Instead every profile summary written by tools/pmc_summary.py / tools/stress_hbm.py / tools/train_summary.py
records `code_hash()` of the tree it measured, and bench.py promotes a committed profile only when its hash
equals the hash of the code it is running (otherwise the line says "stale": true).

usage: python tools/provenance.py          (prints the hash of this tree)
"""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "collaborative_nonstationary_multivariate_gaussian_process_amd"


def source_files(root=ROOT):
    """The HIP sources, the C ABI header and the package's Python (what a kernel trace of bench.py measures)."""
    out = []
    for base, exts in ((os.path.join(PKG, "csrc"), (".hip", ".hpp", "Makefile")), ("include", (".h",)),
                       (PKG, (".py",)), (os.path.join(PKG, "Utility"), (".py",))):
        d = os.path.join(root, base)
        if not os.path.isdir(d):
            continue
        for f in sorted(os.listdir(d)):
            if f.endswith(exts) and os.path.isfile(os.path.join(d, f)):
                out.append(os.path.join(base, f))
    return out


def code_hash(root=ROOT):
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.encode())
        with open(os.path.join(root, rel), "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(code_hash())
